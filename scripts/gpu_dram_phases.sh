#!/usr/bin/env bash
# DRAM fit timing: rocprofv3 kernel stats of the shipped build, then the phase-stamp variants
# (build/ab/libtci_{chainprof,adaptprof}.so: s_memtime cycles per k_chain / k_adapt_mfma phase).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${1:-dph}"; STEPS="${2:-20000}"
mkdir -p "$OUT"; cd /tmp; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_ship" -o trace -- \
  python3 "$ROOT/scripts/dram_time.py" "$STEPS" auto 20 > "$OUT/${TAG}_ship.json" 2> "$OUT/${TAG}_ship.err" || exit $?
cat "$OUT/${TAG}_ship.json"
for v in ${VARIANTS:-chainprof adaptprof}; do
  TCI_LIB="$ROOT/build/ab/libtci_$v.so" timeout -k 10 200 python3 "$ROOT/scripts/dram_time.py" "$STEPS" auto 20 \
    > "$OUT/${TAG}_$v.json" 2> "$OUT/${TAG}_$v.err" || exit $?
  cat "$OUT/${TAG}_$v.json"; grep cycles "$OUT/${TAG}_$v.err"
done
exit 0
