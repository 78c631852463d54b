#!/usr/bin/env bash
# rocprofv3 kernel stats of the DRAM fit for the shipped build and the build/ab adaptation ablations.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${1:-dab}"; STEPS="${2:-20000}"
mkdir -p "$OUT"; cd /tmp; export TMPDIR=/tmp
for v in ${VARIANTS:-ship adapt_nochol adapt_nocov}; do
  lib=""; [ "$v" = ship ] || lib="$ROOT/build/ab/libtci_$v.so"
  TCI_LIB="$lib" timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_$v" -o trace -- \
    python3 "$ROOT/scripts/dram_time.py" "$STEPS" auto 20 > "$OUT/${TAG}_$v.json" 2> "$OUT/${TAG}_$v.err" || exit $?
  cat "$OUT/${TAG}_$v.json"
done
