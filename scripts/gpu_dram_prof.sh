#!/usr/bin/env bash
# rocprofv3 kernel statistics of the 299-cell DRAM fit (20k steps by default) for library variants
# (VARIANTS: "main" = the in-tree build, or build/ab/libtci_<name>.so).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${1:-dprof}"; STEPS="${2:-20000}"
mkdir -p "$OUT"; cd /tmp; export TMPDIR=/tmp
for v in ${VARIANTS:-main}; do
  lib=""; [ "$v" = main ] || lib="$ROOT/build/ab/libtci_$v.so"
  TCI_LIB="$lib" timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_$v" -o trace -- \
    python3 "$ROOT/scripts/dram_time.py" "$STEPS" auto 20 > "$OUT/${TAG}_$v.json" 2> "$OUT/${TAG}_$v.err" || exit $?
  echo "== $v"; cat "$OUT/${TAG}_$v.json"
  f=$(find "$OUT/${TAG}_$v" -name "*kernel_stats.csv" | head -1); cut -d, -f1-5 "$f" | cut -c1-160 | head -12
done
