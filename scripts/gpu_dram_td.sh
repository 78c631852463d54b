#!/usr/bin/env bash
# 299-cell TestData DRAM fit timing per library variant, two interleaved repeats (no profiler).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${1:-dtd}"; STEPS="${2:-20000}"
mkdir -p "$OUT"; cd "$ROOT"
for rep in 1 2; do
  for v in ${VARIANTS:-main}; do
    lib=""; [ "$v" = main ] || lib="$ROOT/build/ab/libtci_$v.so"
    TCI_LIB="$lib" timeout -k 10 200 python3 scripts/dram_time.py "$STEPS" auto 20 > "$OUT/${TAG}_${v}_$rep.json" 2>/dev/null || exit $?
    echo "$v $rep $(python3 -c "import json;print(round(json.load(open('$OUT/${TAG}_${v}_$rep.json'))['us_per_step'],3))")"
  done
done
