#!/usr/bin/env bash
# End-to-end DRAM fit timing per library variant (no profiler): the 299-cell TestData fit and the
# config-4/5 synthetic fits. VARIANTS: names of build/ab/libtci_<name>.so ("main" = in-tree build).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${1:-dlibs}"; STEPS="${2:-20000}"; SSTEPS="${3:-1000}"
mkdir -p "$OUT"; cd "$ROOT"
for v in ${VARIANTS:-main}; do
  lib=""; [ "$v" = main ] || lib="$ROOT/build/ab/libtci_$v.so"
  echo "== $v"
  TCI_LIB="$lib" timeout -k 10 200 python3 scripts/dram_time.py "$STEPS" auto 20 > "$OUT/${TAG}_${v}_td.json" 2> "$OUT/${TAG}_${v}_td.err" || exit $?
  cat "$OUT/${TAG}_${v}_td.json"
  TCI_LIB="$lib" timeout -k 10 300 python3 scripts/synth_dram_time.py 4 "$SSTEPS" 5 "$SSTEPS" > "$OUT/${TAG}_${v}_syn.json" 2> "$OUT/${TAG}_${v}_syn.err" || exit $?
  cat "$OUT/${TAG}_${v}_syn.json"
done
