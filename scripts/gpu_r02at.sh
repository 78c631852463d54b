#!/usr/bin/env bash
# Round-2 A/B of k_adapt_gt's scatter: 10 tiles per wave and pass (2 passes over the window at
# P = 257 instead of 3) and window loads in flight per thread, on the 250-point config-4-style fit.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TCI_SYNTH_POINTS=250 timeout -k 10 300 python3 scripts/dram_lib_equal.py main build/ab/libtci_gtt10p4.so 300 300 4 > "$OUT/r02at_eq_250.json" 2>&1 || exit $?
cat "$OUT/r02at_eq_250.json"
for v in main gtt10p4 gtt10 gtper4 main gtt10p4 gtt10 gtper4; do
  lib=""; [ "$v" = main ] || lib="$ROOT/build/ab/libtci_$v.so"
  TCI_LIB="$lib" TCI_SYNTH_POINTS=250 timeout -k 10 300 python3 scripts/synth_dram_time.py 4 1000 > "$OUT/r02at_250_$v.json" 2> "$OUT/r02at_250_$v.err" || exit $?
  echo "== 250 $v"; cut -c300-420 "$OUT/r02at_250_$v.json"
done
