#!/usr/bin/env bash
# Long-row adaptation (k_adapt_gt) variants on the 250-point config-4-style fit, plus bitwise check.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TCI_SYNTH_POINTS=250 timeout -k 10 300 python3 scripts/dram_lib_equal.py main build/ab/libtci_prev.so 300 300 4 > "$OUT/r02aa_eq_250.json" 2>&1 || exit $?
cat "$OUT/r02aa_eq_250.json"
for v in ${VARIANTS:-main prev gtper1 gtper4 gtmg2 grp2 grp7 main prev}; do
  lib=""; [ "$v" = main ] || lib="$ROOT/build/ab/libtci_$v.so"
  TCI_LIB="$lib" TCI_SYNTH_POINTS=250 timeout -k 10 300 python3 scripts/synth_dram_time.py 4 1000 > "$OUT/r02aa_250_$v.json" 2> "$OUT/r02aa_250_$v.err" || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('$v', round(d['us_per_step'],1))" "$OUT/r02aa_250_$v.json"
done
