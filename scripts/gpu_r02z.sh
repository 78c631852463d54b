#!/usr/bin/env bash
# Round-2 A/B of the draws-pass R address space and the long-row adaptation's batched loads:
# bitwise equality against the previous commit's build, then fit timings per library.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
P=build/ab/libtci_prev.so
timeout -k 10 200 python3 scripts/dram_lib_equal.py main $P 2000 80 0 > "$OUT/r02z_eq_td.json" 2>&1 || exit $?
timeout -k 10 300 python3 scripts/dram_lib_equal.py main $P 300 400 5 > "$OUT/r02z_eq_c5.json" 2>&1 || exit $?
TCI_SYNTH_POINTS=250 timeout -k 10 300 python3 scripts/dram_lib_equal.py main $P 300 300 4 > "$OUT/r02z_eq_250.json" 2>&1 || exit $?
cat "$OUT"/r02z_eq_*.json
VARIANTS="main prev drawsflat main prev" bash scripts/gpu_dram_libs.sh r02z 20000 1000 > "$OUT/r02z_libs.log" 2>&1 || exit $?
for v in main prev gt1 gt4 main prev; do
  lib=""; [ "$v" = main ] || lib="$ROOT/build/ab/libtci_$v.so"
  TCI_LIB="$lib" TCI_SYNTH_POINTS=250 timeout -k 10 300 python3 scripts/synth_dram_time.py 4 1000 > "$OUT/r02z_250_$v.json" 2> "$OUT/r02z_250_$v.err" || exit $?
  echo "== 250 $v"; cut -c1-60,300-420 "$OUT/r02z_250_$v.json"
done
