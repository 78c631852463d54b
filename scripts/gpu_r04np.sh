#!/usr/bin/env bash
# Round 4: fused-engine draws passes per workgroup (np1/np3/np4 against main = 2): kernel stats of
# the 299-cell TestData fit (20k steps), then bitwise equality of each variant with main.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
VARIANTS="main np1 np3 np4 main" bash scripts/gpu_dram_prof.sh r04np 20000 || exit $?
cd "$ROOT"
for v in np1 np3 np4; do
  timeout -k 10 200 python3 scripts/dram_lib_equal.py main "$ROOT/build/ab/libtci_$v.so" 2000 40 0 > "$OUT/r04np_eq_$v.json" 2>&1 || exit $?
  cat "$OUT/r04np_eq_$v.json"
done
