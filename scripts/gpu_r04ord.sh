#!/usr/bin/env bash
# Round 4: k_adapt_mfma workgroup order (o1 longest rows first, o2 with the CU-sharing chains paired
# among the shortest rows) against main: kernel stats of the TestData fit (20k steps), then bitwise
# equality with main.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
VARIANTS="main o1 o2 main o2" bash scripts/gpu_dram_prof.sh r04ord 20000 || exit $?
cd "$ROOT"
for v in o1 o2; do
  timeout -k 10 200 python3 scripts/dram_lib_equal.py main "$ROOT/build/ab/libtci_$v.so" 2000 299 0 > "$OUT/r04ord_eq_$v.json" 2>&1 || exit $?
  cat "$OUT/r04ord_eq_$v.json"
done
