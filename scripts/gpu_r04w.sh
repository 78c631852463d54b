#!/usr/bin/env bash
# Round 4: WALK draws passes per workgroup (w1/w2 against main = 4): kernel stats of the config-4
# fit (10,000 chains, 1k steps), then bitwise equality on config-4 cells.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
WORK=syn4 VARIANTS="main w1 w2 main" bash scripts/gpu_dram_prof.sh r04w 1000 || exit $?
cd "$ROOT"
for v in w1 w2; do
  TCI_ENGINE=walk timeout -k 10 300 python3 scripts/dram_lib_equal.py main "$ROOT/build/ab/libtci_$v.so" 1000 64 4 > "$OUT/r04w_eq_$v.json" 2>&1 || exit $?
  cat "$OUT/r04w_eq_$v.json"
done
