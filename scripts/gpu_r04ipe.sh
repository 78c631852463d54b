#!/usr/bin/env bash
# Round 4: k_walk the 1/s2 division ahead of the stage-1 evaluation (ipe) against main: kernel
# stats of the config-4 fit (10,000 chains, 1k steps), then bitwise equality (WALK on TestData and
# config-4 cells).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
WORK=syn4 VARIANTS="main ipe main ipe" bash scripts/gpu_dram_prof.sh r04ipe 1000 || exit $?
cd "$ROOT"
TCI_ENGINE=walk timeout -k 10 200 python3 scripts/dram_lib_equal.py main "$ROOT/build/ab/libtci_ipe.so" 2000 40 0 > "$OUT/r04ipe_eq_td.json" 2>&1 || exit $?
TCI_ENGINE=walk timeout -k 10 300 python3 scripts/dram_lib_equal.py main "$ROOT/build/ab/libtci_ipe.so" 1000 64 4 > "$OUT/r04ipe_eq_cfg4.json" 2>&1 || exit $?
cat "$OUT/r04ipe_eq_td.json" "$OUT/r04ipe_eq_cfg4.json"
