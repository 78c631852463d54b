#!/usr/bin/env bash
# Round 4: k_chain with the record / s2 waves' work ahead of the evaluation (early) against main:
# kernel stats of the TestData fit (20k steps), then bitwise equality with main.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
VARIANTS="main early main early" bash scripts/gpu_dram_prof.sh r04early 20000 || exit $?
cd "$ROOT"
timeout -k 10 200 python3 scripts/dram_lib_equal.py main "$ROOT/build/ab/libtci_early.so" 2000 299 0 > "$OUT/r04early_eq.json" 2>&1 || exit $?
cat "$OUT/r04early_eq.json"
