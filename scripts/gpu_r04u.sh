#!/usr/bin/env bash
# Round 4 session u: WALK draws passes of 64 rows (main) vs 32 (narrow) on config 4 and 5;
# TestData draws at a 3-wave register budget (wpe3) vs 4 (main); the DRAM GPU tests.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; OUT="$ROOT/gpurun_out"
WORK=syn4 VARIANTS="main narrow main narrow" bash scripts/gpu_dram_prof.sh r04u_syn4 2000 || exit $?
WORK=syn5 VARIANTS="main narrow" bash scripts/gpu_dram_prof.sh r04u_syn5 2000 || exit $?
VARIANTS="main wpe3 main wpe3" bash scripts/gpu_dram_prof.sh r04u 20000 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_dram_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/r04u_pytest.log" 2>&1
rc=$?; tail -4 "$OUT/r04u_pytest.log"; exit $rc
