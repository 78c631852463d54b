#!/usr/bin/env bash
# Round 4 session m: the split draws (k_normals on a second stream beside the adaptation, k_draws
# only multiplying) in main against nosplit, TestData fit 20k steps and config 4 (2,000 steps);
# the DRAM GPU tests on main.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
VARIANTS="nosplit main nosplit main" bash scripts/gpu_dram_prof.sh r04m 20000 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_dram_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/r04m_pytest.log" 2>&1
rc=$?; tail -4 "$OUT/r04m_pytest.log"
[ $rc -le 1 ] || exit $rc
WORK=syn4 VARIANTS="nosplit main" bash scripts/gpu_dram_prof.sh r04m_syn4 2000 || exit $?
exit $rc
