#!/usr/bin/env bash
# Round 4 session i: HEAD (head) vs the Box-Muller pair in plain arithmetic (nrm) vs main (nrm +
# the owned-tile covariance layout of k_adapt_mfma, the diagonal-tile factorization through LDS,
# k_chain's s2 sums from the log at the window end), TestData fit 20k steps; the adaptation's
# phase profile (adaptprof); then the DRAM GPU tests on main.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
VARIANTS="head nrm main head nrm main adaptprof" bash scripts/gpu_dram_prof.sh r04i 20000 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_dram_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/r04i_pytest.log" 2>&1
rc=$?; tail -4 "$OUT/r04i_pytest.log"
[ $rc -le 1 ] || exit $rc
# config 4 (10,000 synthetic chains, P = 207, WALK): 2,000 steps
WORK=syn4 VARIANTS="head main" bash scripts/gpu_dram_prof.sh r04i_syn4 2000 || exit $?
exit $rc
