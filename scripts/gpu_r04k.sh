#!/usr/bin/env bash
# Round 4 sessions k, l (TAG): HEAD (head) vs main (the Box-Muller pair in plain arithmetic, the owned-tile
# covariance layout; l: + the look-ahead diagonal factorization), TestData fit 20k steps; the
# adaptation's phase profile; the DRAM GPU tests; config 4 (2,000 steps).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
VARIANTS="head main head main adaptprof" bash scripts/gpu_dram_prof.sh ${TAG:-r04k} 20000 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_dram_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/${TAG:-r04k}_pytest.log" 2>&1
rc=$?; tail -4 "$OUT/${TAG:-r04k}_pytest.log"
[ $rc -le 1 ] || exit $rc
WORK=syn4 VARIANTS="head main" bash scripts/gpu_dram_prof.sh ${TAG:-r04k}_syn4 2000 || exit $?
exit $rc
