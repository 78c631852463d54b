#!/usr/bin/env bash
# Round 4 session g: k_draws with the pipelined z*R loop (mfma_zr_pf) and a 128-VGPR budget
# (main; wpe3: the 3-wave budget) against HEAD (head), TestData fit 20k steps; DRAM GPU tests.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
VARIANTS="head main wpe3 head main wpe3" bash scripts/gpu_dram_prof.sh r04g 20000 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_dram_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/r04g_pytest.log" 2>&1
rc=$?; tail -4 "$OUT/r04g_pytest.log"; exit $rc
