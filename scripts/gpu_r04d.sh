#!/usr/bin/env bash
# Round-4 session d: DRAM GPU tests, library A/B (prev = round 3, main4 = k_chain LDS diet,
# main = + padded draws stride), D / group timing, rcp accuracy, per-wave chain profiles.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 900 python -u -m pytest tests/test_dram_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/r04d_pytest.log" 2>&1
rc=$?; tail -6 "$OUT/r04d_pytest.log"; [ $rc -le 1 ] || exit $rc
VARIANTS="prev main4 main" bash scripts/gpu_dram_prof.sh r04d 20000 || exit $?
bash scripts/gpu_dg.sh r04d_dg 20000 || exit $?
timeout -k 10 60 ./scripts/calib/rcp_f64 > "$OUT/r04d_rcp.json" || exit $?
bash scripts/gpu_cp3.sh r04d_cp3 20000 || exit $?
TCI_CHAIN_D=3 bash scripts/gpu_cp3.sh r04d_cp3d3 20000
VARIANTS="main xcd xcd2" bash scripts/gpu_lk_pmc.sh r04d_lk
