#!/usr/bin/env bash
# Round-4 session e: k_chain streamlined proposal phase and records (A/B against round 3), the DRAM
# GPU tests, per-wave phase profile.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
VARIANTS="prev main prev main" bash scripts/gpu_dram_prof.sh r04e 20000 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_dram_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/r04e_pytest.log" 2>&1
rc=$?; tail -4 "$OUT/r04e_pytest.log"; [ $rc -le 1 ] || exit $rc
CELLS="0" bash scripts/gpu_cp3.sh r04e_cp3 20000
