#!/usr/bin/env bash
# Round 4 session v: k_chain with the exchanged values read in one LDS round trip after the
# barrier (main) against HEAD (head), TestData fit 20k steps; the DRAM GPU tests.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; OUT="$ROOT/gpurun_out"
VARIANTS="head main head main" bash scripts/gpu_dram_prof.sh ${TAG:-r04v} 20000 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_dram_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/${TAG:-r04v}_pytest.log" 2>&1
rc=$?; tail -4 "$OUT/${TAG:-r04v}_pytest.log"; exit $rc
