#!/usr/bin/env bash
# Round 4 sessions g, h (TAG): k_draws variants (main; wpe3: the 3-wave register budget) against
# HEAD (head), TestData fit 20k steps; then the DRAM GPU tests.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
VARIANTS="head main wpe3 head main wpe3" bash scripts/gpu_dram_prof.sh ${TAG:-r04g} 20000 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_dram_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/${TAG:-r04g}_pytest.log" 2>&1
rc=$?; tail -4 "$OUT/${TAG:-r04g}_pytest.log"; exit $rc
