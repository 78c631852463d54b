#!/usr/bin/env bash
# Kernel A/B (old vs current vs variants), DRAM-fit timing of the same builds, then the GPU tests.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${1:-lean}"
mkdir -p "$OUT"; cd "$ROOT"
RUN_TESTS=0 bash scripts/gpu_ab.sh "${TAG}_ab" "${AB:-old,ship}" || exit $?
VARIANTS="${DV:-old}" bash scripts/gpu_dram_variants.sh "${TAG}_dram" "${DSTEPS:-20000}" || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1
rc=$?; tail -5 "$OUT/${TAG}_pytest.log"; exit $rc
