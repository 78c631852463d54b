#!/usr/bin/env bash
# Round 4 session j: which change broke the adaptation -- head vs nolds (the covariance tile
# layout + k_chain's s2 sums, lane-broadcast diagonal factorization) vs main (+ LDS exchange).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
VARIANTS="head nolds main" bash scripts/gpu_dram_prof.sh r04j 20000 || exit $?
