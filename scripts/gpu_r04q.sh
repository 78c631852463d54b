#!/usr/bin/env bash
# Round 4 session q: config 4 adaptation with k_adapt_gt (tiles in global memory, two chains per CU)
# instead of k_adapt_mfma<8, 13, 12> (tiles in registers, one chain per CU): gt vs main, 2,000 steps.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
WORK=syn4 VARIANTS="main gt main gt" bash scripts/gpu_dram_prof.sh r04q_syn4 2000 || exit $?
