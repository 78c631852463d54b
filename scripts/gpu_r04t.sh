#!/usr/bin/env bash
# Round 4 session t: config 4 draws-pass ablations (no normals / no z*R; the chains are wrong, only
# the k_draws time is read), 1,000 steps.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
WORK=syn4 VARIANTS="main draws_nonorm draws_nomfma" bash scripts/gpu_dram_prof.sh r04t_syn4 1000 || exit $?
