#!/usr/bin/env bash
# Round 4 session f: k_draws ablations (normals / MFMA / scalar draws removed; the chains are wrong,
# only the k_draws time is read), TestData fit 20k steps.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
VARIANTS="main draws_nonorm draws_nomfma draws_noscal draws_none" bash scripts/gpu_dram_prof.sh r04f 20000 || exit $?
