#!/usr/bin/env bash
# Round 4 session s: config 4 with an 8 GiB draws buffer (100-step chunks: one walk launch per
# adaptation window instead of 64 + 36) -- big8 vs main, 2,000 steps; config 5 likewise.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
WORK=syn4 VARIANTS="main big8 main big8" bash scripts/gpu_dram_prof.sh r04s_syn4 2000 || exit $?
WORK=syn5 VARIANTS="main big8" bash scripts/gpu_dram_prof.sh r04s_syn5 2000 || exit $?
