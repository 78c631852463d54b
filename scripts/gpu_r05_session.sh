#!/usr/bin/env bash
# Round-5 measurement session: round-end style check, likelihood A/B, config-4 k_walk A/B with
# bitwise equality, PMC passes of the likelihood kernel.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
T="${1:-r05}"
bash scripts/gpu_check.sh "$T" || exit $?
LK="${LKV:-old,ship}" LK_ARGS="--distinct 8 --rounds 15 --launches 40" bash scripts/gpu_ab_session.sh "$T" || exit $?
if [ -n "${DRAMV:-}" ]; then
  DRAM="$DRAMV" WORK=syn4 STEPS=1000 bash scripts/gpu_ab_session.sh "$T" || exit $?
  TCI_ENGINE=walk EQ="${EQV:-}" EQ_CFG=4 EQ_CELLS=2000 EQ_STEPS=300 bash scripts/gpu_ab_session.sh "$T" || exit $?
fi
[ "${PMC:-1}" = "1" ] && { bash scripts/gpu_pmc.sh "${T}pmc" || exit $?; }
exit 0
