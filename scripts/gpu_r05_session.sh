#!/usr/bin/env bash
# Round-5 measurement session: round-end style check, likelihood A/B, DRAM A/Bs with bitwise
# equality against the round-4 build, PMC passes of the likelihood kernel. Every step optional:
#   CHECK=1 (gpu_check.sh), LKV="old,ship,..", TDV="main nw6" (TestData fit, FUSED), TDEQ="nw6",
#   C4V="main walk1" (config-4 fit), C4EQ="walk1", PMC=1
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
T="${1:-r05}"
if [ "${CHECK:-1}" = "1" ]; then bash scripts/gpu_check.sh "$T" || exit $?; fi
if [ -n "${LKV:-}" ]; then
  LK="$LKV" LK_ARGS="--distinct 8 --rounds 15 --launches 40" bash scripts/gpu_ab_session.sh "${T}" || exit $?
fi
if [ -n "${TDEQ:-}" ]; then
  TCI_ENGINE=fused EQ="$TDEQ" EQ_CFG=0 EQ_CELLS=299 EQ_STEPS=1000 bash scripts/gpu_ab_session.sh "${T}td" || exit $?
fi
if [ -n "${TDV:-}" ]; then DRAM="$TDV" WORK=td STEPS=20000 bash scripts/gpu_ab_session.sh "${T}td" || exit $?; fi
if [ -n "${C4EQ:-}" ]; then
  TCI_ENGINE=walk EQ="$C4EQ" EQ_CFG=4 EQ_CELLS=2000 EQ_STEPS=300 bash scripts/gpu_ab_session.sh "${T}c4" || exit $?
fi
if [ -n "${C4V:-}" ]; then DRAM="$C4V" WORK=syn4 STEPS=1000 bash scripts/gpu_ab_session.sh "${T}c4" || exit $?; fi
if [ "${PMC:-0}" = "1" ]; then bash scripts/gpu_pmc.sh "${T}pmc" || exit $?; fi
exit 0
