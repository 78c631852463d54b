#!/usr/bin/env bash
# Issue/stall breakdown of the likelihood kernel (SQ counters, two rocprofv3 --pmc passes over
# ab_variants.py --run). Usage on the GPU box: bash scripts/sq_stalls.sh [variants]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp
V="${1:-ship}"

run() {
  timeout -k 10 400 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/sq_$1" -o pmc -- \
    python3 "$ROOT/scripts/ab_variants.py" --run --variants "$V" --rounds 1 --launches 2 > /dev/null 2>> "$OUT/sq.err"
}
run SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAVES &&
run SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES &&
run GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_WAVES
