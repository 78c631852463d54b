#!/usr/bin/env bash
# Issue/stall breakdown of the likelihood kernel: SQ counters in separate rocprofv3 --pmc passes
# (--pmc only, at most 8 SQ counters a pass) over ab_variants.py --run on the K=256 workload.
# Usage on the GPU box: bash scripts/sq_stalls.sh [variant (default: main = the in-tree libtci.so)] [tag]
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp
V="${1:-main}"; TAG="${2:-sq}"
i=0
run() {
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/${TAG}_p$i" -o pmc -- \
    python3 "$ROOT/scripts/ab_variants.py" --run --variants "$V" --rounds 1 --launches 4 > /dev/null 2>> "$OUT/${TAG}.err"
}
run SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAVES &&
run SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS &&
run GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64 SQ_WAVES &&
run SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT &&
run FETCH_SIZE &&
run WRITE_SIZE
