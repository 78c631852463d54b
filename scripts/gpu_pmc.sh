#!/usr/bin/env bash
# rocprofv3 PMC passes over the bench workload (one counter group per pass, --pmc only).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
TAG="${1:-pmc}"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT" \
           "TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE" \
           "TCC_HIT_sum TCC_MISS_sum SQ_INSTS_SMEM SQ_INSTS_FLAT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/${TAG}_p$i" -o pmc -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline --dram-steps 0 --no-configs --no-sweep --no-latency > "$OUT/${TAG}_p$i.json" 2> "$OUT/${TAG}_p$i.err"
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i status $rc"; tail -5 "$OUT/${TAG}_p$i.err"; exit $rc; fi
done
exit 0
