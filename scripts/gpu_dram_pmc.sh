#!/usr/bin/env bash
# rocprofv3 PMC passes (one counter group per pass, --pmc only) over a short DRAM fit (WORK=td:
# TestData, default; syn4 / syn5: BASELINE config 4 / 5): per-dispatch counters of k_chain /
# k_walk / k_draws / k_adapt_* (scripts/dram_pmc_summary.py). PMC_SET=fetch: FETCH_SIZE and WRITE_SIZE only.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${1:-dpmc}"; STEPS="${2:-2000}"
mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
lib=""; [ "${VARIANT:-main}" = main ] || lib="$ROOT/build/ab/libtci_${VARIANT}.so"
case "${WORK:-td}" in
  td) CMD=("$ROOT/scripts/dram_time.py" "$STEPS" auto 20) ;;
  syn4) CMD=("$ROOT/scripts/synth_dram_time.py" 4 "$STEPS") ;;
  syn5) CMD=("$ROOT/scripts/synth_dram_time.py" 5 "$STEPS") ;;
  *) echo "unknown WORK=$WORK"; exit 2 ;;
esac
GRPS=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_MFMA_F64 GRBM_GUI_ACTIVE" \
      "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
      "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_INT64" \
      "FETCH_SIZE")
[ "${PMC_SET:-all}" = fetch ] && GRPS=("FETCH_SIZE" "WRITE_SIZE")
i=0
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  TCI_LIB="$lib" timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/${TAG}_p$i" -o pmc -- \
    python3 "${CMD[@]}" > "$OUT/${TAG}_p$i.json" 2> "$OUT/${TAG}_p$i.err"
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i status $rc"; tail -5 "$OUT/${TAG}_p$i.err"; exit $rc; fi
done
python3 "$ROOT/scripts/dram_pmc_summary.py" "$OUT/${TAG}" > "$OUT/${TAG}_summary.json" && cat "$OUT/${TAG}_summary.json"
