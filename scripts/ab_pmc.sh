#!/usr/bin/env bash
# Dynamic instruction counts per A/B variant (one rocprofv3 --pmc pass over ab_variants.py --run).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp; cd /tmp
V="${1:-ship,abl_rows,abl_bounds,abl_interp,abl_scan,abl_all}"
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES --output-format csv \
  -d "$OUT/abpmc" -o pmc -- python3 "$ROOT/scripts/ab_variants.py" --run --variants "$V" --rounds 1 --launches 2 \
  > "$OUT/abpmc.json" 2> "$OUT/abpmc.err"
