#!/usr/bin/env bash
# rocprofv3 kernel-trace summary of the bench's end-to-end DRAM fit (299 cells, n_burn = n_steps/20).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${1:-dprof}"; STEPS="${2:-200000}"
mkdir -p "$OUT"; cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}" -o trace -- \
  python3 "$ROOT/scripts/dram_time.py" "$STEPS" auto 20 > "$OUT/${TAG}.json" 2> "$OUT/${TAG}.err"
rc=$?; cat "$OUT/${TAG}.json"; exit $rc
