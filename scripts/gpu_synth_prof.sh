#!/usr/bin/env bash
# rocprofv3 kernel-trace summary of the config-4 DRAM fit (10,000 synthetic chains x 200 points).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${1:-sprof}"; CFG="${2:-4}"; STEPS="${3:-500}"
mkdir -p "$OUT"; cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}" -o trace -- \
  python3 "$ROOT/scripts/synth_dram_time.py" "$CFG" "$STEPS" > "$OUT/${TAG}.json" 2> "$OUT/${TAG}.err"
rc=$?; cat "$OUT/${TAG}.json"; exit $rc
