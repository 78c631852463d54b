#!/usr/bin/env bash
# DRAM engine check on one GPU: its GPU tests, then timed fits (20k and 200k steps, 299 cells).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${1:-dram}"
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_dram_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/${TAG}_pytest.log" 2>&1
rc=$?; tail -4 "$OUT/${TAG}_pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/dram_time.py 20000 fused > "$OUT/${TAG}_t20k.json" 2>&1 && cat "$OUT/${TAG}_t20k.json" || exit 1
timeout -k 10 120 python scripts/dram_time.py 200000 fused > "$OUT/${TAG}_t200k.json" 2>&1 && cat "$OUT/${TAG}_t200k.json" || exit 1
