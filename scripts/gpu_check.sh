#!/usr/bin/env bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script (no retries).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
TAG="${1:-run}"
mkdir -p "$OUT"
cd "$ROOT"
stop_if_fault() {  # $1 = exit status of a GPU step; 0/1 (test failures) continue, anything else stops
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "GPU step ended with status $1 -- stopping" ; exit "$1"; fi
}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
echo "== pytest -m gpu"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/${TAG}_pytest_gpu.log" 2>&1
rc=$?; tail -5 "$OUT/${TAG}_pytest_gpu.log"; stop_if_fault $rc
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/${TAG}_smoke.log" 2>&1
rc=$?; tail -3 "$OUT/${TAG}_smoke.log"; stop_if_fault $rc
fi
echo "== bench"; timeout -k 10 600 python bench.py > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err"
rc=$?; cat "$OUT/${TAG}_bench.json"; stop_if_fault $rc
echo "== rocprofv3 kernel trace"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_prof" -o trace -- \
  python3 "$ROOT/bench.py" --no-cpu-baseline --dram-steps 0 --no-configs --no-sweep --no-latency > "$OUT/${TAG}_prof_bench.json" 2> "$OUT/${TAG}_prof.err"
rc=$?; stop_if_fault $rc
find "$OUT/${TAG}_prof" -name "*stats*" | head -5
exit 0
