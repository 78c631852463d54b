#!/usr/bin/env bash
# DRAM engine tests + 299-cell fit timing (+ the k_chain phase profile build when present).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${1:-dq}"; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 400 python -u -m pytest tests/test_dram_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1
rc=$?; tail -3 "$OUT/${TAG}_pytest.log"; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python3 scripts/dram_time.py 200000 auto 20 > "$OUT/${TAG}_fit.json" 2>&1 || exit $?
cat "$OUT/${TAG}_fit.json"
if [ -f build/ab/libtci_chainprof.so ]; then VARIANTS=chainprof bash scripts/gpu_chainprof.sh "${TAG}_cp" 20000 || exit $?; fi
exit $rc
