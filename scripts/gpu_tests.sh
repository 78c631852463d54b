#!/usr/bin/env bash
# GPU tests by selection: scripts/gpu_tests.sh TAG [pytest -k expression] [test files...]
# Writes gpurun_out/TAG_pytest.log; every step under its own time limit.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${1:-t}"; K="${2:-}"; shift 2 2>/dev/null || shift $#
FILES="${*:-tests}"
mkdir -p "$OUT"; cd "$ROOT"
if [ -n "$K" ]; then
  timeout -k 10 1000 python -u -m pytest $FILES -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "$K" > "$OUT/${TAG}_pytest.log" 2>&1
else
  timeout -k 10 1000 python -u -m pytest $FILES -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1
fi
rc=$?; tail -25 "$OUT/${TAG}_pytest.log"; exit $rc
