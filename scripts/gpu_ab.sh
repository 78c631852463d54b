#!/usr/bin/env bash
# A/B timing of prebuilt likelihood-kernel variants (build/ab/libtci_<name>.so), then the GPU tests.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${1:-ab}"; VARS="${2:-old,ship}"
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 300 python scripts/ab_variants.py --run --variants "$VARS" > "$OUT/${TAG}.json" 2> "$OUT/${TAG}.err"
rc=$?; cat "$OUT/${TAG}.json"; [ $rc -eq 0 ] || { tail -20 "$OUT/${TAG}.err"; exit $rc; }
if [ "${RUN_TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1
  rc=$?; tail -5 "$OUT/${TAG}_pytest.log"; exit $rc
fi
