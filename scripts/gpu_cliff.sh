#!/usr/bin/env bash
# Long-cell tests + config-4-style fit timing at several cell lengths (the P > 208 cliff).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${1:-cliff}"; STEPS="${2:-1000}"; mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_dram_gpu.py -m gpu -k "long" -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > "$OUT/${TAG}_pytest.log" 2>&1
rc=$?; tail -3 "$OUT/${TAG}_pytest.log"; [ $rc -eq 0 ] || exit $rc
for n in ${POINTS:-200 250}; do
  TCI_SYNTH_POINTS=$n timeout -k 10 300 python3 scripts/synth_dram_time.py 4 "$STEPS" >> "$OUT/${TAG}_fit.txt" 2>> "$OUT/${TAG}_fit.err" || exit $?
  tail -1 "$OUT/${TAG}_fit.txt"
done
