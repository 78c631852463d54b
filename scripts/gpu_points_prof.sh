#!/usr/bin/env bash
# rocprofv3 kernel stats of the config-4-style DRAM fit at several cell lengths (POINTS).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${1:-pts}"; STEPS="${2:-1000}"; mkdir -p "$OUT"; cd /tmp; export TMPDIR=/tmp
for n in ${POINTS:-200 250}; do
  TCI_SYNTH_POINTS=$n timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_$n" -o trace -- \
    python3 "$ROOT/scripts/synth_dram_time.py" 4 "$STEPS" > "$OUT/${TAG}_$n.json" 2> "$OUT/${TAG}_$n.err" || exit $?
  cat "$OUT/${TAG}_$n.json"
done
