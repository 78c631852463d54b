#!/usr/bin/env bash
# rocprofv3 kernel stats of the config-4-style fit at 200 and 250 points (1000 steps, 10,000 chains).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"; export TMPDIR=/tmp
for n in 200 250; do
  TCI_SYNTH_POINTS=$n timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/r02as_$n" -o trace -- \
    python3 scripts/synth_dram_time.py 4 1000 > "$OUT/r02as_$n.json" 2> "$OUT/r02as_$n.err" || exit $?
done
