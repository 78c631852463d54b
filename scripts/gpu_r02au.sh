#!/usr/bin/env bash
# PMC passes (FETCH_SIZE, WRITE_SIZE; one counter group per run) over the 250-point config-4-style
# fit (1000 steps, 10 adaptations): HBM-side bytes per k_adapt_gt / k_draws / k_walk dispatch.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; export TMPDIR=/tmp
cd /tmp
i=0
for grp in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  TCI_SYNTH_POINTS=250 timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/r02au_p$i" -o pmc -- \
    python3 "$ROOT/scripts/synth_dram_time.py" 4 1000 > "$OUT/r02au_p$i.json" 2> "$OUT/r02au_p$i.err" || exit $?
done
