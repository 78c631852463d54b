#!/usr/bin/env bash
# Round 4: likelihood kernel XCD-contiguous block order (xcd) against main, 25 interleaved rounds
# of 40 launches on the bench workload (same process), to settle the within-noise r04a result.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
timeout -k 10 300 python scripts/ab_variants.py --run --variants "main,xcd=TCI_LK_XCD=1" --rounds 25 --launches 40 > "$OUT/r04xcd_ab.json" 2> "$OUT/r04xcd_ab.err" || exit $?
cat "$OUT/r04xcd_ab.json"
