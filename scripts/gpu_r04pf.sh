#!/usr/bin/env bash
# Round 4: likelihood kernel touching the theta row TCI_LK_PF rows ahead (pf4k/pf8k/pf16k) against
# main, bench-like: 8 distinct resident batches cycled, 25 interleaved rounds of 64 launches.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"; OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
timeout -k 10 300 python scripts/ab_variants.py --run --variants "main,pf4k,pf8k,pf16k" --rounds 25 --launches 64 --distinct 8 \
  > "$OUT/r04pf_ab.json" 2> "$OUT/r04pf_ab.err" || exit $?
cat "$OUT/r04pf_ab.json"
