#!/usr/bin/env bash
# k_adapt_gt without the tile-grid write of the scatter (first touches read cov): bitwise equality
# (TCI_GT_DIRECT=1 variant) against the in-tree build at 250 and 300 points, then timings at 250 points.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
P=build/ab/libtci_gtdirect.so
TCI_SYNTH_POINTS=250 timeout -k 10 300 python3 scripts/dram_lib_equal.py main $P 300 300 4 > "$OUT/r02av_eq_250.json" 2>&1 || exit $?
cat "$OUT/r02av_eq_250.json"
TCI_SYNTH_POINTS=300 timeout -k 10 300 python3 scripts/dram_lib_equal.py main $P 300 200 4 > "$OUT/r02av_eq_300.json" 2>&1 || exit $?
cat "$OUT/r02av_eq_300.json"
for v in main gtdirect main gtdirect; do
  lib=""; [ "$v" = main ] || lib="$ROOT/build/ab/libtci_$v.so"
  TCI_LIB="$lib" TCI_SYNTH_POINTS=250 timeout -k 10 300 python3 scripts/synth_dram_time.py 4 1000 > "$OUT/r02av_250_$v.json" 2> "$OUT/r02av_250_$v.err" || exit $?
  echo "== 250 $v"; cut -c300-420 "$OUT/r02av_250_$v.json"
done
exit 0

