#!/usr/bin/env bash
# Round-2 A/B of k_adapt_gt panels per trailing pass (3 vs 4) and waves per EU (4 vs 3) on the
# 250-point config-4-style fit: bitwise equality against the in-tree build, then fit timings.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TCI_SYNTH_POINTS=250 timeout -k 10 300 python3 scripts/dram_lib_equal.py main build/ab/libtci_gtp4w3.so 300 300 4 > "$OUT/r02ar_eq_250.json" 2>&1 || exit $?
cat "$OUT/r02ar_eq_250.json"
for v in main gtp4 gtp4w3 gtp3w3 main gtp4w3 gtp3w3; do
  lib=""; [ "$v" = main ] || lib="$ROOT/build/ab/libtci_$v.so"
  TCI_LIB="$lib" TCI_SYNTH_POINTS=250 timeout -k 10 300 python3 scripts/synth_dram_time.py 4 1000 > "$OUT/r02ar_250_$v.json" 2> "$OUT/r02ar_250_$v.err" || exit $?
  echo "== 250 $v"; cut -c1-60,300-420 "$OUT/r02ar_250_$v.json"
done
