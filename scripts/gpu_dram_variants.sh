#!/usr/bin/env bash
# Device time of the 299-cell DRAM fit for the shipped build and build/ab variants, interleaved
# (3 rounds), so variants are compared on the same box.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${1:-dv}"; STEPS="${2:-20000}"
mkdir -p "$OUT"
for r in 1 2 3; do
  for v in ship ${VARIANTS:-}; do
    lib=""; [ "$v" = ship ] || lib="$ROOT/build/ab/libtci_$v.so"
    echo -n "$v " >> "$OUT/${TAG}.txt"
    TCI_LIB="$lib" timeout -k 10 120 python3 "$ROOT/scripts/dram_time.py" "$STEPS" auto 20 >> "$OUT/${TAG}.txt" 2>> "$OUT/${TAG}.err" || exit $?
  done
done
cat "$OUT/${TAG}.txt"
