#!/usr/bin/env bash
# Per-wave k_chain phase cycles (TCI_CHAIN_PROFILE=3 build under build/ab) on the TestData fit for
# CELLS chain counts (0 = all 299).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${1:-cp3}"; STEPS="${2:-20000}"; mkdir -p "$OUT"
for n in ${CELLS:-0 64}; do
  echo "== cells $n" >> "$OUT/${TAG}.txt"
  TCI_LIB="$ROOT/build/ab/libtci_${VARIANT:-cp3}.so" timeout -k 10 120 python3 "$ROOT/scripts/dram_time.py" "$STEPS" auto 20 "$n" >> "$OUT/${TAG}.txt" 2>> "$OUT/${TAG}.txt" || exit $?
done
cat "$OUT/${TAG}.txt"
