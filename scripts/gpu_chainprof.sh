#!/usr/bin/env bash
# k_chain phase cycles (TCI_CHAIN_PROFILE builds under build/ab) on the 299-cell fit.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${1:-cp}"; STEPS="${2:-20000}"; mkdir -p "$OUT"
for v in ${VARIANTS:-chainprof chainprof2}; do
  echo "== $v" >> "$OUT/${TAG}.txt"
  TCI_LIB="$ROOT/build/ab/libtci_$v.so" timeout -k 10 120 python3 "$ROOT/scripts/dram_time.py" "$STEPS" auto 20 >> "$OUT/${TAG}.txt" 2>> "$OUT/${TAG}.txt" || exit $?
done
cat "$OUT/${TAG}.txt"
