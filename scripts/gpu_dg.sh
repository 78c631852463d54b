#!/usr/bin/env bash
# Wall/device time of the TestData DRAM fit (STEPS steps) for k_chain depths D (TCI_CHAIN_D) and
# chain-group counts G (TCI_DRAM_GROUPS), one process per setting, interleaved twice.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${1:-dg}"; STEPS="${2:-20000}"; mkdir -p "$OUT"
for rep in 1 2; do
  for dg in ${DG_LIST:-2:1 3:1 2:2 3:2 2:3 3:3}; do
    d=${dg%%:*}; g=${dg##*:}
    echo "== D $d G $g" >> "$OUT/${TAG}.txt"
    TCI_CHAIN_D=$d TCI_DRAM_GROUPS=$g timeout -k 10 120 python3 "$ROOT/scripts/dram_time.py" "$STEPS" auto 20 >> "$OUT/${TAG}.txt" 2>&1 || exit $?
  done
done
cat "$OUT/${TAG}.txt"
