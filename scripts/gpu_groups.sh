#!/usr/bin/env bash
# Wall time of the TestData DRAM fit (STEPS steps) for chain-group counts GROUPS (TCI_DRAM_GROUPS),
# one process per setting, no profiler; then a rocprofv3 kernel trace of the last setting.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${1:-grp}"; STEPS="${2:-20000}"; mkdir -p "$OUT"
for g in ${GROUPS_LIST:-1 2 3 1 2 3}; do
  echo "== groups $g" >> "$OUT/${TAG}.txt"
  TCI_DRAM_GROUPS=$g timeout -k 10 120 python3 "$ROOT/scripts/dram_time.py" "$STEPS" auto 20 >> "$OUT/${TAG}.txt" 2>&1 || exit $?
done
cat "$OUT/${TAG}.txt"
