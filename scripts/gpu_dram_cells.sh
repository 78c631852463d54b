#!/usr/bin/env bash
# rocprofv3 kernel statistics of the TestData DRAM fit on the first N cells (CELLS list; 0 = all
# 299), STEPS steps: how the per-chunk kernel times scale with the chains per CU.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${1:-cells}"; STEPS="${2:-20000}"
mkdir -p "$OUT"; cd /tmp; export TMPDIR=/tmp
for n in ${CELLS:-0 256 128}; do
  lib=""; [ "${VARIANT:-main}" = main ] || lib="$ROOT/build/ab/libtci_${VARIANT}.so"
  TCI_LIB="$lib" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_$n" -o trace -- \
    python3 "$ROOT/scripts/dram_time.py" "$STEPS" auto 20 "$n" > "$OUT/${TAG}_$n.json" 2> "$OUT/${TAG}_$n.err" || exit $?
  echo "== cells $n"; cat "$OUT/${TAG}_$n.json"
  f=$(find "$OUT/${TAG}_$n" -name "*kernel_stats.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].replace("tci::(anonymous namespace)::", "").replace("void ", "").split("(tci::")[0]
    print(f"  {n[:44]:44s} {r['Calls']:>6s} {float(r['AverageNs']) / 1000:10.2f} us  {float(r['TotalDurationNs']) / 1e6:9.2f} ms")
PY
done
