#!/usr/bin/env bash
# rocprofv3 kernel statistics of a DRAM fit for library variants (VARIANTS: "main" = the in-tree
# build, or build/ab/libtci_<name>.so). WORK=td (default): the 299-cell TestData fit, STEPS steps
# (20k default); WORK=syn4 / syn5: BASELINE config 4 / 5 (10,000 synthetic chains), STEPS steps.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${1:-dprof}"; STEPS="${2:-20000}"; WORK="${WORK:-td}"
mkdir -p "$OUT"; cd /tmp; export TMPDIR=/tmp
case "$WORK" in
  td) CMD=("$ROOT/scripts/dram_time.py" "$STEPS" auto 20) ;;
  syn4) CMD=("$ROOT/scripts/synth_dram_time.py" 4 "$STEPS") ;;
  syn5) CMD=("$ROOT/scripts/synth_dram_time.py" 5 "$STEPS") ;;
  *) echo "unknown WORK=$WORK"; exit 2 ;;
esac
for v in ${VARIANTS:-main}; do
  lib=""; [ "$v" = main ] || lib="$ROOT/build/ab/libtci_$v.so"
  TCI_LIB="$lib" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_$v" -o trace -- \
    python3 "${CMD[@]}" > "$OUT/${TAG}_$v.json" 2> "$OUT/${TAG}_$v.err" || exit $?
  echo "== $v"; cat "$OUT/${TAG}_$v.json"; grep -h "cycles_per_chain" "$OUT/${TAG}_$v.err" || true
  f=$(find "$OUT/${TAG}_$v" -name "*kernel_stats.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].replace("tci::(anonymous namespace)::", "").replace("void ", "").split("(tci::")[0]
    print(f"  {n[:44]:44s} {r['Calls']:>6s} {float(r['AverageNs']) / 1000:10.2f} us  {float(r['TotalDurationNs']) / 1e6:9.2f} ms")
PY
done
