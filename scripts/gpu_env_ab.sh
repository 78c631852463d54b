#!/usr/bin/env bash
# A/B of an environment switch of the in-tree build (e.g. AB_VAR=TCI_DRAM_OVERLAP): bitwise equality
# of the fits with the switch off and on (FUSED on 299 TestData cells), then the 299-cell fit timed
# under rocprofv3 kernel traces with each setting (STEPS steps, default 20k), then without the
# profiler (its kernel tracing serialises the streams) at WALL_STEPS steps (default 200k; 0 skips).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${1:-envab}"; STEPS="${2:-20000}"; VAR="${AB_VAR:-TCI_DRAM_OVERLAP}"
mkdir -p "$OUT"; cd "$ROOT"
timeout -k 10 300 python3 scripts/dram_lib_equal.py "main@$VAR=0" "main@$VAR=1" 2000 299 0 > "$OUT/${TAG}_eq.json" 2> "$OUT/${TAG}_eq.err"
rc=$?; echo "== eq rc=$rc"; cat "$OUT/${TAG}_eq.json"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { tail -5 "$OUT/${TAG}_eq.err"; exit $rc; }
cd /tmp; export TMPDIR=/tmp
for v in ${AB_VALUES:-0 1 0 1}; do
  n="${TAG}_${VAR}_$v"; [ -e "$OUT/$n" ] && n="${n}_b"
  env "$VAR=$v" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$n" -o trace -- \
    python3 "$ROOT/scripts/dram_time.py" "$STEPS" auto 20 > "$OUT/$n.json" 2> "$OUT/$n.err" || exit $?
  echo "== $VAR=$v"; cat "$OUT/$n.json"
  f=$(find "$OUT/$n" -name "*kernel_stats.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].replace("tci::(anonymous namespace)::", "").replace("void ", "").split("(tci::")[0]
    print(f"  {n[:44]:44s} {r['Calls']:>6s} {float(r['AverageNs']) / 1000:10.2f} us  {float(r['TotalDurationNs']) / 1e6:9.2f} ms")
PY
done
W="${WALL_STEPS:-200000}"
[ "$W" -gt 0 ] || exit 0
for v in ${AB_VALUES:-0 1 0 1}; do
  env "$VAR=$v" timeout -k 10 300 python3 "$ROOT/scripts/dram_time.py" "$W" auto 20 > "$OUT/${TAG}_wall_$v.json" 2>&1 || exit $?
  echo "== wall $VAR=$v"; tail -1 "$OUT/${TAG}_wall_$v.json"
done
exit 0
