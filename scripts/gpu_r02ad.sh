#!/usr/bin/env bash
# Draws-pass R staging by LDS-DMA: bitwise equality vs the previous commit, then fit timings.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
T="${TAG:-r02ad}"; P=build/ab/libtci_prev.so
timeout -k 10 200 python3 scripts/dram_lib_equal.py main $P 2000 80 0 > "$OUT/${T}_eq_td.json" 2>&1 || exit $?
timeout -k 10 300 python3 scripts/dram_lib_equal.py main $P 300 400 5 > "$OUT/${T}_eq_c5.json" 2>&1 || exit $?
TCI_SYNTH_POINTS=250 timeout -k 10 300 python3 scripts/dram_lib_equal.py main $P 300 300 4 > "$OUT/${T}_eq_250.json" 2>&1 || exit $?
cat "$OUT"/${T}_eq_*.json
VARIANTS="${VARIANTS:-main prev glds0 main prev}" bash scripts/gpu_dram_libs.sh $T 20000 1000 > "$OUT/${T}_libs.log" 2>&1 || exit $?
grep -h "us_per_step" "$OUT/${T}_libs.log" | python3 -c "
import sys,json
for l in sys.stdin:
    l=l.strip()
    if l.startswith('{'):
        d=json.loads(l); print(d.get('workload','td')[:8], round(d['us_per_step'],2))
"
for v in ${VARIANTS:-main prev glds0 main prev}; do
  lib=""; [ "$v" = main ] || lib="$ROOT/build/ab/libtci_$v.so"
  TCI_LIB="$lib" TCI_SYNTH_POINTS=250 timeout -k 10 300 python3 scripts/synth_dram_time.py 4 1000 > "$OUT/${T}_250_$v.json" 2> "$OUT/${T}_250_$v.err" || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('250', '$v', round(d['us_per_step'],1))" "$OUT/${T}_250_$v.json"
done
