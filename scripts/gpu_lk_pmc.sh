#!/usr/bin/env bash
# HBM traffic of likelihood-kernel variants (VARIANTS: build/ab/libtci_<name>.so, or main): one
# rocprofv3 --pmc pass per counter group and variant over the bench workload (ab_variants.py --run).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${1:-lkpmc}"; mkdir -p "$OUT"; export TMPDIR=/tmp; cd /tmp
for v in ${VARIANTS:-main xcd}; do
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/${TAG}_${v}_p$i" -o pmc -- \
      python3 "$ROOT/scripts/ab_variants.py" --run --variants "$v" --rounds 2 --launches 10 > "$OUT/${TAG}_${v}_p$i.json" 2> "$OUT/${TAG}_${v}_p$i.err"
    rc=$?; if [ $rc -ne 0 ]; then echo "$v pass $i status $rc"; tail -5 "$OUT/${TAG}_${v}_p$i.err"; exit $rc; fi
  done
  python3 - "$OUT/${TAG}_${v}" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "_p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "tci_cohort_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in agg.items()}
print(sys.argv[1].split("/")[-1], {k: round(v, 1) for k, v in m.items()},
      "hbm_bytes_per_launch", (2 * m.get("FETCH_SIZE", 0) + m.get("WRITE_SIZE", 0)) * 1024)
PY
done
