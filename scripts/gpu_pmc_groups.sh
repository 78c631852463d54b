#!/usr/bin/env bash
# rocprofv3 PMC passes over the kernel-mode bench workload, one counter group per pass (--pmc only,
# every pass in its own time limit). Usage: gpu_pmc_groups.sh TAG "CNT CNT .." ["CNT ..." ...]
# LIST=1 first writes the agent's available counters to gpurun_out/TAG_avail.txt.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"
TAG="$1"; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
if [ "${LIST:-0}" = "1" ]; then
  timeout -k 10 120 rocprofv3 --list-avail > "$OUT/${TAG}_avail.txt" 2>&1 || echo "list-avail status $?"
fi
i=0
for grp in "$@"; do
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/${TAG}_p$i" -o pmc -- \
    python3 "$ROOT/bench.py" --steps 2 --warmup 1 --launches-per-step 8 --no-cpu-baseline --dram-steps 0 --no-configs --no-sweep --no-latency > "$OUT/${TAG}_p$i.json" 2> "$OUT/${TAG}_p$i.err"
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i status $rc"; tail -5 "$OUT/${TAG}_p$i.err"; exit $rc; fi
done
exit 0
