#!/usr/bin/env bash
# Round-end style GPU session: scripts/gpu_check.sh (pytest -m gpu, smoke, bench, rocprofv3 of the
# bench's kernel leg), then the two-rank launcher rehearsal on one GPU (gloo) with --no-configs.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${1:-rc}"
cd "$ROOT"
bash scripts/gpu_check.sh "$TAG" || exit $?
echo "== rehearsal --gpus 2 (gloo, one GPU)"
TCI_BENCH_REHEARSAL=1 timeout -k 10 300 python bench.py --gpus 2 --no-configs --dram-steps 20000 --steps 5 --warmup 2 \
  > "$OUT/${TAG}_rehearsal.json" 2> "$OUT/${TAG}_rehearsal.err"
rc=$?; cat "$OUT/${TAG}_rehearsal.json" | cut -c1-400; echo "rehearsal rc=$rc"
exit 0
