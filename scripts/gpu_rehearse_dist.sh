#!/usr/bin/env bash
# Rehearse bench.py's multi-process path on ONE GPU: 2 ranks over gloo, both on cuda:0.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"; cd "$ROOT"
TCI_BENCH_REHEARSAL=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 --dram-steps "${DSTEPS:-0}" --synth-dram-steps "${SSTEPS:-2000}" --no-cpu-baseline \
  > "$OUT/rehearse_dist.json" 2> "$OUT/rehearse_dist.err"
rc=$?; cat "$OUT/rehearse_dist.json"; tail -5 "$OUT/rehearse_dist.err"; exit $rc
