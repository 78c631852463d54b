#!/usr/bin/env bash
# A DRAM change that must not move any bit: bitwise fit comparison against build/ab/libtci_prev.so
# (TestData, configs 4 and 5), end-to-end timing of both builds, then the DRAM GPU tests.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="${1:-dab}"
cd "$ROOT"; mkdir -p gpurun_out
for cfg in 0 4 5; do
  timeout -k 10 300 python3 scripts/dram_lib_equal.py build/ab/libtci_prev.so main 2000 40 $cfg > gpurun_out/${TAG}_eq$cfg.json 2> gpurun_out/${TAG}_eq$cfg.err
  rc=$?; cat gpurun_out/${TAG}_eq$cfg.json; [ $rc -le 1 ] || exit $rc
done
VARIANTS="main prev" bash scripts/gpu_dram_libs.sh "$TAG" 20000 1000 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_dram_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; tail -2 gpurun_out/${TAG}_pytest.log
