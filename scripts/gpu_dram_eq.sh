#!/usr/bin/env bash
# A sampler change that must not move any bit: each library in LIBS ("main" = the in-tree build, or
# build/ab/libtci_<name>.so) against build/ab/libtci_old.so on the same fits (FUSED and WALK on
# TestData cells, WALK on config-4 cells), the DRAM GPU tests, then the 299-cell fit timed with every
# build (20k steps) and the 10,000-chain config-4 fit (1k steps).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${1:-deq}"; mkdir -p "$OUT"; cd "$ROOT"
LIBS="${LIBS:-main}"
OLD="$ROOT/build/ab/libtci_old.so"
lib_of() { [ "$1" = main ] && echo main || { [ "$1" = old ] && echo "$OLD" || echo "$ROOT/build/ab/libtci_$1.so"; }; }
run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/${TAG}_${name}.json" 2> "$OUT/${TAG}_${name}.err"
  local rc=$?; echo "== $name rc=$rc"; cat "$OUT/${TAG}_${name}.json"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -5 "$OUT/${TAG}_${name}.err"; exit $rc; fi
}
for l in $LIBS; do
  run "eq_fused_$l" 200 python3 scripts/dram_lib_equal.py "$OLD" "$(lib_of $l)" 2000 40 0
  TCI_ENGINE=walk run "eq_walk_$l" 200 python3 scripts/dram_lib_equal.py "$OLD" "$(lib_of $l)" 2000 40 0
  TCI_ENGINE=walk run "eq_cfg4_$l" 300 python3 scripts/dram_lib_equal.py "$OLD" "$(lib_of $l)" 1000 64 4
done
if [ "${RUN_TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_dram_gpu.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > "$OUT/${TAG}_pytest.log" 2>&1
  rc=$?; tail -3 "$OUT/${TAG}_pytest.log"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
for v in old $LIBS; do
  lib=""; [ "$v" = main ] || lib="$(lib_of $v)"
  TCI_LIB="$lib" run "td_$v" 200 python3 scripts/dram_time.py 20000 auto 20
done
for v in old $LIBS; do
  lib=""; [ "$v" = main ] || lib="$(lib_of $v)"
  TCI_LIB="$lib" run "syn_$v" 300 python3 scripts/synth_dram_time.py 4 1000
done
exit 0
