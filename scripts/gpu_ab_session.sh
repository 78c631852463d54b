#!/usr/bin/env bash
# One parameterised A/B session on the GPU box (replaces the one-off gpu_r04*.sh launchers).
# Every step is optional, runs under its own time limit, and a fault / abort / timeout ends the
# session (no retries). Libraries: "main" = the in-tree build, NAME = build/ab/libtci_NAME.so
# (built here beforehand: python scripts/ab_variants.py --build --variants ...).
#   LK="old,ship"        likelihood-kernel A/B in one process (scripts/ab_variants.py --run)
#   DRAM="main new"      rocprofv3 kernel stats of a DRAM fit per library (scripts/gpu_dram_prof.sh),
#     WORK=td|syn4|syn5  the 299-cell TestData fit or the config-4/5 fits, STEPS steps
#   EQ="new"             each library bitwise against build/ab/libtci_old.so on the same fits
#     EQ_STEPS=1000 EQ_CELLS=299 EQ_CFG=0|4|5 TCI_ENGINE=auto|fused|walk|batched
#   TESTS="expr"         pytest -m gpu -k expr (TESTS=all: the whole GPU suite)
# Usage: LK=old,ship TESTS=parity bash scripts/gpu_ab_session.sh TAG
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out"; TAG="${1:-ab}"
mkdir -p "$OUT"; cd "$ROOT"
stop() { echo "step ended with status $1 -- stopping"; exit "$1"; }
if [ -n "${LK:-}" ]; then
  echo "== likelihood A/B: $LK"
  timeout -k 10 300 python scripts/ab_variants.py --run --variants "$LK" ${LK_ARGS:-} > "$OUT/${TAG}_lk.json" 2> "$OUT/${TAG}_lk.err"
  rc=$?; cat "$OUT/${TAG}_lk.json"; [ $rc -eq 0 ] || { tail -20 "$OUT/${TAG}_lk.err"; stop $rc; }
fi
if [ -n "${DRAM:-}" ]; then
  echo "== DRAM kernel stats: $DRAM (WORK=${WORK:-td}, STEPS=${STEPS:-20000})"
  VARIANTS="$DRAM" WORK="${WORK:-td}" bash scripts/gpu_dram_prof.sh "${TAG}_dram" "${STEPS:-20000}" || stop $?
fi
if [ -n "${EQ:-}" ]; then
  for v in $EQ; do
    lib="$v"; [ "$v" = main ] || lib="$ROOT/build/ab/libtci_$v.so"
    echo "== bitwise: $v against old"
    timeout -k 10 300 python3 scripts/dram_lib_equal.py "$ROOT/build/ab/libtci_old.so" "$lib" "${EQ_STEPS:-1000}" \
      "${EQ_CELLS:-299}" "${EQ_CFG:-0}" > "$OUT/${TAG}_eq_$v.json" 2>&1
    rc=$?; cat "$OUT/${TAG}_eq_$v.json"; [ $rc -eq 0 ] || stop $rc
  done
fi
if [ -n "${TESTS:-}" ]; then
  echo "== pytest -m gpu ${TESTS}"
  K=(); [ "$TESTS" = all ] || K=(-k "$TESTS")
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    "${K[@]}" > "$OUT/${TAG}_pytest.log" 2>&1
  rc=$?; tail -8 "$OUT/${TAG}_pytest.log"; [ $rc -eq 0 ] || stop $rc
fi
exit 0
