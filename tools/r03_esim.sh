#!/bin/bash
# GPU iteration: ESIM A/B (previous librf.so in tools/abl vs the working tree), plus the fp32 GEMM lab.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-esim}
mkdir -p "$OUT"
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest -q --timeout 200 $TESTS -m gpu > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -8 "$OUT/pytest.log"
  case $rc in 0|1) ;; *) exit $rc;; esac
fi
for r in 1 2; do
  for v in prev new; do
    if [ $v = prev ]; then export RF_LIB=$PWD/tools/abl/librf_prev.so; else unset RF_LIB; fi
    timeout -k 10 120 python tools/esim_probe.py ${ESIM_ARGS:-} > "$OUT/esim_${v}_$r.json" 2>&1; rc=$?
    echo "$v round $r rc=$rc: $(tail -1 $OUT/esim_${v}_$r.json)"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
unset RF_LIB
if [ -x tools/gemm_lab_f32 ] && [ -n "${LAB:-}" ]; then
  timeout -k 10 240 ./tools/gemm_lab_f32 5 > "$OUT/gemm_lab_f32.txt" 2>&1; rc=$?; echo "lab rc=$rc"; cat "$OUT/gemm_lab_f32.txt"
fi
