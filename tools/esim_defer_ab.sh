#!/bin/bash
# ESIM deferred-store A/B: parity of the ESIM paths on the new build, then the probe on the new build and on
# the previous build (RF_LIB=recommendflow_amd/lib/ab/librf_prev.so), alternating. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/esim_defer; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dense_gpu.py -k "esim" tests/test_models_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for args in "" "--f16" "--L 128" "--L 64 --d 64"; do
  for r in 1 2; do
    echo "new $args: $(timeout -k 10 120 python tools/esim_probe.py --reps 100 $args | tail -1)" || exit 1
    echo "prev $args: $(RF_LIB=recommendflow_amd/lib/ab/librf_prev.so timeout -k 10 120 python tools/esim_probe.py --reps 100 $args | tail -1)" || exit 1
  done
done 2>&1 | tee $OUT/ab.txt
