#!/bin/bash
# GPU iteration: fp32 GEMM variants (LDS-DMA ring, split-K counts, register-staged) on the GEMM yardstick.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-f32}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -q --timeout 300 ${TESTS:-tests/test_dense_gpu.py tests/test_models_gpu.py} -m gpu > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 "$OUT/pytest.log"
case $rc in 0|1) ;; *) exit $rc;; esac
for v in "default" "RF_SPLITK=1" "RF_SPLITK=4" "RF_GEMM_LDS=0"; do
  env_args=""; [ "$v" != default ] && env_args="$v"
  env $env_args timeout -k 10 200 python tools/gemm_probe.py > "$OUT/gemm_probe_${v}.json" 2>&1; rc=$?
  echo "$v rc=$rc"; tail -1 "$OUT/gemm_probe_${v}.json"
  case $rc in 0) ;; *) exit $rc;; esac
done
