#!/bin/bash
# GPU iteration: parity tests of the touched areas, the GEMM yardstick vs hipBLASLt, a full bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-dense}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -q --timeout 300 ${TESTS:-tests/test_sharded_gpu.py tests/test_dense_gpu.py tests/test_models_gpu.py tests/test_embed_gpu.py} -m gpu > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 "$OUT/pytest.log"
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 200 python tools/gemm_probe.py > "$OUT/gemm_probe.json" 2>&1; rc=$?; echo "gemm_probe rc=$rc"; tail -1 "$OUT/gemm_probe.json"
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 "$OUT/bench.log" | cut -c1-1500
