#!/bin/bash
# dense-stage GPU session: dense/graph/model/cascade tests, the per-launch probe, the GEMM yardstick
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-dense}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_dense_gpu.py tests/test_graphs_gpu.py tests/test_models_gpu.py tests/test_cascade_gpu.py tests/test_attention_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python tools/dense_probe.py > "$OUT/probe.json" 2>&1 || exit 1
timeout -k 10 100 python tools/gemm_probe.py > "$OUT/gemm.json" 2>&1; exit $?
