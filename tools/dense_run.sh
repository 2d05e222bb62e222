#!/bin/bash
# dense-stage GPU session: norm / MLP / graph tests, then the per-launch probe (graph-timed)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-dense}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_dense_gpu.py tests/test_graphs_gpu.py tests/test_models_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python tools/dense_probe.py > "$OUT/probe.json" 2>&1; rc=$?; cat "$OUT/probe.json"; exit $rc
