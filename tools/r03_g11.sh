#!/bin/bash
# GPU iteration: model / cascade / graph parity with the gather path as default, then the full bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=gpurun_out/${TAG:-g11}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_models_gpu.py tests/test_cascade_gpu.py tests/test_graphs_gpu.py tests/test_factory_gpu.py tests/test_library.py -m gpu > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest.log"
[ $rc = 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 "$OUT/bench.log" > "$OUT/bench.json"; exit $rc
