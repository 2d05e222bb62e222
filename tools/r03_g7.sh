#!/bin/bash
# GPU iteration: dense/model parity tests, then the cfg3 forward (input MLP concurrent / serial) kernel traces.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=gpurun_out/${TAG:-g7}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread ${TESTS:-tests/test_dense_gpu.py tests/test_models_gpu.py} -m gpu > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"
[ $rc = 0 ] || exit $rc
TAG=${TAG:-g7} bash tools/r03_g5.sh
