#!/bin/bash
# GPU iteration: dense/model parity (mlp2 v2), mlp_probe kernel durations, cfg3 forward traces.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=gpurun_out/${TAG:-g9}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dense_gpu.py tests/test_models_gpu.py -m gpu > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"
[ $rc = 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$R/$OUT/mlp" -o run --output-format csv -- python3 "$R/tools/mlp_probe.py" > "$R/$OUT/mlp.log" 2>&1
rc=$?; echo "mlp probe rc=$rc"; grep -i "mlp2\|Name" "$R/$OUT/mlp/run_kernel_stats.csv" | cut -d, -f1-4
[ $rc = 0 ] || exit $rc
cd "$R"
TAG=${TAG:-g9} bash tools/r03_g5.sh
