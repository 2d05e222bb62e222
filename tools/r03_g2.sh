#!/bin/bash
# GPU iteration: GEMM epilogue A/B (prod_lab), dense/model parity tests, the cfg3 forward's kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=gpurun_out/${TAG:-g2}
mkdir -p "$OUT"
timeout -k 10 120 ./tools/prod_lab 3 > "$OUT/prod.txt" 2>&1; rc=$?; echo "prod_lab rc=$rc"; head -12 "$OUT/prod.txt"
[ $rc = 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread ${TESTS:-tests/test_dense_gpu.py tests/test_models_gpu.py} -m gpu > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"
[ $rc = 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/$OUT/prof" -o run --output-format csv -- python3 "$R/tools/cfg3_gaps.py" > "$R/$OUT/prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; grep forward "$R/$OUT/prof.log"
python3 "$R/tools/trace_gaps.py" "$R/$OUT/prof/run_kernel_trace.csv" --last 200
