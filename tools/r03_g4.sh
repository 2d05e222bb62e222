#!/bin/bash
# GPU iteration: prod_lab (isolated + chained GEMM pair), its kernel trace; dense parity tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=gpurun_out/${TAG:-g4}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread ${TESTS:-tests/test_dense_gpu.py tests/test_models_gpu.py} -m gpu > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"
[ $rc = 0 ] || exit $rc
timeout -k 10 120 ./tools/prod_lab 3 > "$OUT/prod.txt" 2>&1; rc=$?; echo "prod_lab rc=$rc"; cat "$OUT/prod.txt"
[ $rc = 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/$OUT/prof" -o run --output-format csv -- "$R/tools/prod_lab" 1 > "$R/$OUT/prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
python3 "$R/tools/trace_gaps.py" "$R/$OUT/prof/run_kernel_trace.csv" --last 40
