#!/bin/bash
# GPU iteration: ESIM gather path parity, then cfg3 forward timing/traces with and without it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=gpurun_out/${TAG:-g10}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_models_gpu.py tests/test_dense_gpu.py tests/test_embed_gpu.py -m gpu > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 "$OUT/pytest.log"
[ $rc = 0 ] || exit $rc
for v in plain gather; do A="--serial-mlp"; [ $v = gather ] && A="--serial-mlp --gather"
  timeout -k 10 200 python3 tools/cfg3_gaps.py $A; rc=$?; [ $rc = 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/$OUT/prof_gather" -o run --output-format csv -- python3 "$R/tools/cfg3_gaps.py" --serial-mlp --gather > "$R/$OUT/prof_gather.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; grep forward "$R/$OUT/prof_gather.log"
python3 "$R/tools/trace_gaps.py" "$R/$OUT/prof_gather/run_kernel_trace.csv" --last 175
