#!/bin/bash
# GPU iteration: example-major id pass (parity via the gather tests), forward timing vs the slot-major pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=gpurun_out/${TAG:-g13}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_models_gpu.py tests/test_cascade_gpu.py -m gpu > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"
[ $rc = 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 python3 tools/cfg3_gaps.py --serial-mlp --gather || exit 1
  RF_IDS_SLOT_MAJOR=1 timeout -k 10 200 python3 tools/cfg3_gaps.py --serial-mlp --gather || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/$OUT/prof" -o run --output-format csv -- python3 "$R/tools/cfg3_gaps.py" --serial-mlp --gather > "$R/$OUT/prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; grep forward "$R/$OUT/prof.log"
python3 "$R/tools/trace_gaps.py" "$R/$OUT/prof/run_kernel_trace.csv" --last 175
