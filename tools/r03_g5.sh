#!/bin/bash
# GPU iteration: cfg3 forward with the input MLP concurrent vs serial (wall + kernel traces); mlp2_small alone.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=gpurun_out/${TAG:-g5}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in conc serial; do
  A=""; [ $v = serial ] && A="--serial-mlp"
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/$OUT/prof_$v" -o run --output-format csv -- python3 "$R/tools/cfg3_gaps.py" $A > "$R/$OUT/prof_$v.log" 2>&1
  rc=$?; echo "$v rocprof rc=$rc"; grep forward "$R/$OUT/prof_$v.log"
  [ $rc = 0 ] || exit $rc
  python3 "$R/tools/trace_gaps.py" "$R/$OUT/prof_$v/run_kernel_trace.csv" --last 200
done
cd "$R"
for v in conc serial; do A=""; [ $v = serial ] && A="--serial-mlp"; timeout -k 10 200 python3 tools/cfg3_gaps.py $A; done
