#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-scorer}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/scorer_probe.py" > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 "$GRAFT_REPO_ROOT/$OUT/prof.log"
head -12 "$GRAFT_REPO_ROOT/$OUT/prof/run_kernel_stats.csv" | cut -d, -f1-4
