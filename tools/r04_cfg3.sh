#!/bin/bash
# GPU: cfg3 forward (gather path, serial input MLP) kernel trace + per-kernel gaps at HEAD.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
OUT=gpurun_out/${TAG:-r04cfg3}
mkdir -p "$OUT"
timeout -k 10 200 python3 tools/cfg3_gaps.py --serial-mlp --gather > "$OUT/plain.txt" 2>&1 || { tail -5 "$OUT/plain.txt"; exit 1; }
tail -2 "$OUT/plain.txt"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$ROOT/$OUT/prof" -o run --output-format csv -- python3 "$ROOT/tools/cfg3_gaps.py" --serial-mlp --gather > "$ROOT/$OUT/prof.log" 2>&1 || { tail -5 "$ROOT/$OUT/prof.log"; exit 1; }
f=$(find "$ROOT/$OUT/prof" -name "*kernel_trace.csv" | head -1)
python3 "$ROOT/tools/trace_gaps.py" "$f" --last 280 > "$ROOT/$OUT/gaps.txt" 2>&1
cat "$ROOT/$OUT/gaps.txt" | head -20
