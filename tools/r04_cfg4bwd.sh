#!/bin/bash
# GPU: cfg4 sharded backward, streamed vs legacy long-row kernel, and its kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
OUT=gpurun_out/${TAG:-r04cfg4bwd}
mkdir -p "$OUT"
for k in 0; do
RF_BWD_LONG_LEGACY=$k timeout -k 10 300 python tools/cfg4_bwd_probe.py 2>&1 | grep -v amdgpu.ids | tail -2 || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o run -- python3 "$ROOT/tools/cfg4_bwd_probe.py" > "$ROOT/$OUT/prof.log" 2>&1 || { tail -5 "$ROOT/$OUT/prof.log"; exit 1; }
f=$(find "$ROOT/$OUT/prof" -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:14]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:100]}")
PY
