#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
OUT=gpurun_out/${TAG:-r04route}
mkdir -p "$OUT"
timeout -k 10 200 python tools/route_probe.py > "$OUT/route.txt" 2>&1 || { tail -5 "$OUT/route.txt"; exit 1; }
tail -1 "$OUT/route.txt"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" -o run --output-format csv -- python3 "$ROOT/tools/route_probe.py" > "$ROOT/$OUT/prof.log" 2>&1 || { tail -5 "$ROOT/$OUT/prof.log"; exit 1; }
f=$(find "$ROOT/$OUT/prof" -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:14]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:100]}")
PY
