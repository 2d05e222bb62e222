#!/bin/bash
# GPU: the cfg2 train-step probe and its rocprofv3 kernel stats at HEAD.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
OUT=gpurun_out/${TAG:-r04train}
mkdir -p "$OUT"
timeout -k 10 300 python tools/train_step_probe.py > "$OUT/probe.json" 2>&1 || { tail -5 "$OUT/probe.json"; exit 1; }
tail -1 "$OUT/probe.json" | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o run -- python3 "$ROOT/tools/train_step_probe.py" --steps 8 > "$ROOT/$OUT/prof.log" 2>&1 || { tail -5 "$ROOT/$OUT/prof.log"; exit 1; }
f=$(find "$ROOT/$OUT/prof" -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
tot=sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:30]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us {100*float(r['TotalDurationNs'])/tot:5.1f}%  {r['Name'][:100]}")
PY
