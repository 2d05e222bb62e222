#!/bin/bash
# GPU: deferred (replayed) dense table Adam — parity tests, the cfg2 train-step probe (deferred line + split A/B),
# and the kernel stats of the deferred step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
OUT=gpurun_out/${TAG:-r04defer}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_gpu.py tests/test_train_step_gpu.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for k in 1 2; do
  timeout -k 10 400 python tools/train_step_probe.py --steps 30 > "$OUT/probe_$k.json" 2>&1 || { tail -5 "$OUT/probe_$k.json"; exit 1; }
  tail -1 "$OUT/probe_$k.json" | cut -c1-900
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o run -- python3 "$ROOT/tools/train_step_probe.py" --steps 8 > "$ROOT/$OUT/prof.log" 2>&1 || { tail -5 "$ROOT/$OUT/prof.log"; exit 1; }
f=$(find "$ROOT/$OUT/prof" -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
tot=sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:25]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.3f} ms {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us {100*float(r['TotalDurationNs'])/tot:5.1f}%  {r['Name'][:100]}")
PY
