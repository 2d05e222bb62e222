#!/bin/bash
# Round 4 final GPU session: the whole -m gpu suite, smoke(), the default bench line, then the same bench command
# under rocprofv3 --kernel-trace --stats (headline timed-window summary), each step under its own time limit;
# stops at the first step that faults, aborts or times out.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
OUT=gpurun_out/${TAG:-r04final}
mkdir -p "$OUT"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 700 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/bench.err"; exit $rc; }
python - "$OUT/bench.json" <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{')][-1]; d=json.loads(l)
r=d['roofline']
print('headline', d['value'], r['kernel_ms'], r['frac'], r.get('frac_of_peak_measured'), 'uniform', (r.get('uniform') or {}).get('kernel_ms'))
e=d.get('extras') or {}
for k in ('cfg3_esim_forward','cfg2_dssm_forward','cfg2_dssm_train_step','feature_pipe'):
    v=e.get(k); print(k, json.dumps(v)[:600] if v else v)
c=d.get('cfg4_sharded') or {}
print('cfg4', c.get('ms_per_step'), json.dumps(c.get('simulated_p8'))[:600])
PY
[ "${SKIP_PROF:-0}" = 1 ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o run -- python3 "$ROOT/bench.py" > "$ROOT/$OUT/bench_prof.json" 2> "$ROOT/$OUT/bench_prof.err"
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$ROOT/$OUT/bench_prof.err"; exit $rc; }
cd "$ROOT"
python tools/headline_summary.py "$OUT/prof" "$OUT/bench_prof.json" --write-trace "$OUT/headline_kernel_trace.csv" > "$OUT/headline_summary.txt" 2>&1
tail -8 "$OUT/headline_summary.txt"
