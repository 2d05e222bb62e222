#!/bin/bash
# GPU suite (all -m gpu tests), ESIM gather probe + stamps, then the full bench line (all legs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04g6}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 180 python tools/esim_gather_probe.py > "$OUT/esimg_zipf_$r.json" 2>&1 || exit $?
  echo "zipf $r: $(tail -1 $OUT/esimg_zipf_$r.json)"
done
timeout -k 10 180 python tools/esim_gather_probe.py --uniform > "$OUT/esimg_uni.json" 2>&1 || exit $?
echo "uniform: $(tail -1 $OUT/esimg_uni.json)"
timeout -k 10 180 python tools/esim_gather_probe.py --stamp --reps 10 > "$OUT/esimg_stamp.json" 2>&1 || exit $?
grep -v amdgpu.ids $OUT/esimg_stamp.json | head -n -1 | python -c "
import sys,json
for k,v in json.loads(sys.stdin.read()).items(): print('  ', k, v)"
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"
python tools/headline_summary.py "$OUT/bench.log" 2>/dev/null | head -0
python - "$OUT/bench.log" <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{')][-1]; d=json.loads(l)
print('headline', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'], 'uniform', (d['roofline'].get('uniform') or {}).get('kernel_ms'))
e=d.get('extras') or {}
for k in ('cfg3_esim_forward','cfg2_dssm_forward','cfg2_dssm_train_step','feature_pipe','cfg1_demo_two_tower','cfg5_cascade'):
    v=e.get(k); print(k, json.dumps(v)[:700] if v else v)
print('cfg4', json.dumps(d.get('cfg4_sharded'))[:1500])
PY
exit $rc
