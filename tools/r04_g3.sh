#!/bin/bash
# ESIM gather A/B: parity tests (default + RF_ESIM_GXM=2), probe timing per variant (zipf x2, uniform), stamps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04g3}
mkdir -p "$OUT"
T="tests/test_models_gpu.py tests/test_dense_gpu.py tests/test_attention_gpu.py"
timeout -k 10 300 python -u -m pytest $T -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
RF_ESIM_GXM=2 timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gxm2.log" 2>&1
rc=$?; echo "pytest gxm2 rc=$rc"; tail -2 "$OUT/pytest_gxm2.log"; [ $rc -eq 0 ] || exit $rc
for v in 1 2; do
  for r in 1 2; do
    RF_ESIM_GXM=$v timeout -k 10 180 python tools/esim_gather_probe.py > "$OUT/esimg_gxm${v}_zipf_$r.json" 2>&1; rc=$?
    echo "gxm$v zipf $r rc=$rc: $(tail -1 $OUT/esimg_gxm${v}_zipf_$r.json)"; [ $rc -eq 0 ] || exit $rc
  done
  RF_ESIM_GXM=$v timeout -k 10 180 python tools/esim_gather_probe.py --uniform > "$OUT/esimg_gxm${v}_uni.json" 2>&1; rc=$?
  echo "gxm$v uniform rc=$rc: $(tail -1 $OUT/esimg_gxm${v}_uni.json)"; [ $rc -eq 0 ] || exit $rc
  RF_ESIM_GXM=$v timeout -k 10 180 python tools/esim_gather_probe.py --stamp --reps 10 > "$OUT/esimg_gxm${v}_stamp.json" 2>&1; rc=$?
  echo "gxm$v stamp rc=$rc"; grep -v amdgpu.ids $OUT/esimg_gxm${v}_stamp.json | python -c "
import sys,json
t=sys.stdin.read(); j=json.loads(t[:t.rfind('}', 0, t.rfind('{'))+1])
for k,v in j.items(): print(k, v)"; [ $rc -eq 0 ] || exit $rc
done
