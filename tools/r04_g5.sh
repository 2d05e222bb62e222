#!/bin/bash
# ESIM v8 (split, 3 WG/CU) vs v6: parity tests, probe timing and stamps per variant; train tests; headline traffic.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04g5}
mkdir -p "$OUT"
T="tests/test_models_gpu.py tests/test_dense_gpu.py tests/test_attention_gpu.py tests/test_train_gpu.py"
timeout -k 10 400 python -u -m pytest $T -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
RF_ESIM_GXM=2 timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gxm2.log" 2>&1
rc=$?; echo "pytest gxm2 rc=$rc"; tail -2 "$OUT/pytest_gxm2.log"; [ $rc -eq 0 ] || exit $rc
probe() {  # name, env...
  local n=$1; shift
  for r in 1 2; do
    env "$@" timeout -k 10 180 python tools/esim_gather_probe.py > "$OUT/esimg_${n}_zipf_$r.json" 2>&1 || return $?
    echo "$n zipf $r: $(tail -1 $OUT/esimg_${n}_zipf_$r.json)"
  done
  env "$@" timeout -k 10 180 python tools/esim_gather_probe.py --uniform > "$OUT/esimg_${n}_uni.json" 2>&1 || return $?
  echo "$n uniform: $(tail -1 $OUT/esimg_${n}_uni.json)"
  env "$@" timeout -k 10 180 python tools/esim_gather_probe.py --stamp --reps 10 > "$OUT/esimg_${n}_stamp.json" 2>&1 || return $?
  grep -v amdgpu.ids $OUT/esimg_${n}_stamp.json | head -n -1 | python -c "
import sys,json
for k,v in json.loads(sys.stdin.read()).items(): print('  ', k, v)"
}
probe v8 RF_ESIM_SPLIT=1 || exit $?
probe v8gxm2 RF_ESIM_SPLIT=1 RF_ESIM_GXM=2 || exit $?
probe v6 RF_ESIM_SPLIT=0 || exit $?
[ "${TRAFFIC:-1}" = 1 ] && { bash tools/r04_traffic.sh || exit $?; }
exit 0
