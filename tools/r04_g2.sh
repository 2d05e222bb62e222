#!/bin/bash
# ESIM gather: parity tests, timing (zipf x2, uniform), the stamped phase breakdown; feature-pipe look-ahead A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04g2}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py tests/test_dense_gpu.py tests/test_attention_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 180 python tools/esim_gather_probe.py > "$OUT/esimg_zipf_$r.json" 2>&1; rc=$?
  echo "zipf $r rc=$rc: $(tail -1 $OUT/esimg_zipf_$r.json)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 180 python tools/esim_gather_probe.py --uniform > "$OUT/esimg_uni.json" 2>&1; rc=$?
echo "uniform rc=$rc: $(tail -1 $OUT/esimg_uni.json)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python tools/esim_gather_probe.py --stamp --reps 10 > "$OUT/esimg_stamp.json" 2>&1; rc=$?
echo "stamp rc=$rc"; cat $OUT/esimg_stamp.json; [ $rc -eq 0 ] || exit $rc
if [ "${PIPE:-1}" = 1 ]; then
  timeout -k 10 300 python tools/pipe_bench.py > "$OUT/pipe_default.json" 2>&1 || exit $?
  RF_TFR_AHEAD_MB=100000 timeout -k 10 300 python tools/pipe_bench.py > "$OUT/pipe_ahead_big.json" 2>&1 || exit $?
  python -c "
import json
for f in ['default', 'ahead_big']:
    d = json.load(open('$OUT/pipe_' + f + '.json'))
    print(f, d['legs_examples_per_s'], d['legs_after_first_batch_examples_per_s'], d['decode_examples_per_s'])"
fi
