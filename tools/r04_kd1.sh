#!/bin/bash
# GPU: D <= 64 streamed long-row kernel, 16 vs 8 waves (RF_BWD_LONG_KD1_8W) — long-segment parity at both, cfg2
# train probe A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04kd1}
mkdir -p "$OUT"
RF_BWD_LONG_KD1_8W=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_gpu.py -k "long_segments or cfg2_full or every_combiner" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for k in 1 0 1 0; do
RF_BWD_LONG_KD1_8W=$k timeout -k 10 400 python tools/train_step_probe.py --steps 40 > "$OUT/probe_$k.json" 2>&1 || { tail -5 "$OUT/probe_$k.json"; exit 1; }
echo "kd1_8w=$k $(tail -1 "$OUT/probe_$k.json" | cut -c1-150)"
done
