#!/bin/bash
# GPU: fused cosine + cosent loss — tower / train-step parity tests and same-box A/Bs of the cfg2 train probe
# (RF_FUSED_LOSS, RF_SMALL_MM_ROCBLAS).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04loss}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tower_train_gpu.py tests/test_train_step_gpu.py tests/test_losses.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for k in "1 0" "0 0" "1 1" "1 0" "0 0" "1 1"; do
set -- $k
RF_FUSED_LOSS=$1 RF_SMALL_MM_ROCBLAS=$2 timeout -k 10 400 python tools/train_step_probe.py --steps 40 > "$OUT/probe_$1$2.json" 2>&1 || { tail -5 "$OUT/probe_$1$2.json"; exit 1; }
echo "fused=$1 rocblas_small=$2 $(tail -1 "$OUT/probe_$1$2.json" | cut -c1-90)"
done
