#!/bin/bash
# GPU: the towers' wide input layers on hipBLASLt vs rf_linear_splitk_fwd — tower parity tests and a same-box
# A/B of the cfg2 train probe (RF_TOWER_BLASLT_WIDE).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04blaslt}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_tower_train_gpu.py tests/test_train_step_gpu.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for k in 1 0 1 0; do
RF_TOWER_BLASLT_WIDE=$k timeout -k 10 400 python tools/train_step_probe.py --steps 40 > "$OUT/probe_$k.json" 2>&1 || { tail -5 "$OUT/probe_$k.json"; exit 1; }
echo "blaslt_wide=$k $(tail -1 "$OUT/probe_$k.json" | cut -c1-90)"
done
