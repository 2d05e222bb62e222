#!/bin/bash
# GPU: D = 128 streamed long-row kernel, <8 waves, 64 positions per chunk> vs <16 waves, 32> (RF_BWD_LONG_KD2_NARROW)
# — train / sharded parity, cfg4 backward probe A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04cfg4bwd5}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_gpu.py tests/test_sharded_gpu.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for k in 0 1 0 1; do
RF_BWD_LONG_KD2_NARROW=$k timeout -k 10 300 python tools/cfg4_bwd_probe.py 2>&1 | grep -v amdgpu.ids | tail -1 | sed "s/^/narrow=$k /" || exit 1
done
