#!/bin/bash
# GPU: streamed long-row kernel with conflict-free column mapping — train + sharded parity, cfg4 backward probe,
# cfg2 train probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04cfg4bwd2}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_gpu.py tests/test_sharded_gpu.py tests/test_train_step_gpu.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python tools/cfg4_bwd_probe.py 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
timeout -k 10 400 python tools/train_step_probe.py --steps 40 > "$OUT/probe.json" 2>&1 || { tail -5 "$OUT/probe.json"; exit 1; }
tail -1 "$OUT/probe.json" | cut -c1-200
