#!/bin/bash
# GPU: deferred Adam with compare-and-swap row claims — train + sharded parity tests, cfg2 train probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04defer2}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train_gpu.py tests/test_train_step_gpu.py tests/test_sharded_gpu.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 400 python tools/train_step_probe.py --steps 30 > "$OUT/probe.json" 2>&1 || { tail -5 "$OUT/probe.json"; exit 1; }
tail -1 "$OUT/probe.json" | cut -c1-700
