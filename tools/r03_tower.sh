#!/bin/bash
# GPU iteration: tower-training parity, the train-step tests, then the bench's DSSM train-step leg alone.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-tower}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -q --timeout 300 ${TESTS:-tests/test_tower_train_gpu.py tests/test_train_step_gpu.py} -m gpu > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 "$OUT/pytest.log"
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python tools/train_step_probe.py > "$OUT/train_probe.json" 2>&1; rc=$?; echo "probe rc=$rc"; tail -3 "$OUT/train_probe.json"
