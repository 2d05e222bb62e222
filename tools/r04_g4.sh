#!/bin/bash
# ESIM A/B (r04_g3), the training-backward tests incl. the tree-reduce mode, then the headline traffic/counters.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04g4}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_train.log" 2>&1
rc=$?; echo "pytest train rc=$rc"; tail -3 "$OUT/pytest_train.log"; [ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r04g4} bash tools/r04_g3.sh || exit $?
bash tools/r04_traffic.sh || exit $?
