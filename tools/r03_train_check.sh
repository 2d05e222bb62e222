#!/bin/bash
# GPU: sparse-backward + Adam + tower + train-step tests, then the train-step probe and its kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-trainchk}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest -q --timeout 300 tests/test_train_gpu.py tests/test_train_step_gpu.py tests/test_tower_train_gpu.py -m gpu > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 "$OUT/pytest.log"
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python tools/train_step_probe.py > "$OUT/probe.json" 2>&1 || exit $?
tail -1 "$OUT/probe.json" | cut -c1-300
[ -n "${PROF:-}" ] || exit 0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python tools/train_step_probe.py --steps 8 > "$OUT/prof.log" 2>&1
echo "prof rc=$?"
