#!/bin/bash
# GPU A/B of the train step: tower-kernel tests, the probe on this tree's librf.so and on tools/abl/librf_head.so
# (the last commit's build), then a kernel trace of this tree's probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab2}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -q --timeout 200 tests/test_tower_train_gpu.py -m gpu > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest.log"
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python tools/train_step_probe.py > "$OUT/probe_new.json" 2>&1 || exit $?
tail -1 "$OUT/probe_new.json" | cut -c1-300
[ -n "${SKIP_HEAD:-}" ] || RF_LIB=tools/abl/librf_head.so timeout -k 10 300 python tools/train_step_probe.py > "$OUT/probe_head.json" 2>&1 || exit $?
[ -n "${SKIP_HEAD:-}" ] || tail -1 "$OUT/probe_head.json" | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python tools/train_step_probe.py --steps 8 > "$OUT/prof.log" 2>&1
echo "prof rc=$?"
