#!/bin/bash
# GPU: train-step tests, then the train-step probe at several side-stream Adam grids (RF_ADAM_SIDE_GRID).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-sidegrid}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -q --timeout 300 tests/test_train_step_gpu.py tests/test_tower_train_gpu.py -m gpu > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"
case $rc in 0|1) ;; *) exit $rc;; esac
# GRIDS entries: <side grid>[:<RF_TRAIN_PRIO>]
for e in ${GRIDS:-256 512 1024}; do
  g=${e%%:*}; p=1; [ "$e" != "$g" ] && p=${e#*:}
  RF_ADAM_SIDE_GRID=$g timeout -k 10 300 python tools/train_step_probe.py > "$OUT/probe_${g}_p$p.json" 2>&1 || exit $?
  echo "grid $g prio $p: $(tail -1 "$OUT/probe_${g}_p$p.json" | cut -c1-120)"
done
