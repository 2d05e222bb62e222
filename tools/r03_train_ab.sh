#!/bin/bash
# GPU: DSSM train-step A/B (table Adam overlapped on a side stream, side-grid sizes) on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-trainab}
mkdir -p "$OUT"
for v in "RF_TRAIN_OVERLAP=0" "RF_ADAM_SIDE_GRID=512" "RF_ADAM_SIDE_GRID=256" "RF_ADAM_SIDE_GRID=128" "RF_ADAM_SIDE_GRID=65536"; do
  env $v timeout -k 10 300 python tools/train_step_probe.py --steps 40 > "$OUT/probe_$v.json" 2>&1; rc=$?
  echo "$v rc=$rc: $(tail -1 $OUT/probe_$v.json | cut -c1-260)"
  case $rc in 0) ;; *) exit $rc;; esac
done
