#!/bin/bash
# GPU A/B of the cfg2 train-step probe over environment settings: CASES="A=1,B=2 A=0 ..." (one probe run each).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-envab}
mkdir -p "$OUT"
i=0
for c in ${CASES:-RF_BWD_FORK=1}; do
  i=$((i+1))
  env $(echo "$c" | tr ',' ' ') timeout -k 10 300 python tools/train_step_probe.py ${PROBE_ARGS:-} > "$OUT/probe_$i.json" 2>&1 || exit $?
  echo "$c: $(tail -1 "$OUT/probe_$i.json" | cut -c1-100)"
done
