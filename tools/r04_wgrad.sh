#!/bin/bash
# GPU: towers' input-layer weight gradient on a side stream — same-box A/B of the cfg2 train probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04wgrad}
mkdir -p "$OUT"
for k in 1 0 1 0; do
RF_WGRAD_OVERLAP=$k timeout -k 10 400 python tools/train_step_probe.py --steps 40 > "$OUT/probe_$k.json" 2>&1 || { tail -5 "$OUT/probe_$k.json"; exit 1; }
echo "overlap=$k $(tail -1 "$OUT/probe_$k.json" | cut -c1-120)"
done
