#!/bin/bash
# GPU: minimum K for the hipBLASLt route of fp32 tower layers — towers forward probe and cfg2 train probe, same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04blaslt3}
mkdir -p "$OUT"
for k in 4096 256 4096 256; do
echo "min_k=$k $(RF_TOWER_BLASLT_MIN_K=$k timeout -k 10 200 python tools/dssm_towers_probe.py 2>&1 | grep towers | tail -1)"
RF_TOWER_BLASLT_MIN_K=$k timeout -k 10 400 python tools/train_step_probe.py --steps 40 > "$OUT/probe_$k.json" 2>&1 || { tail -5 "$OUT/probe_$k.json"; exit 1; }
echo "min_k=$k train $(tail -1 "$OUT/probe_$k.json" | cut -c1-70)"
done
