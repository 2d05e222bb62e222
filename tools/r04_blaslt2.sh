#!/bin/bash
# GPU: fp32 deep-K layers on hipBLASLt (RF_TOWER_BLASLT_WIDE) — the GPU suite, then a same-box A/B of the DSSM
# towers forward probe.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04blaslt2}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for k in 1 0 1 0; do
echo "blaslt_wide=$k"
RF_TOWER_BLASLT_WIDE=$k timeout -k 10 200 python tools/dssm_towers_probe.py 2>&1 | grep -v amdgpu.ids | tail -3 || exit 1
done
