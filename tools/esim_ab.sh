#!/bin/bash
# ESIM kernel A/B on one GPU box: parity tests of the ESIM paths, the probe on the default build (v5: x from the
# selector MFMA, scalar statistics) and on RF_ESIM_XM=2 (v5, packed statistics) / RF_ESIM_XM=0 (v3), then PMC
# passes on the default. Stops at the first failing step.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
OUT=gpurun_out/${TAG:-esim_ab}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_dense_gpu.py -m gpu -x -q -k "esim" --timeout 120 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for args in "" "--f16" "--L 128" "--L 64 --d 64"; do
  for xm in 1 2 0; do
    RF_ESIM_XM=$xm timeout -k 10 120 python tools/esim_probe.py $args > "$OUT/probe.json" 2>&1 || { cat "$OUT/probe.json"; exit 1; }
    echo "xm=$xm $args: $(tail -1 $OUT/probe.json)"
  done
done
if [ "${PMC:-1}" = 1 ]; then
  PROBE="tools/esim_probe.py --reps 5" TAG="${TAG:-esim_ab}/pmc" PMC_GROUPS="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU
SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
    bash tools/pmc_probe.sh || exit 1
  python tools/pmc_summary.py "$OUT/pmc" esim > "$OUT/pmc_summary.txt"; cat "$OUT/pmc_summary.txt"
fi
