#!/bin/bash
# GPU: PMC counters of every kernel of the cfg3 forward (gather path, fused scorer), two passes over
# tools/cfg3_gaps.py --serial-mlp --gather; summary per kernel by tools/pmc_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
OUT=gpurun_out/${TAG:-r04cfg3pmc}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
n=0
while read -r group; do
  [ -z "$group" ] && continue
  n=$((n+1))
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $group -d "$ROOT/$OUT/pmc_$n" -o run --output-format csv -- \
     python3 $ROOT/tools/cfg3_gaps.py --serial-mlp --gather > "$ROOT/$OUT/pmc_$n.log" 2>&1
  rc=$?; echo "pmc pass $n rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$ROOT/$OUT/pmc_$n.log"; exit $rc; fi
done <<LIST
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES
SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE
LIST
cd "$ROOT"
python tools/pmc_summary.py "$OUT" > "$OUT/summary.txt" 2>&1
grep -A17 "mlp2_small\|single_token_ids_multi\|gemm_lds_kernel<64, 3\|gemm_lds_kernel<64, 4\|head_softmax" "$OUT/summary.txt" | head -120
