#!/bin/bash
# ESIM training step (tools/esim_train_probe.py): PMC passes, one counter group per rocprofv3 run, kernel-trace only.
set -u
ROOT="${GRAFT_REPO_ROOT}"
OUT="$ROOT/gpurun_out/${TAG:-tpmc}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
n=0
while read -r group; do
  [ -z "$group" ] && continue
  n=$((n+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $group -d "$OUT/pmc_$n" -o run --output-format csv -- \
     python3 "$ROOT/tools/esim_train_probe.py" 5 > "$OUT/pmc_$n.log" 2>&1
  rc=$?; echo "pmc pass $n ($group) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/pmc_$n.log"; exit $rc; fi
done <<LIST
FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_BUSY_CYCLES
TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
LIST
