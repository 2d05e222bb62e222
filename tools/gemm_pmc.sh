#!/bin/bash
# GPU: counter passes over the cfg3 1280->1024 GEMM (one pass per counter group).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/gemmpmc
for v in 0 1; do
  export RF_GEMM_PP=$v
  i=0
  for pmc in "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS" "FETCH_SIZE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $pmc --kernel-trace --output-format csv -d gpurun_out/gemmpmc/pp${v}_p$i -o run -- python3 tools/gemm_one.py 4096 1280 1024 30 > gpurun_out/gemmpmc/pp${v}_p$i.log 2>&1 || exit 1
  done
done
