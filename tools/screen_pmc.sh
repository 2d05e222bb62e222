# tools/screen_pmc.sh: SQ counters of ip_screen_bf16_kernel (tools/flat_search_trace.py), librf and the lab
# variant librf_nolist (RF_LAB_SCR=8: pre-filter without the list); diagnostics
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM"
for v in base nolist; do
  lib=""; [ "$v" != base ] && lib="$GRAFT_REPO_ROOT/recommendflow_amd/lib/var/librf_$v.so"
  RF_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_$v -o run -- python3 tools/flat_search_trace.py > gpurun_out/pmc_$v.log 2>&1
done
