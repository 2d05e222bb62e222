# tools/screen_ablate.sh: ip_screen_bf16_kernel time per launch for librf and the lab variants built by
#   bash tools/build_variants.sh rf_dense.hip noepi "-DRF_LAB_SCR=1" onlydma "-DRF_LAB_SCR=3" nodma "-DRF_LAB_SCR=4"
# (rocprofv3 kernel stats of tools/flat_search_trace.py; diagnostics)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base ${VARIANTS:-noepi onlydma nodma}; do
  lib=""; [ "$v" != base ] && lib="$GRAFT_REPO_ROOT/recommendflow_amd/lib/var/librf_$v.so"
  RF_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sa_$v -o run -- python3 tools/flat_search_trace.py > gpurun_out/sa_$v.log 2>&1
  f=$(find gpurun_out/sa_$v -name "*kernel_stats.csv" | head -1)
  echo "$v $(grep ip_screen_bf16 $f | awk -F'","' '{print $0}' | python3 -c 'import sys,csv; r=list(csv.reader(sys.stdin)); print([(x[0][:40], x[1], x[3]) for x in r])')"
done
