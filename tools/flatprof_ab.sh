# tools/flatprof_ab.sh: rocprofv3 kernel stats of the screened Flat search (tools/flat_search_trace.py), the default
# bf16 screen kernel and RF_SCREEN_GEMM=1 (the tile GEMM form), into gpurun_out/fp_new and gpurun_out/fp_old
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fp_new -o run -- python3 tools/flat_search_trace.py > gpurun_out/fp_new.log 2>&1
RF_SCREEN_GEMM=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fp_old -o run -- python3 tools/flat_search_trace.py > gpurun_out/fp_old.log 2>&1
