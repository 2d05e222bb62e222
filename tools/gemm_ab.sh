set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_dense_gpu.py tests/test_models_gpu.py -m gpu -x -q -k "dense or mlp or model" --timeout 120 --timeout-method thread > gpurun_out/gemm_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/gemm_pytest.log; [ $rc -eq 0 ] || exit $rc
for v in "" "RF_GEMM_BM=64" "RF_GEMM_BM=128" "RF_GEMM_LDS=0"; do echo "== $v"; env $v timeout -k 10 100 python tools/gemm_probe.py || exit 1; done
