set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_cascade_gpu.py tests/test_sharded_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/cas_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/cas_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-extras --no-train --no-pipe --no-sharded --cascade-sharded --catalog 200000 > gpurun_out/cas_bench.log 2>&1; rc=$?; tail -c 1500 gpurun_out/cas_bench.log; exit $rc
