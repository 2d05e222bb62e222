#!/bin/bash
# GPU: model / graph / dense tests, then bench's cfg3 and DSSM extras only.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cfg3
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py tests/test_graphs_gpu.py tests/test_dense_gpu.py tests/test_cascade_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/cfg3/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/cfg3/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 40 --warmup 10 --cpu-seconds 0 --no-train --no-pipe --no-sharded --no-cascade > gpurun_out/cfg3/bench.log 2>&1; rc=$?; tail -1 gpurun_out/cfg3/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['extras']; print(json.dumps({k: e[k] for k in ('cfg3_esim_forward','cfg2_dssm_forward')}, indent=1))"; exit $rc
