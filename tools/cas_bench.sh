#!/bin/bash
# GPU: bench's cascade (cfg5) and DSSM extras only.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cas2
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-train --no-pipe --no-sharded > gpurun_out/cas2/bench.log 2>&1; rc=$?; tail -1 gpurun_out/cas2/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['extras']; print(json.dumps({k: e[k] for k in ('cfg5_cascade','cfg2_dssm_forward')}, indent=1))"; exit $rc
