#!/bin/bash
# GPU: dense probe + bench's cfg3/DSSM extras (no tests).
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cfg3p
timeout -k 10 200 python tools/dense_probe.py > gpurun_out/cfg3p/probe.json 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 40 --warmup 10 --cpu-seconds 0 --no-train --no-pipe --no-sharded --no-cascade > gpurun_out/cfg3p/bench.log 2>&1; rc=$?; tail -1 gpurun_out/cfg3p/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['extras']; print(json.dumps({k: e[k] for k in ('cfg3_esim_forward','cfg2_dssm_forward')}, indent=1))"; exit $rc
