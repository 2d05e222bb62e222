#!/bin/bash
# GPU: device-parse pipe breakdown (host half, H2D, parse kernels, whole pipe) at 16 and 32 threads.
set -o pipefail
mkdir -p gpurun_out/pipeprof
timeout -k 10 300 python -u tools/pipe_probe_gpu.py 16 > gpurun_out/pipeprof/probe16.json 2>&1 &&
timeout -k 10 300 python -u tools/pipe_probe_gpu.py 32 > gpurun_out/pipeprof/probe32.json 2>&1 &&
timeout -k 10 300 python -u tools/pipe_bench.py > gpurun_out/pipeprof/bench.json 2>&1
