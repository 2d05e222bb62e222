#!/bin/bash
# GPU: device-parse parity tests, the pipe tests, then the feature-pipe bench leg alone.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_tfrecord_device_gpu.py tests/test_pipe_gpu.py > gpurun_out/pipe_pytest.log 2>&1 &&
timeout -k 10 400 python -u tools/pipe_bench.py > gpurun_out/pipe_bench.log 2>&1
