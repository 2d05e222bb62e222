#!/bin/bash
# Multiply-high bucket modulus A/B: the bit-exact embedding suites on the new build, then the headline bench
# (no extras) on the new build and on the previous one (RF_LIB=recommendflow_amd/lib/ab/librf_prev.so), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/hashmod; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_embed_gpu.py tests/test_train_gpu.py tests/test_sharded_gpu.py tests/test_factory_gpu.py tests/test_pipe_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
A="--cpu-seconds 0 --no-extras --no-sharded --no-pipe --no-train --no-shard-train --no-cascade --steps 200"
for r in 1 2 3; do
  echo "new: $(timeout -k 10 200 python bench.py $A | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"], d["roofline"]["frac"])')" || exit 1
  echo "prev: $(RF_LIB=recommendflow_amd/lib/ab/librf_prev.so timeout -k 10 200 python bench.py $A | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_ms"], d["roofline"]["frac"])')" || exit 1
done 2>&1 | grep -v amdgpu.ids | tee $OUT/ab.txt
