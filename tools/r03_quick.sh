#!/bin/bash
# Quick GPU iteration for round 3: GEMM lab, the sharded/graph parity tests, the cfg4 bench leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-quick}
mkdir -p "$OUT"
if [ "${LAB:-1}" = 1 ]; then
  timeout -k 10 240 ./tools/gemm_lab 5 > "$OUT/gemm_lab.txt" 2>&1; rc=$?; echo "gemm_lab rc=$rc"; cat "$OUT/gemm_lab.txt"
  case $rc in 0) ;; *) exit $rc;; esac
fi
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 ${TESTS:-tests/test_sharded_gpu.py tests/test_graphs_gpu.py tests/test_embed_gpu.py tests/test_cfg1_gpu.py} -m gpu > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 "$OUT/pytest.log"
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 600 python bench.py --no-extras --no-cascade --no-pipe --cpu-seconds 0 --no-probes --no-uniform-leg ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 "$OUT/bench.log" | cut -c1-3000
timeout -k 10 300 python tools/cfg3_encoder_probe.py > "$OUT/cfg3_probe.json" 2>&1; rc=$?; echo "cfg3 probe rc=$rc"; tail -2 "$OUT/cfg3_probe.json"
