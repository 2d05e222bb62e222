#!/bin/bash
# sparse-encoder GPU session: embed parity tests, then the cfg3 encoder probe
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-enc}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_embed_gpu.py tests/test_models_gpu.py tests/test_graphs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/cfg3_encoder_probe.py > "$OUT/probe.json" 2>&1; rc=$?; tail -1 "$OUT/probe.json"; exit $rc
