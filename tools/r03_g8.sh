#!/bin/bash
# GPU iteration: encoder parity (lean-path rule hoist), mlp2_small counters, full bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
OUT=gpurun_out/${TAG:-g8}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_embed_gpu.py tests/test_models_gpu.py tests/test_graphs_gpu.py tests/test_sharded_gpu.py tests/test_train_gpu.py -m gpu > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"
[ $rc = 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
i=0
for pmc in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_BUSY_CYCLES" "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pmc --kernel-trace --output-format csv -d "$R/$OUT/pmc$i" -o run -- python3 "$R/tools/mlp_probe.py" > "$R/$OUT/pmc$i.log" 2>&1
  rc=$?; echo "pmc $i rc=$rc"; [ $rc = 0 ] || exit $rc
done
cd "$R"
timeout -k 10 900 python -u bench.py > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 "$OUT/bench.log" > "$OUT/bench.json"; exit $rc
