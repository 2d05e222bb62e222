#!/bin/bash
# Headline kernel at HEAD (round 6): PMC traffic (FETCH_SIZE / WRITE_SIZE, gfx950 corrections in tools/traffic.py) and
# occupancy / stall / request counters, for Zipf ids and for uniform ids. One counter group per rocprofv3 pass.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
BA="--no-extras --no-sharded --no-pipe --no-train --no-shard-train --no-cascade --no-probes --no-uniform-leg --sim-ranks 0"
G=$'FETCH_SIZE\nWRITE_SIZE\nSQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_BUSY_CYCLES\nTCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE'
for ids in zipf uniform; do
  extra=""; [ $ids = uniform ] && extra="--uniform"
  PMC_GROUPS="$G" TAG=r06_traffic_$ids BENCH_ARGS="$BA $extra" bash tools/pmc.sh || exit 1
  cd "$ROOT" && python3 tools/traffic.py "gpurun_out/r06_traffic_$ids" "gpurun_out/r06_traffic_$ids/traffic_cfg2.json" > /dev/null || exit 1
  echo "$ids: $(python3 -c "import json;d=json.load(open('gpurun_out/r06_traffic_$ids/traffic_cfg2.json'));print(d['hbm_bytes_per_launch'], d['counters_per_launch'])")"
done
