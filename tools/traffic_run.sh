#!/bin/bash
# PMC traffic of the headline kernel (FETCH_SIZE / WRITE_SIZE passes over a short headline-only bench), turned
# into per-launch HBM bytes by tools/traffic.py (gfx950 corrections). Writes gpurun_out/${TAG}/traffic_cfg2.json.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
TAG=${TAG:-traffic_r02}
PMC_GROUPS=$'FETCH_SIZE\nWRITE_SIZE' TAG=$TAG \
  BENCH_ARGS="--no-extras --no-sharded --no-pipe --no-train --no-shard-train --no-cascade" bash tools/pmc.sh || exit 1
cd "$ROOT" && python3 tools/traffic.py "gpurun_out/$TAG" "gpurun_out/$TAG/traffic_cfg2.json" && cat "gpurun_out/$TAG/traffic_cfg2.json"
