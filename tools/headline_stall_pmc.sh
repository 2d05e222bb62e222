#!/bin/bash
# Where the headline kernel's time goes below the SQ: TA / TD busy and stall cycles, TCP->TCC request latency and
# stalls, TCC tag / DRAM-credit stalls, for Zipf and uniform ids (one counter group per rocprofv3 pass).
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOT"
BA="--no-extras --no-sharded --no-pipe --no-train --no-shard-train --no-cascade --no-probes --no-uniform-leg --sim-ranks 0"
G=$'TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE\nTCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum\nTCC_TAG_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_BUSY_sum TCC_LATENCY_FIFO_FULL_sum'
for ids in zipf uniform; do
  extra=""; [ $ids = uniform ] && extra="--uniform"
  PMC_GROUPS="$G" TAG=r06_stall_$ids BENCH_ARGS="$BA $extra" bash tools/pmc.sh || exit 1
done
