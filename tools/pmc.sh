#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only — never combined with sys/runtime trace)
# over a short bench.py run. Writes gpurun_out/$TAG/pmc_<n>/.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-pmc}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
n=0
while read -r group; do
  [ -z "$group" ] && continue
  n=$((n+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $group -d "$OUT/pmc_$n" -o run --output-format csv -- \
     python3 "$ROOT/bench.py" --steps 5 --warmup 1 --cpu-seconds 0 ${BENCH_ARGS:-} > "$OUT/pmc_$n.log" 2>&1
  rc=$?; echo "pmc pass $n ($group) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/pmc_$n.log"; exit $rc; fi
done <<LIST
${PMC_GROUPS:-FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES
TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE}
LIST
