#!/bin/bash
# Round 4, first GPU session: the GPU suite, the ESIM gather-kernel baseline (timing, zipf + uniform) and its PMC
# counters, then one bench line. Stops at the first step that faults, aborts or times out.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
OUT=gpurun_out/${TAG:-r04g1}
mkdir -p "$OUT"
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -6 "$OUT/pytest_gpu.log"
  if [ $rc -ne 0 ]; then echo "stopping after pytest rc=$rc"; exit $rc; fi
fi
for r in 1 2; do
  timeout -k 10 180 python tools/esim_gather_probe.py > "$OUT/esimg_zipf_$r.json" 2>&1; rc=$?
  echo "esim gather zipf $r rc=$rc: $(tail -1 $OUT/esimg_zipf_$r.json)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 180 python tools/esim_gather_probe.py --uniform > "$OUT/esimg_uni.json" 2>&1; rc=$?
echo "esim gather uniform rc=$rc: $(tail -1 $OUT/esimg_uni.json)"; [ $rc -eq 0 ] || exit $rc
if [ "${SKIP_PMC:-0}" != 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  n=0
  while read -r group; do
    [ -z "$group" ] && continue
    n=$((n+1))
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $group -d "$ROOT/$OUT/pmc_$n" -o run --output-format csv -- \
       python3 $ROOT/tools/esim_gather_probe.py --reps 20 > "$ROOT/$OUT/pmc_$n.log" 2>&1
    rc=$?; echo "pmc pass $n ($group) rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$ROOT/$OUT/pmc_$n.log"; exit $rc; fi
  done <<LIST
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES
SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
LIST
  cd "$ROOT"
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
  rc=$?; echo "bench rc=$rc"; tail -c 600 "$OUT/bench.log"
fi
