#!/bin/bash
# Round 6 GPU session runner. Steps (space-separated in STEPS): tests, smoke, bench, prof, lab.
# The tests step is the DRIVER's command (python3 -m pytest tests/ -x -q -m gpu -p no:cacheprovider, no timeout
# plugin), under an outer time limit only; TESTS narrows it to a selection for lab iterations.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
OUT=gpurun_out/${TAG:-r06}
mkdir -p "$OUT"
for step in ${STEPS:-tests smoke bench}; do
  case $step in
  tests)
    timeout -k 10 ${TEST_TIMEOUT:-900} python3 -m pytest ${TESTS:-tests/} -x -q -m gpu -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
    rc=$?; echo "pytest rc=$rc"; grep -v '^\.*s*RUN ' "$OUT/pytest_gpu.log" | tail -4; cp gpurun_out/faulthandler_*.txt "$OUT/" 2>/dev/null
    [ $rc -eq 0 ] || { tail -3 "$OUT/pytest_gpu.log"; exit $rc; } ;;
  smoke)
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
    rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc ;;
  bench)
    timeout -k 10 700 python3 bench.py ${BENCH_ARGS:---warmup 5 --steps 20} > "$OUT/bench.json" 2> "$OUT/bench.err"
    rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/bench.err"; exit $rc; }
    python3 tools/bench_brief.py "$OUT/bench.json" ;;
  prof)
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/prof" -o run -- python3 "$ROOT/bench.py" ${PROF_ARGS:---warmup 5 --steps 20} > "$ROOT/$OUT/bench_prof.json" 2> "$ROOT/$OUT/bench_prof.err")
    rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/bench_prof.err"; exit $rc; }
    python3 tools/headline_summary.py "$OUT/prof" "$OUT/bench_prof.json" --write-trace "$OUT/headline_kernel_trace.csv" > "$OUT/headline_summary.txt" 2>&1
    tail -8 "$OUT/headline_summary.txt" ;;
  lab)
    timeout -k 10 ${LAB_TIMEOUT:-300} bash -c "$LAB" > "$OUT/lab.log" 2>&1
    rc=$?; echo "lab rc=$rc"; tail -${LAB_TAIL:-60} "$OUT/lab.log"; [ $rc -eq 0 ] || exit $rc ;;
  esac
done
