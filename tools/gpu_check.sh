#!/bin/bash
# One GPU session: parity tests -> smoke -> bench -> rocprofv3 kernel trace. Stops at the first step that
# faults, aborts or times out (exit codes >= 2 from pytest, or 124/134/137/139 from anything).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }
echo "== host: $(nproc) cpus, $(lscpu | grep 'Model name' | sed 's/ \+/ /g')" | tee "$OUT/host.txt"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -m gpu -q -ra ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -25 "$OUT/pytest_gpu.log"
  if fatal $rc; then echo "stopping after pytest rc=$rc"; exit $rc; fi
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 "$OUT/smoke.log"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 "$OUT/bench.log"
if [ $rc -ne 0 ]; then exit $rc; fi
if [ "${SKIP_PROF:-0}" != 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- \
      python3 "$GRAFT_REPO_ROOT/bench.py" ${PROF_ARGS:---cpu-seconds 0} > "$GRAFT_REPO_ROOT/$OUT/prof.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 "$GRAFT_REPO_ROOT/$OUT/prof.log"
  find "$GRAFT_REPO_ROOT/$OUT/prof" -name "*stats*" | head
fi
