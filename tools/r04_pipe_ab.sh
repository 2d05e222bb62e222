#!/bin/bash
# GPU box: the feature-pipe leg with the default reader look-ahead budget vs an unbounded one, plus nproc / affinity.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04pipe}
mkdir -p "$OUT"
python -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"
timeout -k 10 300 python tools/pipe_bench.py > "$OUT/pipe_default.json" 2>&1 || { tail -5 "$OUT/pipe_default.json"; exit 1; }
RF_TFR_AHEAD_MB=100000 timeout -k 10 300 python tools/pipe_bench.py > "$OUT/pipe_unbounded.json" 2>&1 || { tail -5 "$OUT/pipe_unbounded.json"; exit 1; }
timeout -k 10 300 python tools/pipe_bench.py --pipe-threads 24 > "$OUT/pipe_t24.json" 2>&1 || { tail -5 "$OUT/pipe_t24.json"; exit 1; }
python -c "
import json
for f in ['default', 'unbounded', 't24']:
    d = json.load(open('$OUT/pipe_' + f + '.json'))
    print(f, d['legs_examples_per_s'], d['legs_after_first_batch_examples_per_s'], d['decode_examples_per_s'])"
