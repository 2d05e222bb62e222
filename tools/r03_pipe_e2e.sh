#!/bin/bash
# GPU box: bench.py's feature-pipe leg alone (tools/pipe_bench.py), libdeflate (default) and zlib.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-pipee2e}
mkdir -p "$OUT"
for m in ${MODES:-libdeflate zlib}; do
  if [ "$m" = zlib ]; then export RF_TFR_INFLATE=zlib; else unset RF_TFR_INFLATE; fi
  timeout -k 10 300 python tools/pipe_bench.py ${PIPE_ARGS:-} > "$OUT/pipe_bench_$m.json" 2>&1 || exit $?
  python - "$OUT/pipe_bench_$m.json" "$m" <<'PY'
import json, sys
t = open(sys.argv[1]).read()
d = json.loads(t[t.index('{'):])
print(sys.argv[2], d['legs_examples_per_s'], d.get('legs_after_first_batch_examples_per_s'), d['decode_examples_per_s'])
PY
done
