#!/bin/bash
# Host-only A/B on the GPU box: the TFRecord reader with libdeflate (default) vs zlib inflate.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-pipeab}
mkdir -p "$OUT"
timeout -k 10 300 python tools/pipe_probe.py --files 16 --per 4096 --threads 16 --modes GZIP > "$OUT/pipe_libdeflate.json" 2>&1 || exit $?
RF_TFR_INFLATE=zlib timeout -k 10 300 python tools/pipe_probe.py --files 16 --per 4096 --threads 16 --modes GZIP > "$OUT/pipe_zlib.json" 2>&1 || exit $?
python -c "
import json
for f in ['libdeflate', 'zlib']:
    print(f, json.dumps(json.load(open('$OUT/pipe_' + f + '.json'))))"
[ -n "${E2E:-}" ] || exit 0
timeout -k 10 300 python tools/pipe_bench.py > "$OUT/pipe_bench_libdeflate.json" 2>&1 || exit $?
RF_TFR_INFLATE=zlib timeout -k 10 300 python tools/pipe_bench.py > "$OUT/pipe_bench_zlib.json" 2>&1 || exit $?
python -c "
import json
for f in ['libdeflate', 'zlib']:
    d = json.load(open('$OUT/pipe_bench_' + f + '.json'))
    print(f, d['legs_examples_per_s'], d['decode_examples_per_s'])"
