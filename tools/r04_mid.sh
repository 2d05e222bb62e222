#!/bin/bash
# GPU: ESIM gather PMC at HEAD (the 'after' of VERDICT r3 item 1), the feature-pipe look-ahead / thread A/B, and one
# default bench line. Each step under its own limit; stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SKIP_TESTS=1 SKIP_BENCH=1 TAG=${TAG:-r04mid}_pmc bash tools/r04_g1.sh || exit $?
TAG=${TAG:-r04mid}_pipe bash tools/r04_pipe_ab.sh || exit $?
OUT=gpurun_out/${TAG:-r04mid}
mkdir -p "$OUT"
timeout -k 10 700 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -5 "$OUT/bench.err"; exit 1; }
python - "$OUT/bench.json" <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{')][-1]; d=json.loads(l)
r=d['roofline']
print('headline', d['value'], r['kernel_ms'], r['frac'], r.get('frac_of_peak_measured'))
e=d.get('extras') or {}
for k in ('cfg3_esim_forward','cfg2_dssm_train_step','feature_pipe'):
    v=e.get(k); print(k, json.dumps(v)[:500] if v else v)
print('cfg4 sim', json.dumps((d.get('cfg4_sharded') or {}).get('simulated_p8'))[:300])
PY
