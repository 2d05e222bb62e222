#!/bin/bash
# Headline kernel A/B over recommendflow_amd/lib/var/librf_<name>.so builds (tools/build_variants.sh): the bench's
# headline leg only (zipf + the uniform leg), each variant twice in alternating order.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04fab}
mkdir -p "$OUT"
BA="--no-extras --no-sharded --no-pipe --no-train --no-shard-train --no-cascade --no-probes --cpu-seconds 0 --sim-ranks 0"
for r in 1 2; do
  for v in ${VARIANTS:-base}; do
    RF_LIB=$PWD/recommendflow_amd/lib/var/librf_$v.so timeout -k 10 300 python bench.py $BA > "$OUT/$v.$r.log" 2>&1 || { echo "$v failed"; tail -5 "$OUT/$v.$r.log"; exit 1; }
    python -c "
import json,sys
l=[x for x in open('$OUT/$v.$r.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('$v r$r', 'kernel_ms', r['kernel_ms'], 'frac', r['frac'], 'uniform_ms', (r.get('uniform') or {}).get('kernel_ms'), 'value', d['value'])"
  done
done
