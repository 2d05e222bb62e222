#!/bin/bash
# Same-box A/B of librf variants on the cfg2 headline (RF_LIB=recommendflow_amd/lib/var/librf_<v>.so), alternating
# variants for ROUNDS rounds: prints kernel_ms / frac per run. Usage: VARIANTS="base nt" ROUNDS=3 tools/r06_lib_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in ${VARIANTS:-base nt}; do
    out=$(RF_LIB=recommendflow_amd/lib/var/librf_$v.so timeout -k 10 300 python3 bench.py --warmup 50 --steps 100 --no-extras \
          --no-sharded --no-cascade --no-train --no-pipe --no-uniform-leg --cpu-seconds 0 ${BENCH_EXTRA:-} 2>/dev/null) || { echo "run failed: $v"; exit 1; }
    echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v', r['kernel_ms'], r['frac'], d['value'])"
  done
done
