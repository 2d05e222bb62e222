#!/bin/bash
# PMC passes over one diagnostic script: PMC_GROUPS (one group per line), PROBE (python script + args), TAG.
# Kernel-trace only; every pass under its own timeout; stops at the first failure.
set -u
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$ROOT/gpurun_out/${TAG:-probe_pmc}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
n=0
while read -r group; do
  [ -z "$group" ] && continue
  n=$((n+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $group -d "$OUT/pmc_$n" -o run --output-format csv -- \
     python3 $ROOT/$PROBE > "$OUT/pmc_$n.log" 2>&1
  rc=$?; echo "pmc pass $n ($group) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/pmc_$n.log"; exit $rc; fi
done <<LIST
$PMC_GROUPS
LIST
