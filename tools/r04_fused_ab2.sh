#!/bin/bash
# GPU: cfg3 forward, fused scorer vs unfused, alternating runs on one box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2 3; do
  echo "fused   $(timeout -k 10 200 python3 tools/cfg3_gaps.py --serial-mlp --gather 2>&1 | grep forward)" || exit 1
  echo "unfused $(timeout -k 10 200 python3 tools/cfg3_gaps.py --serial-mlp --gather --unfused 2>&1 | grep forward)" || exit 1
done
