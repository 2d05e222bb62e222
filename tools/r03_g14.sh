#!/bin/bash
# GPU: cfg3 forward with uniform ids (no locality), gather path vs encoders + attention.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2; do
  timeout -k 10 200 python3 tools/cfg3_gaps.py --serial-mlp --gather --uniform || exit 1
  timeout -k 10 200 python3 tools/cfg3_gaps.py --serial-mlp --uniform || exit 1
  timeout -k 10 200 python3 tools/cfg3_gaps.py --serial-mlp --gather || exit 1
done
