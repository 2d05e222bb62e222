#!/bin/bash
# GEMM yardstick across the kernel choices (measurement only).
set -u
cd $GRAFT_REPO_ROOT
for v in "RF_GEMM_LDS=1" "RF_GEMM_LDS=0" "RF_GEMM_LDS=0 RF_GEMM_BT=128" "RF_GEMM_LDS=0 RF_GEMM_BT=64"; do echo "== $v"; env $v timeout -k 10 100 python tools/gemm_probe.py 2>&1 | grep -v amdgpu || exit 1; done
