#!/bin/bash
# rf_gemm_f32 lab: every tower shape after a warm-up pass (the first GEMMs of a process run on cold clocks / TLBs)
set -e
L=${LIB:-tools/gemm32/libg32.so}
python tools/gemm32_probe.py --lib $L --only fwd > /dev/null
python tools/gemm32_probe.py --lib $L --reps 30
