#!/bin/bash
# rf_gemm_f32 ablation (diagnostics): mode 0 full loop; 1 no barrier; 2 no global loads; 3 no LDS copies;
# 4 no half-1 fragment reads; 5 no next-step half-0 reads (results wrong for 1-5; timing only)
for m in 0 1 2 3 4 5; do
  echo "== mode $m"
  RF_G32_MODE=$m python tools/gemm32_probe.py --lib tools/gemm32/libablate.so --reps 30 --cases "w:4096:1024:20480:1:1:3,fwd_ad:4096:1024:20480:1:1:3,dz_ad:4096:20480:1024:1:0:0,dw_ad:1024:20480:4096:0:0:0" | grep -v "\"w\"" | python3 -c "
import sys,json
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print(d['case'], round(d['frac'],4), round(d['blaslt_frac'],4))"
done
