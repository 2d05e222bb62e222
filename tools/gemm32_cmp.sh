#!/bin/bash
# rf_gemm_f32 lab: two builds on the big tower shapes, each process warmed up first (diagnostics)
C="w:4096:1024:20480:1:1:3,fwd_user:4096:1024:8704:1:1:3,fwd_ad:4096:1024:20480:1:1:3,dw_user:1024:8704:4096:0:0:0,dw_ad:1024:20480:4096:0:0:0,dz_user:4096:8704:1024:1:0:0,dz_ad:4096:20480:1024:1:0:0,fwd_l2:4096:512:1024:1:1:3,dz_l2:4096:1024:512:1:0:0"
for L in ${LIBS:-tools/gemm32/libg32.so tools/gemm32/libbk64.so}; do
  echo "== $L"
  python tools/gemm32_probe.py --lib $L --reps 30 --cases "$C" | grep -v '"w"' | python3 -c "
import sys,json
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print(d['case'], 'err', '%.1e' % d['rel_err'], d['nan'], d['deterministic'], 'frac', round(d['frac'],4), 'blaslt', round(d['blaslt_frac'],4))
    else: print(l.strip())"
done
