#!/bin/bash
# Instruction mix per basic block (MFMA-carrying blocks) of each gemm32_kernel instantiation in a -save-temps .s file
S=${1:-/tmp/rf_gemm32-hip-amdgcn-amd-amdhsa-gfx950.s}
for k in ILb1ELb1E ILb1ELb0E ILb0ELb0E ILb0ELb1E; do
  awk -v pat="^_ZN12_GLOBAL__N_113gemm32_kernel${k}EEvNS_8GemmArgsE:" '$0 ~ pat {f=1} f{print} f&&/^\.Lfunc_end/{exit}' "$S" > /tmp/kk.s
  echo "== $k $(grep -m1 -A0 'NumVgprs' /tmp/kk.s) $(grep -m1 'NumAgprs' /tmp/kk.s)"
  awk '/^\.LBB[0-9_]+:/{lab=$1} /v_mfma/{c[lab]++} /v_accvgpr/{a[lab]++} /ds_read/{r[lab]++} /ds_write/{w[lab]++} /buffer_load/{l[lab]++} /v_mov_b32/{mv[lab]++} /s_nop/{n[lab]++} /s_waitcnt/{wt[lab]++} /^\s+v_/{va[lab]++} END{for (x in c) print x, "mfma", c[x], "acc", a[x]+0, "rd", r[x]+0, "wr", w[x]+0, "ld", l[x]+0, "mov", mv[x]+0, "nop", n[x]+0, "wait", wt[x]+0, "valu(all v_)", va[x]+0}' /tmp/kk.s | sort
done
