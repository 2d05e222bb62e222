"""ESIM attention micro-benchmark (diagnostics): rf_esim_soft_attention_fwd on cfg3's shape
(B = 4096, L = 100, d = 128, bf16), HIP-event timed on the launch stream. Usage:
    python tools/esim_probe.py [--batch 4096] [--L 100] [--d 128] [--reps 50] [--f16]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch

from recommendflow_amd.backend.layers.attention_layers import esim_soft_attention_pool


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--L", type=int, default=100)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--f16", action="store_true")
    a = ap.parse_args()
    dt = torch.float16 if a.f16 else torch.bfloat16
    g = torch.Generator(device="cuda").manual_seed(0)
    q = (0.5 * torch.randn((a.batch, a.L, a.d), generator=g, device="cuda")).to(dt)
    k = (0.5 * torch.randn((a.batch, a.L, a.d), generator=g, device="cuda")).to(dt)
    out = torch.empty((a.batch, 6 * a.d), device="cuda")
    for _ in range(5):
        esim_soft_attention_pool(q, k, out=out)
    s = [torch.cuda.Event(enable_timing=True) for _ in range(a.reps)]
    e = [torch.cuda.Event(enable_timing=True) for _ in range(a.reps)]
    for i in range(a.reps):
        s[i].record()
        esim_soft_attention_pool(q, k, out=out)
        e[i].record()
    torch.cuda.synchronize()
    t = sorted(x.elapsed_time(y) for x, y in zip(s, e))
    ms = t[len(t) // 2]
    flops = 2 * a.L * a.L * a.d * 3 * a.batch
    by = 2 * a.batch * a.L * a.d * q.element_size() + a.batch * 6 * a.d * 4
    print(json.dumps({"ms": round(ms, 4), "TFLOPs": round(flops / ms / 1e9, 1), "GBs": round(by / ms / 1e6, 1),
                      "batch": a.batch, "L": a.L, "d": a.d, "dtype": str(dt)}))


if __name__ == "__main__":
    main()
