"""Which MFMA-internal order reproduces rf_linear_fwd's fp32 scores (diagnostics): rf_ip_rescore_f32 with lane-group
order 0 (ascending) and 1 (descending) against the full rf_linear_fwd score matrix, bit for bit, on random candidates.
    python tools/rescore_check.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from recommendflow_amd.runtime import lib as L  # noqa: E402

res = {}
for K in (256, 512):
    g = torch.Generator(device="cuda").manual_seed(K)
    B, N, cap = 64, 40000, 2048
    q = torch.randn((B, K), device="cuda", generator=g)
    items = torch.randn((N, K), device="cuda", generator=g)
    full = torch.empty((B, N), device="cuda")
    L.call("rf_linear_fwd", L.ptr(q), L.DT_F32, B, K, K, L.ptr(items), N, None, 0, L.ptr(full), N, L.stream_ptr())
    idx = torch.stack([torch.randperm(N, generator=torch.Generator().manual_seed(r))[:cap] for r in range(B)]).cuda()
    cidx = idx.to(torch.int32).contiguous()
    count = torch.full((B,), cap, dtype=torch.int32, device="cuda")
    want = torch.gather(full, 1, idx)
    for order in (0, 1):
        cval = torch.empty((B, cap), device="cuda")
        L.call("rf_ip_rescore_f32", L.ptr(q), K, B, L.ptr(items), K, L.ptr(count), cap, L.ptr(cval), L.ptr(cidx), order,
               L.stream_ptr())
        torch.cuda.synchronize()
        same = (cval.view(torch.int32) == want.view(torch.int32)).float().mean().item()
        res[f"K{K}_order{order}_bit_equal_frac"] = round(same, 6)
        res[f"K{K}_order{order}_max_abs_diff"] = float((cval - want).abs().max().item())
print(json.dumps(res))
