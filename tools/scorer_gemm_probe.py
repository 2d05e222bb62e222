"""cfg3 scorer GEMMs in isolation (diagnostics): the output MLP's two LN-folded bf16 GEMMs as the fused forward runs
them (rf_linear_lnfold_stats_fwd 4096 x 1280 -> 1024, rf_linear_lnfold_head_fwd 4096 x 1024 -> 512 + Dense(2)
softmax), the plain bf16 GEMM of the same shapes (rf_linear_fwd, fp32 out) and torch.mm (hipBLASLt) beside them.
Each call captured 20 times into one hipGraph, HIP events around 10 replays after a 0.3 s warm-up.
    python tools/scorer_gemm_probe.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from recommendflow_amd.backend.encoder.sparse_encoder import SlotSpec  # noqa: E402
from recommendflow_amd.models.ranking.esim import Esim  # noqa: E402
from recommendflow_amd.runtime import lib as L  # noqa: E402
from recommendflow_amd.runtime.graphs import CapturedGraph  # noqa: E402


def window(fn, per_graph=20, replays=10, warm_s=0.3):
    """us per call: fn captured per_graph times into one hipGraph (no host launch cost in the window), replayed"""
    g = CapturedGraph(lambda: [fn() for _ in range(per_graph)])
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < warm_s:
        g.replay()
        torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(replays):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / (per_graph * replays) * 1e3


def slice_stats(x):
    M, K = x.shape
    v = x.float().view(M, K // 32, 32)
    s = v.sum(-1)
    m2 = ((v - (s / 32)[..., None]) ** 2).sum(-1)
    return torch.stack([s, m2], -1).contiguous()


B, Ls = 4096, 100
model = Esim([SlotSpec(f"u{i:03d}", 1000, (2022, 2023)) for i in range(Ls)],
             [SlotSpec(f"a{i:03d}", 1000, (2022, 2023)) for i in range(Ls)], n_dense=16, dim=64,
             table_dtype=torch.bfloat16, seed=3)
mlp, head = model.output_mlp, model.dense_output
d0, d1 = mlp.denses
n0, n1 = mlp.norms
K0 = d0.in_features
xb = (torch.randn(B, K0, device="cuda") * 0.5).to(torch.bfloat16)
xst = slice_stats(xb)
wg0, sv0, tv0 = mlp._ln_folded(0)
wg1, sv1, tv1 = mlp._ln_folded(1)
yb = torch.empty((B, d0.units), dtype=torch.bfloat16, device="cuda")
st1 = torch.empty((B, 4 * ((d0.units + 127) // 128), 2), device="cuda")
act = L.ACT[mlp.activation]
ws_bytes = int(L.load().rf_linear_lnfold_head_ws_bytes(B, d1.units))
ws = torch.zeros(ws_bytes, dtype=torch.uint8, device="cuda")
out = torch.empty((B, head.units), device="cuda")


def g0():
    L.call("rf_linear_lnfold_stats_fwd", L.ptr(xb), B, K0, xb.stride(0), L.ptr(wg0), d0.units, L.ptr(sv0), L.ptr(tv0),
           L.ptr(xst), n0.eps, act, L.ptr(yb), yb.stride(0), L.ptr(st1), L.stream_ptr(None))


def g1():
    L.call("rf_linear_lnfold_head_fwd", L.ptr(yb), B, d1.in_features, yb.stride(0), L.ptr(wg1), d1.units, L.ptr(sv1),
           L.ptr(tv1), L.ptr(st1), n1.eps, act, None, 0, L.ptr(head.weight), head.units,
           L.ptr(head.bias) if head.bias is not None else None, L.ACT[head.activation], L.ptr(out), out.stride(0),
           L.ptr(ws), ws.numel(), L.stream_ptr(None))


y0 = torch.empty((B, d0.units), device="cuda")
y1 = torch.empty((B, d1.units), device="cuda")


def p0():
    L.call("rf_linear_fwd", L.ptr(xb), L.DT_BF16, B, K0, xb.stride(0), L.ptr(wg0), d0.units, None, 0, L.ptr(y0),
           y0.stride(0), L.stream_ptr(None))


def p1():
    L.call("rf_linear_fwd", L.ptr(yb), L.DT_BF16, B, d1.in_features, yb.stride(0), L.ptr(wg1), d1.units, None, 0,
           L.ptr(y1), y1.stride(0), L.stream_ptr(None))


t0 = torch.empty((B, d0.units), dtype=torch.bfloat16, device="cuda")
t1 = torch.empty((B, d1.units), dtype=torch.bfloat16, device="cuda")
g0()
res = {}
for name, fn, flops in [("lnfold_stats_1280_1024", g0, 2 * B * K0 * d0.units),
                        ("lnfold_head_1024_512", g1, 2 * B * d1.in_features * d1.units),
                        ("plain_1280_1024_f32out", p0, 2 * B * K0 * d0.units),
                        ("plain_1024_512_f32out", p1, 2 * B * d1.in_features * d1.units),
                        ("torch_mm_1280_1024_bf16", lambda: torch.mm(xb, wg0.t(), out=t0), 2 * B * K0 * d0.units),
                        ("torch_mm_1024_512_bf16", lambda: torch.mm(yb, wg1.t(), out=t1), 2 * B * d1.in_features * d1.units),
                        ("both_lnfold", lambda: (g0(), g1()), 2 * B * (K0 * d0.units + d1.in_features * d1.units))]:
    us = window(fn)
    res[name] = {"us": round(us, 2), "TFLOPs": round(flops / us / 1e6, 1), "frac_2500": round(flops / us / 1e6 / 2500, 3)}
    print(json.dumps({name: res[name]}), flush=True)
