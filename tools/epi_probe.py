"""GEMM epilogue ablation (diagnostics): the cfg3 scorer GEMMs with each epilogue of gemm_lds_kernel
(plain fp32 without / with gelu, bf16 + row statistics, LN fold) and hipBLASLt on the same shapes, graph-timed
(tools/dense_probe.timeit), plus the whole mlp_scorer stage (output MLP + Dense(2, softmax)).
    python tools/epi_probe.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch

from dense_probe import timeit
from recommendflow_amd.backend.blocks.mlp import create_mlp
from recommendflow_amd.backend.layers.core import Dense, LayerNormalization
from recommendflow_amd.runtime import lib as L


def stream_time(fn, it=20, reps=5):
    """back-to-back launches on the current stream between two events (no graph), median of reps"""
    for _ in range(3):
        fn()
    t = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(it):
            fn()
        b.record()
        torch.cuda.synchronize()
        t.append(a.elapsed_time(b) / it)
    return sorted(t)[len(t) // 2]


def main():
    res = {}
    g = torch.Generator(device="cuda").manual_seed(0)
    for M, K, N in ((4096, 1280, 1024), (4096, 1024, 512)):
        x = (torch.randn((M, K), generator=g, device="cuda") * 0.5).to(torch.bfloat16)
        fl = 2 * M * N * K
        r = {}
        for act in ("none", "gelu"):
            d = Dense(K, N, act, dtype=torch.bfloat16, seed=1)
            ms = timeit(lambda: d(x))
            r[f"plain_{act}"] = {"ms": round(ms, 4), "TF": round(fl / ms / 1e9, 1)}
            ms = stream_time(lambda: d(x))
            r[f"plain_{act}_stream"] = {"ms": round(ms, 4), "TF": round(fl / ms / 1e9, 1)}
        d = Dense(K, N, "gelu", dtype=torch.bfloat16, seed=1)
        yb = torch.empty((M, N), dtype=torch.bfloat16, device="cuda")
        st = torch.empty((M, 4 * ((N + 127) // 128), 2), dtype=torch.float32, device="cuda")
        stats = lambda: L.call("rf_linear_stats_fwd", L.ptr(x), M, K, x.stride(0), L.ptr(d.weight), N, L.ptr(d.bias),
                               L.ACT["gelu"], L.ptr(yb), yb.stride(0), L.ptr(st), L.stream_ptr(None))
        ms = timeit(stats)
        r["stats_gelu"] = {"ms": round(ms, 4), "TF": round(fl / ms / 1e9, 1)}
        # LN fold on x as the previous layer's raw output: stats of x from a stats GEMM of width K
        xs = torch.empty((M, 4 * ((K + 127) // 128), 2), dtype=torch.float32, device="cuda")
        d0 = Dense(512, K, "gelu", dtype=torch.bfloat16, seed=2)
        x0 = (torch.randn((M, 512), generator=g, device="cuda")).to(torch.bfloat16)
        L.call("rf_linear_stats_fwd", L.ptr(x0), M, 512, x0.stride(0), L.ptr(d0.weight), K, L.ptr(d0.bias),
               L.ACT["gelu"], L.ptr(x), x.stride(0), L.ptr(xs), L.stream_ptr(None))
        sv = torch.randn(N, generator=g, device="cuda")
        tv = torch.randn(N, generator=g, device="cuda")
        yo = torch.empty((M, N), dtype=torch.float32, device="cuda")
        lnf = lambda: L.call("rf_linear_lnfold_fwd", L.ptr(x), M, K, x.stride(0), L.ptr(d.weight), N, L.ptr(sv),
                             L.ptr(tv), L.ptr(xs), 1e-6, L.ACT["gelu"], L.ptr(yo), yo.stride(0), L.stream_ptr(None))
        ms = timeit(lnf)
        r["lnfold_gelu"] = {"ms": round(ms, 4), "TF": round(fl / ms / 1e9, 1)}
        Wt = d.weight
        ms = timeit(lambda: torch.nn.functional.linear(x, Wt))
        r["hipblaslt_bf16_out"] = {"ms": round(ms, 4), "TF": round(fl / ms / 1e9, 1)}
        res[f"{M}x{K}->{N}"] = r
    ln = LayerNormalization(epsilon=1e-6)
    out_mlp = create_mlp([1024, 512], 0.3, "gelu", ln, in_features=1280, dtype=torch.bfloat16, seed=1)
    head = Dense(512, 2, activation="softmax", dtype=torch.bfloat16, seed=2)
    xp = torch.randn((4096, 1280), generator=g, device="cuda") * 0.3
    res["mlp_scorer_ms"] = round(timeit(lambda: head(out_mlp(xp))), 4)
    n0 = out_mlp.norms[0]
    res["ln0_1280_ms"] = round(timeit(lambda: n0(xp, out_dtype=torch.bfloat16)), 4)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
