"""Dense-stage micro-benchmark (diagnostics): every Norm / Dense launch of the cfg3 ESIM scorer
(input_mlp 16->256->512, output_mlp 1280->1024->512, Dense(2, softmax); bf16 MFMA, LayerNorm) and of the cfg2
DSSM towers (8704 / 20480 -> 1024 -> 512 -> 256, fp32, BatchNorm), HIP-event timed on the launch stream.
    python tools/dense_probe.py [--batch 4096]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch

from recommendflow_amd.backend.blocks.mlp import create_mlp
from recommendflow_amd.backend.layers.core import BatchNormalization, Dense, LayerNormalization


def timeit(fn, reps=30, warm=5, inner=10):
    """GPU time of one fn(): `inner` calls captured in one hipGraph (no per-launch host path), median of
    `reps` replays / inner."""
    from recommendflow_amd.runtime.graphs import CapturedGraph

    g = CapturedGraph(lambda: [fn() for _ in range(inner)], warmup=1)
    for _ in range(warm):
        g.replay()
    s = [torch.cuda.Event(enable_timing=True) for _ in range(reps)]
    e = [torch.cuda.Event(enable_timing=True) for _ in range(reps)]
    for i in range(reps):
        s[i].record()
        g.replay()
        e[i].record()
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in zip(s, e))
    return t[len(t) // 2] / inner


def mlp_stages(tag, mlp, x, res):
    total = 0.0
    for i, (norm, dense) in enumerate(zip(mlp.norms, mlp.denses)):
        h = norm(x, out_dtype=mlp.dtype)
        ms_n = timeit(lambda: norm(x, out_dtype=mlp.dtype))
        by = x.numel() * 4 + h.numel() * h.element_size()
        res[f"{tag}.norm{i}[{x.shape[1]}]"] = {"ms": round(ms_n, 4), "GBs": round(by / ms_n / 1e6, 1)}
        y = dense(h)
        ms_d = timeit(lambda: dense(h))
        fl = 2 * x.shape[0] * dense.in_features * dense.units
        res[f"{tag}.dense{i}[{dense.in_features}->{dense.units}]"] = {"ms": round(ms_d, 4), "TFLOPs": round(fl / ms_d / 1e9, 1)}
        total += ms_n + ms_d
        x = y
    res[f"{tag}.sum_of_stages_ms"] = round(total, 4)
    return x


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    a = ap.parse_args()
    B = a.batch
    res = {}
    g = torch.Generator(device="cuda").manual_seed(0)
    ln = LayerNormalization(epsilon=1e-6)
    # cfg3 output MLP + head
    out_mlp = create_mlp([1024, 512], 0.3, "gelu", ln, in_features=1280, dtype=torch.bfloat16, seed=1)
    x = torch.randn((B, 1280), generator=g, device="cuda")
    y = mlp_stages("cfg3.output_mlp", out_mlp, x, res)
    head = Dense(512, 2, activation="softmax", dtype=torch.bfloat16, seed=2)
    ms = timeit(lambda: head(y))
    res["cfg3.head[512->2 softmax]"] = {"ms": round(ms, 4)}
    full = lambda: head(out_mlp(x))
    res["cfg3.output_mlp+head_ms"] = round(timeit(full), 4)
    in_mlp = create_mlp([256, 512], 0.3, "gelu", ln, in_features=16, dtype=torch.bfloat16, seed=3)
    xd = torch.randn((B, 16), generator=g, device="cuda")
    mlp_stages("cfg3.input_mlp", in_mlp, xd, res)
    res["cfg3.input_mlp.fused_ms"] = round(timeit(lambda: in_mlp(xd)), 4)
    # cfg2 DSSM towers
    bn = BatchNormalization(epsilon=1e-6)
    for name, width in (("user", 8704), ("ad", 20480)):
        t = create_mlp([1024, 512, 256], 0.3, "selu", bn, in_features=width, dtype=torch.float32, seed=4)
        xt = torch.randn((B, width), generator=g, device="cuda") * 0.05
        mlp_stages(f"cfg2.{name}_tower", t, xt, res)
        res[f"cfg2.{name}_tower_ms"] = round(timeit(lambda: t(xt)), 4)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
