"""GEMM yardstick (diagnostics): rf_linear_fwd vs torch (hipBLASLt) on the cfg3 scorer shapes, bf16 in,
fp32 out, graph-timed (tools/dense_probe.timeit)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch

from dense_probe import timeit
from recommendflow_amd.backend.layers.core import Dense


def main():
    res = {}
    g = torch.Generator(device="cuda").manual_seed(0)
    for M, K, N in ((4096, 1280, 1024), (4096, 1024, 512), (51200, 1280, 1024), (4096, 256, 512), (4096, 8704, 1024), (4096, 20480, 1024)):
        dt = torch.float32 if K in (8704, 20480) else torch.bfloat16
        x = torch.randn((M, K), generator=g, device="cuda").to(dt)
        d = Dense(K, N, "gelu" if dt == torch.bfloat16 else "selu", dtype=dt, seed=1)
        fl = 2 * M * N * K
        ms = timeit(lambda: d(x))
        Wt = d.weight
        ms_t = timeit(lambda: torch.nn.functional.linear(x, Wt))
        res[f"{M}x{K}->{N} {str(dt)[6:]}"] = {"rf_ms": round(ms, 4), "rf_TF": round(fl / ms / 1e9, 1),
                                             "torch_ms": round(ms_t, 4), "torch_TF": round(fl / ms_t / 1e9, 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
