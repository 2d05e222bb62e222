"""Runs one rf_linear_fwd GEMM shape N times (for rocprofv3 counter passes). Usage: gemm_one.py M K N [reps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from recommendflow_amd.backend.layers.core import Dense  # noqa: E402

M, K, N = (int(v) for v in sys.argv[1:4])
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 50
x = torch.randn((M, K), generator=torch.Generator(device="cuda").manual_seed(0), device="cuda").to(torch.bfloat16)
d = Dense(K, N, "gelu", dtype=torch.bfloat16, seed=1)
for _ in range(reps):
    d(x)
torch.cuda.synchronize()
print("ok")
