"""rocprof target (diagnostics): the cfg3 output MLP + head (the bench's mlp_scorer stage) eagerly, 100 times,
so `rocprofv3 --kernel-trace --stats` splits the stage per kernel (LN, stats GEMM, LN-folded GEMM, head)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch

from recommendflow_amd.backend.encoder.sparse_encoder import SlotSpec
from recommendflow_amd.models.ranking.esim import Esim

B, Ls = 4096, 100
model = Esim([SlotSpec(f"u{i:03d}", 1000, (2022, 2023)) for i in range(Ls)],
             [SlotSpec(f"a{i:03d}", 1000, (2022, 2023)) for i in range(Ls)], n_dense=16, dim=64,
             table_dtype=torch.bfloat16, seed=3)
pooled = torch.randn(B, model.pooled_width, device="cuda") * 0.3
for _ in range(100):
    model.dense_output(model.output_mlp(pooled))
torch.cuda.synchronize()
print("ok")
