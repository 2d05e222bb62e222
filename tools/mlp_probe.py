"""rocprof target (diagnostics): the ESIM input MLP, fused (rf_mlp2_small_fwd) with gelu and with relu, and
layer by layer, 50 times each."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch

from recommendflow_amd.backend.blocks.mlp import create_mlp
from recommendflow_amd.backend.layers.core import LayerNormalization
from recommendflow_amd.runtime import lib as L

m = create_mlp([256, 512], 0.3, "gelu", LayerNormalization(epsilon=1e-6), in_features=16, dtype=torch.bfloat16, seed=3)
x = torch.randn(4096, 16, device="cuda")
out = torch.empty(4096, 512, device="cuda")
for _ in range(50):
    m(x, out=out)
m.activation = "relu"
for _ in range(50):
    m(x, out=out)
m.activation = "gelu"
for _ in range(50):
    h = x
    for nm, dn in zip(m.norms, m.denses):
        h = dn(nm(h))
torch.cuda.synchronize()
print("ok")
