"""Two-tower DSSM recall scorer on the MI355X hot path (reference: models/matching/dssm.py:11-64).

The reference builds the towers `create_mlp([1024, 512, 256], 0.3, "selu", BatchNormalization(1e-6))`
(dssm.py:25-26) and `K.l2_normalize` (:35-36) but its `call` never wires them (:38-60); deviation
D-dssm-wiring defines the forward the class intends:
  u = l2norm(user_tower([pool_s]_{s in user}))  v = l2norm(ad_tower([pool_s]_{s in ad}))  score = <u, v>
(the dot-product score of que2search.py:137 / match_losses.py:46). Towers run in fp32 (the reference
dtype) on the exact-fp32 MFMA path; the sparse part is one fused encoder launch per tower.
"""
from __future__ import annotations

from typing import Optional

import torch

from ...backend.blocks.mlp import create_mlp
from ...backend.encoder.sparse_encoder import FusedSparseEncoder
from ...backend.layers.core import BatchNormalization
from ...runtime.batch import SparseBatch


class Dssm(torch.nn.Module):
    def __init__(self, user_encoder: FusedSparseEncoder, ad_encoder: FusedSparseEncoder, units=(1024, 512, 256),
                 tower_dtype=torch.float32, seed: int = 0, device="cuda"):
        super().__init__()
        self.enc_u, self.enc_a = user_encoder, ad_encoder
        bn = BatchNormalization(epsilon=1e-6)
        self.user_dense = create_mlp(list(units), 0.3, "selu", bn, name="user_dense_tower",
                                     in_features=user_encoder.out_width, dtype=tower_dtype, seed=seed + 1, device=device)
        self.ad_dense = create_mlp(list(units), 0.3, "selu", bn, name="ad_dense_tower",
                                   in_features=ad_encoder.out_width, dtype=tower_dtype, seed=seed + 2, device=device)

    def embed(self, user: SparseBatch, ad: SparseBatch):
        u = self.user_dense(self.enc_u(user))
        a = self.ad_dense(self.enc_a(ad))
        return torch.nn.functional.normalize(u, dim=-1, eps=1e-6), torch.nn.functional.normalize(a, dim=-1, eps=1e-6)

    def forward(self, user: SparseBatch, ad: SparseBatch) -> torch.Tensor:
        u, a = self.embed(user, ad)
        return (u * a).sum(dim=-1)

    def flops_per_example(self) -> float:
        f = 0
        for m in (self.user_dense, self.ad_dense):
            for dn in m.denses:
                f += 2 * dn.in_features * dn.units
        return float(f)
