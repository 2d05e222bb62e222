"""create_mlp (reference: backend/blocks/mlp.py:4-15): per hidden size  Norm -> Dense(act) -> Dropout.

Dropout is the identity at inference. Each layer runs rf_norm_fwd (fp32 -> MFMA operand dtype) then
rf_linear_fwd (MFMA GEMM with bias + activation fused in the epilogue).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch

from ..layers.core import Dense, Norm, act_name


class MLP(torch.nn.Module):
    def __init__(self, hidden_units: Sequence[int], dropout_rate: float, activation, normalization_layer,
                 name: Optional[str] = None, in_features: Optional[int] = None, dtype=torch.bfloat16, seed: int = 0,
                 device="cuda"):
        super().__init__()
        self.hidden_units = [int(u) for u in hidden_units]
        self.dropout_rate = dropout_rate
        self.activation = act_name(activation)
        self.norm_spec = normalization_layer
        self.name = name
        self.dtype = dtype
        self.seed = seed
        self.device = device
        self.norms: List[Norm] = []
        self.denses: List[Dense] = []
        if in_features is not None:
            self.build(in_features)

    def build(self, in_features: int):
        width = int(in_features)
        self.norms, self.denses = [], []
        for i, u in enumerate(self.hidden_units):
            self.norms.append(Norm(self.norm_spec, width, device=self.device) if self.norm_spec is not None else None)
            self.denses.append(Dense(width, u, self.activation, dtype=self.dtype, seed=self.seed * 1000 + i, device=self.device))
            width = u
        self.out_features = width
        return self

    def forward(self, x: torch.Tensor, stream=None) -> torch.Tensor:
        if not self.denses:
            self.build(x.shape[-1])
        for norm, dense in zip(self.norms, self.denses):
            h = norm(x, out_dtype=self.dtype, stream=stream) if norm is not None else x
            x = dense(h, stream=stream)
        return x


def create_mlp(hidden_units, dropout_rate, activation, normalization_layer, name=None, **kw) -> MLP:
    return MLP(hidden_units, dropout_rate, activation, normalization_layer, name=name, **kw)
