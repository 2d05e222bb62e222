"""Attention operators with the reference API (backend/layers/attention_layers.py), on librf.so MFMA kernels.

* ``esim_soft_attention_pool(q, a)``  — the fused hot-path op: SoftAttention + ESIM combine + avg/max pooling
  (attention_layers.py:15-74 + models/ranking/esim.py:79-84) -> [B, 6d] fp32, in one launch.
* ``SoftAttention()([a, b]) -> (align_a, align_b)`` — the reference callable (:10-80); same kernel with the
  aligned sequences written out.
* ``MultiHeadAttention(d_model, num_heads).call(q, k, v, mask)`` (:137-168): Dense q/k/v with bias in fp32
  (the reference's Dense dtype; exact-fp32 MFMA, rf_linear_fwd), then rf_sdpa_fwd with split_heads/merge
  folded into addressing; no output projection (as the reference).
* ``SelfAttention(add_pos)([q, k, v, mask])`` (:83-134): sinusoid PE, shared relu(xW) in fp32, masked SDPA,
  mean over the sequence.
Both run the attention core (QK^T, softmax, PV) with `dtype` (fp16 by default, cfg5's "fp16 MFMA
attention") operands and fp32 logits/softmax/accumulation; tests/test_attention_gpu.py states the
tolerance against the float64 oracle.
"""
from __future__ import annotations

import math
from typing import Optional, Sequence

import numpy as np
import torch

from ...runtime import lib as L
from .core import Dense
from .layer_utils import scaled_dot_product_attention


def _half(x: torch.Tensor) -> torch.Tensor:
    if x.dtype not in (torch.bfloat16, torch.float16):
        x = x.to(torch.bfloat16)
    return x


def esim_soft_attention_pool(q: torch.Tensor, a: torch.Tensor, out: Optional[torch.Tensor] = None, out_col: int = 0,
                             att_out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
    """q, a: [B, L, d] bf16/f16 on the GPU (views with unit stride on d are fine). Returns (or fills
    out[:, out_col:out_col+6d]) [avg_q, max_q, avg_a, max_a, avg_q-avg_a, max_q-max_a] in fp32."""
    L.require_gpu()
    q, a = _half(q), _half(a)
    if a.dtype != q.dtype:
        a = a.to(q.dtype)
    if q.shape != a.shape:
        raise ValueError(f"q {tuple(q.shape)} and a {tuple(a.shape)} must match (the reference needs L0 == L1)")
    B, Ln, d = q.shape
    if q.stride() != a.stride() or q.stride(2) != 1:
        q, a = q.contiguous(), a.contiguous()
    if out is None:
        out = torch.empty((B, 6 * d), dtype=torch.float32, device=q.device)
        out_col = 0
    L.call("rf_esim_soft_attention_fwd", L.ptr(q), L.ptr(a), L.torch_dtype_code(q.dtype), B, Ln, d, q.stride(0),
           q.stride(1), L.ptr(out), out.stride(0), out_col, L.ptr(att_out), L.stream_ptr(stream))
    return out


def esim_soft_attention_pool_idx(q: torch.Tensor, q_rep: int, a_table: torch.Tensor, a_rows: torch.Tensor,
                                 out: torch.Tensor, out_col: int = 0, stream=None) -> torch.Tensor:
    """esim_soft_attention_pool over B * q_rep pairs without materialising them: pair e takes q[e // q_rep]
    ([Bq, L, d]) and a_table[a_rows[e]] ([N, L, d]); fills out[:, out_col:out_col + 6d] (rf_esim_soft_attention_idx_fwd).
    A row id outside [0, N) is caught on the device: that pair's features are NaN (no read past the table)."""
    L.require_gpu()
    if q.dtype != a_table.dtype or q.dtype not in (torch.bfloat16, torch.float16):
        raise ValueError("q and a_table must share a bf16 / f16 dtype")
    if q.dim() != 3 or a_table.dim() != 3 or q.shape[1:] != a_table.shape[1:] or not q.is_contiguous() or not a_table.is_contiguous():
        raise ValueError("q [Bq, L, d] and a_table [N, L, d] must be contiguous with the same (L, d)")
    a_rows = a_rows.reshape(-1).to(torch.int64).contiguous()
    P = a_rows.numel()
    if P != q.shape[0] * q_rep or out.shape[0] != P:
        raise ValueError(f"{P} pairs need q with {P // max(q_rep, 1)} rows x q_rep {q_rep} and out with {P} rows")
    _, Ln, d = q.shape
    L.call("rf_esim_soft_attention_idx_fwd", L.ptr(q), int(q_rep), L.ptr(a_table), L.ptr(a_rows), a_table.shape[0], Ln * d,
           L.torch_dtype_code(q.dtype), P, Ln, d, Ln * d, d, L.ptr(out), out.stride(0), out_col, L.stream_ptr(stream))
    return out


class SoftAttention:
    """SoftAttention()([x0, x1]) -> (S @ x0, S @ x1), E[n,i,j] = x1[n,i] . x0[n,j], S = softmax_j(E)."""

    def __call__(self, inputs: Sequence[torch.Tensor]):
        q, a = inputs[0], inputs[1]
        B, Ln, d = q.shape
        att = torch.empty((B, 2, Ln, d), dtype=torch.float32, device=q.device)
        esim_soft_attention_pool(q, a, att_out=att)
        return att[:, 0], att[:, 1]


class MultiHeadAttention(torch.nn.Module):
    def __init__(self, d_model: int, num_heads: int, dtype=torch.float16, seed: int = 0, device="cuda",
                 proj_dtype=torch.float32, in_features: Optional[int] = None):
        super().__init__()
        if d_model % num_heads:
            raise ValueError("d_model must be divisible by num_heads")
        self.d_model, self.num_heads = d_model, num_heads
        self.dtype = dtype
        k_in = in_features or d_model
        self.wq = Dense(k_in, d_model, activation=None, dtype=proj_dtype, seed=seed + 1, device=device)
        self.wk = Dense(k_in, d_model, activation=None, dtype=proj_dtype, seed=seed + 2, device=device)
        self.wv = Dense(k_in, d_model, activation=None, dtype=proj_dtype, seed=seed + 3, device=device)

    def call(self, q, k, v, mask=None):
        B, Lq, _ = q.shape
        Lk = k.shape[1]
        qp = self.wq(q.reshape(B * Lq, -1)).reshape(B, Lq, self.d_model)
        kp = self.wk(k.reshape(B * Lk, -1)).reshape(B, Lk, self.d_model)
        vp = self.wv(v.reshape(B * Lk, -1)).reshape(B, Lk, self.d_model)
        return scaled_dot_product_attention(qp, kp, vp, mask, heads=self.num_heads, dtype=self.dtype)

    forward = call


class SelfAttention(torch.nn.Module):
    def __init__(self, add_pos: bool = True, dim: Optional[int] = None, seed: int = 0, device="cuda",
                 dtype=torch.float16):
        super().__init__()
        self.add_pos = add_pos
        self.dim = dim
        self.seed = seed
        self.device = device
        self.dtype = dtype
        self.W = None

    def build(self, dim: int):
        self.dim = dim
        g = torch.Generator().manual_seed(self.seed)
        w = torch.randn((dim, dim), generator=g) * 0.05  # keras 'random_normal' (stddev 0.05)
        self.W = Dense(dim, dim, activation="relu", use_bias=False, dtype=torch.float32, device=self.device,
                       weight=w.T.contiguous())

    @staticmethod
    def positional_encoding(length: int, dim: int) -> np.ndarray:
        pos = np.arange(length)[:, None]
        i = np.arange(dim)[None, :]
        ang = pos / np.power(10000, (2 * (i // 2)) / np.float32(dim))
        ang[:, 0::2] = np.sin(ang[:, 0::2])
        ang[:, 1::2] = np.cos(ang[:, 1::2])
        return ang.astype(np.float32)

    def forward(self, inputs):
        q, k, v, mask = inputs
        if self.W is None:
            self.build(q.shape[-1])
        B, Ln, dim = q.shape
        if self.add_pos:
            pe = torch.from_numpy(self.positional_encoding(Ln, dim)).to(q.device)
            q = q.float() + pe
            k = k.float() + torch.from_numpy(self.positional_encoding(k.shape[1], dim)).to(q.device)
        qn = self.W(q.reshape(B * Ln, dim)).reshape(B, Ln, dim)
        kn = self.W(k.reshape(B * k.shape[1], dim)).reshape(B, k.shape[1], dim)
        m = None if mask is None else mask.reshape(B, Ln)
        o = scaled_dot_product_attention(qn, kn, v, m, heads=1, dtype=self.dtype)
        return o.mean(dim=1)

    __call__ = torch.nn.Module.__call__
