"""Dense and normalisation layers on librf.so (the building blocks of create_mlp, backend/blocks/mlp.py).

Dense(units, activation)  tf.keras.layers.Dense: y = act(x @ W + b); W kept as [N][K] (transposed Keras
                          kernel) in the compute dtype (bf16 -> bf16 MFMA, fp32 -> exact fp32 MFMA);
                          glorot_uniform kernel, zero bias (Keras defaults), deterministic by seed.
LayerNormalization(eps)   tf.keras.layers.LayerNormalization over the last axis (gamma 1, beta 0).
BatchNormalization(eps)   tf.keras.layers.BatchNormalization at inference (running mean 0, var 1).
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch

from ...runtime import gemm as G
from ...runtime import lib as L


def act_name(activation) -> Optional[str]:
    if activation is None:
        return None
    if isinstance(activation, str):
        name = activation.lower()
    else:
        name = getattr(activation, "__name__", str(activation)).lower()
    if name not in L.ACT:
        raise ValueError(f"unsupported activation {activation!r}")
    return name



# fp32 layers run on rf_gemm_f32 (librf). RF_TOWER_BLASLT_WIDE=1 is an A/B switch only: fp32 layers with K >= 4096
# then take hipBLASLt (torch.addmm) instead
_BLASLT_WIDE = os.environ.get("RF_TOWER_BLASLT_WIDE", "0") == "1"
_BLASLT_MIN_K = int(os.environ.get("RF_TOWER_BLASLT_MIN_K", "4096"))


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False

class Dense(torch.nn.Module):
    def __init__(self, in_features: int, units: int, activation=None, use_bias: bool = True, dtype=torch.bfloat16,
                 seed: int = 0, device="cuda", weight: Optional[torch.Tensor] = None, bias: Optional[torch.Tensor] = None):
        super().__init__()
        self.in_features, self.units = int(in_features), int(units)
        self.activation = act_name(activation)
        self.dtype = dtype
        L.load()
        L.require_gpu()
        if weight is None:
            g = torch.Generator().manual_seed(int(seed))
            lim = math.sqrt(6.0 / (self.in_features + self.units))
            weight = (torch.rand((self.units, self.in_features), generator=g) * 2 - 1) * lim
        self.weight = weight.to(device=device, dtype=dtype).contiguous()  # [N][K]
        if bias is None and use_bias:
            bias = torch.zeros(self.units)
        self.bias = None if bias is None else bias.to(device=device, dtype=torch.float32).contiguous()

    def forward(self, x: torch.Tensor, out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
        M = x.shape[0]
        if (self.units <= 16 or self.activation == "softmax") and x.dtype == torch.float32 and self.units <= 64 \
                and self.in_features % 4 == 0 and x.stride(-1) == 1 and x.stride(0) % 4 == 0 and x.data_ptr() % 16 == 0:
            # small head on fp32 activations: no bf16 round trip of x (rf_dense_head_fwd)
            if out is None:
                out = torch.empty((M, self.units), dtype=torch.float32, device=self.weight.device)
            L.call("rf_dense_head_fwd", L.ptr(x), M, self.in_features, x.stride(0), L.ptr(self.weight),
                   L.torch_dtype_code(self.dtype), self.units, L.ptr(self.bias), L.ACT[self.activation], L.ptr(out),
                   out.stride(0), L.stream_ptr(stream))
            return out
        if x.dtype != self.dtype:
            x = x.to(self.dtype)
        if x.stride(-1) != 1:
            x = x.contiguous()
        if out is None:
            out = torch.empty((M, self.units), dtype=torch.float32, device=self.weight.device)
        return self._linear(x, self.weight, self.bias, out, stream)

    def _linear(self, x, weight, bias, out, stream):
        """fp32: rf_gemm_f32 (stream-K, bias + activation in the epilogue; hipBLASLt only behind
        RF_TOWER_BLASLT_WIDE=1). bf16, and fp32 shapes rf_gemm_f32 refuses: rf_linear_fwd, or its split-K form
        when rf_linear_splitk_ws_bytes > 0 (workspace from the caching allocator on the launch stream)."""
        M, dt = x.shape[0], L.torch_dtype_code(self.dtype)
        blaslt = (_BLASLT_WIDE and self.dtype == torch.float32 and self.in_features >= _BLASLT_MIN_K
                  and out.is_contiguous() and self.activation in (None, "none", "linear", "relu", "selu"))
        if self.dtype == torch.float32 and not blaslt and self.activation != "softmax" and \
                G.supported_gemm(x, weight, trans_b=True, out=out):
            # fp32 layers (the DSSM towers, dssm.py:25-26): rf_gemm_f32, stream-K exact-fp32 MFMA with the bias
            # and activation in its epilogue
            return G.gemm_f32(x, weight, trans_b=True, bias=bias, act=self.activation or "none", out=out,
                              stream=stream)
        if blaslt:
            # A/B only: hipBLASLt's fp32 kernel with its bias epilogue, SELU / ReLU in place after
            G.note_torch_fallback("a Dense layer (RF_TOWER_BLASLT_WIDE=1)")
            with torch.cuda.stream(stream) if isinstance(stream, torch.cuda.Stream) else _nullctx():
                if bias is None:
                    torch.mm(x, weight.t(), out=out)
                else:
                    torch.addmm(bias, x, weight.t(), out=out)
                if self.activation == "selu":
                    torch.selu_(out)
                elif self.activation == "relu":
                    torch.relu_(out)
            return out
        ws_bytes = int(L.load().rf_linear_splitk_ws_bytes(dt, M, self.in_features, self.units)) \
            if self.dtype == torch.float32 else 0
        if ws_bytes:
            ws = torch.empty(ws_bytes // 4, dtype=torch.float32, device=self.weight.device)
            L.call("rf_linear_splitk_fwd", L.ptr(x), dt, M, self.in_features, x.stride(0), L.ptr(weight), self.units,
                   L.ptr(bias), L.ACT[self.activation], L.ptr(out), out.stride(0), L.ptr(ws), ws_bytes,
                   L.stream_ptr(stream))
            return out
        L.call("rf_linear_fwd", L.ptr(x), dt, M, self.in_features, x.stride(0), L.ptr(weight), self.units,
               L.ptr(bias), L.ACT[self.activation], L.ptr(out), out.stride(0), L.stream_ptr(stream))
        return out


    def forward_with(self, x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor],
                     out: Optional[torch.Tensor] = None, stream=None) -> torch.Tensor:
        """This layer's GEMM + activation with substitute parameters ([N][K] weight of this layer's dtype,
        fp32 bias): the path MLP takes with a normalisation folded into the weights."""
        if x.dtype != self.dtype:
            x = x.to(self.dtype)
        if x.stride(-1) != 1:
            x = x.contiguous()
        M = x.shape[0]
        if out is None:
            out = torch.empty((M, self.units), dtype=torch.float32, device=self.weight.device)
        return self._linear(x, weight, bias, out, stream)


class LayerNormalization:
    mode = 0

    def __init__(self, epsilon: float = 1e-3, name: Optional[str] = None):
        self.epsilon = float(epsilon)
        self.name = name


class BatchNormalization:
    mode = 1

    def __init__(self, epsilon: float = 1e-3, name: Optional[str] = None):
        self.epsilon = float(epsilon)
        self.name = name


class Norm(torch.nn.Module):
    """One normalisation instance with its own parameters (deviation D-shared-norm: the reference appends
    the SAME Keras layer before every Dense, mlp.py:10-11, which only works when all widths match)."""

    def __init__(self, spec, width: int, device="cuda"):
        super().__init__()
        self.mode, self.eps, self.width = spec.mode, spec.epsilon, int(width)
        self.gamma = torch.ones(width, device=device)
        self.beta = torch.zeros(width, device=device)
        self.mean = torch.zeros(width, device=device) if self.mode == 1 else None
        self.var = torch.ones(width, device=device) if self.mode == 1 else None

    def forward(self, x: torch.Tensor, out_dtype=torch.bfloat16, stream=None) -> torch.Tensor:
        x = x.float()
        if x.stride(-1) != 1:
            x = x.contiguous()
        M = x.shape[0]
        y = torch.empty((M, self.width), dtype=out_dtype, device=x.device)
        L.call("rf_norm_fwd", L.ptr(x), M, self.width, x.stride(0), self.mode, self.eps, L.ptr(self.gamma),
               L.ptr(self.beta), L.ptr(self.mean), L.ptr(self.var), L.ptr(y), L.torch_dtype_code(out_dtype),
               y.stride(0), L.stream_ptr(stream))
        return y
