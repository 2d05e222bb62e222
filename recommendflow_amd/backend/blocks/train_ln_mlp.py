"""create_mlp(units, rate, gelu, LayerNormalization(eps)) under model.fit, exact fp32 on librf (reference:
backend/blocks/mlp.py:4-15 as models/ranking/esim.py:45-48,52 builds it; trained by example/ranking_search/train.py:96-104).

Per layer (deviation D-shared-norm: one LayerNormalization per layer, the reference's single shared instance only
builds when every width matches):
    z   = LayerNorm(x)                 rf_norm_fwd (mode 0, fp32 out)
    pre = z W^T + b                    rf_gemm_f32 (exact fp32 MFMA, bias in the epilogue)
    h   = Dropout(rate)(gelu(pre))     rf_act_dropout_fwd (rf_dropout_fwd's counter-hash keep mask)
and backward
    dpre, db = rf_act_dropout_bwd(dh, pre)
    dW = dpre^T z, dz = dpre W         rf_gemm_f32 (weight-gradient and input-gradient layouts)
    dx, dgamma, dbeta = rf_layernorm_bwd(dz, x)
Explicit forward / backward (no torch autograd): the caches are the layer inputs, the normalised inputs and the
pre-activations. Parameters are fp32 tensors with .grad set by backward() (backend.optim.KerasAdam steps them).
Keras initialisers: Dense glorot_uniform kernel, zero bias; LayerNorm gamma 1, beta 0.
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence

import torch

from ...runtime import gemm as GM
from ...runtime import lib as L
from .train_mlp import layer_seed


class TrainLNMLP:
    def __init__(self, in_features: int, units: Sequence[int], rate: float = 0.3, activation: str = "gelu",
                 eps: float = 1e-6, seed: int = 0, generator: Optional[torch.Generator] = None, device="cuda"):
        L.load()
        L.require_gpu()
        if activation not in ("gelu", "relu", "selu", "none"):
            raise ValueError(f"TrainLNMLP: unsupported activation {activation!r}")
        self.in_features, self.units = int(in_features), [int(u) for u in units]
        self.rate, self.act, self.eps, self.seed = float(rate), L.ACT[activation], float(eps), int(seed)
        g = generator if generator is not None else torch.Generator().manual_seed(seed)
        self.gamma: List[torch.Tensor] = []
        self.beta: List[torch.Tensor] = []
        self.W: List[torch.Tensor] = []
        self.b: List[torch.Tensor] = []
        k = self.in_features
        for u in self.units:
            lim = math.sqrt(6.0 / (k + u))
            self.gamma.append(torch.ones(k, device=device))
            self.beta.append(torch.zeros(k, device=device))
            self.W.append(((torch.rand((u, k), generator=g) * 2 - 1) * lim).to(device).contiguous())  # [out][in]
            self.b.append(torch.zeros(u, device=device))
            k = u
        self.out_features = k
        self._cache = None

    def parameters(self) -> List[torch.Tensor]:
        out = []
        for i in range(len(self.units)):
            out += [self.W[i], self.b[i], self.gamma[i], self.beta[i]]
        return out

    def layer_seeds(self, step: int) -> List[int]:
        return [layer_seed(self.seed, step, l) for l in range(len(self.units))]

    def forward(self, x: torch.Tensor, step: int = 0, out: Optional[torch.Tensor] = None, training: bool = True,
                stream=None) -> torch.Tensor:
        """x [M, in] fp32 (unit column stride, any row stride) -> [M, units[-1]]; `out` (optional view, any row
        stride) receives the last layer. Dropout runs only with training=True; the caches for backward() are kept."""
        st = L.stream_ptr(stream)
        M = x.shape[0]
        if x.dtype != torch.float32 or x.stride(-1) != 1:
            x = x.float().contiguous()
        rate = self.rate if training else 0.0
        seeds = self.layer_seeds(step)
        cache = []
        last = len(self.units) - 1
        for l, u in enumerate(self.units):
            K = x.shape[1]
            z = torch.empty((M, K), dtype=torch.float32, device=x.device)
            L.call("rf_norm_fwd", L.ptr(x), M, K, x.stride(0), 0, self.eps, L.ptr(self.gamma[l]), L.ptr(self.beta[l]), None,
                   None, L.ptr(z), L.DT_F32, z.stride(0), st)
            pre = GM.gemm_f32(z, self.W[l], trans_b=True, bias=self.b[l], stream=st)
            h = out if (l == last and out is not None) else torch.empty((M, u), dtype=torch.float32, device=x.device)
            L.call("rf_act_dropout_fwd", L.ptr(pre), pre.stride(0), M, u, self.act, rate, seeds[l], L.ptr(h), h.stride(0), st)
            cache.append((x, z, pre))
            x = h
        self._cache = (cache, rate, seeds)
        return x

    def backward(self, dh: torch.Tensor, need_dx: bool = True, stream=None) -> Optional[torch.Tensor]:
        """dh [M, units[-1]] (unit column stride) -> dx [M, in] (None when need_dx is False); sets every
        parameter's .grad."""
        if self._cache is None:
            raise RuntimeError("TrainLNMLP.backward before forward")
        cache, rate, seeds = self._cache
        st = L.stream_ptr(stream)
        lib = L.load()
        if dh.stride(-1) != 1:
            dh = dh.contiguous()
        dx = None
        for l in reversed(range(len(self.units))):
            x, z, pre = cache[l]
            M, N = pre.shape
            K = z.shape[1]
            dpre = torch.empty((M, N), dtype=torch.float32, device=pre.device)
            db = torch.empty(N, dtype=torch.float32, device=pre.device)
            ws = torch.empty(max(int(lib.rf_tower_ws_bytes(M, N)), 4), dtype=torch.uint8, device=pre.device)
            L.call("rf_act_dropout_bwd", L.ptr(dh), dh.stride(0), L.ptr(pre), pre.stride(0), M, N, self.act, rate, seeds[l],
                   L.ptr(dpre), dpre.stride(0), L.ptr(db), L.ptr(ws), ws.numel(), st)
            self.W[l].grad = GM.gemm_f32(dpre, z, trans_a=True, stream=st)
            self.b[l].grad = db
            dz = GM.gemm_f32(dpre, self.W[l], stream=st)
            dxl = torch.empty((M, K), dtype=torch.float32, device=pre.device)
            dg = torch.empty(K, dtype=torch.float32, device=pre.device)
            dbt = torch.empty(K, dtype=torch.float32, device=pre.device)
            wsl = torch.empty(max(int(lib.rf_layernorm_bwd_ws_bytes(M, K)), 4), dtype=torch.uint8, device=pre.device)
            L.call("rf_layernorm_bwd", L.ptr(dz), dz.stride(0), L.ptr(x), x.stride(0), M, K, L.ptr(self.gamma[l]), self.eps,
                   L.ptr(dxl), dxl.stride(0), L.ptr(dg), L.ptr(dbt), L.ptr(wsl), wsl.numel(), st)
            self.gamma[l].grad, self.beta[l].grad = dg, dbt
            dh = dxl
            dx = dxl
        self._cache = None
        return dx if need_dx else None
