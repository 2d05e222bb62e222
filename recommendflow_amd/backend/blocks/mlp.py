"""create_mlp (reference: backend/blocks/mlp.py:4-15): per hidden size  Norm -> Dense(act) -> Dropout.

Dropout is the identity at inference. Each layer runs rf_norm_fwd (fp32 -> MFMA operand dtype) then
rf_linear_fwd (MFMA GEMM with bias + activation fused in the epilogue); an fp32 layer behind a
BatchNormalization runs as ONE GEMM with the normalisation folded into its weights (MLP._bn_folded).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch

from ...runtime import lib as L
from ..layers.core import Dense, Norm, act_name


def _param_key(ts):
    """Cache key of a folded-weight entry: the source tensors themselves (strong references, so a freed
    tensor's id can never be reused by a replacement) with their in-place versions."""
    return tuple((t, t._version) if isinstance(t, torch.Tensor) else t for t in ts)


def _same_key(a, b) -> bool:
    if a is None or b is None or len(a) != len(b):
        return False
    for x, y in zip(a, b):
        if isinstance(x, tuple) and isinstance(y, tuple):
            if x[0] is not y[0] or x[1] != y[1]:
                return False
        elif x != y:
            return False
    return True


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

    def forward(self, x: torch.Tensor, out: Optional[torch.Tensor] = None, stream=None,
                normed=False) -> torch.Tensor:
        """x [M, in] -> [M, hidden_units[-1]] fp32; `out` (optional) receives the last layer (any row stride).
        A two-layer LayerNorm MLP on a narrow input runs as ONE launch (rf_mlp2_small_fwd); otherwise
        each layer is rf_norm_fwd -> rf_linear_fwd. normed=True: x is the first layer's normalisation output
        already (its producer applied norms[0]), in the layers' dtype."""
        if not self.denses:
            self.build(x.shape[-1])
        if not normed and self._fusable(x):
            return self._forward_fused(x, out, stream)
        last = len(self.denses) - 1
        i = 0
        while i <= last:
            norm, dense = self.norms[i], self.denses[i]
            if normed and i == 0:
                norm = None
            o = out if i == last else None
            if norm is not None and norm.mode == 1 and self.dtype == torch.float32 and x.dtype == torch.float32:
                w, b = self._bn_folded(i)  # no normalisation pass: BatchNorm lives in the weights
                x = dense.forward_with(x, w, b, out=o, stream=stream)
                i += 1
                continue
            h = norm(x, out_dtype=self.dtype, stream=stream) if norm is not None else x
            if self._ln_pair_ok(i, h):
                x = self._ln_pair(i, h, out if i + 1 == last else None, stream)
                i += 2
                continue
            x = dense(h, out=o, stream=stream)
            i += 1
        return x

    fold_ln = True  # set False to run every LayerNorm as its own pass (A/B and tests)

    def _ln_pair_ok(self, i: int, h: torch.Tensor) -> bool:
        """Layers i, i+1 as rf_linear_stats_fwd -> rf_linear_lnfold_fwd: bf16 GEMMs on the LDS-DMA path
        (K >= 512, K % 64 == 0 for both), a LayerNorm in front of layer i+1, an elementwise activation."""
        if not self.fold_ln or i + 1 >= len(self.denses) or self.dtype != torch.bfloat16 or self.activation == "softmax":
            return False
        n1 = self.norms[i + 1]
        k0, k1 = self.denses[i].in_features, self.denses[i + 1].in_features
        return (n1 is not None and n1.mode == 0 and k0 >= 512 and k0 % 64 == 0 and k1 >= 512 and k1 % 64 == 0
                and h.dtype == torch.bfloat16 and h.dim() == 2 and h.stride(-1) == 1 and h.stride(0) % 8 == 0
                and h.data_ptr() % 16 == 0)

    def _ln_pair(self, i, h, out, stream):
        """act(LN(act(h W0^T + b0)) W1^T + b1) without the LayerNorm pass: the first GEMM writes its output
        as bf16 plus per-row, per-32-column-slice (sum, squared deviations from the slice mean) from its
        epilogue, the second combines them (Chan) and applies the normalisation after the product (W1
        diag(gamma) and the per-column terms from _ln_folded). Precision: the second GEMM multiplies the
        UNCENTERED bf16 activations, so its error grows with |row mean| / row std (about 2^-9 of that ratio,
        relative); fold_ln = False runs the LayerNorm as its own fp32 pass for such rows."""
        d0, d1, n1 = self.denses[i], self.denses[i + 1], self.norms[i + 1]
        M = h.shape[0]
        yb = torch.empty((M, d0.units), dtype=torch.bfloat16, device=h.device)
        st = torch.empty((M, 4 * ((d0.units + 127) // 128), 2), dtype=torch.float32, device=h.device)
        w0, b0 = d0.weight, d0.bias
        L.call("rf_linear_stats_fwd", L.ptr(h), M, d0.in_features, h.stride(0), L.ptr(w0), d0.units,
               L.ptr(b0), L.ACT[self.activation], L.ptr(yb), yb.stride(0), L.ptr(st), L.stream_ptr(stream))
        wg, sv, tv = self._ln_folded(i + 1)
        if out is None:
            out = torch.empty((M, d1.units), dtype=torch.float32, device=h.device)
        L.call("rf_linear_lnfold_fwd", L.ptr(yb), M, d1.in_features, yb.stride(0), L.ptr(wg), d1.units, L.ptr(sv),
               L.ptr(tv), L.ptr(st), n1.eps, L.ACT[self.activation], L.ptr(out), out.stride(0), L.stream_ptr(stream))
        return out

    def prenormed_head_ok(self, in_features: int, head) -> bool:
        """forward_prenormed_head applies: two bf16 layers, each behind a LayerNormalization, both folded (K >= 512,
        K % 128 == 0 for the first: its producers' 32-column slices fill every partial slot), an elementwise
        activation, and a bf16 Dense(2) head on the last layer's output."""
        if not self.fold_ln or len(self.denses) != 2 or self.dtype != torch.bfloat16 or self.activation == "softmax":
            return False
        if any(n is None or n.mode != 0 for n in self.norms):
            return False
        k0, k1 = self.denses[0].in_features, self.denses[1].in_features
        return (k0 == in_features and k0 >= 512 and k0 % 128 == 0 and k1 >= 512 and k1 % 64 == 0
                and head is not None and head.units == 2 and head.in_features == self.denses[1].units
                and head.weight.dtype == torch.bfloat16 and head.weight.is_contiguous())

    def forward_prenormed_head(self, xb: torch.Tensor, xstats: torch.Tensor, head, out: Optional[torch.Tensor] = None,
                               stream=None) -> torch.Tensor:
        """head(mlp(x)) where x arrives as its producers wrote it for an LN-folded consumer: bf16 values xb [M, K]
        and per-row, per-32-column-slice (sum, squared deviations) partials xstats [M, K / 32, 2] fp32. Layer 0:
        LN0 folded into its GEMM, its output written as bf16 + slice partials (rf_linear_lnfold_stats_fwd); layer 1:
        LN1 folded, the Dense(2) head's per-tile partial logits in its epilogue, then the head's softmax
        (rf_linear_lnfold_head_fwd): no LayerNorm pass and no [M, units] fp32 round trip anywhere (mlp.py:10-13,
        esim.py:84-88). Precision: both GEMMs multiply uncentered bf16 activations (_ln_pair's note)."""
        d0, d1 = self.denses
        n0, n1 = self.norms
        M, K0 = xb.shape
        if xb.dtype != torch.bfloat16 or xb.stride(1) != 1 or xb.stride(0) % 8 or xb.data_ptr() % 16:
            raise ValueError("xb must be a row-major bf16 [M, K] tensor with 16-byte rows")
        if xstats.dtype != torch.float32 or not xstats.is_contiguous() or tuple(xstats.shape) != (M, K0 // 32, 2):
            raise ValueError(f"xstats must be contiguous fp32 [{M}, {K0 // 32}, 2]")
        wg0, sv0, tv0 = self._ln_folded(0)
        yb = torch.empty((M, d0.units), dtype=torch.bfloat16, device=xb.device)
        st1 = torch.empty((M, 4 * ((d0.units + 127) // 128), 2), dtype=torch.float32, device=xb.device)
        act = L.ACT[self.activation]
        L.call("rf_linear_lnfold_stats_fwd", L.ptr(xb), M, K0, xb.stride(0), L.ptr(wg0), d0.units, L.ptr(sv0), L.ptr(tv0),
               L.ptr(xstats), n0.eps, act, L.ptr(yb), yb.stride(0), L.ptr(st1), L.stream_ptr(stream))
        wg1, sv1, tv1 = self._ln_folded(1)
        # the workspace starts with one counter per 64-row block that the launch needs zero and leaves zero (the
        # row block's last tile runs the softmax) and keeps the partial logits at its far end, so one zeroed ws
        # serves every M up to the one it was sized for (N = d1.units is fixed per module): allocated zeroed when
        # too small and reused (one stream at a time per module)
        ws_bytes = int(L.load().rf_linear_lnfold_head_ws_bytes(M, d1.units))
        ws = getattr(self, "_head_ws", None)
        if ws is None or ws.numel() < ws_bytes or ws.device != xb.device:
            ws = self._head_ws = torch.zeros(max(ws_bytes, 1), dtype=torch.uint8, device=xb.device)
        if out is None:
            out = torch.empty((M, head.units), dtype=torch.float32, device=xb.device)
        L.call("rf_linear_lnfold_head_fwd", L.ptr(yb), M, d1.in_features, yb.stride(0), L.ptr(wg1), d1.units, L.ptr(sv1),
               L.ptr(tv1), L.ptr(st1), n1.eps, act, None, 0, L.ptr(head.weight), head.units,
               L.ptr(head.bias) if head.bias is not None else None, L.ACT[head.activation], L.ptr(out), out.stride(0),
               L.ptr(ws), ws.numel(), L.stream_ptr(stream))
        return out

    def _ln_folded(self, i: int):
        """(W diag(gamma) in bf16, s = its row sums, t = W beta + b) of denses[i] behind LayerNorm norms[i];
        cached until a parameter changes (replaced tensor or in-place version)."""
        n, d = self.norms[i], self.denses[i]
        ts = (d.weight, d.bias, n.gamma, n.beta)
        key = _param_key(ts)
        cache = getattr(self, "_fold_cache", None)
        if cache is None:
            cache = self._fold_cache = {}
        hit = cache.get(("ln", i))
        if hit is not None and _same_key(hit[0], key):
            return hit[1]
        w64 = d.weight.double()
        wg = (w64 * n.gamma.double()[None, :]).to(torch.bfloat16).contiguous()
        sv = wg.double().sum(dim=1).float().contiguous()
        tv = (w64 @ n.beta.double() + (d.bias.double() if d.bias is not None else 0.0)).float().contiguous()
        cache[("ln", i)] = (key, (wg, sv, tv))
        return wg, sv, tv

    def _bn_folded(self, i: int):
        """denses[i] with norms[i] folded in, for fp32 layers. BatchNormalization at inference is a per-column
        affine x a + c (a = gamma / sqrt(var + eps), c = beta - mean a), so
            BN(x) W^T + b = x (W diag(a))^T + (W c + b)
        and the GEMM reads the raw activations: the [M, K] normalisation pass (and its HBM round trip)
        disappears. Cached until a parameter changes (replaced tensor or in-place version)."""
        n, d = self.norms[i], self.denses[i]
        ts = (d.weight, d.bias, n.gamma, n.beta, n.mean, n.var)
        key = _param_key(ts + (n.eps,))
        cache = getattr(self, "_fold_cache", None)
        if cache is None:
            cache = self._fold_cache = {}
        hit = cache.get(i)
        if hit is not None and _same_key(hit[0], key):
            return hit[1], hit[2]
        a = n.gamma.double() / torch.sqrt(n.var.double() + n.eps)
        c = n.beta.double() - n.mean.double() * a
        w64 = d.weight.double()
        w = (w64 * a[None, :]).to(d.dtype).contiguous()
        b = (w64 @ c + (d.bias.double() if d.bias is not None else 0.0)).float().contiguous()
        cache[i] = (key, w, b)
        return w, b

    def _fusable(self, x: torch.Tensor) -> bool:
        return (len(self.denses) == 2 and self.dtype == torch.bfloat16 and x.dtype == torch.float32
                and all(n is not None and n.mode == 0 for n in self.norms) and self.activation != "softmax"
                and self.denses[0].in_features <= 32 and self.denses[0].units in (128, 256)
                and x.dim() == 2 and x.stride(-1) == 1)

    def _forward_fused(self, x, out, stream):
        n0, n1 = self.norms
        d0, d1 = self.denses
        M = x.shape[0]
        if out is None:
            out = torch.empty((M, d1.units), dtype=torch.float32, device=x.device)
        L.call("rf_mlp2_small_fwd", L.ptr(x), M, d0.in_features, x.stride(0), n0.eps, L.ptr(n0.gamma), L.ptr(n0.beta),
               L.ptr(d0.weight), L.ptr(d0.bias), d0.units, L.ptr(n1.gamma), L.ptr(n1.beta), L.ptr(d1.weight),
               L.ptr(d1.bias), d1.units, L.ACT[self.activation], L.ptr(out), out.stride(0), L.stream_ptr(stream))
        return out

    def forward_stats(self, x: torch.Tensor, outb: torch.Tensor, stats: torch.Tensor, p0: int, stream=None):
        """The fused two-layer forward (rf_mlp2_small_stats_fwd) writing its output as bf16 into outb [M, O] (any row
        stride) and its per-32-column-slice partials into stats[:, p0 : p0 + O / 32] (stats contiguous [M, P, 2]):
        the input MLP's half of cfg3's pooled row for an LN-folded consumer (forward_prenormed_head)."""
        if not self.denses:
            self.build(x.shape[-1])
        if not self._fusable(x):
            raise ValueError("forward_stats needs the fused two-layer form (rf_mlp2_small_fwd's conditions)")
        n0, n1 = self.norms
        d0, d1 = self.denses
        M = x.shape[0]
        if outb.dtype != torch.bfloat16 or outb.shape != (M, d1.units) or outb.stride(1) != 1:
            raise ValueError(f"outb must be bf16 [{M}, {d1.units}] with unit column stride")
        if stats.dtype != torch.float32 or not stats.is_contiguous() or stats.dim() != 3 or stats.shape[0] != M:
            raise ValueError("stats must be contiguous fp32 [M, P, 2]")
        L.call("rf_mlp2_small_stats_fwd", L.ptr(x), M, d0.in_features, x.stride(0), n0.eps, L.ptr(n0.gamma), L.ptr(n0.beta),
               L.ptr(d0.weight), L.ptr(d0.bias), d0.units, L.ptr(n1.gamma), L.ptr(n1.beta), L.ptr(d1.weight),
               L.ptr(d1.bias), d1.units, L.ACT[self.activation], L.ptr(outb), outb.stride(0), L.ptr(stats),
               stats.shape[1], p0, L.stream_ptr(stream))
        return outb


def forward_towers(mlps: Sequence[MLP], xs: Sequence[torch.Tensor], stream=None) -> List[torch.Tensor]:
    """The forward of several fp32 BatchNormalization MLPs of equal depth (the DSSM user and ad towers,
    dssm.py:25-26) layer by layer: each layer's GEMMs of every tower through runtime.gemm.gemm_f32_layer (ONE
    rf_gemm_f32_grouped launch for the small layers, whose tiles then fill the chip together; one launch each for
    layers with a tile per CU), BatchNormalization folded into the weights (MLP._bn_folded), bias + activation in the
    epilogue. Any other MLP mix runs each MLP on its own."""
    from ...runtime import gemm as G

    for m, x in zip(mlps, xs):
        if not m.denses:
            m.build(x.shape[-1])
    depth = {len(m.denses) for m in mlps}
    ok = (len(depth) == 1 and all(m.dtype == torch.float32 and m.activation not in ("softmax",)
                                  and all(n is not None and n.mode == 1 for n in m.norms) for m in mlps)
          and all(x.dtype == torch.float32 and G.supported(x) for x in xs))
    if not ok:
        return [m(x, stream=stream) for m, x in zip(mlps, xs)]
    hs = list(xs)
    for i in range(depth.pop()):
        probs = []
        for m, h in zip(mlps, hs):
            w, b = m._bn_folded(i)
            probs.append((h, w, b, m.activation or "none", None))
        hs = G.gemm_f32_layer(probs, trans_b=True, stream=stream)
    return hs


def create_mlp(hidden_units, dropout_rate, activation, normalization_layer, name=None, **kw) -> MLP:
    return MLP(hidden_units, dropout_rate, activation, normalization_layer, name=name, **kw)
