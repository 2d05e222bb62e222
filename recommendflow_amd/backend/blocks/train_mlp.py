"""create_mlp under model.fit for the DSSM towers (reference: backend/blocks/mlp.py:4-15 with
models/matching/dssm.py:25-26 `create_mlp([1024, 512, 256], 0.3, "selu", BatchNormalization(1e-6))`, trained by
example/ranking_search/train.py:96-104) on librf.so, replacing torch.nn.BatchNorm1d / Linear / SELU / Dropout.

Per layer, forward (training):
  mean, var = rf_col_stats(h)                          batch statistics (Keras tf.nn.moments: biased variance)
  W', b'    = rf_bn_fold(W, b, gamma, beta, mean, var) BatchNormalization folded into the Dense
  y         = selu(h W'^T + b')                        rf_gemm_f32, exact-fp32 MFMA, bias + SELU in its epilogue
  h_next    = rf_dropout_fwd(y)                        Keras Dropout(rate): kept / (1 - rate), counter-hash mask
and the moving statistics move as Keras does (moving = moving * momentum + batch * (1 - momentum), momentum
0.99, the biased batch variance). Backward: rf_selu_dropout_bwd (dpre and the bias gradient), the Dense weight
gradient G = dpre^T h (rf_gemm_f32) through rf_bn_fold_grad, dz = dpre W (rf_gemm_f32), rf_bn_bwd. In eval mode
the moving statistics fold into the weights (no dropout).
"""
from __future__ import annotations

import math
import os
from typing import List, Optional, Sequence

import torch

from ...runtime import gemm as GM
from ...runtime import lib as L

_ACT_NAME = {0: "none", 1: "gelu", 2: "relu", 3: "selu"}

_SEED_MIX = 0x9E3779B97F4A7C15


def layer_seed(base: int, step: int, layer: int) -> int:
    """The dropout mask seed of (tower seed, training step, layer): a 64-bit mix, any value is valid."""
    x = (base * 0x100000001B3 + step * _SEED_MIX + layer * 0xC2B2AE3D27D4EB4F) & 0xFFFFFFFFFFFFFFFF
    return x


# Every GEMM of the towers (forward, weight gradient, input gradient) runs on rf_gemm_f32 (librf: stream-K
# exact-fp32 MFMA). A/B switches only: RF_TOWER_BLASLT_WIDE=1 sends the forward of layers with K >= 4096 to
# hipBLASLt (torch.addmm + an in-place SELU); RF_TOWER_BWD_BLAS=1 sends the backward products to torch.mm.
_BLASLT_WIDE = os.environ.get("RF_TOWER_BLASLT_WIDE", "0") == "1"
_BLASLT_MIN_K = int(os.environ.get("RF_TOWER_BLASLT_MIN_K", "4096"))
_BWD_BLAS = os.environ.get("RF_TOWER_BWD_BLAS", "0") == "1"


def _linear_f32(x: torch.Tensor, W: torch.Tensor, b: torch.Tensor, act: int, out: torch.Tensor, stream: int):
    M, K = x.shape
    N = W.shape[0]
    if _BLASLT_WIDE and K >= _BLASLT_MIN_K and act == L.ACT["selu"] and out.is_contiguous():
        GM.note_torch_fallback("a tower forward layer (RF_TOWER_BLASLT_WIDE=1)")
        torch.addmm(b, x, W.t(), out=out)
        torch.selu_(out)
        return
    if GM.supported_gemm(x, W, trans_b=True, out=out):
        GM.gemm_f32(x, W, trans_b=True, bias=b, act=_ACT_NAME[act], out=out, stream=stream)
        return
    ws_bytes = int(L.load().rf_linear_splitk_ws_bytes(L.DT_F32, M, K, N))
    if ws_bytes:
        ws = torch.empty(ws_bytes // 4, dtype=torch.float32, device=x.device)
        L.call("rf_linear_splitk_fwd", L.ptr(x), L.DT_F32, M, K, x.stride(0), L.ptr(W), N, L.ptr(b), act, L.ptr(out),
               out.stride(0), L.ptr(ws), ws_bytes, stream)
    else:
        L.call("rf_linear_fwd", L.ptr(x), L.DT_F32, M, K, x.stride(0), L.ptr(W), N, L.ptr(b), act, L.ptr(out),
               out.stride(0), stream)


# Input-layer weight gradient on a side stream (opt-in, overlap_input_wgrad()): the widest GEMM of the backward
# (G = dpre^T x over the 8704 / 20480-wide tower inputs) is not on the path to the input gradient, so it can run
# beside what follows it on the main stream — the other tower's backward, the sparse table's reduce and Adam.
# join_input_wgrad() makes a stream wait for it before anything reads those gradients.
_WGRAD = {"on": False, "side": {}, "events": []}


class overlap_input_wgrad:
    # off by default: measured slower (cfg2 step 9.56-9.59 vs 9.75-9.78 ms same box, profiles/r04/wgrad_overlap_ab.txt):
    # the side GEMM slows the BN backward and the sparse reduce it runs beside more than it saves
    enabled = os.environ.get("RF_WGRAD_OVERLAP", "0") == "1"

    def __enter__(self):
        _WGRAD["on"] = self.enabled
        return self

    def __exit__(self, *exc):
        _WGRAD["on"] = False
        return False


def join_input_wgrad(stream=None):
    cur = torch.cuda.current_stream() if stream is None else stream
    for ev in _WGRAD["events"]:
        cur.wait_event(ev)
    _WGRAD["events"].clear()


def _side_stream(dev) -> torch.cuda.Stream:
    s = _WGRAD["side"].get(dev)
    if s is None:
        s = _WGRAD["side"][dev] = torch.cuda.Stream(device=dev)
    return s


# The small layers' backward GEMMs (K, N <= 1024) are host-bound: hipBLASLt's per-call algorithm query costs more
# host time than their kernels take. RF_SMALL_MM_ROCBLAS=1 routes them to rocBLAS (A/B; the large input-layer
# GEMMs stay on hipBLASLt).
_SMALL_MM_ROCBLAS = os.environ.get("RF_SMALL_MM_ROCBLAS", "0") == "1"


def _mm(a: torch.Tensor, b: torch.Tensor, small: bool) -> torch.Tensor:
    GM.note_torch_fallback("a tower backward product (RF_TOWER_BWD_BLAS=1)")
    if not (small and _SMALL_MM_ROCBLAS):
        return torch.mm(a, b)
    prev = torch.backends.cuda.preferred_blas_library()
    torch.backends.cuda.preferred_blas_library("cublas")
    try:
        return torch.mm(a, b)
    finally:
        torch.backends.cuda.preferred_blas_library(prev)


def _ws(M: int, K: int, device) -> torch.Tensor:
    return torch.empty(max(int(L.load().rf_tower_ws_bytes(M, K)), 4), dtype=torch.uint8, device=device)


def _gemm_layer(probs, trans_a: bool, trans_b: bool, stream):
    """One layer's GEMMs of every tower: probs = [(a, b, bias, act name, out)]. librf (rf_gemm_f32, grouped into one
    launch where runtime.gemm.group_pays) when every operand qualifies; otherwise torch one by one."""
    if all(GM.supported_gemm(a, b, trans_a, trans_b, o) for a, b, _, _, o in probs):
        return GM.gemm_f32_layer(probs, trans_a=trans_a, trans_b=trans_b, stream=stream)
    GM.note_torch_fallback("a tower backward layer (operand layout or size outside rf_gemm_f32's checks)")
    outs = []
    for a, b, bias, act, o in probs:
        A = a.t() if trans_a else a
        B = b.t() if trans_b else b
        r = torch.mm(A, B) if bias is None else torch.addmm(bias, A, B)
        r = {"selu": torch.selu, "relu": torch.relu, "none": lambda t: t}[act](r)
        if o is not None:
            o.copy_(r)
            r = o
        outs.append(r)
    return outs


def _towers_forward(towers, xs, params_list):
    """The training forward of several towers of equal depth on their inputs xs (2-D fp32 views with unit column
    stride; any row stride), layer by layer: per tower the batch statistics and the BatchNormalization fold, then ONE
    grouped GEMM (bias + SELU epilogue) for the layer of every tower, then per tower the dropout.
    Returns per tower (outputs per layer, batch means, batch variances, the step number that seeded the masks)."""
    for x in xs:
        if x.dim() != 2 or x.stride(1) != 1 or x.dtype != torch.float32:
            raise ValueError("TrainTower input must be a 2-D fp32 tensor with unit column stride")
    n = len(towers[0].units)
    if any(len(t.units) != n for t in towers):
        raise ValueError("towers of one grouped forward need equal depth")
    dev, st = xs[0].device, L.stream_ptr(None)
    steps = []
    for t in towers:
        steps.append(t.steps)
        t.steps += 1
    hs = list(xs)
    res = [([], [], []) for _ in towers]
    for l in range(n):
        probs, folded = [], []
        for ti, (tower, h, params) in enumerate(zip(towers, hs, params_list)):
            W, b, g, be = params[4 * l: 4 * l + 4]
            N, K = W.shape
            M = h.shape[0]
            mean = torch.empty(K, dtype=torch.float32, device=dev)
            var = torch.empty(K, dtype=torch.float32, device=dev)
            ws = _ws(M, K, dev)
            L.call("rf_col_stats", L.ptr(h), M, K, h.stride(0), L.ptr(mean), L.ptr(var), L.ptr(ws), ws.numel(), st)
            Wf = torch.empty_like(W)
            bf = torch.empty(N, dtype=torch.float32, device=dev)
            L.call("rf_bn_fold", L.ptr(W), N, K, L.ptr(b), L.ptr(g), L.ptr(be), L.ptr(mean), L.ptr(var), tower.eps,
                   L.ptr(Wf), L.ptr(bf), st)
            y = torch.empty((M, N), dtype=torch.float32, device=dev)
            res[ti][1].append(mean)
            res[ti][2].append(var)
            folded.append(Wf)
            probs.append((h, Wf, bf, "selu", y))
        if _BLASLT_WIDE and any(p[0].shape[1] >= _BLASLT_MIN_K for p in probs):
            for (h, Wf, bf, _, y) in probs:  # A/B: the forward GEMMs on hipBLASLt / librf one by one
                _linear_f32(h, Wf, bf, L.ACT["selu"], y, st)
            ys = [p[4] for p in probs]
        else:
            ys = _gemm_layer(probs, False, True, st)
        for ti, (tower, y) in enumerate(zip(towers, ys)):
            M, N = y.shape
            L.call("rf_dropout_fwd", L.ptr(y), M, N, N, tower.rate, layer_seed(tower.seed, steps[ti], l), L.ptr(y), N, st)
            with torch.no_grad():
                tower.moving_mean[l].mul_(tower.momentum).add_(res[ti][1][l], alpha=1.0 - tower.momentum)
                tower.moving_var[l].mul_(tower.momentum).add_(res[ti][2][l], alpha=1.0 - tower.momentum)
            res[ti][0].append(y)
        hs = ys
    return [(o, m, v, stp) for (o, m, v), stp in zip(res, steps)]


def _towers_backward(towers, steps, xs, params_list, outs_l, means_l, vars_l, douts, dx_outs):
    """Backward of _towers_forward: per tower the parameter gradients (W, b, gamma, beta per layer) returned, the
    input gradients written into dx_outs (views of the xs' shapes; any row stride). Per layer, last to first: per tower
    the SELU / dropout backward (dpre, the bias gradient); ONE grouped GEMM for every tower's Dense weight gradient
    G = dpre^T h, per tower its fold (rf_bn_fold_grad); ONE grouped GEMM for dz = dpre W; per tower the
    BatchNormalization backward."""
    n = len(towers[0].units)
    dev, st = xs[0].device, L.stream_ptr(None)
    dhs = [d if d.stride(1) == 1 else d.contiguous() for d in douts]
    grads = [[None] * (4 * n) for _ in towers]
    for l in reversed(range(n)):
        dpres, dbs, wss, hins = [], [], [], []
        for ti, tower in enumerate(towers):
            W = params_list[ti][4 * l]
            N, K = W.shape
            h_in = xs[ti] if l == 0 else outs_l[ti][l - 1]
            M = h_in.shape[0]
            ws = _ws(M, max(K, N), dev)
            dpre = torch.empty((M, N), dtype=torch.float32, device=dev)
            db = torch.empty(N, dtype=torch.float32, device=dev)
            dh = dhs[ti]
            L.call("rf_selu_dropout_bwd", L.ptr(dh), dh.stride(0), L.ptr(outs_l[ti][l]), N, M, N, tower.rate,
                   layer_seed(tower.seed, steps[ti], l), L.ptr(dpre), N, L.ptr(db), L.ptr(ws), ws.numel(), st)
            dpres.append(dpre)
            dbs.append(db)
            wss.append(ws)
            hins.append(h_in)
        dWs = [torch.empty_like(params_list[ti][4 * l]) for ti in range(len(towers))]

        def wgrad(stream, stream_ptr):
            if _BWD_BLAS:
                Gs = [_mm(dp.t(), h, h.shape[1] <= 1024 and dp.shape[1] <= 1024) for dp, h in zip(dpres, hins)]
            else:
                Gs = _gemm_layer([(dp, h, None, "none", None) for dp, h in zip(dpres, hins)], True, False, stream_ptr)
            for ti, tower in enumerate(towers):
                W, b, g, be = params_list[ti][4 * l: 4 * l + 4]
                N, K = W.shape
                L.call("rf_bn_fold_grad", L.ptr(Gs[ti]), N, K, L.ptr(dbs[ti]), L.ptr(g), L.ptr(be),
                       L.ptr(means_l[ti][l]), L.ptr(vars_l[ti][l]), tower.eps, L.ptr(dWs[ti]), stream_ptr)

        def igrad(stream_ptr):
            if _BWD_BLAS:
                return [_mm(dp, params_list[ti][4 * l], True) for ti, dp in enumerate(dpres)]
            return _gemm_layer([(dp, params_list[ti][4 * l], None, "none", None) for ti, dp in enumerate(dpres)],
                               False, False, stream_ptr)

        if l == 0 and _WGRAD["on"]:
            dzs = igrad(st)  # the input gradient's GEMM first, on the main stream
            main = torch.cuda.current_stream()
            side = _side_stream(dev)
            side.wait_stream(main)  # after dz: the weight gradient runs beside the BN backward and what follows
            with torch.cuda.stream(side):
                wgrad(side, L.stream_ptr(side))
                done = torch.cuda.Event()
                done.record(side)
            for ti in range(len(towers)):  # read / written on the side stream
                for t in (dpres[ti], hins[ti], dbs[ti], means_l[ti][l], vars_l[ti][l], dWs[ti], *params_list[ti][4 * l: 4 * l + 4]):
                    t.record_stream(side)
            _WGRAD["events"].append(done)
        else:
            wgrad(None, st)
            dzs = igrad(st)
        for ti, tower in enumerate(towers):
            W, b, g, be = params_list[ti][4 * l: 4 * l + 4]
            N, K = W.shape
            h_in = hins[ti]
            M = h_in.shape[0]
            dx = dx_outs[ti] if l == 0 else torch.empty((M, K), dtype=torch.float32, device=dev)
            dgamma = torch.empty(K, dtype=torch.float32, device=dev)
            dbeta = torch.empty(K, dtype=torch.float32, device=dev)
            dz = dzs[ti]
            L.call("rf_bn_bwd", L.ptr(dz), dz.stride(0), L.ptr(h_in), h_in.stride(0), M, K, L.ptr(means_l[ti][l]),
                   L.ptr(vars_l[ti][l]), L.ptr(g), tower.eps, L.ptr(dx), dx.stride(0), L.ptr(dgamma), L.ptr(dbeta),
                   L.ptr(wss[ti]), wss[ti].numel(), st)
            grads[ti][4 * l: 4 * l + 4] = [dWs[ti], dbs[ti], dgamma, dbeta]
            dhs[ti] = dx
    return grads


class _TowersFn(torch.autograd.Function):
    """Towers over column blocks of ONE input (the DSSM user and ad blocks of the fused encoder's output):
    the backward writes every tower's input gradient into its block of one full-width gradient, so autograd
    never materialises zero-filled slice gradients and adds them. Towers of equal depth run layer by layer
    together (one grouped GEMM per layer and pass)."""

    @staticmethod
    def forward(ctx, x, blocks, *params):
        towers = [t for t, _, _ in blocks]
        plist, p0 = [], 0
        for t in towers:
            np_ = 4 * len(t.units)
            plist.append(params[p0: p0 + np_])
            p0 += np_
        xs = [x[:, off: off + width] for _, off, width in blocks]
        groups = [[i] for i in range(len(towers))]
        if len({len(t.units) for t in towers}) == 1:
            groups = [list(range(len(towers)))]
        res = [None] * len(towers)
        for grp in groups:
            for i, r in zip(grp, _towers_forward([towers[i] for i in grp], [xs[i] for i in grp], [plist[i] for i in grp])):
                res[i] = r
        saved, meta = [], []
        p0 = 0
        for (tower, off, width), (outs, means, vars_, step) in zip(blocks, res):
            np_ = 4 * len(tower.units)
            meta.append((tower, off, width, step, p0, np_, len(saved)))
            saved += [*outs, *means, *vars_]
            p0 += np_
        ctx.meta = meta
        ctx.groups = groups
        ctx.save_for_backward(x, *params, *saved)
        return tuple(r[0][-1] for r in res)

    @staticmethod
    def backward(ctx, *douts):
        x = ctx.saved_tensors[0]
        nparams = sum(m[5] for m in ctx.meta)
        params = ctx.saved_tensors[1: 1 + nparams]
        saved = ctx.saved_tensors[1 + nparams:]
        dx = torch.zeros_like(x) if sum(m[2] for m in ctx.meta) != x.shape[1] else torch.empty_like(x)
        grads: List[Optional[torch.Tensor]] = [None] * nparams
        per = []
        for (tower, off, width, step, p0, np_, s0), dout in zip(ctx.meta, douts):
            n = len(tower.units)
            outs, means, vars_ = saved[s0: s0 + n], saved[s0 + n: s0 + 2 * n], saved[s0 + 2 * n: s0 + 3 * n]
            if dout is None:
                dout = torch.zeros_like(outs[-1])
            per.append((tower, step, x[:, off: off + width], params[p0: p0 + np_], outs, means, vars_, dout,
                        dx[:, off: off + width], p0, np_))
        for grp in ctx.groups:
            sel = [per[i] for i in grp]
            gs = _towers_backward([p[0] for p in sel], [p[1] for p in sel], [p[2] for p in sel], [p[3] for p in sel],
                                  [p[4] for p in sel], [p[5] for p in sel], [p[6] for p in sel], [p[7] for p in sel],
                                  [p[8] for p in sel])
            for p, g in zip(sel, gs):
                grads[p[9]: p[9] + p[10]] = g
        return (dx, None, *grads)


def towers_forward(x: torch.Tensor, blocks) -> tuple:
    """blocks: [(TrainTower, column offset, width)]: each tower's training forward on its block of x."""
    params = [p for t, _, _ in blocks for p in t.params()]
    return _TowersFn.apply(x, list(blocks), *params)


class TrainTower(torch.nn.Module):
    """One DSSM tower: [BatchNormalization(eps) -> Dense(units, selu) -> Dropout(rate)] per hidden size, fp32,
    glorot_uniform kernels and zero biases (Keras Dense defaults), gamma 1 / beta 0 / moving stats 0 and 1."""

    def __init__(self, in_features: int, units: Sequence[int], rate: float = 0.3, eps: float = 1e-6,
                 momentum: float = 0.99, seed: int = 0, generator: Optional[torch.Generator] = None, device="cuda"):
        super().__init__()
        L.load()
        L.require_gpu()
        self.units, self.rate, self.eps, self.momentum, self.seed = list(units), float(rate), float(eps), float(momentum), int(seed)
        self.steps = 0
        g = generator if generator is not None else torch.Generator().manual_seed(seed)
        self.W, self.b, self.gamma, self.beta = (torch.nn.ParameterList() for _ in range(4))
        self.moving_mean, self.moving_var = [], []
        width = int(in_features)
        for i, u in enumerate(self.units):
            lim = math.sqrt(6.0 / (width + u))
            self.W.append(torch.nn.Parameter(((torch.rand(u, width, generator=g) * 2 - 1) * lim).to(device)))
            self.b.append(torch.nn.Parameter(torch.zeros(u, device=device)))
            self.gamma.append(torch.nn.Parameter(torch.ones(width, device=device)))
            self.beta.append(torch.nn.Parameter(torch.zeros(width, device=device)))
            mm = torch.zeros(width, device=device)
            mv = torch.ones(width, device=device)
            self.register_buffer(f"moving_mean_{i}", mm)
            self.register_buffer(f"moving_var_{i}", mv)
            self.moving_mean.append(mm)
            self.moving_var.append(mv)
            width = u
        self.out_features = width

    def _apply(self, fn, *args, **kw):  # keep the moving-stat lists pointing at the registered buffers
        r = super()._apply(fn, *args, **kw)
        self.moving_mean = [getattr(self, f"moving_mean_{i}") for i in range(len(self.units))]
        self.moving_var = [getattr(self, f"moving_var_{i}") for i in range(len(self.units))]
        return r

    def params(self) -> List[torch.nn.Parameter]:
        out = []
        for l in range(len(self.units)):
            out += [self.W[l], self.b[l], self.gamma[l], self.beta[l]]
        return out

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.training:
            if x.stride(1) != 1:
                x = x.contiguous()
            return towers_forward(x, [(self, 0, x.shape[1])])[0]
        # inference: the moving statistics folded into the weights, no dropout
        st = L.stream_ptr(None)
        h = x if x.stride(1) == 1 else x.contiguous()
        for l in range(len(self.units)):
            W = self.W[l].detach()
            N, K = W.shape
            Wf = torch.empty_like(W)
            bf = torch.empty(N, dtype=torch.float32, device=x.device)
            L.call("rf_bn_fold", L.ptr(W), N, K, L.ptr(self.b[l]), L.ptr(self.gamma[l]), L.ptr(self.beta[l]),
                   L.ptr(self.moving_mean[l]), L.ptr(self.moving_var[l]), self.eps, L.ptr(Wf), L.ptr(bf), st)
            y = torch.empty((h.shape[0], N), dtype=torch.float32, device=x.device)
            _linear_f32(h, Wf, bf, L.ACT["selu"], y, st)
            h = y
        return h
