"""Exact-fp32 GEMM of the DSSM towers on librf.so (rf_gemm_f32, include/rf_api.h).

Reference: every fp32 Dense of the towers (models/matching/dssm.py:25-26, create_mlp -> backend/blocks/mlp.py:4-15)
and, under model.fit (example/ranking_search/train.py:96-104), the two MatMuls of its gradient. One entry point
covers the three layouts:
    forward        y  = act(x W^T + b)   gemm_f32(x, W, trans_b=True)      A k-contiguous, B k-contiguous
    weight grad    G  = dpre^T h         gemm_f32(dpre, h, trans_a=True)   A m-contiguous, B n-contiguous
    input grad     dz = dpre W           gemm_f32(dpre, W)                 A k-contiguous, B n-contiguous
gemm_f32_grouped runs up to 4 such GEMMs of one layout in one launch (the same layer of both towers).
The workspace (per-tile counters that every launch leaves zero, then the stream-K partial tiles) is allocated
zeroed once per (device, stream) and grown as needed; calls on one stream share it.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch

from . import lib as L

_WS = {}
_RETIRED = []
calls = 0  # launches since import (tests assert the tower paths run here)


def _workspace(dev: torch.device, stream_handle: int, need: int) -> torch.Tensor:
    key = (dev.index, stream_handle)
    ws = _WS.get(key)
    if ws is None or ws.numel() < need:
        # a grown ws starts zeroed (its counters); the old one may still be read by launches queued on this stream,
        # so it is never released (growth happens a handful of times per process)
        if ws is not None:
            _RETIRED.append(ws)
        ws = _WS[key] = torch.zeros(max(need, 256), dtype=torch.uint8, device=dev)
        cur = torch.cuda.current_stream(dev)
        if stream_handle not in (cur.cuda_stream, 0) and not torch.cuda.is_current_stream_capturing():
            # the memset ran on torch's current stream: the launch stream waits for it
            torch.cuda.ExternalStream(stream_handle, device=dev).wait_stream(cur)
    return ws


def _op(t: torch.Tensor, kc: bool):
    """(pointer source, leading dimension) of an operand given as a 2-D view: kc = its rows are the contraction
    index's neighbours (unit column stride either way)."""
    if t.dim() != 2 or t.stride(1) != 1 or t.dtype != torch.float32:
        raise ValueError("rf_gemm_f32 operands are 2-D fp32 views with unit column stride")
    return t, t.stride(0)


def supported(*ts: torch.Tensor) -> bool:
    """Operand views rf_gemm_f32 accepts: fp32, unit column stride, leading dimension % 4 == 0, 16-byte aligned."""
    return all(t.dtype == torch.float32 and t.dim() == 2 and t.stride(1) == 1 and t.stride(0) % 4 == 0
               and t.data_ptr() % 16 == 0 for t in ts)


def _block_ok(t: torch.Tensor, kc: bool, K: int) -> bool:
    # rf_gemm_f32's 32-bit buffer offsets (rf_gemm32.hip RF_REQUIRE): a k-contiguous operand's 128-row tile block,
    # an m/n-contiguous operand's K + 192 k-rows, each under 2 GiB
    return (128 if kc else K + 192) * t.stride(0) * 4 < (1 << 31)


def supported_gemm(a: torch.Tensor, b: torch.Tensor, trans_a: bool = False, trans_b: bool = False,
                   out: Optional[torch.Tensor] = None) -> bool:
    """Whether rf_gemm_f32 takes this problem as laid out: supported() operands, K % 4 == 0, and every operand block
    inside the 2 GiB limit of the C check (the tower weight gradient dpre^T h at batch x width x 4 B near
    2 GiB must go to the fallback, not raise)."""
    if not supported(a, b) or (out is not None and not supported(out)):
        return False
    K = a.shape[0] if trans_a else a.shape[1]
    return K % 4 == 0 and _block_ok(a, not trans_a, K) and _block_ok(b, trans_b, K)


torch_fallbacks = 0  # tower / Dense fp32 GEMMs that went to torch (hipBLASLt) instead of librf; tests assert 0
_warned = [False]


def note_torch_fallback(what: str):
    """Counts (and warns once about) an fp32 tower GEMM leaving librf for torch.mm / addmm."""
    global torch_fallbacks
    torch_fallbacks += 1
    if not _warned[0]:
        _warned[0] = True
        import warnings
        warnings.warn(f"rf_gemm_f32 fallback to torch for {what}", RuntimeWarning, stacklevel=3)


def gemm_f32(a: torch.Tensor, b: torch.Tensor, trans_a: bool = False, trans_b: bool = False,
             bias: Optional[torch.Tensor] = None, act: str = "none", out: Optional[torch.Tensor] = None,
             stream=None) -> torch.Tensor:
    """out[M][N] = act(op(a) op(b) + bias) with op(a) = a^T if trans_a (a stored [K][M]) else a ([M][K]) and
    op(b) = b^T if trans_b (b stored [N][K]) else b ([K][N]); fp32 products and accumulation (exact MFMA)."""
    global calls
    M, K = (a.shape[1], a.shape[0]) if trans_a else (a.shape[0], a.shape[1])
    N, Kb = (b.shape[0], b.shape[1]) if trans_b else (b.shape[1], b.shape[0])
    if Kb != K:
        raise ValueError(f"rf_gemm_f32: inner dimensions differ ({K} vs {Kb})")
    A, lda = _op(a, not trans_a)
    B, ldb = _op(b, trans_b)
    if out is None:
        out = torch.empty((M, N), dtype=torch.float32, device=a.device)
    st = stream if isinstance(stream, int) else L.stream_ptr(stream)
    need = int(L.load().rf_gemm_f32_ws_bytes(M, N, K))
    ws = _workspace(a.device, st, need)
    L.call("rf_gemm_f32", L.ptr(A), lda, int(not trans_a), L.ptr(B), ldb, int(trans_b), M, N, K, L.ptr(bias),
           L.ACT[act], L.ptr(out), out.stride(0), L.ptr(ws), ws.numel(), st)
    calls += 1
    return out


def gemm_f32_grouped(problems, trans_a: bool = False, trans_b: bool = False, stream=None):
    """One launch for every (a, b, bias, act, out) of `problems` (1..4, one layout for all): out = act(op(a) op(b) +
    bias) as gemm_f32 computes it. Returns the outputs."""
    global calls
    if not 1 <= len(problems) <= 4:
        raise ValueError("rf_gemm_f32_grouped: 1..4 problems")
    arr = (L.GemmProblem * len(problems))()
    outs = []
    for i, (a, b, bias, act, out) in enumerate(problems):
        M, K = (a.shape[1], a.shape[0]) if trans_a else (a.shape[0], a.shape[1])
        N, Kb = (b.shape[0], b.shape[1]) if trans_b else (b.shape[1], b.shape[0])
        if Kb != K:
            raise ValueError(f"rf_gemm_f32_grouped: inner dimensions differ ({K} vs {Kb}) in problem {i}")
        _op(a, not trans_a)
        _op(b, trans_b)
        if out is None:
            out = torch.empty((M, N), dtype=torch.float32, device=a.device)
        arr[i] = L.GemmProblem(L.ptr(a), a.stride(0), L.ptr(b), b.stride(0), L.ptr(out), out.stride(0), L.ptr(bias),
                               M, N, K, L.ACT[act], 0)
        outs.append(out)
    st = stream if isinstance(stream, int) else L.stream_ptr(stream)
    lib = L.load()
    need = int(lib.rf_gemm_f32_grouped_ws_bytes(ctypes.cast(arr, ctypes.c_void_p), len(problems)))
    ws = _workspace(problems[0][0].device, st, need)
    L.call("rf_gemm_f32_grouped", ctypes.cast(arr, ctypes.c_void_p), len(problems), int(not trans_a), int(trans_b), L.ptr(ws), ws.numel(), st)
    calls += 1
    return outs


def _tiles(M: int, N: int) -> int:
    return ((M + 127) // 128) * ((N + 127) // 128)


def group_pays(shapes, cus: int = None) -> bool:
    """Whether one grouped launch beats one launch per problem for these (M, N) output shapes: grouping fills the
    chip with problems too small to fill it alone (the towers' 512- and 256-wide layers: 0.61 -> 0.79 and 0.27 ->
    0.45 of peak, tools/gemm32_group_probe.py), but a problem with a tile per CU already runs each CU's tile whole,
    and sharing its grid with another problem cuts tiles between workgroups (the 1024-wide input layers: 0.915 ->
    0.849)."""
    if cus is None:
        cus = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
    return len(shapes) > 1 and max(_tiles(M, N) for M, N in shapes) < cus


def gemm_f32_layer(problems, trans_a: bool = False, trans_b: bool = False, stream=None):
    """The same layer of several towers: one grouped launch when group_pays, else one launch per problem."""
    shapes = []
    for a, b, _, _, _ in problems:
        M = a.shape[1] if trans_a else a.shape[0]
        N = b.shape[0] if trans_b else b.shape[1]
        shapes.append((M, N))
    if group_pays(shapes):
        return gemm_f32_grouped(problems, trans_a=trans_a, trans_b=trans_b, stream=stream)
    return [gemm_f32(a, b, trans_a=trans_a, trans_b=trans_b, bias=bias, act=act, out=out, stream=stream)
            for a, b, bias, act, out in problems]
