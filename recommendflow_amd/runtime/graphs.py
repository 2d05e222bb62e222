"""hipGraph capture of whole forwards (torch.cuda.CUDAGraph is a hipGraph on ROCm).

A forward here is a chain of short launches through the C ABI (cfg3: 2 fused encoders, the ESIM
kernel, 9 norm / GEMM launches). Eager, every launch pays the Python + ctypes path on the host
(~13-15 us), which is longer than most of the kernels: the chain is host-bound. Captured once and
replayed, the chain costs one graph launch; the kernels run back to back.

Nothing in librf synchronises with the host or allocates (rf_api.h: caller-owned buffers, stream-ordered
launches), so every hot-path op is capturable as-is. Inputs live in static device buffers:
  * tensors: one static copy (or the caller's own tensor when it is passed again);
  * SparseBatch: the CSR arrays with a CAPACITY (token bytes and token count vary per batch; the kernels
    find every token through bag_off, and the launch parameters depend only on B and the slot count), so
    any batch of the same B / slot count that fits is loaded by device-to-device copies, no recapture.
"""
from __future__ import annotations

import gc
from typing import Callable, List, Optional, Sequence

import torch

from .batch import SparseBatch


class StaticSparseBatch(SparseBatch):
    """Device CSR buffers with room for `tok_bytes_cap` bytes and `tok_cap` tokens."""

    def __init__(self, like: SparseBatch, tok_bytes_cap: Optional[int] = None, tok_cap: Optional[int] = None,
                 device="cuda"):
        nb = int(len(like.tok_bytes))
        nt = like.n_tokens
        tok_bytes_cap = max(16, int(tok_bytes_cap if tok_bytes_cap is not None else nb + nb // 4 + 64))
        tok_cap = int(tok_cap if tok_cap is not None else nt + nt // 4 + 16)
        super().__init__(torch.zeros(tok_bytes_cap, dtype=torch.uint8, device=device),
                         torch.zeros(tok_cap + 1, dtype=torch.int32, device=device),
                         torch.zeros(like.batch * like.n_slots + 1, dtype=torch.int32, device=device),
                         torch.zeros(like.n_slots, dtype=torch.int32, device=device), like.batch, like.n_slots)
        self.n_tok_live = 0
        self.single_token_capture = False
        self.load(like)
        # FusedSparseEncoder picks the single-token kernel (RF_FLAG_SINGLE_TOKEN) from the host Lmax of the
        # batch it sees, so a graph captured on this batch bakes that choice in: remember it, and refuse a
        # later batch the single-token kernel cannot pool (load below)
        hl = self.host_lmax
        self.single_token_capture = hl is not None and len(hl) > 0 and int(max(hl)) <= 1

    @property
    def n_tokens(self) -> int:  # the live batch's token count (the buffers hold capacity)
        return self.n_tok_live

    def load(self, b: SparseBatch) -> "StaticSparseBatch":
        if b is self:
            return self
        if b.batch != self.batch or b.n_slots != self.n_slots:
            raise ValueError(f"static batch is B={self.batch} x {self.n_slots} slots, got B={b.batch} x {b.n_slots}")
        if self.single_token_capture:
            hl = b.lmax if not b.is_device() else b.host_lmax
            if hl is None or (len(hl) and int(max(hl)) > 1):
                raise ValueError("this static batch was captured on a batch whose slots hold at most one token "
                                 "(single-token kernel); a batch with Lmax > 1 (or without a host copy of lmax) "
                                 "needs a graph captured on a multi-token batch")
        nb, nt = int(len(b.tok_bytes)), b.n_tokens
        if nb > self.tok_bytes.numel() or nt + 1 > self.tok_off.numel():
            raise ValueError(f"batch needs {nb} token bytes / {nt} tokens; capacity {self.tok_bytes.numel()} / "
                             f"{self.tok_off.numel() - 1}: capture with a larger capacity")
        dev = b if b.is_device() else b.to(self.tok_off.device)
        self.tok_bytes[:nb].copy_(dev.tok_bytes[:nb], non_blocking=True)
        self.tok_off[: nt + 1].copy_(dev.tok_off, non_blocking=True)
        self.bag_off.copy_(dev.bag_off, non_blocking=True)
        self.lmax.copy_(dev.lmax, non_blocking=True)
        self.host_lmax = b.lmax if not b.is_device() else b.host_lmax  # never a device sync
        self.n_tok_live = nt
        return self


class CapturedGraph:
    """`fn()` (reading and writing fixed device buffers) captured once; replay() re-runs its launches."""

    def __init__(self, fn: Callable[[], object], warmup: int = 2):
        self.fn = fn
        # warm-up and capture on this graph's own stream: lazy init, LDS attributes, the allocator, and the
        # per-stream state librf's callers key on the stream (runtime/gemm.py's zeroed stream-K workspace) all
        # exist, eagerly initialised, before the capture starts (torch's shared default capture stream would give
        # every graph one workspace, first zeroed by a memset captured into whichever graph came first)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                fn()
        torch.cuda.current_stream().wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        # No Python garbage collection inside the capture: a cycle collected there runs destructors (a pinned host
        # buffer's free records and queries events) that are illegal while a stream captures, and the process
        # aborts. torch >= 2.6 no longer collects before a capture (force_cudagraph_gc), so collect here, then hold
        # the collector off until capture_end (GPUTEST_r05's SIGABRT: "Garbage-collecting" inside rf_gemm_f32_grouped
        # under test_graphs_gpu's capture). thread_local: other threads' HIP calls (a FeaturePipe's producer) are
        # not capture violations.
        gc.collect()
        was_enabled = gc.isenabled()
        gc.disable()
        try:
            with torch.cuda.graph(self.graph, stream=side, capture_error_mode="thread_local"):
                self.out = fn()
        finally:
            if was_enabled:
                gc.enable()

    def replay(self):
        self.graph.replay()
        return self.out


class GraphedForward:
    """A module forward captured on static inputs; __call__(*inputs) loads the inputs and replays.

    Tensor inputs are copied into the static buffers unless the caller passes the static tensors
    themselves (`static_inputs`); SparseBatch inputs go through StaticSparseBatch.load. The returned
    output tensor is the graph's own buffer, overwritten by the next call (clone it to keep it)."""

    def __init__(self, forward: Callable[..., torch.Tensor], *inputs, warmup: int = 2, capacity_slack: float = 0.25):
        self.static_inputs: List[object] = []
        for x in inputs:
            if isinstance(x, SparseBatch):
                nb, nt = int(len(x.tok_bytes)), x.n_tokens
                self.static_inputs.append(StaticSparseBatch(x, int(nb * (1 + capacity_slack)) + 64,
                                                            int(nt * (1 + capacity_slack)) + 16))
            elif isinstance(x, torch.Tensor):
                self.static_inputs.append(x.detach().clone())
            else:
                self.static_inputs.append(x)
        self._g = CapturedGraph(lambda: forward(*self.static_inputs), warmup=warmup)

    def __call__(self, *inputs: Sequence[object]) -> torch.Tensor:
        if len(inputs) != len(self.static_inputs):
            raise ValueError(f"expected {len(self.static_inputs)} inputs, got {len(inputs)}")
        for s, x in zip(self.static_inputs, inputs):
            if isinstance(s, StaticSparseBatch):
                s.load(x)
            elif isinstance(s, torch.Tensor):
                if x is not s:
                    if x.shape != s.shape:
                        raise ValueError(f"input shape {tuple(x.shape)} != captured {tuple(s.shape)}")
                    s.copy_(x, non_blocking=True)
        return self._g.replay()
