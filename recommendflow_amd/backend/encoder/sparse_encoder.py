"""Fused multi-slot sparse encoder: every hashing feature of a tower in ONE kernel launch.

Replaces the per-feature loop the reference runs inside a model: for each hashing feature f of
get_preprocess_layers (backend/utils/preprocess_utils.py:10-20), DoubleHashingEmbedding.call
(backend/layers/preprocess_layers.py:94-97) = 2 x Hashing + 2 x (Embedding gather + combiner) + concat,
i.e. 2 string-hash ops + 2 gathers + 2 reductions per feature per step (456 + 456 + 456 TF ops for
base_recall_sdpa.yaml). Here all slots of a tower share one fused table; slot s owns two segments
[row_base[k], row_base[k] + N_s) (k = seeds[0], seeds[1]); its output [pool(T1) | pool(T2)] lands at
a fixed column offset of one [B, sum_s 2*D] tensor (the concat of the reference's per-feature outputs
in feature order).
"""
from __future__ import annotations

import zlib
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch

from ...runtime import lib as L
from ...runtime.batch import SparseBatch

# rf_slot_desc (include/rf_api.h), 64 bytes
SLOT_DTYPE = np.dtype(
    [
        ("row_base", "<i8", (2,)),
        ("num_bins", "<i8"),
        ("salt", "<u8", (2,)),
        ("out_off", "<i8"),
        ("dim", "<i4"),
        ("combiner", "<i4"),
        ("mask_empty", "<i4"),
        ("reserved", "<i4"),
    ]
)
assert SLOT_DTYPE.itemsize == 64

POOLED = ("sum", "avg", "max", "min", "first", "last")


def normalize_seeds(seeds) -> Tuple[int, int]:
    """DoubleHashingEmbedding seeds: [s0, s1]; an int s means [s, s + 7] (preprocess_layers.py:88; the
    reference then indexes the raw int and crashes — deviation D-int-seed keeps the stated intent)."""
    if seeds is None:
        raise ValueError("DoubleHashingEmbedding needs hash seeds (Keras Hashing without a salt uses FarmHash64, "
                         "which this build does not implement)")
    if isinstance(seeds, (int, np.integer)):
        return int(seeds), int(seeds) + 7
    s = list(seeds)
    if len(s) < 2:
        raise ValueError(f"seeds must hold two salts, got {seeds}")
    return int(s[0]), int(s[1])


def name_seed(name: str, base: int = 0) -> int:
    return (zlib.crc32(name.encode()) ^ (base * 0x9E3779B1)) & 0xFFFFFFFF


@dataclass
class SlotSpec:
    name: str
    num_bins: int
    seeds: Tuple[int, int]
    combiner: str = "sum"
    mask_empty: bool = True  # get_preprocess_layers builds Hashing with mask_value="" (preprocess_utils.py:15)


def init_table(table: torch.Tensor, row0: int = 0, row_stride: int = 1, seed: int = 0, lo: float = -0.05,
               hi: float = 0.05, stream=None) -> torch.Tensor:
    """Counter-based U(lo, hi) init on the GPU (rf_table_init_uniform): identical rows for any sharding."""
    L.require_gpu()
    rows, dim = table.shape
    L.call("rf_table_init_uniform", L.ptr(table), L.torch_dtype_code(table.dtype), rows, dim, row0, row_stride,
           seed, lo, hi, L.stream_ptr(stream))
    return table


@dataclass
class BwdPlan:
    """FusedSparseEncoder.backward_plan's state: the device batch, the distinct rows (rows[:n_uniq]) and the
    workspace the reduce half continues from."""
    batch: SparseBatch
    n_pos: int
    cap: int
    rows: torch.Tensor
    n_uniq: torch.Tensor
    ws: torch.Tensor
    flags: int


@dataclass
class SparseGrad:
    """Deduplicated gradient of a fused table (device): rows[:n] ascending, grad[:n] [n, dim]; n = n_uniq
    (a device int32; negative = invalid batch, see rf_fused_hash_embed_bwd)."""
    rows: torch.Tensor
    grad: torch.Tensor
    n_uniq: torch.Tensor
    cap: int

    def count(self) -> int:
        n = int(self.n_uniq.item())
        if n < 0:
            raise ValueError(f"invalid batch for the embedding backward (error bits {-n})")
        if n > self.cap:
            raise ValueError(f"{n} distinct rows exceed uniq_cap {self.cap}")
        return n


class FusedSparseEncoder(torch.nn.Module):
    """All hashing slots of one tower -> [B, sum_s 2*D] with one rf_fused_hash_embed_fwd launch."""

    def __init__(self, slots: Sequence[SlotSpec], dim: int, table_dtype=torch.float32, out_dtype=None,
                 seed: int = 0, mask_padding: bool = False, device="cuda", init_range=(-0.05, 0.05),
                 table: Optional[torch.Tensor] = None, row_base0: int = 0, spec_rows: bool = False):
        super().__init__()
        if not slots:
            raise ValueError("FusedSparseEncoder needs at least one slot")
        self.slots = list(slots)
        self.dim = int(dim)
        self.table_dtype = table_dtype
        self.out_dtype = out_dtype or table_dtype
        self.mask_padding = bool(mask_padding)
        self.seed = int(seed)
        self.single_token = True  # RF_FLAG_SINGLE_TOKEN when a batch's host-side Lmax allows it (A/B: False)
        # backward: rows with > 256 positions summed as fixed-order partials + a tree (RF_FLAG_TREE_REDUCE: within
        # SURVEY §8d's L 2^-23 sum|x| of the reference's CPU order, not bit-exact with it); default: the CPU order
        self.tree_reduce = False
        self.extra_flags = 0  # diagnostic bits (rf_api.h RF_FLAG_DIAG_*; ablations 12-14 go to rf_diag_fused_hash_embed_fwd)
        desc = np.zeros(len(self.slots), SLOT_DTYPE)
        base = int(row_base0)
        for i, sp in enumerate(self.slots):
            if sp.num_bins is None or sp.num_bins <= 0:
                raise ValueError("`num_bins` cannot be `None` or non-positive values.")
            if sp.num_bins >= 2 ** 31:
                raise ValueError("num_bins must be < 2^31")
            if sp.combiner not in POOLED:
                raise ValueError(f"Do not support combiner = '{sp.combiner}' in a fused encoder, supported: "
                                 f"[{', '.join(POOLED)}] (null pooling runs per feature)")
            desc[i]["row_base"] = (base, base + sp.num_bins)
            desc[i]["num_bins"] = sp.num_bins
            desc[i]["salt"] = (sp.seeds[0] & (2 ** 64 - 1), sp.seeds[1] & (2 ** 64 - 1))
            desc[i]["out_off"] = i * 2 * self.dim
            desc[i]["dim"] = self.dim
            desc[i]["combiner"] = L.COMB[sp.combiner]
            desc[i]["mask_empty"] = int(sp.mask_empty)
            base += 2 * sp.num_bins
        self.host_desc = desc
        self.table_rows = base
        self.out_width = 2 * self.dim * len(self.slots)
        L.load()
        L.require_gpu()
        self.register_buffer("desc", torch.from_numpy(desc.view(np.uint8).copy()).to(device), persistent=False)
        # spec_rows: the allocation holds two more rows right after the table, a NaN row (id table_rows) and a zero
        # row (table_rows + 1), which the ESIM gather path's ids address directly (RF_FLAG_SPEC_ROWS); self.table
        # stays the [table_rows, dim] view, so every other operator sees the same table
        self.spec_rows = bool(spec_rows) and table is None
        if table is None:
            full = torch.empty((self.table_rows + (2 if self.spec_rows else 0), self.dim), dtype=table_dtype, device=device)
            table = full[: self.table_rows]
            init_table(table, 0, 1, self.seed, *init_range)
            if self.spec_rows:
                full[self.table_rows] = float("nan")
                full[self.table_rows + 1] = 0.0
        elif table.shape[0] < self.table_rows or table.shape[1] != self.dim:
            raise ValueError(f"shared table {tuple(table.shape)} too small for {self.table_rows} x {self.dim}")
        self.table = table

    def _single_token_batch(self, batch: SparseBatch) -> bool:
        """True when the batch's per-slot Lmax is known on the host without a device sync and is <= 1, and the
        row width suits the single-token kernel (4, 8 or 16 chunks of 16 bytes)."""
        lm = batch.lmax if not batch.is_device() else batch.host_lmax
        if lm is None:
            return False
        chunks = self.dim * self.table.element_size() // 16
        return chunks in (4, 8, 16) and int(np.max(lm, initial=0)) <= 1

    def slot_offsets(self) -> List[Tuple[str, int, int]]:
        return [(sp.name, i * 2 * self.dim, (i + 1) * 2 * self.dim) for i, sp in enumerate(self.slots)]

    def forward(self, batch: SparseBatch, out: Optional[torch.Tensor] = None, out_col: int = 0,
                emit_idx: bool = False, stream=None):
        if batch.n_slots != len(self.slots):
            raise ValueError(f"batch has {batch.n_slots} slots, encoder {len(self.slots)}")
        if not batch.is_device():
            batch = batch.to(self.table.device)
        B = batch.batch
        if out is None:
            out = torch.empty((B, self.out_width), dtype=self.out_dtype, device=self.table.device)
            out_col = 0
        if out_col:
            raise ValueError("out_col is reserved; pass a column slice through the descriptors instead")
        flags = (L.FLAG_MASK_PADDING if self.mask_padding else 0) | (L.FLAG_EMIT_IDX if emit_idx else 0) | self.extra_flags
        if not emit_idx and not self.extra_flags and self.single_token and self._single_token_batch(batch):
            flags |= L.FLAG_SINGLE_TOKEN  # every slot's batch Lmax <= 1: the low-register single-token kernel
        idx = torch.empty((max(batch.n_tokens, 1), 2), dtype=torch.int64, device=self.table.device) if emit_idx else None
        entry = "rf_diag_fused_hash_embed_fwd" if self.extra_flags & L.DIAG_ABLATIONS else "rf_fused_hash_embed_fwd"
        L.call(entry, L.ptr(self.desc), len(self.slots), L.ptr(batch.tok_bytes),
               L.ptr(batch.tok_off), L.ptr(batch.bag_off), L.ptr(batch.lmax), B, L.ptr(self.table),
               L.torch_dtype_code(self.table.dtype), self.table.shape[0], self.dim, L.ptr(out),
               L.torch_dtype_code(out.dtype), out.stride(0), flags, L.ptr(idx), L.stream_ptr(stream))
        if emit_idx:
            return out, idx[: batch.n_tokens]
        return out

    # ---- training -------------------------------------------------------------
    def backward(self, batch: SparseBatch, dout: torch.Tensor, out: Optional[torch.Tensor] = None,
                 uniq_cap: Optional[int] = None, stream=None) -> "SparseGrad":
        """Deduplicated sparse gradient of the fused table from dout [B, out_width] (fp32), exactly the
        IndexedSlices Keras' optimizer sums per row (rf_fused_hash_embed_bwd). `out` (the forward
        output) is needed when a slot pools max/min."""
        if self.table.dtype != torch.float32 or dout.dtype != torch.float32:
            raise ValueError("backward needs an fp32 table and an fp32 output gradient")
        if batch.n_slots != len(self.slots):
            raise ValueError(f"batch has {batch.n_slots} slots, encoder {len(self.slots)}")
        lm = batch.lmax_numpy()
        if not batch.is_device():
            batch = batch.to(self.table.device)
        B = batch.batch
        dev = self.table.device
        n_pos = B * int(2 * np.asarray(lm, np.int64).sum())
        cap = int(uniq_cap) if uniq_cap is not None else max(1, min(n_pos, self.table.shape[0]))
        rows = torch.empty(max(cap, 1), dtype=torch.int64, device=dev)
        grad = torch.empty((max(cap, 1), self.dim), dtype=torch.float32, device=dev)
        n_uniq = torch.zeros(1, dtype=torch.int32, device=dev)
        need_mm = any(sp.combiner in ("max", "min") for sp in self.slots)
        if need_mm and out is None:
            raise ValueError("max/min pooling: backward needs the forward output `out`")
        dout = dout.contiguous()
        if out is not None and (out.stride(0) != dout.stride(0) or out.dtype != torch.float32):
            out = out.contiguous().float()
        cnt = torch.empty(dout.shape, dtype=torch.int32, device=dev) if need_mm else None
        wsb = L.load().rf_embed_bwd_ws_bytes(n_pos, len(self.slots), self.table.shape[0])
        ws = torch.empty(max(int(wsb), 256), dtype=torch.uint8, device=dev)
        flags = (L.FLAG_MASK_PADDING if self.mask_padding else 0) | (L.FLAG_TREE_REDUCE if self.tree_reduce else 0)
        L.call("rf_fused_hash_embed_bwd", L.ptr(self.desc), len(self.slots), L.ptr(batch.tok_bytes), L.ptr(batch.tok_off),
               L.ptr(batch.bag_off), L.ptr(batch.lmax), B, n_pos, L.ptr(self.table), self.table.shape[0], self.dim,
               L.ptr(out) if need_mm else None, L.ptr(dout), dout.stride(0), flags, L.ptr(cnt), L.ptr(rows), L.ptr(grad),
               cap, L.ptr(n_uniq), L.ptr(ws), ws.numel(), L.stream_ptr(stream))
        return SparseGrad(rows, grad, n_uniq, cap)

    def backward_plan(self, batch: SparseBatch, uniq_cap: Optional[int] = None, stream=None) -> "BwdPlan":
        """The batch-only half of backward() (rf_fused_hash_embed_bwd_plan): the distinct rows the gradient will
        hold (plan.rows[:n], ascending; n = plan.n_uniq on the device), before dout exists."""
        if batch.n_slots != len(self.slots):
            raise ValueError(f"batch has {batch.n_slots} slots, encoder {len(self.slots)}")
        lm = batch.lmax_numpy()
        if not batch.is_device():
            batch = batch.to(self.table.device)
        B, dev = batch.batch, self.table.device
        n_pos = B * int(2 * np.asarray(lm, np.int64).sum())
        cap = int(uniq_cap) if uniq_cap is not None else max(1, min(n_pos, self.table.shape[0]))
        rows = torch.empty(max(cap, 1), dtype=torch.int64, device=dev)
        n_uniq = torch.zeros(1, dtype=torch.int32, device=dev)
        wsb = L.load().rf_embed_bwd_ws_bytes(n_pos, len(self.slots), self.table.shape[0])
        ws = torch.empty(max(int(wsb), 256), dtype=torch.uint8, device=dev)
        flags = (L.FLAG_MASK_PADDING if self.mask_padding else 0) | (L.FLAG_TREE_REDUCE if self.tree_reduce else 0)
        L.call("rf_fused_hash_embed_bwd_plan", L.ptr(self.desc), len(self.slots), L.ptr(batch.tok_bytes),
               L.ptr(batch.tok_off), L.ptr(batch.bag_off), L.ptr(batch.lmax), B, n_pos, self.table.shape[0], self.dim,
               self.out_width, flags, L.ptr(rows), cap, L.ptr(n_uniq), L.ptr(ws), ws.numel(), L.stream_ptr(stream))
        return BwdPlan(batch, n_pos, cap, rows, n_uniq, ws, flags)

    def backward_reduce(self, plan: "BwdPlan", dout: torch.Tensor, out: Optional[torch.Tensor] = None,
                        stream=None) -> "SparseGrad":
        """The dout half of backward() on a plan from backward_plan (same stream order or joined): the result
        equals backward(plan.batch, dout, out) bit for bit."""
        if self.table.dtype != torch.float32 or dout.dtype != torch.float32:
            raise ValueError("backward needs an fp32 table and an fp32 output gradient")
        dout = dout.contiguous()
        if dout.stride(0) != self.out_width:
            raise ValueError("backward_reduce: dout must be [B, out_width] (the plan's row stride)")
        need_mm = any(sp.combiner in ("max", "min") for sp in self.slots)
        if need_mm and out is None:
            raise ValueError("max/min pooling: backward needs the forward output `out`")
        if out is not None and (out.stride(0) != dout.stride(0) or out.dtype != torch.float32):
            out = out.contiguous().float()
        cnt = torch.empty(dout.shape, dtype=torch.int32, device=dout.device) if need_mm else None
        grad = torch.empty((max(plan.cap, 1), self.dim), dtype=torch.float32, device=dout.device)
        b = plan.batch
        L.call("rf_fused_hash_embed_bwd_reduce", L.ptr(self.desc), len(self.slots), L.ptr(b.tok_bytes), L.ptr(b.tok_off),
               L.ptr(b.bag_off), L.ptr(b.lmax), b.batch, plan.n_pos, L.ptr(self.table), self.table.shape[0], self.dim,
               L.ptr(out) if need_mm else None, L.ptr(dout), dout.stride(0), plan.flags, L.ptr(cnt), L.ptr(plan.rows),
               L.ptr(grad), plan.cap, L.ptr(plan.n_uniq), L.ptr(plan.ws), plan.ws.numel(), L.stream_ptr(stream))
        return SparseGrad(plan.rows, grad, plan.n_uniq, plan.cap)

    def algorithmic_bytes(self, batch: SparseBatch, pad_rows: bool = False) -> int:
        """HBM bytes one forward must move, SURVEY §8d exactly: bytes = sum_s 2 L_s D e_T (every row occurrence, no
        dedup credit) + sum_s 2 D e_out (pooled output) + sum_s L_s (token length + 4) (token bytes and their i32
        offsets), summed over the batch's examples.

        pad_rows=True is the round-5 form: one extra pad-row read per padded bag and table (the
        reference gathers T[0] at every pad position; the kernel reads row 0 once per bag) plus the i32 bag
        offsets. bench.py prints both and takes the roofline fraction from the §8d form."""
        h = batch.numpy()
        esz = torch.tensor([], dtype=self.table_dtype).element_size()
        osz = torch.tensor([], dtype=self.out_dtype).element_size()
        lens = np.diff(h.bag_off).reshape(h.batch, h.n_slots)
        rows = int(lens.sum())
        out = h.batch * self.out_width * osz
        if not pad_rows:
            return 2 * rows * self.dim * esz + out + int(h.tok_off[-1]) + 4 * h.n_tokens
        if not self.mask_padding:
            rows += int((lens < h.lmax[None, :]).sum())
        return 2 * rows * self.dim * esz + out + int(len(h.tok_bytes)) + 4 * (h.n_tokens + 1) + 4 * (h.batch * h.n_slots + 1)
