"""Row-sharded fused sparse encoder: the fused table of one tower split over P ranks.

The reference never shards a table: it runs MirroredStrategy (one full replica per device, gradients
all-reduced; run/train.py) and its largest table is what fits one device. Here the fused
table of `FusedSparseEncoder` is row-sharded over the P ranks of the job so a 1e9 x 128 table (512 GB
fp32) spans 8 x 288 GB of HBM:

* owner(g) = g mod P, local(g) = g div P (round-robin rows: hot low bins and hot slots spread evenly);
* shard r holds rows g = r, r + P, ... and is initialised with the same counter-based generator as the
  unsharded table (rf_table_init_uniform, row0 = r, row_stride = P), so for a given seed every P
  produces the same logical table, and the pooled output is bit-identical to the single-GPU kernel.

One forward per rank (requester) is four C-ABI launches and two all-to-alls:

  route   : rf_hash_rows (2 global rows per token) + 2*S padding rows -> rf_route_rows (each distinct
            row once, sorted owner-major: local ids, per-owner counts, and the row map from each
            logical row to its slot in the receive buffer); dedup=False uses rf_bucketize_owner instead
  exchange: all_to_all(counts); all_to_all_single(local ids)           -> owners
  serve   : rf_gather_rows on the local shard                           (owner side)
  exchange: all_to_all_single(row vectors)                              -> requesters
  combine : rf_pool_rows_fwd straight from the receive buffer, reading logical row j at row_map[j]
            (the un-permute is fused into the pooling loads; same pooling code and accumulation order as
            rf_fused_hash_embed_fwd, so the result is bit-identical)

The communication object is pluggable: `TorchDistComm` (torch.distributed; RCCL on the GPU box, gloo in
the CPU tests) and `simulate_sharded_forward` (P shards in one process, for single-GPU parity tests).
The kernel ops are pluggable the same way (`GpuShardOps` = librf; the CPU tests pass oracle-backed ops
from tests/, never the product).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np
import torch

from ...runtime import lib as L
from ...runtime.batch import SparseBatch, from_lists
from .sparse_encoder import POOLED, SLOT_DTYPE, SlotSpec


def shard_rows(total_rows: int, rank: int, nranks: int) -> int:
    """Rows of the global table owned by `rank` (g = rank, rank + P, ...)."""
    return max(0, (total_rows - rank + nranks - 1) // nranks)


def build_slot_desc(slots: Sequence[SlotSpec], dim: int, row_base0: int = 0):
    """Descriptors of the fused layout (identical to FusedSparseEncoder's)."""
    desc = np.zeros(len(slots), SLOT_DTYPE)
    base = int(row_base0)
    for i, sp in enumerate(slots):
        if sp.num_bins is None or sp.num_bins <= 0:
            raise ValueError("`num_bins` cannot be `None` or non-positive values.")
        if sp.combiner not in POOLED:
            raise ValueError(f"Do not support combiner = '{sp.combiner}' in a sharded encoder")
        desc[i]["row_base"] = (base, base + sp.num_bins)
        desc[i]["num_bins"] = sp.num_bins
        desc[i]["salt"] = (sp.seeds[0] & (2 ** 64 - 1), sp.seeds[1] & (2 ** 64 - 1))
        desc[i]["out_off"] = i * 2 * dim
        desc[i]["dim"] = dim
        desc[i]["combiner"] = L.COMB[sp.combiner]
        desc[i]["mask_empty"] = int(sp.mask_empty)
        base += 2 * sp.num_bins
    return desc, base


class GpuShardOps:
    """The four device stages of the sharded lookup, through librf (include/rf_api.h)."""

    def __init__(self, device="cuda"):
        L.load()
        L.require_gpu()
        self.device = torch.device(device)

    def prepare_batch(self, batch: SparseBatch) -> SparseBatch:
        return batch if batch.is_device() else batch.to(self.device)

    def upload_desc(self, desc: np.ndarray):
        return torch.from_numpy(desc.view(np.uint8).copy()).to(self.device)

    def init_shard(self, rows: int, dim: int, dtype, rank: int, nranks: int, seed: int, lo: float, hi: float):
        t = torch.empty((max(rows, 1), dim), dtype=dtype, device=self.device)
        if rows:
            L.call("rf_table_init_uniform", L.ptr(t), L.torch_dtype_code(dtype), rows, dim, rank, nranks, seed, lo, hi,
                   L.stream_ptr(None))
        return t[:rows]

    def hash_rows(self, desc, n_slots: int, batch: SparseBatch, tail: Optional[torch.Tensor] = None) -> torch.Tensor:
        """rf_hash_rows -> int64 [2 n_tok] (+ `tail` appended in the same buffer: the pad rows, without a cat)."""
        n = 2 * batch.n_tokens
        nt = 0 if tail is None else tail.numel()
        out = torch.empty(max(n + nt, 1), dtype=torch.int64, device=self.device)
        if nt:
            out[n:n + nt].copy_(tail)
        if n:
            L.call("rf_hash_rows", L.ptr(desc), n_slots, L.ptr(batch.tok_bytes), L.ptr(batch.tok_off),
                   L.ptr(batch.bag_off), batch.batch, L.ptr(out), L.stream_ptr(None))
        return out[: n + nt]

    def bucketize(self, rows: torch.Tensor, nranks: int):
        n = rows.numel()
        counts = torch.empty(nranks, dtype=torch.int32, device=self.device)
        perm = torch.empty(max(n, 1), dtype=torch.int32, device=self.device)
        inv = torch.empty(max(n, 1), dtype=torch.int32, device=self.device)
        local = torch.empty(max(n, 1), dtype=torch.int64, device=self.device)
        ws_bytes = L.load().rf_bucketize_ws_bytes(n, nranks)
        ws = torch.empty(max(int(ws_bytes), 1), dtype=torch.uint8, device=self.device)
        L.call("rf_bucketize_owner", L.ptr(rows), n, nranks, L.ptr(counts), L.ptr(perm), L.ptr(inv), L.ptr(local), L.ptr(ws),
               ws_bytes, L.stream_ptr(None))
        return counts, perm[:n], local[:n], inv[:n]

    def route(self, rows: torch.Tensor, nranks: int, table_rows: int):
        """Dedup + owner-major routing (rf_route_rows) -> (counts int32 [P], local int64 [U], row_map int32 [n])."""
        n = rows.numel()
        counts = torch.empty(nranks, dtype=torch.int32, device=self.device)
        local = torch.empty(max(n, 1), dtype=torch.int64, device=self.device)
        row_map = torch.empty(max(n, 1), dtype=torch.int32, device=self.device)
        ws_bytes = L.load().rf_route_ws_bytes(n, nranks, table_rows)
        ws = torch.empty(max(int(ws_bytes), 1), dtype=torch.uint8, device=self.device)
        L.call("rf_route_rows", L.ptr(rows), n, nranks, table_rows, L.ptr(counts), L.ptr(local), L.ptr(row_map), None,
               L.ptr(ws), ws_bytes, L.stream_ptr(None))
        return counts, local, row_map[:n]

    def route_hash_build(self, rows: torch.Tensor, nranks: int, rank: int, table_rows: int):
        """rf_route_hash_build: -> (counts int32 [P] device, state for route_hash_finish). rank >= 0: rows that
        rank owns are not routed (row_map = 0x80000000 | local, pooled in place from the shard)."""
        n = rows.numel()
        counts = torch.empty(nranks, dtype=torch.int32, device=self.device)
        row_map = torch.empty(max(n, 1), dtype=torch.int32, device=self.device)
        ws_bytes = int(L.load().rf_route_hash_ws_bytes(n, nranks, table_rows))
        ws = torch.empty(max(ws_bytes, 256), dtype=torch.uint8, device=self.device)
        L.call("rf_route_hash_build", L.ptr(rows), n, nranks, rank, table_rows, L.ptr(row_map), L.ptr(counts), L.ptr(ws),
               ws_bytes, L.stream_ptr(None))
        return counts, (n, nranks, table_rows, row_map, ws, ws_bytes)

    def route_hash_build_tokens(self, desc, n_slots: int, batch: SparseBatch, tail: torch.Tensor, nranks: int,
                                rank: int, table_rows: int):
        """rf_route_hash_build_tokens: hash_rows(batch, tail) + route_hash_build in one launch (no request list in
        HBM) -> (counts, state, n requests)."""
        n = 2 * batch.n_tokens + tail.numel()
        counts = torch.empty(nranks, dtype=torch.int32, device=self.device)
        row_map = torch.empty(max(n, 1), dtype=torch.int32, device=self.device)
        ws_bytes = int(L.load().rf_route_hash_ws_bytes(n, nranks, table_rows))
        ws = torch.empty(max(ws_bytes, 256), dtype=torch.uint8, device=self.device)
        L.call("rf_route_hash_build_tokens", L.ptr(desc), n_slots, L.ptr(batch.tok_bytes), L.ptr(batch.tok_off),
               L.ptr(batch.bag_off), batch.batch, batch.n_tokens, L.ptr(tail), tail.numel(), nranks, rank, table_rows,
               L.ptr(row_map), L.ptr(counts), L.ptr(ws), ws_bytes, L.stream_ptr(None))
        return counts, (n, nranks, table_rows, row_map, ws, ws_bytes), n

    def route_hash_finish(self, state, n_uniq: int):
        """rf_route_hash_finish -> (local int64 [n_uniq], row_map int32 [n]). n_uniq = -1 (nranks <= 64): the
        distinct total is read on the device, so this can be enqueued before the host reads the counts; local then
        has n entries, of which the first sum(counts) are the distinct rows."""
        n, nranks, table_rows, row_map, ws, ws_bytes = state
        local = torch.empty(max(n if n_uniq < 0 else n_uniq, 1), dtype=torch.int64, device=self.device)
        L.call("rf_route_hash_finish", n, nranks, table_rows, n_uniq, L.ptr(local), L.ptr(row_map), L.ptr(ws), ws_bytes,
               L.stream_ptr(None))
        return (local if n_uniq < 0 else local[:n_uniq]), row_map[:n]

    # -- owner-side partial pooling (rf_partial.hip) ---------------------------------------------------
    def pp_plan(self, desc, n_slots: int, batch: SparseBatch, rows: torch.Tensor, flags: int, nranks: int):
        """Requester: pooling entries in (unit, position) order, then owner-major (stable) ->
        (ent int32 [n][3] = (local, unit, mult) owner-major, entry counts int32 [P], segment counts int32 [P],
        seg_of int32 [n_units][P]). One host read (the entry count)."""
        B, S = batch.batch, n_slots
        n_units = 2 * B * S
        cap = max(2 * batch.n_tokens + n_units, 1)
        dev = self.device
        ent_off = torch.empty(n_units + 1, dtype=torch.int32, device=dev)
        ent_row = torch.empty(cap, dtype=torch.int64, device=dev)
        ent_unit = torch.empty(cap, dtype=torch.int32, device=dev)
        ent_mult = torch.empty(cap, dtype=torch.int32, device=dev)
        n_ent = torch.empty(1, dtype=torch.int32, device=dev)
        wsb = int(L.load().rf_pp_ws_bytes(max(n_units, cap)))
        ws = torch.empty(max(wsb, 256), dtype=torch.uint8, device=dev)
        L.call("rf_pp_plan", L.ptr(desc), S, L.ptr(batch.bag_off), L.ptr(batch.lmax), B, batch.n_tokens, L.ptr(rows),
               flags, L.ptr(ent_off), L.ptr(ent_row), L.ptr(ent_unit), L.ptr(ent_mult), L.ptr(n_ent), L.ptr(ws), wsb,
               L.stream_ptr(None))
        n = int(n_ent.item())
        counts, perm, local, _ = self.bucketize(ent_row[:n], nranks)
        perm = perm.long()
        ent = torch.stack([local.to(torch.int32), ent_unit[:n][perm], ent_mult[:n][perm]], dim=1).contiguous()
        seg_counts = torch.empty(nranks, dtype=torch.int32, device=dev)
        seg_of = torch.empty((max(n_units, 1), nranks), dtype=torch.int32, device=dev)
        L.call("rf_pp_heads", L.ptr(ent[:, 1].contiguous()), n, L.ptr(counts), nranks, L.ptr(seg_counts), L.ptr(seg_of),
               n_units, None, L.ptr(ws), wsb, L.stream_ptr(None))
        return ent, counts, seg_counts, seg_of

    def pp_owner_pool(self, desc, n_slots: int, ent: torch.Tensor, recv_counts: List[int], shard: torch.Tensor):
        """Owner: one partial per segment of the received entries -> fp32 [n_seg, D]."""
        n = ent.shape[0]
        dev = self.device
        P = len(recv_counts)
        cnt = torch.tensor(recv_counts, dtype=torch.int32).to(dev)
        seg_counts = torch.empty(P, dtype=torch.int32, device=dev)
        seg_start = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        wsb = int(L.load().rf_pp_ws_bytes(max(n, 1)))
        ws = torch.empty(max(wsb, 256), dtype=torch.uint8, device=dev)
        L.call("rf_pp_heads", L.ptr(ent[:, 1].contiguous()) if n else None, n, L.ptr(cnt), P, L.ptr(seg_counts), None, 0,
               L.ptr(seg_start), L.ptr(ws), wsb, L.stream_ptr(None))
        return seg_counts, seg_start

    def pp_owner_partials(self, desc, n_slots: int, ent, seg_start, n_seg: int, shard):
        D = shard.shape[1]
        part = torch.empty((max(n_seg, 1), D), dtype=torch.float32, device=self.device)
        L.call("rf_pp_owner_pool", L.ptr(desc), n_slots, L.ptr(ent), ent.shape[0], L.ptr(seg_start), n_seg, L.ptr(shard),
               L.torch_dtype_code(shard.dtype), shard.shape[0], D, L.ptr(part), L.stream_ptr(None))
        return part[:n_seg]

    def pp_combine(self, desc, n_slots: int, batch: SparseBatch, flags: int, nranks: int, seg_of, part, out):
        if part.numel() == 0:
            part = torch.zeros((1, out.shape[1] if out.dim() == 2 else 4), dtype=torch.float32, device=self.device)
        L.call("rf_pp_combine", L.ptr(desc), n_slots, L.ptr(batch.bag_off), L.ptr(batch.lmax), batch.batch, flags, nranks,
               L.ptr(seg_of), L.ptr(part), part.shape[1], L.ptr(out), L.torch_dtype_code(out.dtype), out.stride(0),
               L.stream_ptr(None))
        return out

    def gather(self, shard: torch.Tensor, local: torch.Tensor) -> torch.Tensor:
        n = local.numel()
        out = torch.empty((max(n, 1), shard.shape[1]), dtype=shard.dtype, device=self.device)
        if n:
            L.call("rf_gather_rows", L.ptr(local), n, L.ptr(shard), L.torch_dtype_code(shard.dtype), shard.shape[0],
                   shard.shape[1], L.ptr(out), L.stream_ptr(None))
        return out[:n]

    def pool(self, desc, n_slots: int, batch: SparseBatch, gathered: torch.Tensor, out: torch.Tensor, flags: int,
             row_map: Optional[torch.Tensor] = None, local_table: Optional[torch.Tensor] = None):
        if gathered.numel() == 0:  # every row is rank-local: any aligned buffer (never read)
            gathered = local_table if local_table is not None and local_table.numel() else \
                torch.empty((1, out.shape[1] if out.dim() == 2 else 4), dtype=out.dtype, device=self.device)
        L.call("rf_pool_rows_fwd", L.ptr(desc), n_slots, L.ptr(batch.bag_off), L.ptr(batch.lmax), batch.batch,
               batch.n_tokens, L.ptr(gathered), L.ptr(row_map), L.ptr(local_table), L.torch_dtype_code(gathered.dtype),
               gathered.shape[1], L.ptr(out), L.torch_dtype_code(out.dtype), out.stride(0), flags, L.stream_ptr(None))
        return out


    # -- training -------------------------------------------------------------
    def pool_bwd(self, desc, n_slots: int, batch: SparseBatch, row_map: torch.Tensor, gathered: torch.Tensor,
                 out: torch.Tensor, dout: torch.Tensor, flags: int, need_minmax: bool, sync: bool = True):
        """rf_pool_rows_bwd -> (rows into `gathered` [U] ascending, grads [U, D]); sync=False: the capacity-sized
        buffers and the DEVICE count (no host read: the caller folds it into its one synchronisation)."""
        lm = batch.lmax_numpy()
        n_pos = batch.batch * int(2 * np.asarray(lm, np.int64).sum())
        R = gathered.shape[0]
        cap = max(1, min(n_pos, R))
        D = gathered.shape[1]
        rows = torch.empty(cap, dtype=torch.int64, device=self.device)
        grad = torch.empty((cap, D), dtype=torch.float32, device=self.device)
        n_uniq = torch.zeros(1, dtype=torch.int32, device=self.device)
        cnt = torch.empty(dout.shape, dtype=torch.int32, device=self.device) if need_minmax else None
        wsb = int(L.load().rf_embed_bwd_ws_bytes(n_pos, n_slots, max(R, 1)))
        ws = torch.empty(max(wsb, 256), dtype=torch.uint8, device=self.device)
        L.call("rf_pool_rows_bwd", L.ptr(desc), n_slots, L.ptr(batch.bag_off), L.ptr(batch.lmax), batch.batch,
               batch.n_tokens, n_pos, L.ptr(row_map), L.ptr(gathered), R, D, L.ptr(out) if need_minmax else None,
               L.ptr(dout), dout.stride(0), flags, L.ptr(cnt), L.ptr(rows), L.ptr(grad), cap, L.ptr(n_uniq), L.ptr(ws),
               ws.numel(), L.stream_ptr(None))
        if not sync:
            return rows, grad, n_uniq
        n = int(n_uniq.item())
        if n < 0:
            raise ValueError(f"rf_pool_rows_bwd: invalid batch (error bits {-n})")
        return rows[:n], grad[:n]

    def segment_sum(self, ids: torch.Tensor, vals: torch.Tensor, id_range: int):
        """rf_segment_sum_rows -> (distinct ids ascending, per-id sums in input order)."""
        n = ids.numel()
        D = vals.shape[1]
        cap = max(1, min(n, id_range))
        uid = torch.empty(cap, dtype=torch.int64, device=self.device)
        uval = torch.empty((cap, D), dtype=torch.float32, device=self.device)
        n_uniq = torch.zeros(1, dtype=torch.int32, device=self.device)
        wsb = int(L.load().rf_segment_sum_ws_bytes(n, id_range))
        ws = torch.empty(max(wsb, 256), dtype=torch.uint8, device=self.device)
        L.call("rf_segment_sum_rows", L.ptr(ids.contiguous()), L.ptr(vals.contiguous()), n, D, id_range, L.ptr(uid),
               L.ptr(uval), cap, L.ptr(n_uniq), L.ptr(ws), ws.numel(), L.stream_ptr(None))
        return uid, uval, n_uniq, cap


class TorchDistComm:
    """Exchange over torch.distributed: RCCL on MI355X (xGMI point-to-point), gloo in the CPU tests."""

    def __init__(self, group=None):
        import torch.distributed as dist

        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)

    def exchange_counts(self, counts: torch.Tensor) -> torch.Tensor:
        recv = torch.empty_like(counts)
        self.dist.all_to_all_single(recv, counts, group=self.group)
        return recv

    def exchange(self, x: torch.Tensor, send_splits: List[int], recv_splits: List[int]) -> torch.Tensor:
        out = torch.empty((sum(recv_splits),) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        self.dist.all_to_all_single(out, x.contiguous(), output_split_sizes=recv_splits, input_split_sizes=send_splits,
                                    group=self.group)
        return out

    def exchange_async(self, x: torch.Tensor, send_splits: List[int], recv_splits: List[int]):
        """exchange() without waiting: (output, work). RCCL runs it on its own stream, ordered after the work
        already queued on the current stream; work.wait() orders the current stream after it."""
        out = torch.empty((sum(recv_splits),) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        work = self.dist.all_to_all_single(out, x.contiguous(), output_split_sizes=recv_splits,
                                           input_split_sizes=send_splits, group=self.group, async_op=True)
        return out, work

    def all_gather_rows(self, x: torch.Tensor) -> torch.Tensor:
        """Every rank's rows concatenated in rank order (row counts may differ: padded to the largest)."""
        n = torch.tensor([x.shape[0]], dtype=torch.int64, device=x.device)
        ns = [torch.zeros_like(n) for _ in range(self.world)]
        self.dist.all_gather(ns, n, group=self.group)
        ns = [int(v.item()) for v in ns]
        m = max(ns)
        xp = torch.zeros((m,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        xp[: x.shape[0]] = x
        bufs = [torch.empty_like(xp) for _ in range(self.world)]
        self.dist.all_gather(bufs, xp, group=self.group)
        return torch.cat([b[:k] for b, k in zip(bufs, ns)])

    def all_gather_ints(self, v: int) -> List[int]:
        t = torch.tensor([int(v)], dtype=torch.int64)
        if self.dist.get_backend(self.group) != "gloo":
            t = t.cuda()
        out = [torch.zeros_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t, group=self.group)
        return [int(o.item()) for o in out]


class LocalComm:
    """P = 1: the exchange is the identity (the sharded pipeline on one GPU, for weak-scaling baselines)."""

    rank, world = 0, 1

    def exchange_counts(self, counts: torch.Tensor) -> torch.Tensor:
        return counts

    def exchange(self, x: torch.Tensor, send_splits: List[int], recv_splits: List[int]) -> torch.Tensor:
        return x

    def exchange_async(self, x: torch.Tensor, send_splits: List[int], recv_splits: List[int]):
        return x, None

    def all_gather_rows(self, x: torch.Tensor) -> torch.Tensor:
        return x

    def all_gather_ints(self, v: int) -> List[int]:
        return [int(v)]


class LoopbackComm:
    """Timing stand-in for rank 0 of a P-rank job on ONE GPU (bench.py cfg4_sharded.simulated_p8): every
    exchange is a device copy of the same bytes, and what rank 0 would receive from rank k is taken to be what it
    sends to k (the requests of P symmetric ranks have the same statistics). The owner side then serves as many
    rows as it would at P, from its own shard (local ids are < the shard's rows for every rank), so route -> id
    exchange -> gather -> row exchange -> row-mapped pool run at the real sizes. The VALUES pooled for remote rows
    come from the wrong shard: timing only, never a parity path."""

    rank = 0

    def __init__(self, world: int):
        self.world = int(world)

    def exchange_counts(self, counts: torch.Tensor) -> torch.Tensor:
        return counts.clone()

    def exchange(self, x: torch.Tensor, send_splits: List[int], recv_splits: List[int]) -> torch.Tensor:
        return x.clone()

    def exchange_async(self, x: torch.Tensor, send_splits: List[int], recv_splits: List[int]):
        return x.clone(), None

    def all_gather_rows(self, x: torch.Tensor) -> torch.Tensor:
        return torch.cat([x] * self.world)

    def all_gather_ints(self, v: int) -> List[int]:
        return [int(v)] * self.world


@dataclass
class RouteState:
    counts: List[int]          # rows this rank requests from each owner
    local: torch.Tensor        # int64: local row id at its owner, owner-major (the id send buffer)
    row_map: torch.Tensor      # int32 [2*n_tok + 2*S]: logical row j arrives at row row_map[j]
    n_requests: int            # rows requested (after dedup)
    n_logical: int             # rows the pooling reads (2*n_tok + 2*S)


class ShardedFusedEncoder(torch.nn.Module):
    """One rank's view of a row-sharded fused table (same slots / output as FusedSparseEncoder)."""

    def __init__(self, slots: Sequence[SlotSpec], dim: int, rank: int, nranks: int, comm=None, ops=None,
                 table_dtype=torch.float32, out_dtype=None, seed: int = 0, mask_padding: bool = False,
                 init_range=(-0.05, 0.05), device="cuda", dedup: bool = True, route: str = "hash"):
        super().__init__()
        if not slots:
            raise ValueError("ShardedFusedEncoder needs at least one slot")
        if not (0 <= rank < nranks):
            raise ValueError(f"rank {rank} outside [0, {nranks})")
        self.slots = list(slots)
        self.dim = int(dim)
        self.rank, self.nranks = int(rank), int(nranks)
        self.comm = comm
        self.ops = ops if ops is not None else GpuShardOps(device)
        self.table_dtype = table_dtype
        self.out_dtype = out_dtype or table_dtype
        self.mask_padding = bool(mask_padding)
        self.dedup = bool(dedup)  # send each distinct row once per step
        if route not in ("hash", "radix"):
            raise ValueError(f"route must be 'hash' or 'radix', got {route!r}")
        # hash: rf_route_hash_build/finish (one atomic per distinct row, only the distinct set sorted) and the
        # forward pools the rows this rank owns in place; radix: rf_route_rows (a sort of every request)
        self.route_mode = route if self.dedup else "radix"
        self.host_desc, self.table_rows = build_slot_desc(self.slots, self.dim)
        self.out_width = 2 * self.dim * len(self.slots)
        self.desc = self.ops.upload_desc(self.host_desc)
        self.local_rows = shard_rows(self.table_rows, self.rank, self.nranks)
        self.shard = self.ops.init_shard(self.local_rows, self.dim, table_dtype, self.rank, self.nranks, int(seed),
                                         *init_range)
        # padding rows of every slot and table: the rows the empty string hashes to (pad positions gather
        # the bin of b"": bin 0 with mask_value="", the SipHash bin otherwise), computed by rf_hash_rows
        # on a one-example batch of empty tokens so the rule lives in one place.
        S = len(self.slots)
        empty = self.ops.prepare_batch(from_lists([[[b""] for _ in range(S)]]))
        self.pad_rows = self.ops.hash_rows(self.desc, S, empty)

    # -- the three local stages -------------------------------------------------------------------
    serve_hook = None  # forward_train calls serve_hook(local ids) before serving them from the shard

    def _route_device(self, batch: SparseBatch):
        req = self.ops.hash_rows(self.desc, len(self.slots), batch, tail=self.pad_rows)
        if self.dedup:
            counts, local, row_map = self.ops.route(req, self.nranks, self.table_rows)
        else:
            counts, _, local, row_map = self.ops.bucketize(req, self.nranks)
        return counts.to(torch.int64), local, row_map, req.numel()

    def _route_state(self, counts: List[int], local, row_map, n_logical: int) -> RouteState:
        if self.dedup:
            local = local[: sum(counts)]  # rf_route_rows sizes the id buffer for the undeduplicated worst case
        return RouteState(counts, local, row_map, int(local.numel()), n_logical)

    def route(self, batch: SparseBatch, local_fast: bool = False) -> RouteState:
        if self.route_mode == "hash":
            st, _ = self._route_hash(batch, local_fast, exchange=False)
            return st
        counts, local, row_map, n = self._route_device(batch)
        return self._route_state([int(c) for c in counts.cpu().tolist()], local, row_map, n)

    def _route_hash(self, batch: SparseBatch, local_fast: bool, exchange: bool):
        """hash route: build (device counts) -> [counts all-to-all] -> ONE host read of send (+ receive) counts
        -> finish. local_fast: this rank's own rows stay out of the exchange (row_map bit 31)."""
        rank = self.rank if local_fast else -1
        if hasattr(self.ops, "route_hash_build_tokens"):  # the hash fused into the insert (GpuShardOps)
            counts, state, n_req = self.ops.route_hash_build_tokens(self.desc, len(self.slots), batch, self.pad_rows,
                                                                    self.nranks, rank, self.table_rows)
        else:
            req = self.ops.hash_rows(self.desc, len(self.slots), batch, tail=self.pad_rows)
            counts, state = self.ops.route_hash_build(req, self.nranks, rank, self.table_rows)
            n_req = req.numel()
        counts = counts.to(torch.int64)
        P = counts.numel()
        recv = self.comm.exchange_counts(counts) if exchange else None
        if isinstance(self.ops, GpuShardOps) and P <= 64:
            # the counts go to pinned host memory first, then the finish (row map + send ids) is enqueued with the
            # distinct total read on the device, and the host waits only for the copies: the finish kernel runs
            # while the host turns the counts into split sizes
            pin = getattr(self, "_counts_pin", None)
            if pin is None or pin.numel() != 2 * P:
                pin = self._counts_pin = torch.empty(2 * P, dtype=torch.int64, pin_memory=True)
            pin[:P].copy_(counts, non_blocking=True)
            if recv is not None:
                pin[P:].copy_(recv.to(counts.device), non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            local, row_map = self.ops.route_hash_finish(state, -1)
            ev.synchronize()
            both = [int(c) for c in pin.tolist()]
            send, recv_l = both[:P], (both[P:] if recv is not None else None)
            local = local[: sum(send)]
        else:
            if recv is not None:
                both = [int(c) for c in torch.cat([counts, recv.to(counts.device)]).cpu().tolist()]
                send, recv_l = both[:P], both[P:]
            else:
                send, recv_l = [int(c) for c in counts.cpu().tolist()], None
            local, row_map = self.ops.route_hash_finish(state, sum(send))
        return RouteState(send, local, row_map, int(local.numel()), n_req), recv_l

    def route_exchange(self, batch: SparseBatch, local_fast: bool = False):
        """route() plus the all-to-all of the per-owner counts with ONE host synchronisation: the counts
        stay on the device for the exchange, and the send and receive counts come back together (the
        split sizes of the id and row all-to-alls are host lists). -> (RouteState, recv_counts)."""
        if self.route_mode == "hash":
            return self._route_hash(batch, local_fast, exchange=True)
        counts, local, row_map, n = self._route_device(batch)
        recv = self.comm.exchange_counts(counts)
        both = [int(c) for c in torch.cat([counts, recv.to(counts.device)]).cpu().tolist()]
        P = counts.numel()
        return self._route_state(both[:P], local, row_map, n), both[P:]

    def serve(self, local_rows: torch.Tensor) -> torch.Tensor:
        # rows beyond the shard come back NaN (rf_gather_rows), poisoning the pooled output loudly
        return self.ops.gather(self.shard, local_rows)

    def combine(self, batch: SparseBatch, st: RouteState, back: torch.Tensor, out: Optional[torch.Tensor] = None,
                local_fast: bool = False):
        if out is None:
            out = torch.empty((batch.batch, self.out_width), dtype=self.out_dtype, device=back.device)
        flags = L.FLAG_MASK_PADDING if self.mask_padding else 0
        return self.ops.pool(self.desc, len(self.slots), batch, back, out, flags, row_map=st.row_map,
                             local_table=self.shard if local_fast else None)

    @property
    def local_fast(self) -> bool:
        """The inference forward pools this rank's own rows in place (hash route only)."""
        return self.route_mode == "hash"

    def forward(self, batch: SparseBatch, out: Optional[torch.Tensor] = None):
        if self.comm is None:
            raise RuntimeError("ShardedFusedEncoder.forward needs a comm (TorchDistComm); "
                               "use simulate_sharded_forward for in-process shards")
        if batch.n_slots != len(self.slots):
            raise ValueError(f"batch has {batch.n_slots} slots, encoder {len(self.slots)}")
        batch = self.ops.prepare_batch(batch)
        lf = self.local_fast
        st, recv_counts = self.route_exchange(batch, local_fast=lf)
        wanted = self.comm.exchange(st.local, st.counts, recv_counts)        # ids other ranks want from me
        vec = self.serve(wanted)
        back = self.comm.exchange(vec, recv_counts, st.counts)               # my rows, owner-major
        return self.combine(batch, st, back, out, local_fast=lf)

    def forward_partial(self, batch: SparseBatch, out: Optional[torch.Tensor] = None):
        """The owner-side partial-pooling exchange (SURVEY §8e alternative; rf_partial.hip): each unit's positions
        go to their owners as (local row, unit, multiplicity) entries, every owner pools the positions it owns per
        unit, one fp32 partial per (unit, owner) comes back and the requester combines them in owner order. Two
        host reads (the entry total, then the exchanged entry / segment counts). Exact at P = 1 and for max / min /
        first / last at any P; sum / avg add the owners' partials in owner order (D-partial-pool-order)."""
        if self.comm is None:
            raise RuntimeError("forward_partial needs a comm")
        batch = self.ops.prepare_batch(batch)
        if out is None:
            out = torch.empty((batch.batch, self.out_width), dtype=self.out_dtype, device=self.ops.device)
        flags = L.FLAG_MASK_PADDING if self.mask_padding else 0
        S, P = len(self.slots), self.nranks
        rows = self.ops.hash_rows(self.desc, S, batch, tail=self.pad_rows)
        ent, counts, seg_counts, seg_of = self.ops.pp_plan(self.desc, S, batch, rows, flags, P)
        both = torch.stack([counts, seg_counts], dim=1).to(torch.int64)           # [P, 2]: entries, segments
        recv = self.comm.exchange_counts(both.reshape(-1)).reshape(P, 2)
        hb = [int(v) for v in torch.cat([both.reshape(-1), recv.reshape(-1).to(both.device)]).cpu().tolist()]
        send_e, send_s = hb[0:2 * P:2], hb[1:2 * P:2]
        recv_e, recv_s = hb[2 * P::2], hb[2 * P + 1::2]
        r_ent = self.comm.exchange(ent, send_e, recv_e)                          # owner side from here
        _, seg_start = self.ops.pp_owner_pool(self.desc, S, r_ent, recv_e, self.shard)
        part = self.ops.pp_owner_partials(self.desc, S, r_ent, seg_start, sum(recv_s), self.shard)
        back = self.comm.exchange(part, recv_s, send_s)                          # requester side again
        return self.ops.pp_combine(self.desc, S, batch, flags, P, seg_of, back, out)

    def forward_pipelined(self, micro: Sequence[SparseBatch], outs: Optional[Sequence[torch.Tensor]] = None):
        """forward() over micro-batches (runtime.batch.split_examples: consecutive examples, the whole batch's
        lmax) with the all-to-alls of one micro-batch overlapping the local stages of the others (SURVEY §5.8
        "Scheduling"). Enqueue order, R = route, A/B = id/row all-to-all (RCCL's stream), G = gather, P = pool:
            R0 | A0 | R1 | A1 | G0 | B0 | G1 | B1 | P0 | P1 ...
        so the compute stream runs R1 and G0 while A0 / A1 are on the wire, and G1 while B0 is. Each micro-batch
        costs one host read of its counts (the split sizes). Same outputs as forward() on each micro-batch."""
        m = len(micro)
        micro = [self.ops.prepare_batch(b) for b in micro]
        lf = self.local_fast
        st, recv, ids, vec = [None] * m, [None] * m, [None] * m, [None] * m
        for i in range(m):
            st[i], recv[i] = self.route_exchange(micro[i], local_fast=lf)
            ids[i] = self.comm.exchange_async(st[i].local, st[i].counts, recv[i])
        for i in range(m):
            wanted, work = ids[i]
            if work is not None:
                work.wait()
            vec[i] = self.comm.exchange_async(self.serve(wanted), recv[i], st[i].counts)
        res = []
        for i in range(m):
            back, work = vec[i]
            if work is not None:
                work.wait()
            res.append(self.combine(micro[i], st[i], back, None if outs is None else outs[i], local_fast=lf))
        return res


@dataclass
class TrainCtx:
    batch: SparseBatch
    st: RouteState
    wanted: torch.Tensor   # local ids the other ranks requested from this shard, rank-major
    recv_counts: List[int]
    back: torch.Tensor     # the rows this rank received (request order)
    out: torch.Tensor


def _grad_exchange_plan(enc, st: RouteState, rows: torch.Tensor):
    """Per-owner counts of the touched requested rows (rows index the owner-major request order)."""
    bounds = torch.tensor(np.cumsum(st.counts), dtype=torch.int64, device=rows.device)
    owner = torch.bucketize(rows, bounds, right=True)
    return [int(c) for c in torch.bincount(owner, minlength=enc.nranks).cpu().tolist()]


def _shard_training_methods():
    def forward_train(self, batch: SparseBatch, out: Optional[torch.Tensor] = None) -> TrainCtx:
        """forward() that keeps what the backward needs (route state, received rows, served ids)."""
        batch = self.ops.prepare_batch(batch)
        st, recv_counts = self.route_exchange(batch)
        wanted = self.comm.exchange(st.local, st.counts, recv_counts)
        if self.serve_hook is not None:  # e.g. SparseAdam(deferred=True).prepare_ids: the rows current before read
            self.serve_hook(wanted)
        back = self.comm.exchange(self.serve(wanted), recv_counts, st.counts)
        out = self.combine(batch, st, back, out)
        return TrainCtx(batch, st, wanted, recv_counts, back, out)

    def requester_grad(self, ctx: TrainCtx, dout: torch.Tensor):
        """(local ids at their owners, grads, per-owner counts) of the rows this rank touched."""
        if self.table_dtype != torch.float32:
            raise ValueError("sharded training needs an fp32 table")
        flags = L.FLAG_MASK_PADDING if self.mask_padding else 0
        mm = any(sp.combiner in ("max", "min") for sp in self.slots)
        rows, grad = self.ops.pool_bwd(self.desc, len(self.slots), ctx.batch, ctx.st.row_map, ctx.back, ctx.out,
                                       dout.float().contiguous(), flags, mm)
        return ctx.st.local[rows], grad, _grad_exchange_plan(self, ctx.st, rows)

    def owner_grad(self, ids: torch.Tensor, grads: torch.Tensor):
        """Sum the gradients other ranks sent for this shard's rows (rank order) -> SparseGrad."""
        from .sparse_encoder import SparseGrad

        uid, uval, n_uniq, cap = self.ops.segment_sum(ids, grads, max(self.local_rows, 1))
        return SparseGrad(uid, uval, n_uniq, cap)

    def backward(self, ctx: TrainCtx, dout: torch.Tensor):
        """Reverse all-to-all of row gradients; returns the SparseGrad of the local shard (feed SparseAdam(shard)).
        ONE host synchronisation: the requester's distinct-row count and its per-owner counts are computed on the
        device, the counts exchanged there, and all three read back together."""
        if not isinstance(self.ops, GpuShardOps):
            ids, grad, send = self.requester_grad(ctx, dout)
            recv = [int(c) for c in self.comm.exchange_counts(torch.tensor(send, dtype=torch.int64, device=ids.device)).cpu().tolist()]
            return self.owner_grad(self.comm.exchange(ids, send, recv), self.comm.exchange(grad, send, recv))
        if self.table_dtype != torch.float32:
            raise ValueError("sharded training needs an fp32 table")
        flags = L.FLAG_MASK_PADDING if self.mask_padding else 0
        mm = any(sp.combiner in ("max", "min") for sp in self.slots)
        rows, grad, n_dev = self.ops.pool_bwd(self.desc, len(self.slots), ctx.batch, ctx.st.row_map, ctx.back, ctx.out,
                                             dout.float().contiguous(), flags, mm, sync=False)
        P = self.nranks
        dev = rows.device
        bounds = torch.tensor(np.cumsum(ctx.st.counts), dtype=torch.int64).to(dev, non_blocking=True)
        owner = torch.bucketize(rows, bounds, right=True).clamp_(max=P - 1)
        valid = (torch.arange(rows.numel(), device=dev) < n_dev.to(torch.int64)).to(torch.int64)
        send_dev = torch.zeros(P, dtype=torch.int64, device=dev).scatter_add_(0, owner, valid)
        recv_dev = self.comm.exchange_counts(send_dev)
        both = [int(v) for v in torch.cat([n_dev.to(torch.int64), send_dev, recv_dev.to(dev)]).cpu().tolist()]
        n, send, recv = both[0], both[1:1 + P], both[1 + P:]
        if n < 0:
            raise ValueError(f"rf_pool_rows_bwd: invalid batch (error bits {-n})")
        ids = ctx.st.local[rows[:n]]
        return self.owner_grad(self.comm.exchange(ids, send, recv), self.comm.exchange(grad[:n], send, recv))

    return forward_train, requester_grad, owner_grad, backward


(ShardedFusedEncoder.forward_train, ShardedFusedEncoder.requester_grad, ShardedFusedEncoder.owner_grad,
 ShardedFusedEncoder.backward) = _shard_training_methods()


def simulate_sharded_backward(encoders: Sequence[ShardedFusedEncoder], batches: Sequence[SparseBatch], douts):
    """All P ranks in one process: forward, requester gradients, the reverse exchange by slicing, owner sums.
    Returns (outputs, [SparseGrad per shard])."""
    P = len(encoders)
    ctxs = []
    batches = [enc.ops.prepare_batch(b) for enc, b in zip(encoders, batches)]
    states = [enc.route(b) for enc, b in zip(encoders, batches)]
    offs = [np.concatenate([[0], np.cumsum(st.counts)]) for st in states]
    vec = []
    for o in range(P):
        wanted = torch.cat([states[r].local[offs[r][o]: offs[r][o + 1]] for r in range(P)])
        vec.append(encoders[o].serve(wanted))
    for r in range(P):
        pos = [int(sum(states[q].counts[o] for q in range(r))) for o in range(P)]
        back = torch.cat([vec[o][pos[o]: pos[o] + states[r].counts[o]] for o in range(P)])
        out = encoders[r].combine(batches[r], states[r], back)
        ctxs.append(TrainCtx(batches[r], states[r], None, None, back, out))
    sent = [encoders[r].requester_grad(ctxs[r], douts[r]) for r in range(P)]
    grads = []
    for o in range(P):
        ids, gs = [], []
        for r in range(P):
            _, _, cnt = sent[r]
            a = int(sum(cnt[:o]))
            ids.append(sent[r][0][a: a + cnt[o]])
            gs.append(sent[r][1][a: a + cnt[o]])
        grads.append(encoders[o].owner_grad(torch.cat(ids), torch.cat(gs)))
    return [c.out for c in ctxs], grads


def simulate_partial_forward(encoders: Sequence[ShardedFusedEncoder], batches: Sequence[SparseBatch]):
    """forward_partial of all P ranks in one process (the exchanges done by slicing), for parity tests."""
    P = len(encoders)
    S = len(encoders[0].slots)
    batches = [enc.ops.prepare_batch(b) for enc, b in zip(encoders, batches)]
    plans = []
    for enc, b in zip(encoders, batches):
        flags = L.FLAG_MASK_PADDING if enc.mask_padding else 0
        rows = torch.cat([enc.ops.hash_rows(enc.desc, S, b), enc.pad_rows])
        ent, counts, seg_counts, seg_of = enc.ops.pp_plan(enc.desc, S, b, rows, flags, P)
        plans.append((ent, [int(c) for c in counts.cpu().tolist()], [int(c) for c in seg_counts.cpu().tolist()], seg_of))
    e_off = [np.concatenate([[0], np.cumsum(p[1])]) for p in plans]
    s_off = [np.concatenate([[0], np.cumsum(p[2])]) for p in plans]
    parts = []
    for o, enc in enumerate(encoders):
        r_ent = torch.cat([plans[r][0][e_off[r][o]: e_off[r][o + 1]] for r in range(P)])
        recv_e = [plans[r][1][o] for r in range(P)]
        _, seg_start = enc.ops.pp_owner_pool(enc.desc, S, r_ent, recv_e, enc.shard)
        parts.append(enc.ops.pp_owner_partials(enc.desc, S, r_ent, seg_start, sum(plans[r][2][o] for r in range(P)),
                                               enc.shard))
    outs = []
    for r, enc in enumerate(encoders):
        flags = L.FLAG_MASK_PADDING if enc.mask_padding else 0
        back = []
        for o in range(P):
            pos = sum(plans[q][2][o] for q in range(r))
            back.append(parts[o][pos: pos + plans[r][2][o]])
        out = torch.empty((batches[r].batch, enc.out_width), dtype=enc.out_dtype, device=enc.ops.device)
        outs.append(enc.ops.pp_combine(enc.desc, S, batches[r], flags, P, plans[r][3], torch.cat(back), out))
    return outs


def simulate_sharded_forward(encoders: Sequence[ShardedFusedEncoder], batches: Sequence[SparseBatch],
                             local_fast: bool = False):
    """All P ranks in one process (no collective): the exchange done by slicing, for parity tests.
    local_fast: each rank pools its own rows in place (hash route), as forward() does."""
    P = len(encoders)
    batches = [enc.ops.prepare_batch(b) for enc, b in zip(encoders, batches)]
    states = [enc.route(b, local_fast=local_fast) for enc, b in zip(encoders, batches)]
    offs = [np.concatenate([[0], np.cumsum(st.counts)]) for st in states]
    vec = []
    for o in range(P):
        wanted = torch.cat([states[r].local[offs[r][o]: offs[r][o + 1]] for r in range(P)])
        vec.append(encoders[o].serve(wanted))
    outs = []
    for r in range(P):
        pos = [int(sum(states[q].counts[o] for q in range(r))) for o in range(P)]
        back = torch.cat([vec[o][pos[o]: pos[o] + states[r].counts[o]] for o in range(P)])
        outs.append(encoders[r].combine(batches[r], states[r], back, local_fast=local_fast))
    return outs
