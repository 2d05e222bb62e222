"""Batched-CSR feature layout (the input format of the fused sparse encoder) and builders.

Reference format: per hashing feature, parse_example (backend/core/dataloader.py:32-33,
77-89) yields a dense [B, Lmax] byte-string tensor padded with b"" to the BATCH max list length; the
writer stores missing values ("-1") as b"" (utils/make_tfrecord.py:36-41). The build keeps the same
information without padding bytes:

    tok_bytes  u8[]          concatenated token bytes
    tok_off    i32[Ntok+1]   byte offsets of tokens
    bag_off    i32[B*S+1]    token offsets of (example b, slot s), example-major
    lmax       i32[S]        per-slot batch max list length (= the reference's padded width)

Padding positions are implied by lmax (the kernel gathers bin 0 for them, as the reference does).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np


@dataclass
class SparseBatch:
    tok_bytes: object  # np.ndarray (host) or torch.Tensor (device)
    tok_off: object
    bag_off: object
    lmax: object
    batch: int
    n_slots: int
    host_lmax: object = None  # numpy copy of lmax kept with a device batch (n_positions of the backward)

    @property
    def n_tokens(self) -> int:
        return int(len(self.tok_off) - 1)

    def is_device(self) -> bool:
        return not isinstance(self.tok_off, np.ndarray)

    def numpy(self) -> "SparseBatch":
        if not self.is_device():
            return self
        return SparseBatch(self.tok_bytes.cpu().numpy(), self.tok_off.cpu().numpy(), self.bag_off.cpu().numpy(),
                           self.lmax.cpu().numpy(), self.batch, self.n_slots)

    def to(self, device="cuda", non_blocking: bool = False, pin: bool = False) -> "SparseBatch":
        import torch

        def cv(a):
            t = torch.from_numpy(np.ascontiguousarray(a)) if isinstance(a, np.ndarray) else a
            if pin and t.device.type == "cpu":
                t = t.pin_memory()
            return t.to(device, non_blocking=non_blocking)

        tb = self.tok_bytes
        if isinstance(tb, np.ndarray) and tb.size == 0:
            tb = np.zeros(16, np.uint8)  # never hand a zero-sized buffer to the kernel
        hl = self.lmax if isinstance(self.lmax, np.ndarray) else self.host_lmax
        return SparseBatch(cv(tb), cv(self.tok_off), cv(self.bag_off), cv(self.lmax), self.batch, self.n_slots,
                           None if hl is None else np.array(hl, np.int32))

    def lmax_numpy(self) -> np.ndarray:
        """lmax on the host (no device sync when the batch came from host memory)."""
        if isinstance(self.lmax, np.ndarray):
            return self.lmax
        if self.host_lmax is None:
            self.host_lmax = self.lmax.cpu().numpy()
        return self.host_lmax

    def slot(self, s: int) -> "SparseBatch":
        """Host-side single-slot view (re-based CSR) for per-feature operators."""
        h = self.numpy()
        starts = h.bag_off[s:-1:h.n_slots][: h.batch]
        ends = h.bag_off[s + 1::h.n_slots][: h.batch]
        lens = (ends - starts).astype(np.int64)
        tok_idx = np.concatenate([np.arange(a, b) for a, b in zip(starts, ends)]) if h.batch else np.zeros(0, np.int64)
        tlen = (h.tok_off[tok_idx + 1] - h.tok_off[tok_idx]).astype(np.int64)
        tok_off = np.zeros(len(tok_idx) + 1, np.int32)
        np.cumsum(tlen, out=tok_off[1:])
        tb = np.concatenate([h.tok_bytes[h.tok_off[t]:h.tok_off[t + 1]] for t in tok_idx]) if len(tok_idx) else np.zeros(0, np.uint8)
        bag = np.zeros(h.batch + 1, np.int32)
        np.cumsum(lens, out=bag[1:])
        return SparseBatch(tb.astype(np.uint8), tok_off, bag, np.array([int(h.lmax[s])], np.int32), h.batch, 1)

    def bytes_per_example(self) -> float:
        return (int(len(self.tok_bytes)) + 4 * self.n_tokens) / max(self.batch, 1)


def split_examples(batch: SparseBatch, parts: int) -> List[SparseBatch]:
    """Host CSR batch -> `parts` micro-batches of consecutive examples (re-based CSR), each keeping the WHOLE
    batch's lmax: the reference pads to the batch max (dataloader.py:32-33), so a micro-batch pools exactly as
    its examples do inside the full batch (the sharded encoder's pipelined forward)."""
    h = batch.numpy()
    S, B = h.n_slots, h.batch
    bounds = [B * i // parts for i in range(parts + 1)]
    out = []
    for b0, b1 in zip(bounds[:-1], bounds[1:]):
        t0, t1 = int(h.bag_off[b0 * S]), int(h.bag_off[b1 * S])
        c0, c1 = int(h.tok_off[t0]), int(h.tok_off[t1])
        out.append(SparseBatch(h.tok_bytes[c0:c1].copy(), (h.tok_off[t0:t1 + 1] - c0).astype(np.int32),
                               (h.bag_off[b0 * S:b1 * S + 1] - t0).astype(np.int32), np.array(h.lmax, np.int32),
                               b1 - b0, S))
    return out


def from_lists(rows: Sequence[Sequence[Sequence[bytes]]], lmax: Optional[Sequence[int]] = None) -> SparseBatch:
    """rows[b][s] = list of tokens (bytes or str) of example b, slot s."""
    B = len(rows)
    S = len(rows[0]) if B else 0
    toks: List[bytes] = []
    bag = [0]
    lm = np.zeros(S, np.int32)
    for b in range(B):
        if len(rows[b]) != S:
            raise ValueError("every example needs the same number of slots")
        for s in range(S):
            vals = [t.encode() if isinstance(t, str) else bytes(t) for t in rows[b][s]]
            toks.extend(vals)
            bag.append(len(toks))
            lm[s] = max(lm[s], len(vals))
    if lmax is not None:
        lm = np.maximum(lm, np.asarray(lmax, np.int32))
    lens = np.array([len(t) for t in toks], np.int64)
    tok_off = np.zeros(len(toks) + 1, np.int32)
    np.cumsum(lens, out=tok_off[1:])
    tb = np.frombuffer(b"".join(toks), np.uint8).copy() if toks else np.zeros(0, np.uint8)
    return SparseBatch(tb, tok_off, np.asarray(bag, np.int32), lm, B, S)


def from_dense(columns: Sequence[Sequence[Sequence[bytes]]]) -> SparseBatch:
    """Per-slot dense [B][Lmax] byte-string columns as parse_example yields them (padding b"" at the end
    of short rows). Trailing b"" are treated as padding (dropped from the CSR, restored via lmax)."""
    S = len(columns)
    B = len(columns[0]) if S else 0
    rows = [[None] * S for _ in range(B)]
    lmax = []
    for s, col in enumerate(columns):
        lmax.append(max((len(r) for r in col), default=0))
        for b, r in enumerate(col):
            r = [t.encode() if isinstance(t, str) else bytes(t) for t in r]
            while r and r[-1] == b"":
                r = r[:-1]
            rows[b][s] = r
    return from_lists(rows, lmax)


# ------------------------------------------------------------------------------------------------
# synthetic batches (BASELINE.md §2 / SURVEY §8d): token f"s{slot:03d}:{id}", id ~ Zipf(1.1) on [1, 1e6]
# ------------------------------------------------------------------------------------------------
def _zipf(rng, a: float, n: int, hi: int) -> np.ndarray:
    out = rng.zipf(a, n)
    bad = out > hi
    while bad.any():
        out[bad] = rng.zipf(a, int(bad.sum()))
        bad = out > hi
    return out.astype(np.int64)


def synthetic_batch(batch: int, multivalued: Sequence[bool], seed: int = 1234, zipf_a: float = 1.1,
                    id_max: int = 1_000_000, poisson_mean: float = 7.0, max_len: int = 64,
                    uniform: bool = False, slot_ids: Optional[Sequence[int]] = None) -> SparseBatch:
    """Deterministic synthetic CSR batch: scalar slots L=1, multi-valued L = 1 + Poisson(7) clipped to [1, 64]."""
    rng = np.random.default_rng(seed)
    S = len(multivalued)
    slot_ids = np.asarray(slot_ids if slot_ids is not None else np.arange(S), np.int64)
    mv = np.asarray(multivalued, bool)
    lens = np.ones((batch, S), np.int64)
    if mv.any():
        k = int(mv.sum())
        lens[:, mv] = np.clip(1 + rng.poisson(poisson_mean, (batch, k)), 1, max_len)
    flat = lens.reshape(-1)
    n = int(flat.sum())
    slot_of_tok = np.repeat(np.tile(slot_ids, batch), flat)
    ids = rng.integers(1, id_max + 1, n) if uniform else _zipf(rng, zipf_a, n, id_max)
    nd = np.floor(np.log10(ids)).astype(np.int64) + 1
    tlen = 5 + nd
    width = 5 + 7
    mat = np.zeros((n, width), np.uint8)
    mat[:, 0] = ord("s")
    mat[:, 1] = ord("0") + (slot_of_tok // 100) % 10
    mat[:, 2] = ord("0") + (slot_of_tok // 10) % 10
    mat[:, 3] = ord("0") + slot_of_tok % 10
    mat[:, 4] = ord(":")
    for k in range(7):
        pos = nd - 1 - k  # digit k from the right goes to column 5 + pos
        valid = pos >= 0
        digit = (ids // (10 ** k)) % 10
        rows_ = np.nonzero(valid)[0]
        mat[rows_, 5 + pos[valid]] = ord("0") + digit[valid]
    keep = np.arange(width)[None, :] < tlen[:, None]
    tok_bytes = mat[keep]
    tok_off = np.zeros(n + 1, np.int32)
    np.cumsum(tlen, out=tok_off[1:])
    bag_off = np.zeros(batch * S + 1, np.int32)
    np.cumsum(flat, out=bag_off[1:])
    lmax = lens.max(axis=0).astype(np.int32) if batch else np.zeros(S, np.int32)
    return SparseBatch(tok_bytes, tok_off, bag_off, lmax, batch, S)


def synthetic_demo_rows(n: int, seed: int = 1234, missing: float = 0.05):
    """cfg1 rows (BASELINE.json configs[0]: conf/demo_conf.yaml's working features) as per-example
    dicts for runtime.tfrecord.columns_from_rows: app_id "app{id}", id ~ Zipf(1.1) over 5,000, a `missing`
    share written as "-1" -> b"" (utils/make_tfrecord.py:40); query / app_name token ids: 8 ints ~ U[1, 21128),
    segment ids 8 ints in {0, 1}; label ~ Bernoulli(0.1); down ~ U(0, 1) float32."""
    rng = np.random.default_rng(seed)
    rows = []
    for _ in range(n):
        z = int(rng.zipf(1.1))
        while z > 5000:
            z = int(rng.zipf(1.1))
        app = "" if rng.random() < missing else f"app{z}"
        rows.append({
            "query_tok_id": rng.integers(1, 21128, 8).tolist(), "query_seg_id": rng.integers(0, 2, 8).tolist(),
            "app_name_tok_id": rng.integers(1, 21128, 8).tolist(), "app_name_seg_id": rng.integers(0, 2, 8).tolist(),
            "app_id": [app], "label": float(rng.random() < 0.1), "down": float(np.float32(rng.random())),
        })
    return rows
