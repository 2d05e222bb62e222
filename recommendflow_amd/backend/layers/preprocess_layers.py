"""Preprocessing operators with the reference's constructor signatures, as torch modules on librf.so.

Reference: backend/layers/preprocess_layers.py (TF/Keras). Inputs are the batched-CSR form of the
reference's padded [B, Lmax] byte-string tensors (runtime/batch.py) — a ``SparseBatch`` with one
slot — or, for convenience, the padded dense rows themselves (list of lists), converted on the host.

Operator                 reference (file:line)          device entry point
Hashing                  keras Hashing (:89-90)         rf_siphash_bucket
EmbeddingBag             :16-76                          rf_embedding_bag_fwd
DoubleHashingEmbedding   :79-106                         rf_fused_hash_embed_fwd (one slot)
LookupEmbedding          :135-169                        rf_lookup_ids (vocab hash table) -> rf_embedding_bag_fwd
DiscreteEmbedding        :172-200                        rf_bucketize_ids -> rf_embedding_bag_fwd
BertEncode               :109-132                        out of scope (BERT), raises
"""
from __future__ import annotations

from typing import Any, List, Optional, Sequence, Union

import numpy as np
import torch

from ...config_parser.config_proto import TYPE_INT, TYPE_STR
from ...runtime import lib as L
from ...runtime.batch import SparseBatch, from_dense
from ..encoder.sparse_encoder import SLOT_DTYPE, init_table, name_seed, normalize_seeds

SUPPORT_POOLING = ["null", "sum", "min", "max", "avg", "first", "last"]


def _as_slot_batch(inputs, device) -> SparseBatch:
    if isinstance(inputs, SparseBatch):
        if inputs.n_slots != 1:
            raise ValueError("a per-feature operator takes a one-slot SparseBatch")
        return inputs if inputs.is_device() else inputs.to(device)
    # padded dense [B][Lmax] rows (the parse_example form)
    return from_dense([inputs]).to(device)


class Hashing(torch.nn.Module):
    """keras.layers.Hashing(num_bins, mask_value, salt) -> dense [B, Lmax] int64 bins.

    salt int s -> SipHash key (s, s); salt [k0, k1] -> key (k0, k1). mask_value "" -> b"" (padding)
    maps to bin 0 and other tokens to 1 + h mod (num_bins - 1). salt=None (FarmHash64) is not
    implemented (no reference call site uses it: preprocess_layers.py:89-90 always passes a seed).
    """

    def __init__(self, num_bins: int, mask_value: Optional[str] = None, salt: Union[int, Sequence[int], None] = None,
                 name: Optional[str] = None, device="cuda"):
        super().__init__()
        if num_bins is None or num_bins <= 0:
            raise ValueError("`num_bins` cannot be `None` or non-positive values.")
        if salt is None:
            raise NotImplementedError("Hashing without salt (FarmHash64) is not implemented")
        if mask_value not in (None, ""):
            raise NotImplementedError("only mask_value None or '' are supported")
        self.num_bins = int(num_bins)
        self.mask_value = mask_value
        self.key = (int(salt), int(salt)) if isinstance(salt, (int, np.integer)) else (int(salt[0]), int(salt[1]))
        self.name = name
        self.device = device

    def hash_tokens(self, batch: SparseBatch) -> torch.Tensor:
        """bins of every CSR token, int64 [Ntok]."""
        L.require_gpu()
        out = torch.empty(max(batch.n_tokens, 1), dtype=torch.int64, device=self.device)
        L.call("rf_siphash_bucket", L.ptr(batch.tok_bytes), L.ptr(batch.tok_off), batch.n_tokens,
               self.key[0] & (2 ** 64 - 1), self.key[1] & (2 ** 64 - 1), self.num_bins,
               int(self.mask_value == ""), L.ptr(out), L.stream_ptr())
        return out[: batch.n_tokens]

    def forward(self, inputs) -> torch.Tensor:
        batch = _as_slot_batch(inputs, self.device)
        flat = self.hash_tokens(batch)
        B, lmax = batch.batch, int(batch.lmax[0].item())
        # padding positions hold b"": bin 0 with mask_value "", else the bin of the empty string
        pad = 0 if self.mask_value == "" else int(self._empty_bin())
        dense = torch.full((B, lmax), pad, dtype=torch.int64, device=self.device)
        lens = (batch.bag_off[1:] - batch.bag_off[:-1]).long()
        rows = torch.repeat_interleave(torch.arange(B, device=self.device), lens)
        cols = torch.arange(batch.n_tokens, device=self.device) - torch.repeat_interleave(batch.bag_off[:-1].long(), lens)
        dense[rows, cols] = flat
        return dense

    def _empty_bin(self):
        one = SparseBatch(np.zeros(16, np.uint8), np.zeros(2, np.int32), np.array([0, 1], np.int32),
                          np.array([1], np.int32), 1, 1).to(self.device)
        return self.hash_tokens(one)[0].item()


class EmbeddingBag(torch.nn.Module):
    """Embedding(input_dim, output_dim) + combiner over axis 1 (preprocess_layers.py:16-76).

    forward(ids [B, L] int64, device) -> [B, D] ([B, L, D] for combiner "null"). Every position is
    pooled (Keras reduce_* ignores the Embedding mask, as in the reference). first/last take position
    0 / L-1 of each example (deviation D-first-last; the reference indexes the batch axis, :51,53).
    """

    def __init__(self, input_dim: int, output_dim: int, mask_zero: bool = False, combiner: str = "sum",
                 embeddings_initializer="uniform", embeddings_regularizer=None, activity_regularizer=None,
                 embeddings_constraint=None, name: Optional[str] = None, dtype=torch.float32, out_dtype=None,
                 seed: Optional[int] = None, device="cuda", table: Optional[torch.Tensor] = None, row_base: int = 0):
        super().__init__()
        self.input_dim, self.output_dim = int(input_dim), int(output_dim)
        self.mask_zero = mask_zero
        self.combiner = combiner
        self.support_pooling = list(SUPPORT_POOLING)
        self.name = name or "embedding_bag"
        self.out_dtype = out_dtype or dtype
        self.row_base = int(row_base)
        L.load()
        L.require_gpu()
        if table is None:
            if embeddings_initializer not in ("uniform", "random_uniform"):
                raise NotImplementedError("only the Keras 'uniform' initializer (U(-0.05, 0.05)) is implemented")
            table = torch.empty((self.input_dim, self.output_dim), dtype=dtype, device=device)
            init_table(table, 0, 1, name_seed(self.name) if seed is None else seed)
        self.table = table

    def forward(self, ids: torch.Tensor, stream=None) -> torch.Tensor:
        if self.combiner not in self.support_pooling:
            raise ValueError(f"Do not support combiner = '{self.combiner}', supported: [{', '.join(self.support_pooling)}]")
        ids = ids.to(device=self.table.device, dtype=torch.int64).contiguous()
        if ids.dim() == 1:
            ids = ids[:, None]
        B, Ln = ids.shape
        D = self.output_dim
        width = Ln * D if self.combiner == "null" else D
        out = torch.empty((B, width), dtype=self.out_dtype, device=self.table.device)
        L.call("rf_embedding_bag_fwd", L.ptr(ids), B, Ln, self.row_base, L.ptr(self.table),
               L.torch_dtype_code(self.table.dtype), self.table.shape[0], D, L.COMB[self.combiner], L.ptr(out),
               L.torch_dtype_code(out.dtype), out.stride(0), 0, L.stream_ptr(stream))
        return out.view(B, Ln, D) if self.combiner == "null" else out

    def get_config(self):
        return {"name": self.name, "combiner": self.combiner, "input_dim": self.input_dim, "output_dim": self.output_dim}


class DoubleHashingEmbedding(torch.nn.Module):
    """Two salted Hashing layers + two EmbeddingBags, concatenated on axis 1 (preprocess_layers.py:79-106).

    The two [num_bins, D] tables are two segments of one table (rows [base, base+N) and [base+N, base+2N));
    ``table``/``row_base`` let get_preprocess_layers place them inside a tower's fused table.
    forward(one-slot SparseBatch | padded dense rows) -> [B, 2D]  (null: [B, 2*Lmax, D]).
    """

    def __init__(self, num_bins, output_dim, seeds, combiner, mask_value=None, mask_zero=False, name="",
                 dtype=torch.float32, out_dtype=None, seed: Optional[int] = None, mask_padding: bool = False,
                 device="cuda", table: Optional[torch.Tensor] = None, row_base: int = 0):
        if num_bins is None or num_bins <= 0:
            raise ValueError("`num_bins` cannot be `None` or non-positive values.")
        super().__init__()
        if mask_value not in (None, ""):
            raise NotImplementedError("only mask_value None or '' are supported")
        self.num_bins = int(num_bins)
        self.output_dim = int(output_dim)
        self.mask_value = mask_value
        self.mask_zero = mask_zero
        self.combiner = combiner
        self.seeds = list(normalize_seeds(seeds))
        self.name = name
        self.mask_padding = mask_padding
        self.out_dtype = out_dtype or dtype
        self.row_base = int(row_base)
        L.load()
        L.require_gpu()
        if table is None:
            table = torch.empty((2 * self.num_bins, self.output_dim), dtype=dtype, device=device)
            init_table(table, 0, 1, name_seed(name) if seed is None else seed)
            self.row_base = 0
        self.table = table
        self._desc_cache = None

    def _desc(self, out_off: int):
        if self.combiner not in SUPPORT_POOLING:
            raise ValueError(f"Do not support combiner = '{self.combiner}', supported: [{', '.join(SUPPORT_POOLING)}]")
        d = np.zeros(1, SLOT_DTYPE)
        d[0]["row_base"] = (self.row_base, self.row_base + self.num_bins)
        d[0]["num_bins"] = self.num_bins
        d[0]["salt"] = (self.seeds[0] & (2 ** 64 - 1), self.seeds[1] & (2 ** 64 - 1))
        d[0]["out_off"] = out_off
        d[0]["dim"] = self.output_dim
        d[0]["combiner"] = L.COMB[self.combiner]
        d[0]["mask_empty"] = int(self.mask_value == "")
        key = (out_off, self.combiner)
        if self._desc_cache is None or self._desc_cache[0] != key:
            self._desc_cache = (key, torch.from_numpy(d.view(np.uint8).copy()).to(self.table.device))
        return self._desc_cache[1]

    def forward(self, inputs, emit_idx: bool = False, stream=None):
        batch = _as_slot_batch(inputs, self.table.device)
        B, D = batch.batch, self.output_dim
        lmax = int(batch.lmax[0].item()) if batch.is_device() else int(batch.lmax[0])
        width = 2 * lmax * D if self.combiner == "null" else 2 * D
        out = torch.empty((B, max(width, 4)), dtype=self.out_dtype, device=self.table.device)
        idx = torch.empty((max(batch.n_tokens, 1), 2), dtype=torch.int64, device=self.table.device) if emit_idx else None
        flags = (L.FLAG_MASK_PADDING if self.mask_padding else 0) | (L.FLAG_EMIT_IDX if emit_idx else 0)
        L.call("rf_fused_hash_embed_fwd", L.ptr(self._desc(0)), 1, L.ptr(batch.tok_bytes), L.ptr(batch.tok_off),
               L.ptr(batch.bag_off), L.ptr(batch.lmax), B, L.ptr(self.table), L.torch_dtype_code(self.table.dtype),
               self.table.shape[0], D, L.ptr(out), L.torch_dtype_code(out.dtype), out.stride(0), flags, L.ptr(idx),
               L.stream_ptr(stream))
        out = out[:, :width]
        if self.combiner == "null":
            out = out.reshape(B, 2 * lmax, D)
        return (out, idx[: batch.n_tokens]) if emit_idx else out

    def get_config(self):
        return {"name": self.name, "combiner": self.combiner, "seeds": self.seeds, "num_bins": self.num_bins}


VOCAB_DTYPE = np.dtype([("key", "<u8"), ("id", "<i4"), ("ref", "<i4")])  # rf_vocab_entry, 16 bytes
assert VOCAB_DTYPE.itemsize == 16


def _ragged_slot(inputs, slot: int, dtype, device):
    """(values, bag_off, n_slots, lmax) of one slot of a ragged group, on `device`. Accepts
    runtime.tfrecord.RaggedColumns (the pipe's int64/float list features) or padded dense host rows
    [B][L] (the parse_example form; every position is a value, padding included)."""
    if hasattr(inputs, "bag_off") and hasattr(inputs, "values"):
        S = len(inputs.names) if getattr(inputs, "names", None) else 1
        lm = inputs.lmax
        lmax = int(lm[slot]) if isinstance(lm, np.ndarray) else int(lm[slot].item())
        vals = inputs.values if isinstance(inputs.values, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(inputs.values))
        bo = inputs.bag_off if isinstance(inputs.bag_off, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(inputs.bag_off))
        vals = vals.to(device=device, dtype=dtype)
        if vals.numel() == 0:
            vals = torch.zeros(1, dtype=dtype, device=device)
        return vals.contiguous(), bo.to(device=device, dtype=torch.int32).contiguous(), S, lmax
    rows = [list(r) if isinstance(r, (list, tuple, np.ndarray)) else [r] for r in inputs]
    L_ = max((len(r) for r in rows), default=0)
    flat = [v for r in rows for v in r]
    bo = np.zeros(len(rows) + 1, np.int32)
    np.cumsum([len(r) for r in rows], out=bo[1:])
    np_dt = np.int64 if dtype == torch.int64 else np.float32
    vals = torch.from_numpy(np.asarray(flat if flat else [0], np_dt)).to(device)
    return vals, torch.from_numpy(bo).to(device), 1, L_


class LookupEmbedding(torch.nn.Module):
    """StringLookup / IntegerLookup + EmbeddingBag (preprocess_layers.py:135-169), index producer on the GPU
    (rf_lookup_ids over a vocabulary hash table).

    Index rule of Keras StringLookup/IntegerLookup (num_oov_indices=1, mask_token=None): vocab[i] -> i+1,
    anything else (including the padding default "" / 0) -> 0. A repeated vocabulary term raises ValueError,
    as Keras does. Deviation D-lookup: the reference calls a missing update_lookup_layer (:158) and compares a
    TF dtype with a type name (:148); its table has len(vocabs) rows for len(vocabs)+1 ids — the build sizes it
    max(vocab_size, len(vocabs)+1).

    forward(inputs, slot=0): inputs = a SparseBatch (string features; `slot` picks the feature of a
    multi-slot group), a RaggedColumns (int features from the TFRecord pipe), or padded dense host rows.
    """

    def __init__(self, embedding_dim: int, dtype: str, vocabs: List[Any], vocab_size: Optional[int] = None,
                 pooling: str = "sum", name: Optional[str] = None, device="cuda", table_dtype=torch.float32):
        super().__init__()
        if dtype not in (TYPE_STR, TYPE_INT):
            raise ValueError(f"Unsupported type for lookup feature: {dtype}")
        L.load()
        L.require_gpu()
        self.vocabulary = list(vocabs)
        self.pooling = pooling
        self.dtype_name = dtype
        self.device = torch.device(device)
        self.kind = 0 if dtype == TYPE_STR else 1  # RF_VOCAB_BYTES / RF_VOCAB_INT64
        n = len(self.vocabulary)
        cap = int(L.load().rf_vocab_capacity(n))
        tab = np.zeros(cap, VOCAB_DTYPE)
        if self.kind == 0:
            terms = [v if isinstance(v, bytes) else str(v).encode() for v in self.vocabulary]
            vb = np.frombuffer(b"".join(terms), np.uint8).copy() if terms else np.zeros(0, np.uint8)
            voff = np.zeros(n + 1, np.int32)
            np.cumsum([len(t) for t in terms], out=voff[1:])
            vbuf = vb if vb.size else np.zeros(1, np.uint8)
            L.call("rf_vocab_build", 0, vbuf.ctypes.data, voff.ctypes.data, n, tab.ctypes.data, cap)
            self.vocab_bytes = torch.from_numpy(vbuf).to(self.device)
            self.vocab_off = torch.from_numpy(voff).to(self.device)
        else:
            iv = np.asarray([int(v) for v in self.vocabulary] or [0], np.int64)
            L.call("rf_vocab_build", 1, iv.ctypes.data, None, n, tab.ctypes.data, cap)
            self.vocab_bytes = self.vocab_off = None
        self.cap = cap
        self.vocab_table = torch.from_numpy(tab.view(np.uint8).copy()).to(self.device)
        rows = max(int(vocab_size or 0), n + 1)
        self.embedding = EmbeddingBag(rows, embedding_dim, True, combiner=pooling, name=(name or "lookup") + "_embedding",
                                      dtype=table_dtype, device=device)

    def lookup_ids(self, inputs, slot: int = 0) -> torch.Tensor:
        """Padded [B, Lmax] int64 ids (the StringLookup/IntegerLookup output)."""
        st = L.stream_ptr()
        if self.kind == 0:
            sb = inputs if isinstance(inputs, SparseBatch) else from_dense([inputs])
            lmax = int(sb.lmax_numpy()[slot])
            if not sb.is_device():
                sb = sb.to(self.device)
            ids = torch.empty((sb.batch, lmax), dtype=torch.int64, device=self.device)
            L.call("rf_lookup_ids", 0, L.ptr(self.vocab_table), self.cap, L.ptr(self.vocab_bytes), L.ptr(self.vocab_off),
                   L.ptr(sb.tok_bytes), L.ptr(sb.tok_off), L.ptr(sb.bag_off), sb.n_slots, slot, sb.batch, lmax,
                   L.ptr(ids), st)
            return ids
        vals, bo, S, lmax = _ragged_slot(inputs, slot, torch.int64, self.device)
        B = (bo.numel() - 1) // S
        ids = torch.empty((B, lmax), dtype=torch.int64, device=self.device)
        L.call("rf_lookup_ids", 1, L.ptr(self.vocab_table), self.cap, None, None, L.ptr(vals), None, L.ptr(bo), S, slot, B,
               lmax, L.ptr(ids), st)
        return ids

    def lookup(self, rows) -> np.ndarray:
        """Host convenience: padded ids of host rows."""
        return self.lookup_ids(rows).cpu().numpy()

    def forward(self, inputs, slot: int = 0):
        ids = inputs if isinstance(inputs, torch.Tensor) else self.lookup_ids(inputs, slot)
        return self.embedding(ids)

    def get_vocabulary(self):
        return ["[UNK]"] + list(self.vocabulary)


class DiscreteEmbedding(torch.nn.Module):
    """Discretization(bin_boundaries) + EmbeddingBag (preprocess_layers.py:172-200), index producer on the GPU
    (rf_bucketize_ids): bin = number of boundaries <= x (tf Bucketize); padding = the float default 0.0."""

    def __init__(self, embedding_dim: int, vocabs: List[float], vocab_size: Optional[int] = None,
                 pooling: str = "sum", name: Optional[str] = None, device="cuda", table_dtype=torch.float32):
        super().__init__()
        L.load()
        L.require_gpu()
        self.vocabulary = [float(v) for v in vocabs]
        self.pooling = pooling
        self.device = torch.device(device)
        rows = max(int(vocab_size or 0), len(self.vocabulary) + 1)
        self.boundaries = torch.tensor(self.vocabulary or [0.0], dtype=torch.float32, device=self.device)
        self.embedding = EmbeddingBag(rows, embedding_dim, True, combiner=pooling,
                                      name=(name or "discrete") + "_disc_lookup_embedding", dtype=table_dtype, device=device)

    def bucket_ids(self, inputs, slot: int = 0) -> torch.Tensor:
        vals, bo, S, lmax = _ragged_slot(inputs, slot, torch.float32, self.device)
        B = (bo.numel() - 1) // S
        ids = torch.empty((B, lmax), dtype=torch.int64, device=self.device)
        L.call("rf_bucketize_ids", L.ptr(vals), L.ptr(bo), S, slot, B, lmax, L.ptr(self.boundaries), len(self.vocabulary),
               0.0, L.ptr(ids), L.stream_ptr())
        return ids

    def forward(self, inputs, slot: int = 0):
        ids = inputs if (isinstance(inputs, torch.Tensor) and inputs.dtype == torch.int64) else self.bucket_ids(inputs, slot)
        return self.embedding(ids)

    def get_vocabulary(self):
        return list(self.vocabulary)


class BertEncode(torch.nn.Module):
    """Out of scope (BERT tokenizer, preprocess_layers.py:109-132; SURVEY §2 marks backend/encoder BERT OOS)."""

    def __init__(self, dict_path: str, max_len: Optional[int] = None, name: Optional[str] = None):
        super().__init__()
        raise NotImplementedError("BertEncode is outside the accelerated hot path (SURVEY §2)")
