"""TFRecord(GZIP) -> batched-CSR feature pipe, host side (include/rf_io.h through ctypes).

Reference surface mirrored here:
  * build_feature_description(conf)      backend/core/dataloader.py:23-44
  * get_label_dict(example, label_names) dataloader.py:47-57
  * TFRecordDataset(paths, compression_type, num_parallel_reads=thread_num).batch(B)
    .map(parse_example)                  dataloader.py:541-578  -> TFRecordReader / FeaturePipe
  * tf.io.TFRecordWriter(path, "GZIP")   utils/make_tfrecord.py:142 -> TFRecordWriter

Decoding happens in librf.so's C++ reader (per-file inflate threads + a parse pool), straight into
pinned host buffers; FeaturePipe then streams each batch to HBM on a side HIP stream while the
model works on the previous one. Bytes features come out as the SparseBatch the fused sparse
encoder consumes; no padding is materialised (the padded width is the batch max `lmax`, as
parse_example's FixedLenSequenceFeature pads to, dataloader.py:32-33).
"""
from __future__ import annotations

import ctypes
import queue
import threading
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import lib as L
from .batch import SparseBatch

BYTES, INT64, FLOAT = 0, 1, 2
SEQ, SCALAR = 0, 1
NONE, GZIP = 0, 1
RF_EDATA, RF_ENOSPC, RF_EIO = -4, -5, -6
_KIND_OF_TYPE = {"str": BYTES, "int": INT64, "float": FLOAT}


@dataclass(frozen=True)
class FeatureSpec:
    """One entry of the feature description (tf.io.FixedLen[Sequence]Feature)."""
    name: str
    kind: int  # BYTES / INT64 / FLOAT
    shape: int  # SEQ (FixedLenSequenceFeature, allow_missing) / SCALAR (FixedLenFeature(()))
    default: object = None


def build_feature_description(conf) -> List[FeatureSpec]:
    """dataloader.py:23-44: numeric/null/image/embedding/bert_encode -> FixedLenFeature (one value,
    default when missing); discrete/hashing/lookup/token_id -> FixedLenSequenceFeature (list,
    missing -> empty). Order = conf.train_features."""
    from ..config_parser.config_proto import DEFAULT_MAP, FeatureDeal

    out = []
    for f in conf.train_features:
        kind = _KIND_OF_TYPE[f.type]
        if f.deal in (FeatureDeal.Discrete, FeatureDeal.Hashing, FeatureDeal.Lookup):
            out.append(FeatureSpec(f.name, kind, SEQ, DEFAULT_MAP[f.type]))
        elif f.deal == FeatureDeal.TokenId:
            out.append(FeatureSpec(f.name, INT64, SEQ, 0))
        elif f.deal == FeatureDeal.BertEncode:
            out.append(FeatureSpec(f.name, BYTES, SCALAR, ""))
        elif f.deal in (FeatureDeal.Numeric, FeatureDeal.Null, FeatureDeal.Image, FeatureDeal.Embedding):
            out.append(FeatureSpec(f.name, kind, SCALAR, DEFAULT_MAP[f.type]))
        else:
            raise Exception(f"Unregister Feature: {f.name}")
    return out


# ---- ctypes mirror of rf_io.h -------------------------------------------------------------------
class _Feat(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("kind", ctypes.c_int32), ("shape", ctypes.c_int32),
                ("default_i", ctypes.c_int64), ("default_f", ctypes.c_double)]


class _Cols(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("tok_bytes", "tok_off", "bag_off", "lmax", "ival", "ibag_off", "ilmax",
                                               "fval", "fbag_off", "flmax", "iscalar", "fscalar")] + \
               [(n, ctypes.c_int64) for n in ("tok_bytes_cap", "tok_cap", "ival_cap", "fval_cap",
                                              "n_tok_bytes", "n_tok", "n_ival", "n_fval")] + \
               [("batch", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class _DevStats(ctypes.Structure):
    _fields_ = [("n_tok_bytes", ctypes.c_int64), ("n_tok", ctypes.c_int64), ("n_ival", ctypes.c_int64),
                ("n_fval", ctypes.c_int64), ("err_b", ctypes.c_int32), ("err_type", ctypes.c_int32),
                ("err_feat", ctypes.c_int32), ("err_kind", ctypes.c_int32), ("err_count", ctypes.c_int64),
                ("reserved", ctypes.c_int64)]


_vp, _i32, _i64, _sz = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t
IO_SIGS = {
    "rf_crc32c": (ctypes.c_uint32, [ctypes.c_uint32, _vp, _sz]),
    "rf_crc32c_masked": (ctypes.c_uint32, [_vp, _sz]),
    "rf_tfw_open": (ctypes.c_int, [ctypes.c_char_p, _i32, _i32, ctypes.POINTER(_vp)]),
    "rf_tfw_write": (ctypes.c_int, [_vp, _vp, _i64]),
    "rf_tfw_close": (ctypes.c_int, [_vp]),
    "rf_tfr_encode_examples": (ctypes.c_int, [ctypes.POINTER(_Feat), _i32, ctypes.POINTER(_Cols), _vp, _i64,
                                              _vp, ctypes.POINTER(_i64)]),
    "rf_tfr_open": (ctypes.c_int, [ctypes.POINTER(ctypes.c_char_p), _i32, _i32, _i32, ctypes.POINTER(_vp)]),
    "rf_tfr_next_batch": (ctypes.c_int, [_vp, ctypes.POINTER(_Feat), _i32, _i32, ctypes.POINTER(_Cols)]),
    "rf_tfr_records_read": (_i64, [_vp]),
    "rf_tfr_close": (ctypes.c_int, [_vp]),
    "rf_tfr_next_records": (ctypes.c_int, [_vp, _i32, _vp, _i64, _vp, ctypes.POINTER(_i32), ctypes.POINTER(_i64)]),
    "rf_tfr_schema_blob": (ctypes.c_int, [ctypes.POINTER(_Feat), _i32, _vp, _i64, ctypes.POINTER(_i64)]),
    "rf_tfr_device_workspace_bytes": (_i64, [_vp, _i32]),
    "rf_tfr_parse_device": (ctypes.c_int, [_vp, _vp, _vp, _vp, _i32, _i64, _i64, ctypes.POINTER(_Cols), _vp, _vp, _i64,
                                           _vp]),
    "rf_tfr_device_check": (ctypes.c_int, [_vp, ctypes.POINTER(_Feat), _i32, _i64]),
}
_io_lock = threading.Lock()
_io_bound = False


def _lib():
    global _io_bound
    lib = L.load()
    if not _io_bound:
        with _io_lock:
            for name, (res, args) in IO_SIGS.items():
                fn = getattr(lib, name)
                fn.restype, fn.argtypes = res, args
            _io_bound = True
    return lib


class DataLossError(RuntimeError):
    """Corrupt / truncated record or malformed Example (TF: tf.errors.DataLossError)."""


def _check(rc: int, what: str):
    if rc == L.RF_OK:
        return
    msg = _lib().rf_last_error().decode(errors="replace")
    if rc == RF_EDATA:
        raise DataLossError(f"{what}: {msg}")
    if rc == RF_EIO:
        raise OSError(f"{what}: {msg}")
    if rc == L.RF_EINVAL:
        raise ValueError(f"{what}: {msg}")
    raise L.RFError(f"{what}: rc {rc}: {msg}")


def crc32c(data: bytes, crc: int = 0) -> int:
    buf = ctypes.create_string_buffer(bytes(data), len(data))
    return int(_lib().rf_crc32c(crc, buf, len(data)))


def masked_crc32c(data: bytes) -> int:
    buf = ctypes.create_string_buffer(bytes(data), len(data))
    return int(_lib().rf_crc32c_masked(buf, len(data)))


def _compression(c) -> int:
    if c in (None, "", "NONE", NONE):
        return NONE
    if c in ("GZIP", GZIP):
        return GZIP
    raise ValueError(f"unsupported compression_type {c!r} (GZIP or none)")


def _feats_array(specs: Sequence[FeatureSpec]):
    arr = (_Feat * len(specs))()
    keep = []
    for i, s in enumerate(specs):
        nm = s.name.encode()
        keep.append(nm)
        di = int(s.default) if s.kind == INT64 and s.shape == SCALAR and s.default is not None else 0
        df = float(s.default) if s.kind == FLOAT and s.shape == SCALAR and s.default is not None else 0.0
        if s.kind == BYTES and s.shape == SCALAR and s.default not in (None, "", b""):
            raise ValueError(f"{s.name}: a bytes FixedLenFeature default must be empty")
        arr[i] = _Feat(nm, s.kind, s.shape, di, df)
    return arr, keep


def _groups(specs: Sequence[FeatureSpec]):
    g = {"bytes": [], "iseq": [], "fseq": [], "iscalar": [], "fscalar": []}
    for s in specs:
        if s.kind == BYTES:
            g["bytes"].append(s.name)
        elif s.shape == SEQ:
            g["iseq" if s.kind == INT64 else "fseq"].append(s.name)
        else:
            g["iscalar" if s.kind == INT64 else "fscalar"].append(s.name)
    return g


# ---- one parsed batch ---------------------------------------------------------------------------
@dataclass
class RaggedColumns:
    """Example-major CSR of the int64 or float list features: values, bag_off[B*S+1], lmax[S]."""
    values: object
    bag_off: object
    lmax: object
    names: List[str]

    def dense(self, name: str, default=0):
        """Padded [B, Lmax] array — what parse_example returns for the feature (host)."""
        s = self.names.index(name)
        S = len(self.names)
        vals, bo, lm = (np.asarray(x.cpu()) if hasattr(x, "cpu") else np.asarray(x)
                        for x in (self.values, self.bag_off, self.lmax))
        B = (len(bo) - 1) // S if S else 0
        out = np.full((B, int(lm[s])), default, dtype=vals.dtype)
        for b in range(B):
            a, e = bo[b * S + s], bo[b * S + s + 1]
            out[b, : e - a] = vals[a:e]
        return out


@dataclass
class FeatureBatch:
    """parse_example's output for one batch, in column form (host numpy or device tensors)."""
    batch: int
    sparse: Optional[SparseBatch]  # BYTES features (hashing / lookup-str / bert / image ...)
    sparse_names: List[str]
    int_seq: Optional[RaggedColumns]
    float_seq: Optional[RaggedColumns]
    int_scalar: object  # [B, Ni]
    int_scalar_names: List[str]
    float_scalar: object  # [B, Nf]
    float_scalar_names: List[str]

    def scalar(self, name: str):
        if name in self.float_scalar_names:
            return self.float_scalar[:, self.float_scalar_names.index(name)]
        if name in self.int_scalar_names:
            return self.int_scalar[:, self.int_scalar_names.index(name)]
        raise KeyError(name)

    def labels(self, label_names: Sequence) -> Dict[str, object]:
        """get_label_dict (dataloader.py:47-57)."""
        return {getattr(f, "name", f): self.scalar(getattr(f, "name", f)) for f in label_names}

    def tokens(self, name: str) -> List[List[bytes]]:
        """Per-example token lists of a bytes feature (host; for tests and debugging)."""
        sb = self.sparse.numpy()
        s = self.sparse_names.index(name)
        S = len(self.sparse_names)
        out = []
        for b in range(self.batch):
            a, e = int(sb.bag_off[b * S + s]), int(sb.bag_off[b * S + s + 1])
            out.append([bytes(sb.tok_bytes[sb.tok_off[t]:sb.tok_off[t + 1]]) for t in range(a, e)])
        return out


class _HostColumns:
    """Capacity-sized host buffers (numpy, or pinned torch tensors) for one batch."""

    def __init__(self, groups, batch: int, caps: Dict[str, int], pinned: bool):
        self.g, self.B, self.pinned = groups, batch, pinned
        self.caps = dict(caps)
        Sb, Si, Sf = len(groups["bytes"]), len(groups["iseq"]), len(groups["fseq"])
        Ni, Nf = len(groups["iscalar"]), len(groups["fscalar"])
        a = self._alloc
        self.bufs = {
            "tok_bytes": a(max(caps["tok_bytes"], 16), np.uint8), "tok_off": a(caps["tok"] + 1, np.int32),
            "bag_off": a(batch * Sb + 1, np.int32), "lmax": a(max(Sb, 1), np.int32),
            "ival": a(max(caps["ival"], 1), np.int64), "ibag_off": a(batch * Si + 1, np.int32), "ilmax": a(max(Si, 1), np.int32),
            "fval": a(max(caps["fval"], 1), np.float32), "fbag_off": a(batch * Sf + 1, np.int32), "flmax": a(max(Sf, 1), np.int32),
            "iscalar": a(max(batch * Ni, 1), np.int64), "fscalar": a(max(batch * Nf, 1), np.float32),
        }

    def _alloc(self, n, dt):
        if not self.pinned:
            return np.empty(int(n), dt)
        import torch
        tdt = {np.uint8: torch.uint8, np.int32: torch.int32, np.int64: torch.int64, np.float32: torch.float32}[dt]
        return torch.empty(int(n), dtype=tdt, pin_memory=True)

    @staticmethod
    def _addr(x):
        return int(x.data_ptr()) if hasattr(x, "data_ptr") else int(x.ctypes.data)

    def struct(self) -> _Cols:
        c = _Cols()
        for k, v in self.bufs.items():
            setattr(c, k, self._addr(v))
        c.tok_bytes_cap, c.tok_cap = self.caps["tok_bytes"], self.caps["tok"]
        c.ival_cap, c.fval_cap = self.caps["ival"], self.caps["fval"]
        return c

    def views(self, c: _Cols) -> Dict[str, object]:
        B = c.batch
        Sb, Si, Sf = len(self.g["bytes"]), len(self.g["iseq"]), len(self.g["fseq"])
        Ni, Nf = len(self.g["iscalar"]), len(self.g["fscalar"])
        b = self.bufs
        return {
            "tok_bytes": b["tok_bytes"][: c.n_tok_bytes], "tok_off": b["tok_off"][: c.n_tok + 1],
            "bag_off": b["bag_off"][: B * Sb + 1], "lmax": b["lmax"][:Sb],
            "ival": b["ival"][: c.n_ival], "ibag_off": b["ibag_off"][: B * Si + 1], "ilmax": b["ilmax"][:Si],
            "fval": b["fval"][: c.n_fval], "fbag_off": b["fbag_off"][: B * Sf + 1], "flmax": b["flmax"][:Sf],
            "iscalar": b["iscalar"][: B * Ni], "fscalar": b["fscalar"][: B * Nf],
        }


def _make_batch(groups, B: int, v: Dict[str, object]) -> FeatureBatch:
    Sb = len(groups["bytes"])
    sparse = SparseBatch(v["tok_bytes"], v["tok_off"], v["bag_off"], v["lmax"], B, Sb) if Sb else None
    iseq = RaggedColumns(v["ival"], v["ibag_off"], v["ilmax"], groups["iseq"]) if groups["iseq"] else None
    fseq = RaggedColumns(v["fval"], v["fbag_off"], v["flmax"], groups["fseq"]) if groups["fseq"] else None
    Ni, Nf = len(groups["iscalar"]), len(groups["fscalar"])
    return FeatureBatch(B, sparse, groups["bytes"], iseq, fseq, v["iscalar"].reshape(B, Ni), groups["iscalar"],
                        v["fscalar"].reshape(B, Nf), groups["fscalar"])


# ---- writer -------------------------------------------------------------------------------------
class TFRecordWriter:
    """tf.io.TFRecordWriter(path, compression) (make_tfrecord.py:142)."""

    def __init__(self, path: str, compression_type: Optional[str] = "GZIP", level: int = -1):
        h = ctypes.c_void_p()
        _check(_lib().rf_tfw_open(str(path).encode(), _compression(compression_type), level, ctypes.byref(h)),
               "rf_tfw_open")
        self._h = h

    def write(self, record: bytes):
        if self._h is None:
            raise ValueError("writer is closed")
        buf = ctypes.create_string_buffer(bytes(record), len(record))
        _check(_lib().rf_tfw_write(self._h, buf, len(record)), "rf_tfw_write")

    def write_many(self, data, rec_off):
        """Writes records data[rec_off[i]:rec_off[i+1]] (the output of encode_examples)."""
        base = data.ctypes.data
        for i in range(len(rec_off) - 1):
            _check(_lib().rf_tfw_write(self._h, base + int(rec_off[i]), int(rec_off[i + 1] - rec_off[i])),
                   "rf_tfw_write")

    def close(self):
        if self._h is not None:
            h, self._h = self._h, None
            _check(_lib().rf_tfw_close(h), "rf_tfw_close")

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def encode_examples(specs: Sequence[FeatureSpec], fb: FeatureBatch):
    """Serialises a host FeatureBatch as tf.train.Example records -> (uint8 data, int64 rec_off[B+1])."""
    g = _groups(specs)
    sb = fb.sparse.numpy() if fb.sparse is not None else None
    arrays = {}

    def keep(name, arr, dt):
        a = np.ascontiguousarray(np.asarray(arr), dtype=dt)
        arrays[name] = a
        return a.ctypes.data

    c = _Cols()
    if g["bytes"]:
        c.tok_bytes = keep("tb", sb.tok_bytes if len(sb.tok_bytes) else np.zeros(1, np.uint8), np.uint8)
        c.tok_off = keep("to", sb.tok_off, np.int32)
        c.bag_off = keep("bo", sb.bag_off, np.int32)
    if g["iseq"]:
        c.ival = keep("iv", fb.int_seq.values if len(fb.int_seq.values) else np.zeros(1, np.int64), np.int64)
        c.ibag_off = keep("ib", fb.int_seq.bag_off, np.int32)
    if g["fseq"]:
        c.fval = keep("fv", fb.float_seq.values if len(fb.float_seq.values) else np.zeros(1, np.float32), np.float32)
        c.fbag_off = keep("fb", fb.float_seq.bag_off, np.int32)
    if g["iscalar"]:
        c.iscalar = keep("is", fb.int_scalar, np.int64)
    if g["fscalar"]:
        c.fscalar = keep("fs", fb.float_scalar, np.float32)
    c.batch = fb.batch
    feats, _names = _feats_array(specs)
    rec_off = np.zeros(fb.batch + 1, np.int64)
    need = ctypes.c_int64(0)
    rc = _lib().rf_tfr_encode_examples(feats, len(specs), ctypes.byref(c), None, 0, rec_off.ctypes.data, ctypes.byref(need))
    if rc not in (L.RF_OK, RF_ENOSPC):
        _check(rc, "rf_tfr_encode_examples")
    out = np.empty(max(int(need.value), 1), np.uint8)
    _check(_lib().rf_tfr_encode_examples(feats, len(specs), ctypes.byref(c), out.ctypes.data, out.size,
                                         rec_off.ctypes.data, ctypes.byref(need)), "rf_tfr_encode_examples")
    return out[: int(need.value)], rec_off


def columns_from_rows(specs: Sequence[FeatureSpec], rows: Sequence[Dict[str, object]]) -> FeatureBatch:
    """Host FeatureBatch from per-example dicts {name: list or scalar} (missing key = empty list /
    default), e.g. to encode Examples. Bytes values may be str (UTF-8 encoded) or bytes."""
    g = _groups(specs)
    by = {s.name: s for s in specs}
    B = len(rows)

    def enc(x):
        return x.encode() if isinstance(x, str) else bytes(x)

    toks, bag = [], [0]
    for r in rows:
        for n in g["bytes"]:
            v = r.get(n, [] if by[n].shape == SEQ else [b""])
            v = [v] if isinstance(v, (str, bytes)) else list(v)
            toks.extend(enc(t) for t in v)
            bag.append(len(toks))
    tok_off = np.zeros(len(toks) + 1, np.int32)
    np.cumsum([len(t) for t in toks], out=tok_off[1:]) if toks else None
    tb = np.frombuffer(b"".join(toks), np.uint8).copy() if toks else np.zeros(0, np.uint8)
    Sb = len(g["bytes"])
    lmax = np.array([max([bag[b * Sb + s + 1] - bag[b * Sb + s] for b in range(B)] or [0]) for s in range(Sb)], np.int32)
    sparse = SparseBatch(tb, tok_off, np.array(bag, np.int32), lmax, B, Sb) if Sb else None

    def ragged(names, dt):
        if not names:
            return None
        vals, bo = [], [0]
        for r in rows:
            for n in names:
                v = r.get(n, [])
                v = [v] if np.isscalar(v) else list(v)
                vals.extend(v)
                bo.append(len(vals))
        bo = np.array(bo, np.int32)
        S = len(names)
        lm = np.array([max([bo[b * S + s + 1] - bo[b * S + s] for b in range(B)] or [0]) for s in range(S)], np.int32)
        return RaggedColumns(np.array(vals, dt), bo, lm, list(names))

    def dense(names, dt):
        return np.array([[r.get(n, by[n].default if by[n].default is not None else 0) for n in names] for r in rows],
                        dt).reshape(B, len(names))

    return FeatureBatch(B, sparse, g["bytes"], ragged(g["iseq"], np.int64), ragged(g["fseq"], np.float32),
                        dense(g["iscalar"], np.int64), g["iscalar"], dense(g["fscalar"], np.float32), g["fscalar"])


def _nbytes(x) -> int:
    return int(x.numel()) if hasattr(x, "numel") else int(x.size)


def _like(x, n: int):
    """A new uint8 host buffer of n bytes, pinned if x is a pinned torch tensor."""
    if hasattr(x, "numel"):
        import torch

        return torch.empty(n, dtype=torch.uint8, pin_memory=x.is_pinned())
    return np.empty(n, np.uint8)


# ---- reader -------------------------------------------------------------------------------------
class TFRecordReader:
    """TFRecordDataset(paths, compression_type, num_parallel_reads=thread_num).batch(B).map(parse_example)
    (dataloader.py:541-578), parsed in C++ into reusable host column buffers."""

    _DEFAULT_TOK_PER_EX, _DEFAULT_BYTES_PER_TOK = 64, 16

    def __init__(self, paths: Sequence[str], specs: Sequence[FeatureSpec], batch_size: int, thread_num: int = 4,
                 compression_type: Optional[str] = "GZIP", drop_remainder: bool = False, pinned: bool = False):
        if isinstance(paths, str):
            paths = [paths]
        if not paths:
            raise AssertionError("Paths must not be empty")
        self.specs, self.B, self.drop_remainder, self.pinned = list(specs), int(batch_size), drop_remainder, pinned
        self.groups = _groups(self.specs)
        self._feats, self._names = _feats_array(self.specs)
        arr = (ctypes.c_char_p * len(paths))(*[str(p).encode() for p in paths])
        h = ctypes.c_void_p()
        _check(_lib().rf_tfr_open(arr, len(paths), _compression(compression_type), int(thread_num), ctypes.byref(h)),
               "rf_tfr_open")
        self._h = h
        S = max(len(self.groups["bytes"]), 1)
        self.caps = {"tok": self.B * S * 4, "tok_bytes": self.B * S * 4 * self._DEFAULT_BYTES_PER_TOK,
                     "ival": self.B * max(len(self.groups["iseq"]), 1) * 16,
                     "fval": self.B * max(len(self.groups["fseq"]), 1) * 16}

    def new_columns(self) -> _HostColumns:
        return _HostColumns(self.groups, self.B, self.caps, self.pinned)

    def read_into(self, cols: _HostColumns):
        """Parses the next batch into `cols` (growing them if needed). Returns (cols, _Cols) or None at end."""
        while True:
            c = cols.struct()
            rc = _lib().rf_tfr_next_batch(self._h, self._feats, len(self.specs), self.B, ctypes.byref(c))
            if rc == RF_ENOSPC:
                grow = {"tok": c.n_tok, "tok_bytes": c.n_tok_bytes, "ival": c.n_ival, "fval": c.n_fval}
                for k, v in grow.items():
                    if v > self.caps[k]:
                        self.caps[k] = int(v * 1.25) + 64
                cols = self.new_columns()
                continue
            _check(rc, "rf_tfr_next_batch")
            if c.batch == 0 or (self.drop_remainder and c.batch < self.B):
                return None
            return cols, c

    def read_records(self, buf, rec_off):
        """Device-parse host half (rf_tfr_next_records): packs the next batch's serialized records into
        `buf` (uint8, pinned torch or numpy; replaced by a larger one when too small) with offsets in
        rec_off[:n+1]. Returns (buf, n, n_bytes); n = 0 at end of data (or a dropped remainder)."""
        n, nb = ctypes.c_int32(0), ctypes.c_int64(0)
        while True:
            rc = _lib().rf_tfr_next_records(self._h, self.B, _HostColumns._addr(buf), _nbytes(buf), _HostColumns._addr(rec_off),
                                            ctypes.byref(n), ctypes.byref(nb))
            if rc == RF_ENOSPC:
                buf = _like(buf, int(nb.value * 1.25) + 4096)
                continue
            _check(rc, "rf_tfr_next_records")
            if n.value == 0 or (self.drop_remainder and n.value < self.B):
                return buf, 0, 0
            return buf, int(n.value), int(nb.value)

    def __iter__(self):
        cols = self.new_columns()
        while True:
            r = self.read_into(cols)
            if r is None:
                return
            cols, c = r
            v = {k: (x.numpy() if hasattr(x, "numpy") else x).copy() for k, x in cols.views(c).items()}
            yield _make_batch(self.groups, c.batch, v)

    @property
    def records_read(self) -> int:
        return int(_lib().rf_tfr_records_read(self._h))

    def close(self):
        if getattr(self, "_h", None) is not None:
            h, self._h = self._h, None
            _check(_lib().rf_tfr_close(h), "rf_tfr_close")

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceParser:
    """parse_example on the GPU (rf_tfr_parse_device): serialized records in HBM -> the same columns
    TFRecordReader's C++ parse produces, as device tensors. The schema is compiled once into a device
    blob (rf_tfr_schema_blob)."""

    def __init__(self, specs: Sequence[FeatureSpec], device):
        import torch

        self.specs, self.device = list(specs), torch.device(device)
        self.groups = _groups(self.specs)
        self._feats, self._names = _feats_array(self.specs)
        need = ctypes.c_int64(0)
        rc = _lib().rf_tfr_schema_blob(self._feats, len(self.specs), None, 0, ctypes.byref(need))
        if rc not in (L.RF_OK, RF_ENOSPC):
            _check(rc, "rf_tfr_schema_blob")
        self.blob_host = np.zeros(int(need.value), np.uint8)
        _check(_lib().rf_tfr_schema_blob(self._feats, len(self.specs), self.blob_host.ctypes.data, self.blob_host.size,
                                         ctypes.byref(need)), "rf_tfr_schema_blob")
        self.blob_dev = torch.from_numpy(self.blob_host).to(self.device)
        self.Sb, self.Si, self.Sf = len(self.groups["bytes"]), len(self.groups["iseq"]), len(self.groups["fseq"])
        self.Ni, self.Nf = len(self.groups["iscalar"]), len(self.groups["fscalar"])
        # one small block read back per batch: stats (64 B = 16 int32) | lmax | ilmax | flmax
        self.small_len = 16 + self.Sb + self.Si + self.Sf

    def parse(self, rec, rec_off, B: int, n_bytes: int, max_rec: int, stream):
        """Enqueues the parse of B records (rec: device uint8 with >= 16 bytes of slack past n_bytes;
        rec_off: device int64 [B+1]) on `stream`. Returns (device column buffers, small), `small` the
        device int32 block holding the stats and lmax arrays."""
        import torch

        dev = self.device
        Sb, Si, Sf = self.Sb, self.Si, self.Sf
        small = torch.empty(self.small_len, dtype=torch.int32, device=dev)
        lm = small[16:]

        def buf(n, dt, need):
            return torch.empty(max(int(n), 1), dtype=dt, device=dev) if need else None

        tok_cap = n_bytes // 2 + B * Sb
        b = {"tok_bytes": buf(n_bytes + 16, torch.uint8, Sb), "tok_off": buf(tok_cap + 1, torch.int32, Sb),
             "bag_off": buf(B * Sb + 1, torch.int32, Sb), "lmax": lm[:Sb] if Sb else None,
             "ival": buf(n_bytes, torch.int64, Si), "ibag_off": buf(B * Si + 1, torch.int32, Si),
             "ilmax": lm[Sb:Sb + Si] if Si else None,
             "fval": buf(n_bytes // 4 + 1, torch.float32, Sf), "fbag_off": buf(B * Sf + 1, torch.int32, Sf),
             "flmax": lm[Sb + Si:] if Sf else None,
             "iscalar": buf(B * self.Ni, torch.int64, self.Ni), "fscalar": buf(B * self.Nf, torch.float32, self.Nf)}
        c = _Cols()
        for k, v in b.items():
            setattr(c, k, int(v.data_ptr()) if v is not None else None)
        c.tok_bytes_cap, c.tok_cap = n_bytes + 16, tok_cap
        c.ival_cap, c.fval_cap = n_bytes, n_bytes // 4 + 1
        ws_n = int(_lib().rf_tfr_device_workspace_bytes(self.blob_host.ctypes.data, B))
        ws = torch.empty(max(ws_n, 1), dtype=torch.uint8, device=dev)
        _check(_lib().rf_tfr_parse_device(self.blob_dev.data_ptr(), self.blob_host.ctypes.data, rec.data_ptr(),
                                          rec_off.data_ptr(), B, n_bytes, max_rec, ctypes.byref(c), small.data_ptr(),
                                          ws.data_ptr(), ws_n, stream.cuda_stream), "rf_tfr_parse_device")
        b["_ws"] = ws
        return b, small

    def check(self, small_host, first_record: int) -> _DevStats:
        """Raises DataLossError with the host reader's message if the batch failed; else the stats."""
        st = _DevStats.from_buffer_copy(np.ascontiguousarray(small_host[:16]).tobytes())
        _check(_lib().rf_tfr_device_check(ctypes.addressof(st), self._feats, len(self.specs), int(first_record)),
               "rf_tfr_next_batch")
        return st

    def views(self, b, st: _DevStats, B: int):
        """Columns trimmed to the batch's counts (the rf_tfr_columns views TFRecordReader hands out)."""
        Sb, Si, Sf, Ni, Nf = self.Sb, self.Si, self.Sf, self.Ni, self.Nf
        v = {}
        if Sb:
            v["tok_bytes"] = b["tok_bytes"][: st.n_tok_bytes] if st.n_tok_bytes else b["tok_bytes"][:16]
            v["tok_off"], v["bag_off"], v["lmax"] = b["tok_off"][: st.n_tok + 1], b["bag_off"][: B * Sb + 1], b["lmax"]
        if Si:
            v["ival"], v["ibag_off"], v["ilmax"] = b["ival"][: st.n_ival], b["ibag_off"][: B * Si + 1], b["ilmax"]
        if Sf:
            v["fval"], v["fbag_off"], v["flmax"] = b["fval"][: st.n_fval], b["fbag_off"][: B * Sf + 1], b["flmax"]
        import torch

        v["iscalar"] = b["iscalar"][: B * Ni] if Ni else torch.empty(0, dtype=torch.int64, device=self.device)
        v["fscalar"] = b["fscalar"][: B * Nf] if Nf else torch.empty(0, dtype=torch.float32, device=self.device)
        return v


class FeaturePipe:
    """Batches from TFRecord files, decoded in C++ into pinned host buffers and streamed to HBM on a
    side HIP stream. Iterating yields device FeatureBatches whose tensors are safe to
    use on the consumer's current stream (it waits on the copy's event; tensors are record_stream'd).

    `prefetch` pinned buffer sets rotate: the decoder thread fills set i+1 while the H2D copy of set
    i runs and the model consumes batch i-1.

    parse="device": the host only frames and packs the serialized records (rf_tfr_next_records); they
    are streamed to HBM as they are and parsed there (DeviceParser), so the host's per-example
    protobuf work leaves the critical path. Same batches, same bytes, same errors.
    """

    _END = object()

    def __init__(self, paths, specs, batch_size: int, thread_num: int = 8, compression_type="GZIP",
                 drop_remainder: bool = False, prefetch: int = 3, device=None, parse: str = "host"):
        import torch

        L.require_gpu()
        if parse not in ("host", "device"):
            raise ValueError(f"parse must be 'host' or 'device', got {parse!r}")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.reader = TFRecordReader(paths, specs, batch_size, thread_num, compression_type, drop_remainder, pinned=True)
        self.groups = self.reader.groups
        self.parse = parse
        self.parser = DeviceParser(specs, self.device) if parse == "device" else None
        self.stream = torch.cuda.Stream(device=self.device)
        self._free: "queue.Queue" = queue.Queue()
        for _ in range(max(1, prefetch)):
            self._free.put(None)  # lazily allocated pinned sets
        self._ready: "queue.Queue" = queue.Queue(maxsize=max(1, prefetch))
        self._stop = False
        self._err: Optional[BaseException] = None
        self._th = threading.Thread(target=self._produce_device if parse == "device" else self._produce, daemon=True)
        self._th.start()

    def _produce(self):
        import torch

        try:
            torch.cuda.set_device(self.device)
            while not self._stop:
                slot = self._free.get()
                if slot is not None:
                    cols, ev = slot
                    ev.synchronize()  # the previous H2D copy out of this pinned set has finished
                else:
                    cols = self.reader.new_columns()
                r = self.reader.read_into(cols)
                if r is None:
                    break
                cols, c = r
                host = cols.views(c)
                if c.n_tok_bytes == 0:  # never hand a zero-sized (NULL) byte buffer to a kernel
                    host["tok_bytes"] = cols.bufs["tok_bytes"][:16]
                with torch.cuda.stream(self.stream):
                    dev = {k: v.to(self.device, non_blocking=True) for k, v in host.items()}
                    ev = torch.cuda.Event()
                    ev.record(self.stream)
                dev["_host_lmax"] = np.array(host["lmax"].numpy(), np.int32)
                self._ready.put(("host", dev, c.batch, ev, cols))
        except BaseException as e:  # surfaced to the consumer
            self._err = e
        self._ready.put(self._END)

    def _produce_device(self):
        """Frames + packs records into a pinned set, streams them to HBM and enqueues the device parse
        and the read-back of its stats, all on the side stream; the consumer waits on the event."""
        import torch

        P, B = self.parser, self.reader.B
        try:
            torch.cuda.set_device(self.device)
            while not self._stop:
                slot = self._free.get()
                if slot is not None:
                    slot["ev"].synchronize()  # the H2D copies out of (and stats into) this set are done
                else:
                    slot = {"rec": torch.empty(B * 4096, dtype=torch.uint8, pin_memory=True),
                            "off": torch.empty(B + 1, dtype=torch.int64, pin_memory=True),
                            "small": torch.empty(P.small_len, dtype=torch.int32, pin_memory=True)}
                slot["rec"], n, nb = self.reader.read_records(slot["rec"], slot["off"])
                if n == 0:
                    break
                first = self.reader.records_read - n
                off = slot["off"][: n + 1]
                max_rec = int(np.diff(off.numpy()).max())
                with torch.cuda.stream(self.stream):
                    rec = torch.empty(nb + 64, dtype=torch.uint8, device=self.device)
                    rec[:nb].copy_(slot["rec"][:nb], non_blocking=True)
                    off_d = off.to(self.device, non_blocking=True)
                    bufs, small = P.parse(rec, off_d, n, nb, max_rec, self.stream)
                    slot["small"].copy_(small, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(self.stream)
                slot["ev"] = ev
                self._ready.put(("device", bufs, n, ev, slot, first))
        except BaseException as e:  # surfaced to the consumer
            self._err = e
        self._ready.put(self._END)

    def __iter__(self):
        import torch

        while True:
            item = self._ready.get()
            if item is self._END:
                if self._err is not None:
                    raise self._err
                return
            cur = torch.cuda.current_stream(self.device)
            if item[0] == "host":
                _, dev, B, ev, cols = item
                host_lmax = dev.pop("_host_lmax")
                cur.wait_event(ev)
                for t in dev.values():
                    t.record_stream(cur)
                self._free.put((cols, ev))
            else:
                _, bufs, B, ev, slot, first = item
                ev.synchronize()  # parse done, stats and lmax are on the host
                small = slot["small"].numpy().copy()
                self._free.put(slot)
                st = self.parser.check(small, first)
                dev = self.parser.views(bufs, st, B)
                host_lmax = small[16:16 + self.parser.Sb].astype(np.int32)
                for t in dev.values():
                    t.record_stream(cur)
            fb = _make_batch(self.groups, B, dev)
            if fb.sparse is not None:
                fb.sparse.host_lmax = host_lmax
            yield fb

    def close(self):
        self._stop = True
        while self._th.is_alive():
            try:
                self._ready.get(timeout=0.05)
            except queue.Empty:
                pass
            if self._free.qsize() == 0:
                self._free.put(None)
        self.reader.close()
