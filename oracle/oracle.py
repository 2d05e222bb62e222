"""CPU oracle for the RecommendFlow hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module; the product (``recommendflow_amd``) never does. It restates the reference semantics:

* integer / byte work (hash, gather, pool) in plain C: ``oracle/rf_oracle.c`` (ctypes below);
* the dense floating-point stages in float64 numpy, each function citing the reference lines it
  follows (backend/layers/attention_layers.py, layer_utils.py, backend/blocks/mlp.py,
  models/ranking/esim.py, models/matching/dssm.py).

Parity pins: see ``tests/test_oracle_kats.py`` (SipHash-2-4 reference vectors, CPython's siphash24,
TF/Keras docstring KATs) and ``tests/golden/`` (config-parser fixtures generated from the reference's
own parser, see tests/golden/make_config_golden.py). The dense stages (ESIM, MLP, SDPA) are restated
from the reference source lines cited; no reference output pins them ("parity unpinned" for those
stages).
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "librf_oracle.so")
_lib = None

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

COMB = {"sum": 0, "avg": 1, "max": 2, "min": 3, "first": 4, "last": 5, "null": 6}
DT_F32, DT_BF16 = 0, 1
FLAG_MASK_PADDING, FLAG_EMIT_IDX = 1, 2


def build(force: bool = False) -> str:
    """Compile oracle/rf_oracle.c (gcc) into oracle/build/librf_oracle.so."""
    src = os.path.join(_HERE, "rf_oracle.c")
    if force or not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE] + (["-B"] if force else []))
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        u64, i64, i32, vp = ctypes.c_uint64, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p
        L.orf_siphash24.restype = u64
        L.orf_siphash24.argtypes = [u64, u64, ctypes.c_char_p, i64]
        L.orf_hash_bucket.restype = i64
        L.orf_hash_bucket.argtypes = [u64, u64, ctypes.c_char_p, i64, i64, i32]
        L.orf_hash_tokens.restype = None
        L.orf_hash_tokens.argtypes = [vp, vp, i64, u64, u64, i64, i32, vp]
        L.orf_table_value.restype = ctypes.c_float
        L.orf_table_value.argtypes = [u64, i64, i32, i32, ctypes.c_float, ctypes.c_float]
        L.orf_table_init_uniform.restype = None
        L.orf_table_init_uniform.argtypes = [vp, i32, i64, i32, i64, i64, u64, ctypes.c_float, ctypes.c_float]
        L.orf_fused_hash_embed_fwd.restype = ctypes.c_int
        L.orf_fused_hash_embed_fwd.argtypes = [vp, i32, vp, vp, vp, vp, i32, vp, i32, i64, i32, vp, i32, i64, i32, vp, i32]
        L.orf_embedding_bag_fwd.restype = ctypes.c_int
        L.orf_embedding_bag_fwd.argtypes = [vp, i32, i32, i64, vp, i32, i64, i32, i32, vp, i32, i64, i64]
        L.orf_hash_rows.restype = None
        L.orf_hash_rows.argtypes = [vp, i32, vp, vp, vp, i32, vp]
        L.orf_pool_rows_fwd.restype = ctypes.c_int
        L.orf_pool_rows_fwd.argtypes = [vp, i32, vp, vp, i32, i64, vp, vp, i32, i32, vp, i32, i64, i32]
        L.orf_fused_hash_embed_bwd.restype = i64
        L.orf_fused_hash_embed_bwd.argtypes = [vp, i32, vp, vp, vp, vp, i32, vp, i64, i32, vp, vp, i64, i32, vp, vp]
        L.orf_pool_rows_bwd.restype = i64
        L.orf_pool_rows_bwd.argtypes = [vp, i32, vp, vp, i32, i64, vp, vp, i64, i32, vp, vp, i64, i32, vp, vp]
        L.orf_adam_apply.restype = None
        L.orf_adam_apply.argtypes = [vp, vp, vp, i64, i32, vp, vp, i64, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                     ctypes.c_float, i32]
        L.orf_bucketize_owner.restype = None
        L.orf_bucketize_owner.argtypes = [vp, i64, i32, vp, vp, vp, vp]
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


# ----------------------------------------------------------------------------------------------
# integer / byte work (C)
# ----------------------------------------------------------------------------------------------
def siphash24(k0: int, k1: int, msg: bytes) -> int:
    return lib().orf_siphash24(k0, k1, msg, len(msg))


def hash_bucket(token: bytes, num_bins: int, salt: int, mask_empty: bool = True) -> int:
    """keras.layers.Hashing(num_bins, mask_value="" if mask_empty else None, salt=salt)(token)."""
    return lib().orf_hash_bucket(salt, salt, token, len(token), num_bins, int(mask_empty))


def hash_tokens(tok_bytes: np.ndarray, tok_off: np.ndarray, k0: int, k1: int, num_bins: int, mask_empty: bool) -> np.ndarray:
    tok_bytes = np.ascontiguousarray(tok_bytes, dtype=np.uint8)
    tok_off = np.ascontiguousarray(tok_off, dtype=np.int32)
    n = len(tok_off) - 1
    out = np.empty(n, dtype=np.int64)
    lib().orf_hash_tokens(_p(tok_bytes), _p(tok_off), n, k0, k1, num_bins, int(mask_empty), _p(out))
    return out


def table_init_uniform(rows: int, dim: int, dtype: int = DT_F32, seed: int = 0, row0: int = 0, row_stride: int = 1,
                       lo: float = -0.05, hi: float = 0.05) -> np.ndarray:
    out = np.empty((rows, dim), dtype=np.float32 if dtype == DT_F32 else np.uint16)
    lib().orf_table_init_uniform(_p(out), dtype, rows, dim, row0, row_stride, seed, lo, hi)
    return out


def fused_hash_embed(slots: np.ndarray, tok_bytes: np.ndarray, tok_off: np.ndarray, bag_off: np.ndarray,
                     lmax: np.ndarray, batch: int, table: np.ndarray, dim: int, out_stride: int,
                     out_dtype: int = DT_F32, flags: int = 0, emit_idx: bool = False, n_threads: int = 0):
    """Restatement of rf_fused_hash_embed_fwd; returns (out, idx or None)."""
    slots = np.ascontiguousarray(slots, dtype=SLOT_DTYPE)
    tok_bytes = np.ascontiguousarray(tok_bytes, dtype=np.uint8)
    if tok_bytes.size == 0:
        tok_bytes = np.zeros(1, np.uint8)
    tok_off = np.ascontiguousarray(tok_off, dtype=np.int32)
    bag_off = np.ascontiguousarray(bag_off, dtype=np.int32)
    lmax = np.ascontiguousarray(lmax, dtype=np.int32)
    table = np.ascontiguousarray(table)
    tdt = DT_F32 if table.dtype == np.float32 else DT_BF16
    out = np.zeros((batch, out_stride), dtype=np.float32 if out_dtype == DT_F32 else np.uint16)
    n_tok = len(tok_off) - 1
    idx = np.zeros((max(n_tok, 1), 2), dtype=np.int64) if emit_idx else None
    if emit_idx:
        flags |= FLAG_EMIT_IDX
    rc = lib().orf_fused_hash_embed_fwd(_p(slots), len(slots), _p(tok_bytes), _p(tok_off), _p(bag_off), _p(lmax),
                                        batch, _p(table), tdt, table.shape[0], dim, _p(out), out_dtype, out_stride,
                                        flags, _p(idx) if emit_idx else None, n_threads)
    if rc != 0:
        raise RuntimeError(f"oracle fused_hash_embed failed rc={rc}")
    return out, (idx[:n_tok] if emit_idx else None)


def fused_hash_embed_bwd(slots, tok_bytes, tok_off, bag_off, lmax, batch, table, dim, out, dout, flags=0):
    """Restatement of rf_fused_hash_embed_bwd (fp32): returns (uniq_rows int64 [U], uniq_grad f32 [U, dim])."""
    slots = np.ascontiguousarray(slots, dtype=SLOT_DTYPE)
    tok_bytes = np.ascontiguousarray(tok_bytes, dtype=np.uint8)
    if tok_bytes.size == 0:
        tok_bytes = np.zeros(1, np.uint8)
    tok_off = np.ascontiguousarray(tok_off, dtype=np.int32)
    bag_off = np.ascontiguousarray(bag_off, dtype=np.int32)
    lmax = np.ascontiguousarray(lmax, dtype=np.int32)
    table = np.ascontiguousarray(table, dtype=np.float32)
    out = np.ascontiguousarray(out, dtype=np.float32)
    dout = np.ascontiguousarray(dout, dtype=np.float32)
    n_pos = int(batch) * int(2 * lmax.astype(np.int64).sum())
    cap = max(min(n_pos, table.shape[0]), 1)
    rows = np.zeros(cap, np.int64)
    grad = np.zeros((cap, dim), np.float32)
    nu = lib().orf_fused_hash_embed_bwd(_p(slots), len(slots), _p(tok_bytes), _p(tok_off), _p(bag_off), _p(lmax), batch,
                                        _p(table), table.shape[0], dim, _p(out), _p(dout), dout.shape[1], flags,
                                        _p(rows), _p(grad))
    if nu < 0:
        raise RuntimeError("oracle fused_hash_embed_bwd: row out of range")
    return rows[:nu], grad[:nu]


def pool_rows_bwd(slots, bag_off, lmax, batch, n_tok, row_map, gathered, dim, out, dout, flags=0):
    """Restatement of rf_pool_rows_bwd (the sharded requester's backward, rf_oracle.c orf_pool_rows_bwd):
    rows index `gathered`; returns (uniq_rows int64 [U], uniq_grad f32 [U, dim])."""
    slots = np.ascontiguousarray(slots, dtype=SLOT_DTYPE)
    bag_off = np.ascontiguousarray(bag_off, dtype=np.int32)
    lmax = np.ascontiguousarray(lmax, dtype=np.int32)
    row_map = np.ascontiguousarray(row_map, dtype=np.int32)
    gathered = np.ascontiguousarray(gathered, dtype=np.float32)
    out = np.ascontiguousarray(out, dtype=np.float32)
    dout = np.ascontiguousarray(dout, dtype=np.float32)
    n_pos = int(batch) * int(2 * lmax.astype(np.int64).sum())
    cap = max(min(n_pos, gathered.shape[0]), 1)
    rows = np.zeros(cap, np.int64)
    grad = np.zeros((cap, dim), np.float32)
    nu = lib().orf_pool_rows_bwd(_p(slots), len(slots), _p(bag_off), _p(lmax), batch, n_tok, _p(row_map), _p(gathered),
                                 gathered.shape[0], dim, _p(out), _p(dout), dout.shape[1], flags, _p(rows), _p(grad))
    if nu < 0:
        raise RuntimeError("oracle pool_rows_bwd: row out of range")
    return rows[:nu], grad[:nu]


def segment_sum_rows(ids, vals):
    """Restatement of rf_segment_sum_rows: distinct ids ascending, each with the fp32 sum of its rows taken
    in input order starting from +0.0 (the owner side of the sharded backward: the senders' rows arrive
    rank-major, so a row's gradient is the sum over ranks r = 0..P-1 in that order)."""
    ids = np.asarray(ids, np.int64)
    vals = np.asarray(vals, np.float32).reshape(len(ids), -1)
    order = np.argsort(ids, kind="stable")
    uid, start = np.unique(ids[order], return_index=True)
    out = np.zeros((len(uid), vals.shape[1]), np.float32)
    bounds = list(start) + [len(ids)]
    for u in range(len(uid)):
        acc = np.zeros(vals.shape[1], np.float32)
        for i in order[bounds[u]: bounds[u + 1]]:
            acc = acc + vals[i]
        out[u] = acc
    return uid, out


def adam_apply(table, m, v, uniq_rows, uniq_grad, lr, beta1, beta2, eps, lazy=False):
    """Restatement of rf_adam_apply, in place on fp32 numpy arrays."""
    for a in (table, m, v):
        assert a.dtype == np.float32 and a.flags.c_contiguous
    uniq_rows = np.ascontiguousarray(uniq_rows, dtype=np.int64)
    uniq_grad = np.ascontiguousarray(uniq_grad, dtype=np.float32)
    lib().orf_adam_apply(_p(table), _p(m), _p(v), table.shape[0], table.shape[1], _p(uniq_rows), _p(uniq_grad),
                         len(uniq_rows), lr, beta1, beta2, eps, int(lazy))


def adam_dense(w, g, m, v, lr, beta1, beta2, eps):
    """Keras Adam._resource_apply_dense (TF ResourceApplyAdam, training_ops: ApplyAdamNonCuda) in place on fp32
    numpy arrays, lr the bias-corrected step size (keras_adam_lr): m += (g - m)(1 - b1); v += (g^2 - v)(1 - b2);
    w -= m lr / (sqrt(v) + eps). numpy float32 ops round each step (no fused multiply-add), as the kernel does."""
    f = np.float32
    for a in (w, g, m, v):
        assert a.dtype == np.float32
    m += (g - m) * (f(1) - f(beta1))
    v += (g * g - v) * (f(1) - f(beta2))
    w -= (m * f(lr)) / (np.sqrt(v) + f(eps))


def keras_adam_lr(lr: float, beta1: float, beta2: float, step: int) -> float:
    """Keras Adam's bias-corrected step size in float32: lr * (sqrt(1 - b2^t) / (1 - b1^t))."""
    f = np.float32
    t = f(step)
    b1p, b2p = np.power(f(beta1), t), np.power(f(beta2), t)
    return float(f(lr) * (np.sqrt(f(1) - b2p) / (f(1) - b1p)))


def embedding_bag(ids: np.ndarray, table: np.ndarray, combiner: str, row_base: int = 0, out_dtype: int = DT_F32):
    ids = np.ascontiguousarray(ids, dtype=np.int64)
    B, L = ids.shape
    table = np.ascontiguousarray(table)
    D = table.shape[1]
    tdt = DT_F32 if table.dtype == np.float32 else DT_BF16
    width = L * D if combiner == "null" else D
    out = np.zeros((B, width), dtype=np.float32 if out_dtype == DT_F32 else np.uint16)
    rc = lib().orf_embedding_bag_fwd(_p(ids), B, L, row_base, _p(table), tdt, table.shape[0], D, COMB[combiner],
                                     _p(out), out_dtype, width, 0)
    if rc != 0:
        raise RuntimeError(f"oracle embedding_bag failed rc={rc}")
    return out


def hash_rows(slots, tok_bytes, tok_off, bag_off, batch) -> np.ndarray:
    """rf_hash_rows restated: int64 [2 * n_tok] global fused-table rows."""
    slots = np.ascontiguousarray(slots, dtype=SLOT_DTYPE)
    tok_bytes = np.ascontiguousarray(tok_bytes, dtype=np.uint8)
    if tok_bytes.size == 0:
        tok_bytes = np.zeros(1, np.uint8)
    tok_off = np.ascontiguousarray(tok_off, dtype=np.int32)
    bag_off = np.ascontiguousarray(bag_off, dtype=np.int32)
    out = np.zeros(2 * (len(tok_off) - 1), np.int64)
    lib().orf_hash_rows(_p(slots), len(slots), _p(tok_bytes), _p(tok_off), _p(bag_off), batch, _p(out))
    return out


def pool_rows(slots, bag_off, lmax, batch, n_tok, gathered, dim, out_stride, flags=0, row_map=None):
    """rf_pool_rows_fwd restated (fp32 gathered rows -> fp32 out; row_map: int32 logical -> gathered row)."""
    rm = None if row_map is None else np.ascontiguousarray(row_map, np.int32)
    slots = np.ascontiguousarray(slots, dtype=SLOT_DTYPE)
    gathered = np.ascontiguousarray(gathered, dtype=np.float32)
    out = np.zeros((batch, out_stride), np.float32)
    rc = lib().orf_pool_rows_fwd(_p(slots), len(slots), _p(np.ascontiguousarray(bag_off, np.int32)),
                                 _p(np.ascontiguousarray(lmax, np.int32)), batch, n_tok, _p(gathered),
                                 None if rm is None else _p(rm), DT_F32, dim,
                                 _p(out), DT_F32, out_stride, flags)
    if rc:
        raise RuntimeError(f"oracle pool_rows failed rc={rc}")
    return out


def bucketize_owner(rows: np.ndarray, nranks: int):
    rows = np.ascontiguousarray(rows, dtype=np.int64)
    counts = np.zeros(nranks, np.int32)
    perm = np.zeros(len(rows), np.int32)
    local = np.zeros(len(rows), np.int64)
    inv = np.zeros(len(rows), np.int32)
    lib().orf_bucketize_owner(_p(rows), len(rows), nranks, _p(counts), _p(perm), _p(inv), _p(local))
    return counts, perm, local, inv


def route_rows(rows: np.ndarray, nranks: int, table_rows: int):
    """rf_route_rows restated: distinct rows sorted by (owner = g mod P, local = g div P).
    Returns (counts int32 [P], local int64 [U], row_map int32 [n])."""
    rows = np.asarray(rows, np.int64)
    lp = -(-table_rows // nranks)
    ok = (rows >= 0) & (rows < table_rows)
    keys = np.where(ok, (rows % nranks) * lp + rows // nranks, nranks * lp)
    uniq, row_map = np.unique(keys, return_inverse=True)
    local = np.where(uniq < nranks * lp, uniq % lp, -1).astype(np.int64)
    owner = np.minimum(uniq // lp, nranks - 1)
    counts = np.bincount(owner, minlength=nranks).astype(np.int32)
    return counts, local, row_map.astype(np.int32).reshape(-1)


def route_rows_local(rows: np.ndarray, nranks: int, rank: int, table_rows: int):
    """rf_route_hash_build + rf_route_hash_finish restated: as route_rows over the rows NOT owned by `rank`
    (rank = -1: every row routed); a row the rank owns keeps row_map = 0x80000000 | local (int32 bits) and is
    read in place from the rank's shard by rf_pool_rows_fwd. Returns (counts int32 [P], local int64, row_map)."""
    rows = np.asarray(rows, np.int64)
    ok = (rows >= 0) & (rows < table_rows)
    own = ok & (rows % nranks == rank) if rank >= 0 else np.zeros(len(rows), bool)
    counts, local, rm = route_rows(rows[~own], nranks, table_rows)
    row_map = np.empty(len(rows), np.int32)
    row_map[~own] = rm
    row_map[own] = (np.uint32(0x80000000) | (rows[own] // nranks).astype(np.uint32)).view(np.int32)
    return counts, local, row_map


def partial_pool(slots, tok_bytes, tok_off, bag_off, lmax, batch, table, dim, out_stride, nranks, flags=0):
    """rf_pp_* (owner-side partial pooling) restated: unit (b, s, k) pools its positions l < L (L = len masked,
    else max(Lmax, len); pad positions read the slot's pad row) per owner (row mod P) in position order from
    +0.0 (sum) / -inf (max) / +inf (min), then adds / maxes / mins the owners' partials in owner order 0..P-1;
    avg divides by L; first / last take position 0 / L-1; an empty unit (L = 0) gets 0 / NaN / -inf / +inf / 0
    as rf_fused_hash_embed_fwd (zeros when masked). float32 arithmetic, fp32 table."""
    f32 = np.float32
    slots = np.ascontiguousarray(slots, dtype=SLOT_DTYPE)
    S = len(slots)
    rows = hash_rows(slots, tok_bytes, tok_off, bag_off, batch)
    mask_pad = bool(flags & FLAG_MASK_PADDING)
    table = np.asarray(table, np.float32)
    out = np.zeros((batch, out_stride), np.float32)
    for s in range(S):
        sd = slots[s]
        comb = int(sd["combiner"])
        pads = []
        for k in range(2):
            nb = int(sd["num_bins"])
            pb = 0 if int(sd["mask_empty"]) else hash_bucket(b"", nb, int(sd["salt"][k]), False)
            pads.append(int(sd["row_base"][k]) + pb)
        for b in range(batch):
            u = b * S + s
            t0, t1 = int(bag_off[u]), int(bag_off[u + 1])
            ln = t1 - t0
            L = ln if mask_pad else max(int(lmax[s]), ln)
            for k in range(2):
                pos = [int(rows[2 * t + k]) for t in range(t0, t1)] + [pads[k]] * (L - ln)
                if comb == COMB["first"]:
                    pos = pos[:1]
                elif comb == COMB["last"]:
                    pos = pos[L - 1:L] if L else []
                if L == 0:
                    v = np.full(dim, 0.0 if mask_pad else {COMB["avg"]: np.nan, COMB["max"]: -np.inf,
                                                           COMB["min"]: np.inf}.get(comb, 0.0), f32)
                else:
                    init = {COMB["max"]: -np.inf, COMB["min"]: np.inf}.get(comb, 0.0)
                    v = np.full(dim, init, f32)
                    for o in range(nranks):
                        mine = [g for g in pos if g % nranks == o]
                        if not mine:
                            continue
                        p = np.full(dim, init, f32)
                        for g in mine:
                            x = table[g]
                            if comb in (COMB["sum"], COMB["avg"]):
                                p = (p + x).astype(f32)
                            elif comb == COMB["max"]:
                                p = np.where(x > p, x, p)
                            elif comb == COMB["min"]:
                                p = np.where(x < p, x, p)
                            else:
                                p = x.copy()
                        if comb in (COMB["sum"], COMB["avg"]):
                            v = (v + p).astype(f32)
                        elif comb == COMB["max"]:
                            v = np.where(p > v, p, v)
                        elif comb == COMB["min"]:
                            v = np.where(p < v, p, v)
                        else:
                            v = p
                    if comb == COMB["avg"]:
                        v = (v / f32(L)).astype(f32)
                off = int(sd["out_off"]) + k * dim
                out[b, off:off + dim] = v
    return out


def bf16_to_f32(u16: np.ndarray) -> np.ndarray:
    return (np.asarray(u16, dtype=np.uint16).astype(np.uint32) << 16).view(np.float32)


def f32_to_bf16(x: np.ndarray) -> np.ndarray:
    """Round-to-nearest-even f32 -> bf16 bits (NaN stays NaN)."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    nan = (u & 0x7FFFFFFF) > 0x7F800000
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    r[nan] = ((u[nan] >> 16) | 0x40).astype(np.uint16)
    return r


# ----------------------------------------------------------------------------------------------
# dense floating-point stages (float64 numpy)
# ----------------------------------------------------------------------------------------------
def soft_attention(x0: np.ndarray, x1: np.ndarray):
    """SoftAttention.__call__ (attention_layers.py:15-30): inputs [x0, x1] = [q, a].

    _attention (:44-47): batch_dot(x0, x1^T) -> [B, L0, L1], permuted -> E[n, i, j] = x1[n,i].x0[n,j].
    _soft_alignment (:69-74): S = exp(E - max_j E) / sum_j;  align_0 = S @ x0, align_1 = S @ x1.
    """
    x0 = np.asarray(x0, np.float64)
    x1 = np.asarray(x1, np.float64)
    E = np.einsum("bjk,bik->bij", x0, x1)
    e = np.exp(E - E.max(axis=-1, keepdims=True))
    S = e / e.sum(axis=-1, keepdims=True)
    return S @ x0, S @ x1


def esim_pool(q: np.ndarray, a: np.ndarray) -> np.ndarray:
    """Esim.call combine (esim.py:78-82): [avg_q, max_q, avg_a, max_a, avg_q-avg_a, max_q-max_a] -> [B, 6d]."""
    att_q, att_a = soft_attention(q, a)
    q = np.asarray(q, np.float64)
    a = np.asarray(a, np.float64)
    m_q = np.concatenate([q, att_q, q - att_q, q * att_q], axis=1)
    m_a = np.concatenate([a, att_a, a - att_a, a * att_a], axis=1)
    avg_q, max_q = m_q.mean(axis=1), m_q.max(axis=1)
    avg_a, max_a = m_a.mean(axis=1), m_a.max(axis=1)
    return np.concatenate([avg_q, max_q, avg_a, max_a, avg_q - avg_a, max_q - max_a], axis=1)


def gelu(x):
    """tf.keras.activations.gelu (approximate=False): 0.5 x (1 + erf(x / sqrt 2))."""
    from scipy.special import erf

    return 0.5 * x * (1.0 + erf(x / math.sqrt(2.0)))


def selu(x):
    alpha, scale = 1.6732632423543772848170429916717, 1.0507009873554804934193349852946
    return scale * np.where(x > 0, x, alpha * (np.exp(np.minimum(x, 0)) - 1.0))


def activation(x, act: str):
    if act in (None, "none", "linear"):
        return x
    if act == "gelu":
        return gelu(x)
    if act == "relu":
        return np.maximum(x, 0)
    if act == "selu":
        return selu(x)
    if act == "softmax":
        e = np.exp(x - x.max(axis=-1, keepdims=True))
        return e / e.sum(axis=-1, keepdims=True)
    raise ValueError(act)


def layer_norm(x, gamma, beta, eps=1e-6):
    """tf.keras.layers.LayerNormalization(epsilon) over the last axis."""
    x = np.asarray(x, np.float64)
    mu = x.mean(axis=-1, keepdims=True)
    var = ((x - mu) ** 2).mean(axis=-1, keepdims=True)
    return (x - mu) / np.sqrt(var + eps) * gamma + beta


def batch_norm_infer(x, gamma, beta, mean, var, eps=1e-6):
    """tf.keras.layers.BatchNormalization(epsilon) at inference."""
    return (np.asarray(x, np.float64) - mean) / np.sqrt(var + eps) * gamma + beta


def mlp(x, layers, act: str, norm: str = "ln", eps: float = 1e-6):
    """create_mlp (mlp.py:4-15): per layer  x = act(Norm(x) @ W + b); Dropout = identity at inference.

    layers: list of dicts {W: [K, N], b: [N], gamma, beta, (mean, var for BN)} — one norm per layer
    (deviation D-shared-norm).
    """
    x = np.asarray(x, np.float64)
    for p in layers:
        if norm == "ln":
            x = layer_norm(x, p["gamma"], p["beta"], eps)
        elif norm == "bn":
            x = batch_norm_infer(x, p["gamma"], p["beta"], p["mean"], p["var"], eps)
        x = activation(x @ np.asarray(p["W"], np.float64) + p["b"], act)
    return x


def esim_scorer_f32(q, a, dense, input_layers, output_layers, W_out, b_out, eps=1e-6):
    """The CPU baseline of cfg3's dense stages (bench.py cpu_baseline): a.5-a.7 in float32
    numpy / BLAS, operation for operation as the reference graph runs them on a CPU (esim.py:69-89):
    SoftAttention (attention_layers.py:44-74, batched matmuls, max-subtracted softmax), the [B, 4L, d]
    concatenations and their mean / max (esim.py:79-84), create_mlp LayerNorm -> Dense(gelu) stacks
    (mlp.py:4-15), Dense(2, softmax) (esim.py:53,88). Not a checker: the float64 functions above are."""
    from scipy.special import erf

    f = np.float32
    q, a, dense = np.asarray(q, f), np.asarray(a, f), np.asarray(dense, f)

    def ln(x, p):
        mu = x.mean(-1, keepdims=True, dtype=f)
        d = x - mu
        var = (d * d).mean(-1, keepdims=True, dtype=f)
        return d / np.sqrt(var + f(eps)) * p["gamma"].astype(f) + p["beta"].astype(f)

    def stack(x, layers):
        for p in layers:
            x = ln(x, p) @ p["W"].astype(f) + p["b"].astype(f)
            x = f(0.5) * x * (f(1.0) + erf(x / f(math.sqrt(2.0))).astype(f))
        return x

    E = np.matmul(a, q.transpose(0, 2, 1))
    E = np.exp(E - E.max(-1, keepdims=True))
    S = E / E.sum(-1, keepdims=True)
    att_q, att_a = np.matmul(S, q), np.matmul(S, a)
    m_q = np.concatenate([q, att_q, q - att_q, q * att_q], axis=1)
    m_a = np.concatenate([a, att_a, a - att_a, a * att_a], axis=1)
    avg_q, max_q, avg_a, max_a = m_q.mean(1, dtype=f), m_q.max(1), m_a.mean(1, dtype=f), m_a.max(1)
    pooled = np.concatenate([stack(dense, input_layers), avg_q, max_q, avg_a, max_a, avg_q - avg_a, max_q - max_a], axis=1)
    z = stack(pooled, output_layers) @ np.asarray(W_out, f) + np.asarray(b_out, f)
    z = np.exp(z - z.max(-1, keepdims=True))
    return z / z.sum(-1, keepdims=True)


def sdpa(q, k, v, mask=None):
    """scaled_dot_product_attention (layer_utils.py:4-24): mask [.., Lq] zero => whole QUERY row filled
    with -4294967295 (the [..., Lq, 1] mask broadcasts over keys), softmax over keys, @ v."""
    q, k, v = (np.asarray(t, np.float64) for t in (q, k, v))
    logits = q @ np.swapaxes(k, -1, -2) / math.sqrt(k.shape[-1])
    if mask is not None:
        m = np.asarray(mask)[..., :, None]
        logits = np.where(m == 0, -4294967295.0, logits)
    e = np.exp(logits - logits.max(axis=-1, keepdims=True))
    return (e / e.sum(axis=-1, keepdims=True)) @ v


def positional_encoding(length: int, dim: int) -> np.ndarray:
    """SelfAttention.get_angles / positional_encoding (attention_layers.py:126-134): angle = pos /
    10000^(2*(i//2) / float32(dim)) in float64, sin on even columns, cos on odd, cast to float32."""
    pos = np.arange(length)[:, None]
    i = np.arange(dim)[None, :]
    ang = pos * (1 / np.power(10000, (2 * (i // 2)) / np.float32(dim)))
    ang[:, 0::2] = np.sin(ang[:, 0::2])
    ang[:, 1::2] = np.cos(ang[:, 1::2])
    return ang.astype(np.float32)


def self_attention(q, k, v, mask, W, add_pos=True):
    """SelfAttention.call (attention_layers.py:98-124): q,k += PE (float32, :101-103); q' = relu(q W),
    k' = relu(k W) with the ONE shared W (:105-106); logits = q' k'^T / sqrt(dim) (:107-110); mask [B, L, 1]
    tiled over the keys (:112), rows with mask == 0 become -2^32 + 1 (:113-114); softmax over keys (:116),
    @ v (:118, v untouched by PE and W), mean over the sequence axis (:119) -> [B, dim]."""
    q = np.asarray(q, np.float32)
    k = np.asarray(k, np.float32)
    dim = q.shape[-1]
    if add_pos:
        k = k + positional_encoding(k.shape[1], dim)
        q = q + positional_encoding(q.shape[1], dim)
    W = np.asarray(W, np.float64)
    qn = np.maximum(q.astype(np.float64) @ W, 0.0)
    kn = np.maximum(k.astype(np.float64) @ W, 0.0)
    logits = qn @ np.swapaxes(kn, -1, -2) / math.sqrt(float(np.float32(dim)))
    if mask is not None:
        m = np.asarray(mask).reshape(q.shape[0], q.shape[1])[:, :, None]
        logits = np.where(m == 0, -4294967295.0, logits)
    e = np.exp(logits - logits.max(axis=-1, keepdims=True))
    out = (e / e.sum(axis=-1, keepdims=True)) @ np.asarray(v, np.float64)
    return out.mean(axis=1)


def multi_head_attention(q, k, v, mask, Wq, bq, Wk, bk, Wv, bv, heads: int):
    """MultiHeadAttention.call (attention_layers.py:153-168): Dense q/k/v with bias, W as [in, d_model] (:148-150,
    :154-156); split_heads (layer_utils.py:27-38) -> [B, h, L, depth]; mask [B, L, 1] tiled over heads (:161);
    scaled_dot_product_attention (layer_utils.py:4-24, row-mask); merge heads (:166-167); NO output projection."""
    f = lambda x, W, b: np.asarray(x, np.float64) @ np.asarray(W, np.float64) + np.asarray(b, np.float64)
    qp, kp, vp = f(q, Wq, bq), f(k, Wk, bk), f(v, Wv, bv)
    B, Lq, dm = qp.shape
    Lk = kp.shape[1]
    depth = dm // heads
    split = lambda x, Ln: x.reshape(B, Ln, heads, depth).transpose(0, 2, 1, 3)
    m = None if mask is None else np.broadcast_to(np.asarray(mask).reshape(B, 1, Lq), (B, heads, Lq))
    o = sdpa(split(qp, Lq), split(kp, Lk), split(vp, Lk), m)
    return o.transpose(0, 2, 1, 3).reshape(B, Lq, dm)


def l2_normalize(x, eps=1e-12):
    """K.l2_normalize (dssm.py:35-36): x / sqrt(max(sum x^2, eps))."""
    x = np.asarray(x, np.float64)
    return x / np.sqrt(np.maximum((x * x).sum(axis=-1, keepdims=True), eps))


# ----------------------------------------------------------------------------------------------
# DSSM tower training (float64): create_mlp([..], rate, "selu", BatchNormalization(eps)) under model.fit
# (dssm.py:25-26, mlp.py:4-15, train.py:96-104): per layer BatchNormalization with batch statistics (Keras
# tf.nn.moments: biased variance) -> Dense -> SELU -> Dropout(rate); the keep mask restates rf_dropout_fwd's
# ----------------------------------------------------------------------------------------------
def _splitmix64_np(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64)
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def dropout_keep(seed: int, M: int, N: int, rate: float) -> np.ndarray:
    """keep(r, c) = top 24 bits of splitmix64(seed ^ (r N + c)) / 2^24 >= rate (float32 compare)."""
    idx = np.arange(M, dtype=np.uint64)[:, None] * np.uint64(N) + np.arange(N, dtype=np.uint64)[None, :]
    h = _splitmix64_np(np.uint64(seed) ^ idx)
    u = (h >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    return u >= np.float32(rate)


def tower_train_fwd(x, layers, rate: float, seeds, eps: float = 1e-6):
    """layers: [{"W": [N][K], "b", "gamma", "beta"}]; returns (output, cache) in float64."""
    h = np.asarray(x, np.float64)
    cache = []
    for p, seed in zip(layers, seeds):
        W = np.asarray(p["W"], np.float64)
        mean, var = h.mean(0), h.var(0)
        xhat = (h - mean) / np.sqrt(var + eps)
        z = xhat * p["gamma"] + p["beta"]
        y = selu(z @ W.T + p["b"])
        keep = dropout_keep(seed, h.shape[0], W.shape[0], rate)
        out = np.where(keep, y / (1.0 - rate), 0.0)
        cache.append({"h": h, "mean": mean, "var": var, "xhat": xhat, "z": z, "y": y, "keep": keep})
        h = out
    return h, cache


def tower_train_bwd(dout, layers, cache, rate: float, eps: float = 1e-6):
    """Backward of tower_train_fwd: returns (dx, [{"W", "b", "gamma", "beta"} gradients]); the SELU gradient is
    TF's SeluGrad on the activations (y < 0: y + scale alpha, else scale)."""
    scale, alpha = 1.0507009873554804934193349852946, 1.6732632423543772848170429916717
    dh = np.asarray(dout, np.float64)
    grads = []
    for p, c in zip(reversed(layers), reversed(cache)):
        W = np.asarray(p["W"], np.float64)
        dy = np.where(c["keep"], dh / (1.0 - rate), 0.0)
        dpre = dy * np.where(c["y"] < 0, c["y"] + scale * alpha, scale)
        dz = dpre @ W
        dxhat = dz * p["gamma"]
        xh = c["xhat"]
        dh = (dxhat - dxhat.mean(0) - xh * (dxhat * xh).mean(0)) / np.sqrt(c["var"] + eps)
        grads.insert(0, {"W": dpre.T @ c["z"], "b": dpre.sum(0), "gamma": (dz * xh).sum(0), "beta": dz.sum(0)})
    return dh, grads


# ----------------------------------------------------------------------------------------------
# ESIM ranking-model training (float64): esim.py:45-53,69-89 under model.fit (example/ranking_search/train.py:96-104).
# create_mlp(units, 0.3, gelu, LayerNormalization(1e-6)) layers (mlp.py:4-15, one norm per layer: deviation
# D-shared-norm), the SoftAttention + combine + pooling block, Dropout(0.3) on the pooled row (esim.py:85),
# Dense(2, softmax) and the sparse categorical cross-entropy of its logits. Dropout masks restate rf_dropout_fwd's.
# ----------------------------------------------------------------------------------------------
def gelu_grad(x):
    """d/dx of the exact erf GELU: 0.5 (1 + erf(x / sqrt 2)) + x phi(x)."""
    from scipy.special import erf

    x = np.asarray(x, np.float64)
    return 0.5 * (1.0 + erf(x / math.sqrt(2.0))) + x * np.exp(-0.5 * x * x) / math.sqrt(2.0 * math.pi)


def ln_mlp_train_fwd(x, layers, rate: float, seeds, eps: float = 1e-6):
    """layers: [{"W": [N][K], "b", "gamma", "beta"}] (W stored [out][in], as librf); per layer LayerNormalization
    (tf.nn.moments: biased variance) -> Dense -> gelu -> Dropout(rate). Returns (h, cache)."""
    h = np.asarray(x, np.float64)
    cache = []
    for p, seed in zip(layers, seeds):
        W = np.asarray(p["W"], np.float64)
        mu = h.mean(-1, keepdims=True)
        var = ((h - mu) ** 2).mean(-1, keepdims=True)
        rstd = 1.0 / np.sqrt(var + eps)
        xhat = (h - mu) * rstd
        z = xhat * p["gamma"] + p["beta"]
        pre = z @ W.T + p["b"]
        keep = dropout_keep(seed, h.shape[0], W.shape[0], rate) if rate > 0 else np.ones(pre.shape, bool)
        out = np.where(keep, gelu(pre) / (1.0 - rate), 0.0)
        cache.append({"h": h, "xhat": xhat, "rstd": rstd, "z": z, "pre": pre, "keep": keep})
        h = out
    return h, cache


def ln_mlp_train_bwd(dout, layers, cache, rate: float):
    """Backward of ln_mlp_train_fwd: (dx, [{"W", "b", "gamma", "beta"} gradients])."""
    dh = np.asarray(dout, np.float64)
    grads = []
    for p, c in zip(reversed(layers), reversed(cache)):
        W = np.asarray(p["W"], np.float64)
        dpre = np.where(c["keep"], dh / (1.0 - rate), 0.0) * gelu_grad(c["pre"])
        dz = dpre @ W
        u = dz * p["gamma"]
        xh = c["xhat"]
        dh = c["rstd"] * (u - u.mean(-1, keepdims=True) - xh * (u * xh).mean(-1, keepdims=True))
        grads.insert(0, {"W": dpre.T @ c["z"], "b": dpre.sum(0), "gamma": (dz * xh).sum(0), "beta": dz.sum(0)})
    return dh, grads


def esim_pool_bwd(q, a, dpooled):
    """float64 backward of esim_pool: (dq, da). The max pooling's gradient follows TF's reduce_max (_MinOrMaxGrad):
    split evenly over every candidate equal to the maximum."""
    q = np.asarray(q, np.float64)
    a = np.asarray(a, np.float64)
    dp = np.asarray(dpooled, np.float64)
    B, L, d = q.shape
    E = np.einsum("bjk,bik->bij", q, a)
    e = np.exp(E - E.max(axis=-1, keepdims=True))
    S = e / e.sum(axis=-1, keepdims=True)
    att = (S @ q, S @ a)
    g = [dp[:, k * d:(k + 1) * d] for k in range(6)]
    gavg = ((g[0] + g[4]) / (4 * L), (g[2] - g[4]) / (4 * L))
    gmax = (g[1] + g[5], g[3] - g[5])
    G, Dx = [], []
    for x, at, ga, gm in zip((q, a), att, gavg, gmax):
        cands = [x, at, x - at, x * at]
        M = np.max([c.max(axis=1) for c in cands], axis=0)  # [B, d]
        eq = [(c == M[:, None, :]).astype(np.float64) for c in cands]
        share = gm / sum(t.sum(axis=1) for t in eq)  # [B, d]
        G.append(x * ga[:, None, :] + share[:, None, :] * (eq[1] - eq[2] + x * eq[3]))
        Dx.append((2.0 + at) * ga[:, None, :] + share[:, None, :] * (eq[0] + eq[2] + at * eq[3]))
    dS = G[0] @ np.swapaxes(q, 1, 2) + G[1] @ np.swapaxes(a, 1, 2)  # [B, i, j]
    dE = S * (dS - (S * dS).sum(axis=-1, keepdims=True))
    St = np.swapaxes(S, 1, 2)
    dq = Dx[0] + St @ G[0] + np.swapaxes(dE, 1, 2) @ a
    da = Dx[1] + St @ G[1] + dE @ q
    return dq, da


def esim_train_loss(q, a, dense, label, input_layers, output_layers, W_out, b_out, rate: float = 0.0, seeds=None,
                    eps: float = 1e-6, grads: bool = False):
    """The ESIM training loss (float64) and, with grads=True, every gradient: returns (loss, probs) or (loss, probs,
    {"q", "a", "input", "output", "W_out", "b_out"}). seeds = (input layer seeds, pooled-dropout seed, output layer
    seeds) of the Dropout(rate) masks; W_out [2][K] stored [out][in]."""
    nin, nout = len(input_layers), len(output_layers)
    if seeds is None:
        seeds = ([0] * nin, 0, [0] * nout)
    s_in, s_pool, s_out = seeds
    label = np.asarray(label).astype(np.int64)
    d_emb, c_in = ln_mlp_train_fwd(dense, input_layers, rate, s_in, eps)
    pooled = np.concatenate([d_emb, esim_pool(q, a)], axis=1)
    keep = dropout_keep(s_pool, pooled.shape[0], pooled.shape[1], rate) if rate > 0 else np.ones(pooled.shape, bool)
    x = np.where(keep, pooled / (1.0 - rate), 0.0)
    h, c_out = ln_mlp_train_fwd(x, output_layers, rate, s_out, eps)
    Wo = np.asarray(W_out, np.float64)
    z = h @ Wo.T + b_out
    m = z.max(axis=-1, keepdims=True)
    lse = m[:, 0] + np.log(np.exp(z - m).sum(axis=-1))
    B = z.shape[0]
    loss = float((lse - z[np.arange(B), label]).mean())
    prob = np.exp(z - lse[:, None])
    if not grads:
        return loss, prob
    dz = prob.copy()
    dz[np.arange(B), label] -= 1.0
    dz /= B
    gWo, gbo = dz.T @ h, dz.sum(0)
    dx, g_out = ln_mlp_train_bwd(dz @ Wo, output_layers, c_out, rate)
    dpooled = np.where(keep, dx / (1.0 - rate), 0.0)
    W = d_emb.shape[1]
    _, g_in = ln_mlp_train_bwd(dpooled[:, :W], input_layers, c_in, rate)
    dq, da = esim_pool_bwd(q, a, dpooled[:, W:])
    return loss, prob, {"q": dq, "a": da, "input": g_in, "output": g_out, "W_out": gWo, "b_out": gbo}


# ----------------------------------------------------------------------------------------------
# training losses (float64), backend/losses/match_losses.py
# ----------------------------------------------------------------------------------------------
def cosent_loss(y: np.ndarray, s: np.ndarray, scale: float = 20.0):
    """match_losses.py:42-56 on scores s_i = <q_i, d_i>: returns (loss, dloss/ds)."""
    y = np.asarray(y, np.float64)
    s = np.asarray(s, np.float64)
    valid = y[:, None] < y[None, :]
    x = scale * (s[:, None] - s[None, :])
    xs = np.where(valid, x, -np.inf)
    m = max(0.0, float(xs.max()) if valid.any() else 0.0)
    e = np.where(valid, np.exp(x - m), 0.0)
    z = np.exp(-m) + e.sum()
    loss = m + np.log(z)
    p = e / z
    ds = scale * (p.sum(axis=1) - p.sum(axis=0))
    return loss, ds


def inbatch_ce_loss(y: np.ndarray, logits: np.ndarray, scale: float = 20.0):
    """match_losses.py:150-165 on logits P = q . d^T: returns (loss, dloss/dP)."""
    y = np.asarray(y, np.float64)
    P = np.asarray(logits, np.float64) * scale
    m = P.max(axis=1, keepdims=True)
    e = np.exp(P - m)
    sm = e / e.sum(axis=1, keepdims=True)
    B = len(y)
    loss = float(np.mean(-np.log(np.diag(sm)) * y))
    d = scale * y[:, None] / B * (sm - np.eye(B))
    return loss, d


# ----------------------------------------------------------------------------------------------
# Lookup / Discrete index producers (preprocess_layers.py:135-200), pure Python
# ----------------------------------------------------------------------------------------------
def lookup_ids(vocab, rows, pad):
    """StringLookup/IntegerLookup(vocabulary, num_oov_indices=1, mask_token=None) on padded rows:
    vocab[i] -> i + 1, else 0; rows shorter than the batch max are padded with `pad` first."""
    index = {v: i + 1 for i, v in enumerate(vocab)}
    width = max((len(r) for r in rows), default=0)
    return np.array([[index.get(v, 0) for v in list(r) + [pad] * (width - len(r))] for r in rows], np.int64).reshape(len(rows), width)


def bucketize_ids(boundaries, rows, pad=0.0):
    """tf Bucketize / Keras Discretization: number of boundaries <= x (bisect_right; NaN -> len). The
    boundaries are a list(float) op attribute, i.e. float32, like the inputs."""
    import bisect

    b = [float(np.float32(x)) for x in boundaries]
    width = max((len(r) for r in rows), default=0)
    return np.array([[bisect.bisect_right(b, float(np.float32(v))) for v in list(r) + [pad] * (width - len(r))]
                     for r in rows], np.int64).reshape(len(rows), width)


# ----------------------------------------------------------------------------------------------
# exact top-k search (faiss IndexFlatIP semantics), float64
# ----------------------------------------------------------------------------------------------
def flat_search(queries, items, k, cos=False):
    """(scores float64 [B, k], indexes int64 [B, k]): inner products, descending, ties by smaller index."""
    q = np.asarray(queries, np.float64)
    x = np.asarray(items, np.float64)
    if cos:
        q = q / np.sqrt((q * q).sum(1, keepdims=True))
        x = x / np.sqrt((x * x).sum(1, keepdims=True))
    s = q @ x.T
    idx = np.argsort(-s, axis=1, kind="stable")[:, :k]
    return np.take_along_axis(s, idx, 1), idx


def attention_fusion(inputs, W, is_norm=True):
    """fusion_layers.py:35-46 in float64: (out, att)."""
    x = np.concatenate([np.asarray(t, np.float64) for t in inputs], axis=1)
    logits = x @ np.asarray(W, np.float64)
    e = np.exp(logits - logits.max(axis=1, keepdims=True))
    att = e / e.sum(axis=1, keepdims=True)
    out = sum(att[:, c:c + 1] * np.asarray(inputs[c], np.float64) for c in range(len(inputs)))
    if is_norm:
        out = out / np.sqrt(np.maximum((out * out).sum(axis=1, keepdims=True), 1e-12))
    return out, att
