"""Pins of the CPU oracle (oracle/rf_oracle.c) — no GPU.

* SipHash-2-4 reference vectors (Aumasson & Bernstein, key 00..0f, messages 00..(n-1)), n = 0..15.
* CPython's own siphash24 (sys.hash_info.algorithm == 'siphash24'; PYTHONHASHSEED=0 => key (0, 0)):
  an independent implementation of the same function, on 2000 random messages.
* TF / Keras API docstring examples: tf.strings.to_hash_bucket_strong and
  keras.layers.Hashing(num_bins=3, salt=...).
* Pooling semantics of the reference padded batch on hand-checked cases.
"""
import struct
import subprocess
import sys

import numpy as np
import pytest

SIP_VECTORS = [0x726fdb47dd0e0e31, 0x74f839c593dc67fd, 0x0d6c8009d9a94f5a, 0x85676696d7fb7e2d, 0xcf2794e0277187b7,
               0x18765564cd99a68d, 0xcbc9466e58fee3ce, 0xab0200f58b01d137, 0x93f5f5799a932462, 0x9e0082df0ba9e4b0,
               0x7a5dbbc594ddb9f3, 0xf4b32f46226bada7, 0x751e8fbc860ee5fb, 0x14ea5627c0843d90, 0xf723ca908e7af2ee,
               0xa129ca6149be45e5]


def test_siphash_reference_vectors(O):
    k0, k1 = struct.unpack("<QQ", bytes(range(16)))
    for n, want in enumerate(SIP_VECTORS):
        assert O.siphash24(k0, k1, bytes(range(n))) == want, n


def test_siphash_matches_cpython(O):
    if sys.hash_info.algorithm != "siphash24":
        pytest.skip("this CPython does not use siphash24")
    rng = np.random.default_rng(0)
    msgs = [bytes(rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8)) for _ in range(2000)]
    code = "import sys\nfor line in sys.stdin.read().split():\n    print(hash(bytes.fromhex(line)))\n"
    res = subprocess.run([sys.executable, "-c", code], input="\n".join(m.hex() for m in msgs), capture_output=True,
                         text=True, env={"PYTHONHASHSEED": "0"}, check=True)
    got = [int(x) for x in res.stdout.split()]
    for m, h in zip(msgs, got):
        mine = O.siphash24(0, 0, m)
        mine = mine - (1 << 64) if mine >= 1 << 63 else mine
        if mine == -1:
            mine = -2
        assert mine == h


def test_tf_docstring_kats(O):
    # tf.strings.to_hash_bucket_strong(["Hello", "TF"], 3, [1, 2]) -> [2, 0]
    assert [O.siphash24(1, 2, t) % 3 for t in (b"Hello", b"TF")] == [2, 0]
    # keras.layers.Hashing(num_bins=3, salt=133)(["A".."E"]) -> [0, 0, 2, 1, 0]   (int salt -> key (s, s))
    assert [O.hash_bucket(bytes([t]), 3, 133, mask_empty=False) for t in b"ABCDE"] == [0, 0, 2, 1, 0]
    # keras.layers.Hashing(num_bins=3, salt=[133, 137]) -> [1, 2, 1, 0, 2]
    assert [O.siphash24(133, 137, bytes([t])) % 3 for t in b"ABCDE"] == [1, 2, 1, 0, 2]


def test_mask_rule(O):
    # mask_value="" (preprocess_utils.py:15): b"" -> 0, else 1 + h mod (N - 1); N == 1 reserves nothing
    assert O.hash_bucket(b"", 3000, 2022) == 0
    for t in (b"com.example.app", b"12345", b"x" * 100):
        h = O.siphash24(2022, 2022, t)
        assert O.hash_bucket(t, 3000, 2022) == 1 + h % 2999
        assert O.hash_bucket(t, 1, 2022) == 0
    assert (O.hash_bucket(b"com.example.app", 3000, 2022), O.hash_bucket(b"com.example.app", 3000, 2023)) == (750, 2359)


def _one_slot(O, combiner, rows, lmax=None, dim=4, flags=0):
    from recommendflow_amd.runtime.batch import from_lists

    hb = from_lists([[r] for r in rows], lmax=None if lmax is None else [lmax])
    N = 11
    table = np.arange(2 * N * dim, dtype=np.float32).reshape(2 * N, dim) / 8.0
    desc = np.zeros(1, O.SLOT_DTYPE)
    desc[0]["row_base"] = (0, N)
    desc[0]["num_bins"] = N
    desc[0]["salt"] = (2022, 2023)
    desc[0]["dim"] = dim
    desc[0]["combiner"] = O.COMB[combiner]
    desc[0]["mask_empty"] = 1
    width = 2 * int(hb.lmax[0]) * dim if combiner == "null" else 2 * dim
    out, idx = O.fused_hash_embed(desc, hb.tok_bytes, hb.tok_off, hb.bag_off, hb.lmax, len(rows), table, dim, width,
                                  flags=flags, emit_idx=True)
    return out, idx, table, N


def test_pool_padding_semantics(O):
    rows = [[b"a", b"b", b"c"], [b"d"], []]
    out, idx, T, N = _one_slot(O, "sum", rows)
    # example 1: one real token + 2 padding positions gathering row 0 of each table
    b1 = idx[3]
    want = np.concatenate([T[b1[0]] + T[0] + T[0], T[N + b1[1]] + T[N] + T[N]])
    np.testing.assert_array_equal(out[1], want)
    # example 2 (empty, len 0 < Lmax 3): three padding rows
    np.testing.assert_array_equal(out[2], np.concatenate([3 * T[0], 3 * T[N]]))
    avg, _, _, _ = _one_slot(O, "avg", rows)
    np.testing.assert_array_equal(avg[1], (want / np.float32(3)).astype(np.float32))
    mx, _, _, _ = _one_slot(O, "max", rows)
    np.testing.assert_array_equal(mx[1], np.concatenate([np.maximum(T[b1[0]], T[0]), np.maximum(T[N + b1[1]], T[N])]))
    masked, _, _, _ = _one_slot(O, "sum", rows, flags=O.FLAG_MASK_PADDING)
    np.testing.assert_array_equal(masked[1], np.concatenate([T[b1[0]], T[N + b1[1]]]))
    np.testing.assert_array_equal(masked[2], np.zeros(8, np.float32))


def test_first_last_null(O):
    rows = [[b"a", b"b", b"c"], [b"d"]]
    f, idx, T, N = _one_slot(O, "first", rows)
    np.testing.assert_array_equal(f[1], np.concatenate([T[idx[3][0]], T[N + idx[3][1]]]))
    last, idx, T, N = _one_slot(O, "last", rows)
    np.testing.assert_array_equal(last[0], np.concatenate([T[idx[2][0]], T[N + idx[2][1]]]))
    np.testing.assert_array_equal(last[1], np.concatenate([T[0], T[N]]))  # position Lmax-1 is padding
    nul, idx, T, N = _one_slot(O, "null", rows)
    got = nul[1].reshape(2, 3, 4)
    np.testing.assert_array_equal(got[0], np.stack([T[idx[3][0]], T[0], T[0]]))
    np.testing.assert_array_equal(got[1], np.stack([T[N + idx[3][1]], T[N], T[N]]))


def test_table_init_is_shard_invariant(O):
    full = O.table_init_uniform(40, 8, seed=99)
    for P in (2, 4):
        for rank in range(P):
            shard = O.table_init_uniform(40 // P, 8, seed=99, row0=rank, row_stride=P)
            np.testing.assert_array_equal(shard, full[rank::P])
    assert full.min() >= -0.05 and full.max() < 0.05


def test_bucketize_owner(O):
    rows = np.array([5, 2, 7, 4, 9, 0, 3, 6], np.int64)
    counts, perm, local, inv = O.bucketize_owner(rows, 3)
    np.testing.assert_array_equal(inv[perm], np.arange(len(rows)))
    assert counts.tolist() == [4, 2, 2]  # owners 2 2 1 1 0 0 0 0
    assert perm.tolist() == [4, 5, 6, 7, 2, 3, 0, 1]  # owner-major, stable
    np.testing.assert_array_equal(local, rows[perm] // 3)
