"""Lookup / Discrete embeddings: GPU index producers rf_lookup_ids / rf_bucketize_ids
against the Python oracle and the TF/Keras docstring examples (public API docs: StringLookup,
IntegerLookup, Discretization, tf.raw_ops.Bucketize)."""
import ctypes

import numpy as np
import pytest

from oracle import oracle as O

KATS_STRING = (["a", "b", "c", "d"], [["a", "c", "d"], ["d", "z", "b"]], [[1, 3, 4], [4, 0, 2]])
KATS_INT = ([12, 36, 1138, 42], [[12, 1138, 42], [42, 1000, 36]], [[1, 3, 4], [4, 0, 2]])
KATS_DISC = ([0.0, 1.0, 2.0], [[-1.5, 1.0, 3.4, 0.5], [0.0, 3.0, 1.3, 0.0]], [[0, 2, 3, 1], [1, 3, 2, 1]])
KATS_BUCKETIZE = ([0, 10, 100], [[-5, 10000], [150, 10], [5, 100]], [[0, 3], [3, 2], [1, 3]])


def test_oracle_kats():
    v, rows, want = KATS_STRING
    assert O.lookup_ids(v, rows, "").tolist() == want
    v, rows, want = KATS_INT
    assert O.lookup_ids(v, rows, 0).tolist() == want
    for v, rows, want in (KATS_DISC, KATS_BUCKETIZE):
        assert O.bucketize_ids(v, rows).tolist() == want
    assert O.bucketize_ids([1.0, 2.0], [[float("nan")]]).tolist() == [[2]]


def test_vocab_build_host_rejects_repeated_terms():
    from recommendflow_amd.runtime import lib as L

    lib = L.load()
    cap = lib.rf_vocab_capacity(3)
    assert cap >= 6 and cap & (cap - 1) == 0
    tab = np.zeros(cap * 16, np.uint8)
    vb = np.frombuffer(b"abcab", np.uint8).copy()
    off = np.array([0, 2, 3, 5], np.int32)  # "ab", "c", "ab"
    assert lib.rf_vocab_build(0, vb.ctypes.data, off.ctypes.data, 3, tab.ctypes.data, cap) == L.RF_EINVAL
    assert b"repeated" in lib.rf_last_error()
    iv = np.array([5, -7, 5], np.int64)
    assert lib.rf_vocab_build(1, iv.ctypes.data, None, 3, tab.ctypes.data, cap) == L.RF_EINVAL
    iv = np.array([5, -7, 9], np.int64)
    assert lib.rf_vocab_build(1, iv.ctypes.data, None, 3, tab.ctypes.data, cap) == 0
    ids = tab.view(np.dtype([("key", "<u8"), ("id", "<i4"), ("ref", "<i4")]))["id"]
    assert sorted(ids[ids >= 0].tolist()) == [1, 2, 3]


@pytest.mark.gpu
def test_lookup_kats_gpu(cuda):
    from recommendflow_amd.backend.layers.preprocess_layers import DiscreteEmbedding, LookupEmbedding

    v, rows, want = KATS_STRING
    assert LookupEmbedding(8, "str", v).lookup_ids(rows).cpu().tolist() == want
    v, rows, want = KATS_INT
    assert LookupEmbedding(8, "int", v).lookup_ids(rows).cpu().tolist() == want
    for v, rows, want in (KATS_DISC, KATS_BUCKETIZE):
        assert DiscreteEmbedding(8, v).bucket_ids(rows).cpu().tolist() == want


@pytest.mark.gpu
@pytest.mark.parametrize("n_vocab", [0, 1, 37, 5000])
def test_lookup_random_vs_oracle(cuda, n_vocab):
    import torch

    from recommendflow_amd.backend.layers.preprocess_layers import LookupEmbedding
    from recommendflow_amd.runtime.batch import from_lists

    rng = np.random.default_rng(n_vocab)
    vocab = [f"t{i}" for i in rng.permutation(3 * n_vocab + 1)[:n_vocab]]
    # strings: bags of varying length incl. empty strings, OOV terms and empty bags
    rows = [[rng.choice(vocab + ["", "oov", "t"]) if vocab else "x" for _ in range(int(rng.integers(0, 7)))] for _ in range(300)]
    sb = from_lists([[r] for r in rows])
    lk = LookupEmbedding(16, "str", vocab, pooling="avg")
    got = lk.lookup_ids(sb).cpu().numpy()
    want = O.lookup_ids(vocab, rows, "")
    np.testing.assert_array_equal(got, want)
    # pooled output = the C oracle's EmbeddingBag over the same ids
    emb = lk(sb).cpu().numpy()
    np.testing.assert_array_equal(emb.view(np.uint32), O.embedding_bag(want, lk.embedding.table.cpu().numpy(), "avg").view(np.uint32))
    # integers, negative values and 0-padding
    ivocab = [int(x) for x in rng.choice(np.arange(-10 ** 12, 10 ** 12, 7919), n_vocab, replace=False)]
    irows = [[int(rng.choice(ivocab + [0, 3, -1])) if ivocab else 5 for _ in range(int(rng.integers(0, 6)))] for _ in range(200)]
    lki = LookupEmbedding(8, "int", ivocab)
    from recommendflow_amd.runtime.tfrecord import RaggedColumns

    bo = np.zeros(201, np.int32)
    np.cumsum([len(r) for r in irows], out=bo[1:])
    flat = np.array([v for r in irows for v in r] or [0], np.int64)
    rc = RaggedColumns(torch.from_numpy(flat).cuda(), torch.from_numpy(bo).cuda(),
                       np.array([max(len(r) for r in irows)], np.int32), ["f"])
    np.testing.assert_array_equal(lki.lookup_ids(rc).cpu().numpy(), O.lookup_ids(ivocab, irows, 0))


@pytest.mark.gpu
def test_discrete_random_vs_oracle(cuda):
    import torch

    from recommendflow_amd.backend.layers.preprocess_layers import DiscreteEmbedding
    from recommendflow_amd.runtime.tfrecord import RaggedColumns

    rng = np.random.default_rng(1)
    bnd = sorted(set(np.round(rng.normal(size=40), 3).tolist()))
    rows = [[float(np.float32(x)) for x in rng.normal(size=int(rng.integers(0, 5)))] for _ in range(500)]
    rows[3] = [float("nan"), bnd[5], -1e30, 1e30]  # NaN, exact boundary hits, extremes
    # two features interleaved example-major; slot 1 is the one under test
    other = [[1.0] for _ in rows]
    flat, bo = [], [0]
    for a, b in zip(other, rows):
        flat += a
        bo.append(len(flat))
        flat += b
        bo.append(len(flat))
    rc = RaggedColumns(torch.tensor(flat, dtype=torch.float32).cuda(), torch.tensor(bo, dtype=torch.int32).cuda(),
                       np.array([1, max(len(r) for r in rows)], np.int32), ["other", "f"])
    de = DiscreteEmbedding(8, bnd, pooling="max")
    got = de.bucket_ids(rc, slot=1).cpu().numpy()
    np.testing.assert_array_equal(got, O.bucketize_ids(bnd, rows))
    emb = de(rc, slot=1).cpu().numpy()
    np.testing.assert_array_equal(emb.view(np.uint32), O.embedding_bag(got, de.embedding.table.cpu().numpy(), "max").view(np.uint32))
