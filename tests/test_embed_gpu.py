"""GPU parity of the sparse hot path (hash -> gather -> pool) against the C oracle, through the C ABI.

Bar: bit-exact for bucket ids and for pooled fp32/bf16 outputs (the kernel accumulates in the oracle's
order, position l = 0..Lmax-1, one fp32 add per position).
"""
import numpy as np
import pytest
import torch

from recommendflow_amd.backend.encoder.sparse_encoder import FusedSparseEncoder, SlotSpec
from recommendflow_amd.backend.layers.preprocess_layers import DoubleHashingEmbedding, EmbeddingBag, Hashing
from recommendflow_amd.runtime import lib as L
from recommendflow_amd.runtime.batch import SparseBatch, from_lists, synthetic_batch

pytestmark = pytest.mark.gpu
COMBS = ["sum", "avg", "max", "min", "first", "last"]


def bits(x):
    return np.ascontiguousarray(x).view(np.uint32 if x.dtype == np.float32 else np.uint16)


def run_both(O, enc, hb, emit=True):
    out, idx = enc(hb.to("cuda"), emit_idx=True) if emit else (enc(hb.to("cuda")), None)
    tdt = enc.table.dtype
    table = enc.table.cpu().view(torch.int16).numpy().view(np.uint16) if tdt == torch.bfloat16 else enc.table.cpu().numpy()
    flags = O.FLAG_MASK_PADDING if enc.mask_padding else 0
    odt = O.DT_F32 if enc.out_dtype == torch.float32 else O.DT_BF16
    ref, ridx = O.fused_hash_embed(enc.host_desc, hb.tok_bytes, hb.tok_off, hb.bag_off, hb.lmax, hb.batch, table,
                                   enc.dim, enc.out_width, out_dtype=odt, flags=flags, emit_idx=True)
    got = out.cpu()
    got = got.view(torch.int16).numpy().view(np.uint16) if got.dtype == torch.bfloat16 else got.numpy()
    return got, ref, (idx.cpu().numpy() if emit else None), ridx


def test_siphash_bucket_matches_oracle(O, cuda):
    rng = np.random.default_rng(1)
    toks = [bytes(rng.integers(0, 256, int(rng.integers(0, 70)), dtype=np.uint8)) for _ in range(5000)]
    hb = from_lists([[[t]] for t in toks])
    # unaligned token starts are the common case (byte-packed CSR); also hit every tail length 0..7
    for nb, salt, mask in [(3000, 2022, True), (1, 7, True), (2, 11, False), (100003, 2 ** 63 + 5, True)]:
        h = Hashing(nb, mask_value="" if mask else None, salt=salt)
        got = h.hash_tokens(hb.to("cuda")).cpu().numpy()
        want = O.hash_tokens(hb.tok_bytes, hb.tok_off, salt, salt, nb, mask)
        np.testing.assert_array_equal(got, want)


def test_hashing_layer_dense_padding(O, cuda):
    h = Hashing(3, salt=133)
    dense = h([[b"A", b"B", b"C"], [b"D"], [b"E"]]).cpu().numpy()
    # keras docstring: salt 133 on A..E -> [0, 0, 2, 1, 0]; padding b"" (no mask) -> hash of b""
    assert dense[:, 0].tolist() == [0, 1, 0] and dense[0].tolist() == [0, 0, 2]
    assert dense[1, 1] == dense[1, 2] == O.hash_bucket(b"", 3, 133, mask_empty=False)


@pytest.mark.parametrize("tdt,odt", [(torch.float32, torch.float32), (torch.bfloat16, torch.bfloat16),
                                     (torch.bfloat16, torch.float32), (torch.float32, torch.bfloat16)])
@pytest.mark.parametrize("dim", [4, 8, 16, 64, 128, 256])
def test_fused_embed_parity_dims(O, cuda, tdt, odt, dim):
    if tdt == torch.bfloat16 and dim % 8:
        pytest.skip("bf16 rows need dim % 8 == 0")
    S, B = 12, 97
    specs = [SlotSpec(f"f{s}", 50 + 131 * s, (2022 + s, 2023 + 3 * s), COMBS[s % 6], mask_empty=(s % 5 != 4))
             for s in range(S)]
    enc = FusedSparseEncoder(specs, dim, table_dtype=tdt, out_dtype=odt, seed=dim)
    hb = synthetic_batch(B, [s % 3 == 0 for s in range(S)], seed=dim, poisson_mean=5)
    got, ref, idx, ridx = run_both(O, enc, hb)
    np.testing.assert_array_equal(idx, ridx)
    np.testing.assert_array_equal(got, bits(ref) if got.dtype != ref.dtype else ref.view(got.dtype))


@pytest.mark.parametrize("mask_padding", [False, True])
def test_fused_embed_edge_cases(O, cuda, mask_padding):
    """empty bags, bags longer than the 256-token LDS bucket, empty tokens, Lmax > every len, B=1."""
    rng = np.random.default_rng(7)
    S = 5
    rows = []
    for b in range(9):
        r = []
        for s in range(S):
            n = [0, 1, 3, 300, 2][s] if b % 2 == 0 else [1, 0, 0, 1, 700][s]
            r.append([b"" if rng.random() < 0.1 else bytes(rng.integers(33, 127, int(rng.integers(0, 20)), dtype=np.uint8))
                      for _ in range(n)])
        rows.append(r)
    hb = from_lists(rows, lmax=[4, 2, 5, 700, 800])
    for comb in COMBS:
        specs = [SlotSpec(f"f{s}", 7 + s, (s, 99 - s), comb, mask_empty=s != 2) for s in range(S)]
        enc = FusedSparseEncoder(specs, 16, seed=3, mask_padding=mask_padding)
        got, ref, idx, ridx = run_both(O, enc, hb)
        np.testing.assert_array_equal(idx, ridx)
        np.testing.assert_array_equal(bits(got), bits(ref), err_msg=comb)
    one = from_lists([[[b"x"]]])
    enc = FusedSparseEncoder([SlotSpec("a", 5, (1, 2), "sum")], 4, seed=1, mask_padding=mask_padding)
    got, ref, _, _ = run_both(O, enc, one)
    np.testing.assert_array_equal(bits(got), bits(ref))


@pytest.mark.parametrize("tdt,odt", [(torch.float32, torch.float32), (torch.bfloat16, torch.bfloat16),
                                     (torch.bfloat16, torch.float32)])
@pytest.mark.parametrize("dim", [8, 64, 128])
@pytest.mark.parametrize("mask_padding", [False, True])
def test_fused_embed_single_token_items(O, cuda, tdt, odt, dim, mask_padding):
    """Items whose bags hold 0 or 1 token with Lmax = 1 take the lean phase 2 (no emit_idx): bit-exact vs
    the oracle and vs the general path (flag bit 15), every combiner, empty bags, b"" tokens, and a slot
    with one 2-token bag (Lmax = 2: general path) beside them; B spans several 64-example items."""
    rng = np.random.default_rng(dim)
    S, B = 7, 150
    rows = []
    for b in range(B):
        r = []
        for s in range(S):
            n = 2 if (s == 6 and b == 77) else int(rng.random() < 0.8)
            r.append([b"" if rng.random() < 0.05 else b"t%d" % rng.integers(0, 400) for _ in range(n)])
        rows.append(r)
    hb = from_lists(rows)
    assert list(hb.lmax[:6]) == [1] * 6 and hb.lmax[6] == 2
    for comb in COMBS:
        specs = [SlotSpec(f"f{s}", 40 + 13 * s, (s, 7 + s), comb, mask_empty=s != 3) for s in range(S)]
        enc = FusedSparseEncoder(specs, dim, table_dtype=tdt, out_dtype=odt, seed=dim + 1, mask_padding=mask_padding)
        got, ref, _, _ = run_both(O, enc, hb, emit=False)
        np.testing.assert_array_equal(bits(got), bits(ref), err_msg=comb)
        enc.extra_flags = 1 << 15
        gen, _, _, _ = run_both(O, enc, hb, emit=False)
        np.testing.assert_array_equal(bits(got), bits(gen), err_msg=comb)


@pytest.mark.parametrize("tdt,odt,dim", [(torch.bfloat16, torch.bfloat16, 64), (torch.bfloat16, torch.bfloat16, 32),
                                         (torch.bfloat16, torch.float32, 128), (torch.float32, torch.float32, 16),
                                         (torch.float32, torch.bfloat16, 64)])
@pytest.mark.parametrize("mask_padding", [False, True])
def test_single_token_kernel(O, cuda, tdt, odt, dim, mask_padding):
    """RF_FLAG_SINGLE_TOKEN (set by the encoder when the batch's host-side Lmax is <= 1): the low-register
    single-token kernel is bit-exact vs the oracle and vs the general kernel, for every combiner, empty
    bags (pad rows / zeros when masked), b"" tokens, unmasked-empty salts, and a slot whose Lmax is 0
    (empty-reduction values). A batch that breaks the promise (a 2-token bag) gets NaN in that slot only."""
    rng = np.random.default_rng(dim)
    S, B = 6, 200
    rows = [[([b"" if rng.random() < 0.05 else b"t%d" % rng.integers(0, 900)] if (s != 5 and rng.random() < 0.85) else [])
             for s in range(S)] for _ in range(B)]
    hb = from_lists(rows)
    assert list(hb.lmax) == [1, 1, 1, 1, 1, 0]
    for comb in COMBS:
        specs = [SlotSpec(f"f{s}", 40 + 13 * s, (s, 7 + s), comb, mask_empty=s != 3) for s in range(S)]
        enc = FusedSparseEncoder(specs, dim, table_dtype=tdt, out_dtype=odt, seed=dim + 1, mask_padding=mask_padding)
        assert enc._single_token_batch(hb)
        got, ref, _, _ = run_both(O, enc, hb, emit=False)
        np.testing.assert_array_equal(bits(got), bits(ref), err_msg=comb)
        enc.single_token = False
        gen, _, _, _ = run_both(O, enc, hb, emit=False)
        np.testing.assert_array_equal(bits(got), bits(gen), err_msg=comb)
    rows[17][2] = [b"a", b"b"]
    bad = from_lists(rows).to("cuda")
    out = torch.empty((B, enc.out_width), dtype=odt, device="cuda")
    L.call("rf_fused_hash_embed_fwd", L.ptr(enc.desc), S, L.ptr(bad.tok_bytes), L.ptr(bad.tok_off), L.ptr(bad.bag_off),
           L.ptr(bad.lmax), B, L.ptr(enc.table), L.torch_dtype_code(tdt), enc.table.shape[0], dim, L.ptr(out),
           L.torch_dtype_code(odt), out.stride(0), L.FLAG_SINGLE_TOKEN | (L.FLAG_MASK_PADDING if mask_padding else 0),
           None, L.stream_ptr())
    o = out.float().cpu().numpy()
    assert np.isnan(o[:, 2 * 2 * dim: 3 * 2 * dim]).all()
    assert not np.isnan(o[:, : 2 * 2 * dim]).any()


@pytest.mark.parametrize("extra", [1 << 11, (1 << 11) | (1 << 15)])
def test_fused_embed_diagnostic_item_order_is_exact(O, cuda, extra):
    """Diagnostic flag bit 11 (slot-interleaved XCD item order, rf_fused.h) only permutes the items: 19
    slots (two full groups of 8 plus a plain-order tail), mixed single/multi-valued, B spanning several
    items — bit-exact vs the oracle and vs the default order."""
    multi = [s % 3 == 0 for s in range(19)]
    hb = synthetic_batch(300, multi, seed=11)
    specs = [SlotSpec(f"f{s}", 50 + 17 * s, (s, 3 + s), COMBS[s % len(COMBS)]) for s in range(19)]
    enc = FusedSparseEncoder(specs, 32, seed=5)
    got, ref, _, _ = run_both(O, enc, hb, emit=False)
    np.testing.assert_array_equal(bits(got), bits(ref))
    enc.extra_flags = extra
    alt, _, _, _ = run_both(O, enc, hb, emit=False)
    np.testing.assert_array_equal(bits(alt), bits(got))


def test_double_hashing_embedding_api(O, cuda):
    with pytest.raises(ValueError):
        DoubleHashingEmbedding(0, 8, [1, 2], "sum")
    d = DoubleHashingEmbedding(3000, 16, [2022, 2023], "sum", mask_value="", mask_zero=True, name="hashing_app_id")
    rows = [[b"com.example.app", b"12345"], [b"12345"], [b""]]
    out = d(rows).cpu().numpy()
    T = d.table.cpu().numpy()
    # ("com.example.app" -> (750, 2359), "12345" -> (2693, 606)), padding -> bin 0
    np.testing.assert_array_equal(out[0, :16], T[750] + T[2693])
    np.testing.assert_array_equal(out[0, 16:], T[3000 + 2359] + T[3000 + 606])
    np.testing.assert_array_equal(out[1, :16], T[2693] + T[0])
    np.testing.assert_array_equal(out[2, :16], T[0] + T[0])
    # int seed -> [s, s + 7] (D-int-seed)
    assert DoubleHashingEmbedding(10, 4, 5, "sum").seeds == [5, 12]
    nul = DoubleHashingEmbedding(3000, 16, [2022, 2023], "null", mask_value="", name="hashing_app_id")
    x = nul(rows)
    assert tuple(x.shape) == (3, 4, 16)
    with pytest.raises(ValueError):
        DoubleHashingEmbedding(10, 4, 5, "median")(rows)


@pytest.mark.parametrize("comb", COMBS + ["null"])
def test_embedding_bag_ids(O, cuda, comb):
    rng = np.random.default_rng(2)
    for tdt in (torch.float32, torch.bfloat16):
        eb = EmbeddingBag(1000, 32, combiner=comb, dtype=tdt, seed=4)
        ids = rng.integers(0, 1000, (33, 7))
        got = eb(torch.from_numpy(ids).cuda()).reshape(33, -1).cpu()
        T = eb.table.cpu()
        Tn = T.view(torch.int16).numpy().view(np.uint16) if tdt == torch.bfloat16 else T.numpy()
        want = O.embedding_bag(ids, Tn, comb, out_dtype=O.DT_F32 if tdt == torch.float32 else O.DT_BF16)
        g = got.view(torch.int16).numpy().view(np.uint16) if tdt == torch.bfloat16 else got.numpy()
        np.testing.assert_array_equal(bits(g), bits(want))


def test_table_init_bit_exact(O, cuda):
    for dt, code in ((torch.float32, O.DT_F32), (torch.bfloat16, O.DT_BF16)):
        t = torch.empty((1000, 24), dtype=dt, device="cuda")
        L.call("rf_table_init_uniform", L.ptr(t), L.torch_dtype_code(dt), 1000, 24, 3, 5, 1234, -0.05, 0.05, L.stream_ptr())
        g = t.cpu().view(torch.int16).numpy().view(np.uint16) if dt == torch.bfloat16 else t.cpu().numpy()
        want = O.table_init_uniform(1000, 24, code, seed=1234, row0=3, row_stride=5)
        np.testing.assert_array_equal(bits(g), bits(want))


def test_cfg2_full_size_parity(O, cuda):
    """BASELINE cfg2 at full size: 229 slots of base_recall_sdpa.yaml, fused 10M x 64 fp32 table, B=4096.
    Every bucket id and every pooled value bit-exact vs the C oracle."""
    import os

    from recommendflow_amd.config_parser.configuration import Configuration

    conf = Configuration(os.path.join(os.path.dirname(__file__), "golden", "conf", "base_recall_sdpa.yaml"))
    feats = conf.features.hashing_features
    n_bins = 10_000_000 // (2 * len(feats))
    specs = [SlotSpec(f.name, n_bins, tuple(f.hash_seeds), f.pooling.value) for f in feats]
    enc = FusedSparseEncoder(specs, 64, seed=2023)
    hb = synthetic_batch(4096, [bool(f.multivalued) for f in feats], seed=1234)
    got, ref, idx, ridx = run_both(O, enc, hb)
    np.testing.assert_array_equal(idx, ridx)
    np.testing.assert_array_equal(bits(got), bits(ref))
    assert idx.min() >= 1 and idx.max() < n_bins
