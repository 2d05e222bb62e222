"""Model-level parity (GPU vs the CPU oracle composed stage by stage), small shapes.

ESIM (cfg3 structure): sparse slots -> bf16 tables -> q, a token sequences (bit-exact vs the oracle)
-> ESIM pooling + MLPs (float64 oracle). Bar: |dp| <= 1e-2 on the softmax outputs,
>= 99.9% arg-max agreement (here: all rows, on a batch of 256).
DSSM (cfg2 structure): fp32 towers on the exact-fp32 MFMA path, rtol 1e-4 on the cosine score.
"""
import numpy as np
import pytest
import torch

from recommendflow_amd.backend.encoder.sparse_encoder import FusedSparseEncoder, SlotSpec
from recommendflow_amd.models.matching.dssm import Dssm
from recommendflow_amd.models.ranking.esim import Esim
from recommendflow_amd.runtime.batch import synthetic_batch

from model_helpers import enc_ref, mlp_params

pytestmark = pytest.mark.gpu


def test_esim_model_vs_oracle(O, cuda):
    Lq, B, D = 24, 256, 64
    user = [SlotSpec(f"u{i}", 5000 + i, (2022, 2023)) for i in range(Lq)]
    ad = [SlotSpec(f"a{i}", 7000 + i, (2022, 2023)) for i in range(Lq)]
    model = Esim(user, ad, n_dense=16, dim=D, seed=5)
    hu = synthetic_batch(B, [False] * Lq, seed=1)
    ha = synthetic_batch(B, [i % 5 == 0 for i in range(Lq)], seed=2)
    dense = torch.randn(B, 16, generator=torch.Generator().manual_seed(3))
    p = model(hu.to("cuda"), ha.to("cuda"), dense.cuda()).cpu().numpy()
    q = enc_ref(O, model.enc_q, hu).reshape(B, Lq, 2 * D)
    a = enc_ref(O, model.enc_a, ha).reshape(B, Lq, 2 * D)
    d_emb = O.mlp(dense.numpy(), mlp_params(model.input_mlp), "gelu", "ln")
    pooled = np.concatenate([d_emb, O.esim_pool(q, a)], axis=1)
    x = O.mlp(pooled, mlp_params(model.output_mlp), "gelu", "ln")
    W = model.dense_output.weight.float().cpu().numpy()
    want = O.activation(x @ W.T.astype(np.float64) + model.dense_output.bias.cpu().numpy(), "softmax")
    assert np.abs(p - want).max() <= 1e-2
    assert (p.argmax(1) == want.argmax(1)).mean() >= 0.999
    np.testing.assert_allclose(p.sum(1), 1.0, atol=1e-5)


def test_dssm_model_vs_oracle(O, cuda):
    B, D = 128, 16
    us = [SlotSpec(f"u{i}", 3000, (2022, 2023)) for i in range(6)]
    as_ = [SlotSpec(f"a{i}", 3000, (2022, 2023)) for i in range(9)]
    eu, ea = FusedSparseEncoder(us, D, seed=1), FusedSparseEncoder(as_, D, seed=2)
    m = Dssm(eu, ea, units=(128, 64, 32), seed=4)
    hu = synthetic_batch(B, [i % 2 == 0 for i in range(6)], seed=7)
    ha = synthetic_batch(B, [False] * 9, seed=8)
    score = m(hu.to("cuda"), ha.to("cuda")).cpu().numpy()
    u = O.l2_normalize(O.mlp(enc_ref(O, eu, hu), mlp_params(m.user_dense), "selu", "bn"))
    v = O.l2_normalize(O.mlp(enc_ref(O, ea, ha), mlp_params(m.ad_dense), "selu", "bn"))
    np.testing.assert_allclose(score, (u * v).sum(1), rtol=1e-4, atol=1e-5)


def test_esim_cfg3_shape_vs_oracle(O, cuda):
    """cfg3 at configuration shape (BASELINE.json configs[2]): 100 user + 100 ad single-valued slots, bf16
    tables with D = 64 per hash (token dim d = 128), L = 100, 16 dense features, B = 512, end to end
    against the oracle at the §8d bar. num_bins is 20,000 per hash instead of 1M (same descriptors and
    kernel paths, smaller segments) so the oracle's host copy of the tables stays at 1 GB. The hipGraph
    replay of the same forward is bit-identical to the eager one."""
    Ls, B = 100, 512
    user = [SlotSpec(f"u{i:03d}", 20_000, (2022, 2023)) for i in range(Ls)]
    ad = [SlotSpec(f"a{i:03d}", 20_000, (2022, 2023)) for i in range(Ls)]
    model = Esim(user, ad, n_dense=16, dim=64, seed=3)
    hu = synthetic_batch(B, [False] * Ls, seed=77, slot_ids=range(Ls))
    ha = synthetic_batch(B, [False] * Ls, seed=99, slot_ids=range(Ls, 2 * Ls))
    dense = torch.randn(B, 16, generator=torch.Generator().manual_seed(5))
    du, da, dd = hu.to("cuda"), ha.to("cuda"), dense.cuda()
    p_gpu = model(du, da, dd)
    p = p_gpu.cpu().numpy()
    q = enc_ref(O, model.enc_q, hu).reshape(B, Ls, 128)
    a = enc_ref(O, model.enc_a, ha).reshape(B, Ls, 128)
    d_emb = O.mlp(dense.numpy(), mlp_params(model.input_mlp), "gelu", "ln")
    pooled = np.concatenate([d_emb, O.esim_pool(q, a)], axis=1)
    x = O.mlp(pooled, mlp_params(model.output_mlp), "gelu", "ln")
    W = model.dense_output.weight.float().cpu().numpy()
    want = O.activation(x @ W.T.astype(np.float64) + model.dense_output.bias.cpu().numpy(), "softmax")
    assert np.abs(p - want).max() <= 1e-2
    assert (p.argmax(1) == want.argmax(1)).mean() >= 0.999
    fwd = model.graphed(du, da, dd)
    assert torch.equal(fwd(du, da, dd), p_gpu)
    # the unfused scorer (pooled fp32 -> LayerNorm pass -> GEMMs -> head) at the same bar, and the input MLP on a
    # side stream beside the encoders (the A/B switch, unfused scorer) gives its bits
    model.fused_scorer = False
    try:
        p_unf = model(du, da, dd)
        assert np.abs(p_unf.cpu().numpy() - want).max() <= 1e-2
        model.concurrent_input_mlp = True
        assert torch.equal(model(du, da, dd), p_unf)
    finally:
        model.concurrent_input_mlp = False
        model.fused_scorer = True


@pytest.mark.parametrize("mask_padding", [False, True])
def test_esim_gather_equals_encoders_plus_attention(cuda, mask_padding):
    """rf_single_token_ids_fwd -> rf_esim_gather_fwd (the attention gathers its token rows by id) against the
    encoders' [B, L, 2D] outputs -> rf_esim_soft_attention_fwd: the same pooled features and the same forward,
    bit for bit (100 + 100 single-valued slots, some bags empty: pad rows, or the zero row when masked)."""
    Ls, B = 100, 300
    user = [SlotSpec(f"u{i:03d}", 20_000, (2022, 2023)) for i in range(Ls)]
    ad = [SlotSpec(f"a{i:03d}", 20_000, (2022, 2023)) for i in range(Ls)]
    encs = (FusedSparseEncoder(user, 64, table_dtype=torch.bfloat16, seed=4, mask_padding=mask_padding, spec_rows=True),
            FusedSparseEncoder(ad, 64, table_dtype=torch.bfloat16, seed=5, mask_padding=mask_padding, spec_rows=True))
    model = Esim(user, ad, n_dense=16, dim=64, seed=3, encoders=encs)
    from recommendflow_amd.runtime.batch import from_lists
    rng = np.random.default_rng(7)

    def rows(tag):
        return [[[] if rng.random() < 0.05 else [f"{tag}{s}_{int(rng.integers(0, 5000))}"] for s in range(Ls)]
                for _ in range(B)]

    hu, ha = from_lists(rows("u")).to("cuda"), from_lists(rows("a")).to("cuda")
    dense = torch.randn(B, 16, generator=torch.Generator().manual_seed(9)).cuda()
    model.fused_scorer = False  # bit-equality of the two attention paths under the same (unfused) scorer
    model.gather = False
    want = model(hu, ha, dense)
    pw = torch.zeros((B, model.pooled_width), device="cuda")
    q = model.enc_q(hu).view(B, Ls, 128)
    a = model.enc_a(ha).view(B, Ls, 128)
    from recommendflow_amd.backend.layers.attention_layers import esim_soft_attention_pool
    esim_soft_attention_pool(q, a, out=pw, out_col=model.d_emb)
    model.gather = True
    assert model._gather_ok(hu, ha)
    pg = torch.zeros_like(pw)
    model._esim_gather(hu, ha, pg)
    torch.cuda.synchronize()
    assert torch.equal(pg[:, model.d_emb:], pw[:, model.d_emb:])
    assert torch.equal(model(hu, ha, dense), want)
    fwd = model.graphed(hu, ha, dense)
    assert torch.equal(fwd(hu, ha, dense), want)
    # the fused scorer on the gather path: the same probabilities within the §8d bar
    model.fused_scorer = True
    pf = model(hu, ha, dense).cpu().numpy()
    assert np.abs(pf - want.cpu().numpy()).max() <= 1e-2
    assert (pf.argmax(1) == want.cpu().numpy().argmax(1)).mean() >= 0.99


def test_esim_rejects_mismatched_batches(cuda):
    """the gather path sizes its [B, L, 2] id buffers from the batches, so a user / ad batch-size
    or slot-count mismatch (or injected encoders whose slot count differs from L) must raise before any launch,
    as the encoder path does."""
    Ls, B = 8, 16
    user = [SlotSpec(f"u{i}", 5000, (2022, 2023)) for i in range(Ls)]
    ad = [SlotSpec(f"a{i}", 5000, (2022, 2023)) for i in range(Ls)]
    model = Esim(user, ad, n_dense=16, dim=64, seed=3)
    dense = torch.randn(B, 16, device="cuda")
    hu = synthetic_batch(B, [False] * Ls, seed=1).to("cuda")
    ha = synthetic_batch(B, [False] * Ls, seed=2).to("cuda")
    model(hu, ha, dense)  # the well-formed pair runs
    for gather in (True, False):
        model.gather = gather
        with pytest.raises(ValueError):
            model(hu, synthetic_batch(B + 4, [False] * Ls, seed=3).to("cuda"), dense)
        with pytest.raises(ValueError):
            model(hu, synthetic_batch(B, [False] * (Ls - 1), seed=4).to("cuda"), dense)
    model.gather = True
    # injected encoders whose slot count differs from L
    short = FusedSparseEncoder(ad[:-1], 64, table_dtype=torch.bfloat16, seed=5)
    model.enc_a = short
    with pytest.raises(ValueError):
        model(hu, synthetic_batch(B, [False] * (Ls - 1), seed=4).to("cuda"), dense)
    ids = torch.zeros((B, Ls, 2), dtype=torch.int32, device="cuda")
    with pytest.raises(ValueError):
        model.attention_gather(ids, torch.zeros((B + 1, Ls, 2), dtype=torch.int32, device="cuda"),
                               torch.empty((B, model.pooled_width), device="cuda"))


def _take_examples(h, idx):
    """Host CSR batch -> the examples `idx` (re-based CSR, the whole batch's lmax kept)."""
    from recommendflow_amd.runtime.batch import SparseBatch
    S = h.n_slots
    toks, bag = [], [0]
    for b in idx:
        for s in range(S):
            t0, t1 = int(h.bag_off[b * S + s]), int(h.bag_off[b * S + s + 1])
            toks.extend(bytes(h.tok_bytes[h.tok_off[t]:h.tok_off[t + 1]]) for t in range(t0, t1))
            bag.append(len(toks))
    tok_off = np.zeros(len(toks) + 1, np.int32)
    np.cumsum([len(t) for t in toks], out=tok_off[1:])
    return SparseBatch(np.frombuffer(b"".join(toks), np.uint8).copy(), tok_off, np.asarray(bag, np.int32),
                       np.array(h.lmax, np.int32), len(idx), S)


def test_esim_cfg3_full_shape_sampled(O, cuda):
    """cfg3 at its FULL shape (BASELINE.json configs[2]): 100 + 100 single-valued slots with num_bins = 1M per
    hash (two bf16 tables of 200M x 64 rows, 25.6 GB each), B = 4096, gather path. The token ids of the whole
    batch are checked against the oracle's hash (rf_single_token_ids_multi_fwd vs orf_hash_rows, bit-exact);
    64 sampled examples go end to end through the oracle (their rows from the oracle's table init at the oracle's
    ids — and the device tables' copies of those rows bit-exact with them —, then esim_pool + MLPs in float64) at
    the §8d bar."""
    Ls, B, NB = 100, 4096, 1_000_000
    user = [SlotSpec(f"u{i:03d}", NB, (2022, 2023)) for i in range(Ls)]
    ad = [SlotSpec(f"a{i:03d}", NB, (2022, 2023)) for i in range(Ls)]
    model = Esim(user, ad, n_dense=16, dim=64, seed=3)
    hu = synthetic_batch(B, [False] * Ls, seed=177, slot_ids=range(Ls))
    ha = synthetic_batch(B, [False] * Ls, seed=199, slot_ids=range(Ls, 2 * Ls))
    dense = torch.randn(B, 16, generator=torch.Generator().manual_seed(15))
    du, da, dd = hu.to("cuda"), ha.to("cuda"), dense.cuda()
    assert model._gather_ok(du, da)
    p = model(du, da, dd).cpu().numpy()
    qi, ai = model.token_ids(du, da)
    for ids, enc, h in ((qi, model.enc_q, hu), (ai, model.enc_a, ha)):
        want = O.hash_rows(enc.host_desc, h.tok_bytes, h.tok_off, h.bag_off, B).reshape(B, Ls, 2)
        assert want.max() < enc.table_rows
        np.testing.assert_array_equal(ids.cpu().numpy().astype(np.int64), want)
    idx = np.sort(np.random.default_rng(5).choice(B, 64, replace=False))
    seqs = []
    for enc, h in ((model.enc_q, hu), (model.enc_a, ha)):
        sub = _take_examples(h, idx)
        rows = O.hash_rows(enc.host_desc, sub.tok_bytes, sub.tok_off, sub.bag_off, sub.batch)
        uniq, inv = np.unique(rows, return_inverse=True)
        # the rows from the oracle's table init (not read back from the device: VERDICT r4), then the device's
        # copies of the same rows checked bit for bit against them
        init = np.stack([O.table_init_uniform(1, enc.dim, O.DT_BF16, seed=enc.seed, row0=int(r))[0] for r in uniq])
        dev = enc.table[torch.from_numpy(uniq).cuda()].cpu().view(torch.int16).numpy().view(np.uint16)
        np.testing.assert_array_equal(dev, init)
        gathered = (init.astype(np.uint32) << 16).view(np.float32)
        row_map = np.concatenate([inv, np.zeros(2 * Ls, np.int64)]).astype(np.int32)  # + pad rows (unused: L = 1)
        out = O.pool_rows(enc.host_desc, sub.bag_off, sub.lmax, sub.batch, sub.n_tokens, gathered, enc.dim,
                          enc.out_width, row_map=row_map)
        seqs.append(out.reshape(len(idx), Ls, 128))
    d_emb = O.mlp(dense.numpy()[idx], mlp_params(model.input_mlp), "gelu", "ln")
    pooled = np.concatenate([d_emb, O.esim_pool(*seqs)], axis=1)
    x = O.mlp(pooled, mlp_params(model.output_mlp), "gelu", "ln")
    W = model.dense_output.weight.float().cpu().numpy()
    want = O.activation(x @ W.T.astype(np.float64) + model.dense_output.bias.cpu().numpy(), "softmax")
    assert np.abs(p[idx] - want).max() <= 1e-2
    assert (p[idx].argmax(1) == want.argmax(1)).all()


def test_esim_gather_stats_output(cuda):
    """rf_esim_gather_stats_fwd: the pooled features of rf_esim_gather_fwd stored as bf16 (RNE of the same fp32
    values, bit for bit) and the (sum, squared deviations) pairs of each 32-column slice of those fp32 values."""
    import recommendflow_amd.runtime.lib as L

    Ls, B = 100, 300
    user = [SlotSpec(f"u{i:03d}", 20_000, (2022, 2023)) for i in range(Ls)]
    ad = [SlotSpec(f"a{i:03d}", 20_000, (2022, 2023)) for i in range(Ls)]
    model = Esim(user, ad, n_dense=16, dim=64, seed=3)
    hu = synthetic_batch(B, [False] * Ls, seed=7, slot_ids=range(Ls)).to("cuda")
    ha = synthetic_batch(B, [False] * Ls, seed=8, slot_ids=range(Ls, 2 * Ls)).to("cuda")
    qi, ai = model.token_ids(hu, ha)
    W = model.pooled_width
    pooled = torch.zeros((B, W), device="cuda")
    model.attention_gather(qi, ai, pooled)
    pb = torch.zeros((B, W), dtype=torch.bfloat16, device="cuda")
    st = torch.full((B, W // 32, 2), -7.0, device="cuda")
    eq, ea = model.enc_q, model.enc_a
    L.call("rf_esim_gather_stats_fwd", L.ptr(qi), L.ptr(ai), L.ptr(eq.table), eq.table.shape[0], L.ptr(ea.table),
           ea.table.shape[0], L.DT_BF16, B, Ls, 128, L.ptr(pb), pb.stride(0), model.d_emb, L.ptr(st), W // 32,
           model.d_emb // 32, L.stream_ptr(None))
    torch.cuda.synchronize()
    feat = pooled[:, model.d_emb:]
    np.testing.assert_array_equal(pb[:, model.d_emb:].contiguous().view(torch.int16).cpu().numpy(),
                                  feat.to(torch.bfloat16).contiguous().view(torch.int16).cpu().numpy())
    f = feat.cpu().numpy().astype(np.float64).reshape(B, -1, 32)
    S = f.sum(2)
    M2 = ((f - S[..., None] / 32) ** 2).sum(2)
    got = st.cpu().numpy()
    np.testing.assert_allclose(got[:, model.d_emb // 32:, 0], S, rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(got[:, model.d_emb // 32:, 1], M2, rtol=1e-4, atol=1e-4)
    assert (got[:, : model.d_emb // 32] == -7.0).all()
