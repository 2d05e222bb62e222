"""GPU: the recall -> prerank -> rank cascade (cfg5 wiring, models/cascade.py), every stage against the
float64 oracle."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from recommendflow_amd.backend.encoder.sparse_encoder import FusedSparseEncoder, SlotSpec
from recommendflow_amd.models.cascade import Cascade, gather_rows, topk_rows
from recommendflow_amd.models.matching.dssm import Dssm
from recommendflow_amd.models.ranking.esim import Esim
from recommendflow_amd.runtime.batch import synthetic_batch

from model_helpers import enc_ref, mlp_params

pytestmark = pytest.mark.gpu


def _build(N=3000, B=16, Ls=8):
    user = [SlotSpec(f"u{i}", 5000, (2022, 2023)) for i in range(6)]
    ad = [SlotSpec(f"a{i}", 5000, (2022, 2023)) for i in range(5)]
    dssm = Dssm(FusedSparseEncoder(user, 16, seed=1), FusedSparseEncoder(ad, 16, seed=2), units=(128, 64), seed=3)
    esim = Esim([SlotSpec(f"q{i}", 1000, (7, 8)) for i in range(Ls)], [SlotSpec(f"k{i}", 1000, (7, 8)) for i in range(Ls)],
                n_dense=16, dim=64, seed=4)
    cas = Cascade(dssm, esim, k_recall=100, k_prerank=20, k_final=5, seed=5)
    cat_r = [c.to("cuda") for c in _catalog_recall_batches(N)]
    cat_k = [c.to("cuda") for c in _catalog_rank_batches(Ls, N)]
    cas.index_catalog(cat_r, cat_k)
    ur = synthetic_batch(B, [i % 2 == 0 for i in range(6)], seed=7).to("cuda")
    uk = synthetic_batch(B, [False] * Ls, seed=9, slot_ids=range(300, 300 + Ls)).to("cuda")
    dense = torch.randn(B, 16, device="cuda")
    return cas, ur, uk, dense


def test_topk_rows_and_gather(cuda):
    s = torch.tensor([[0.5, 2.0, 2.0, -1.0], [3.0, 1.0, 0.0, 1.0]], device="cuda")
    v, i = topk_rows(s, 3)
    assert i.cpu().tolist() == [[1, 2, 0], [0, 1, 3]]
    src = torch.arange(40, dtype=torch.float32, device="cuda").view(10, 4)
    assert torch.equal(gather_rows(src, torch.tensor([[3, 0], [9, 3]], device="cuda")), src[[3, 0, 9, 3]])


def test_cascade_stages(cuda):
    """Every stage against the float64 oracle composed from the ORACLE's encodings (not the model's own
    modules): recall towers + exact inner-product top-100, prerank Dense(64, relu) -> Dense(1) scores and
    their top-20, rank ESIM p(click) (fp16 attention) of the prerank candidates and the best 5 (§8d bar:
    |dp| <= 1e-2; selections equal up to near-ties)."""
    cas, ur, uk, dense = _build()
    res = cas(ur, uk, dense)
    B = ur.batch
    urh, ukh = ur.numpy(), uk.numpy()
    # recall: oracle user tower, exact search over the catalog vectors
    un = O.l2_normalize(O.mlp(enc_ref(O, cas.recall.enc_u, urh), mlp_params(cas.recall.user_dense), "selu", "bn"), eps=1e-6)
    with torch.no_grad():
        ug = torch.nn.functional.normalize(cas.recall.user_dense(cas.recall.enc_u(ur)), dim=-1, eps=1e-6).cpu().numpy()
    np.testing.assert_allclose(ug, un, rtol=1e-4, atol=1e-5)
    items = np.concatenate([O.l2_normalize(O.mlp(enc_ref(O, cas.recall.enc_a, c), mlp_params(cas.recall.ad_dense), "selu",
                                                 "bn"), eps=1e-6) for c in _catalog_recall_batches()])
    np.testing.assert_allclose(cas.searcher.index.cpu().numpy(), items, rtol=1e-4, atol=1e-5)
    want_s, _ = O.flat_search(un, items, 100)
    got1 = res.recall_items.cpu().numpy()
    np.testing.assert_allclose((un[:, None, :] * items[got1]).sum(-1), want_s, rtol=1e-4, atol=1e-5)
    # prerank: float64 scores of the recall candidates, top-20 (ties within the fp32 error excepted)
    p1, p2 = cas.pre1, cas.pre2
    W1, b1 = p1.weight.cpu().numpy().T.astype(np.float64), p1.bias.cpu().numpy()
    W2, b2 = p2.weight.cpu().numpy().T.astype(np.float64), p2.bias.cpu().numpy()
    s2 = (np.maximum((un[:, None, :] * items[got1]) @ W1 + b1, 0.0) @ W2 + b2)[..., 0]  # [B, 100]
    got2 = res.prerank_items.cpu().numpy()
    pos = {b: {int(i): k for k, i in enumerate(got1[b])} for b in range(B)}
    for b in range(B):
        srt = np.sort(s2[b])[::-1]
        kth = srt[19]
        sel = np.array([s2[b, pos[b][int(i)]] for i in got2[b]])
        assert np.all(sel >= kth - 1e-5), b  # every selected candidate is within tolerance of the top 20
        assert np.all(np.diff(sel) <= 1e-5), b  # in descending order
    # rank: oracle encodings of the user / item sequences (bf16 tables -> fp16 operands, exact), ESIM + MLPs
    rk = cas.ranker
    q = enc_ref(O, rk.enc_q, ukh).reshape(B, rk.L, rk.d)
    cat = np.concatenate([enc_ref(O, rk.enc_a, c.numpy()) for c in _catalog_rank_batches(rk.L)]).reshape(-1, rk.L, rk.d)
    np.testing.assert_array_equal(cat.astype(np.float16), cas.a_item.cpu().numpy().reshape(cat.shape))
    d_emb = O.mlp(dense.cpu().numpy(), mlp_params(rk.input_mlp), "gelu", "ln")
    Wo = rk.dense_output.weight.float().cpu().numpy().T.astype(np.float64)
    bo = rk.dense_output.bias.cpu().numpy()
    got3, s3 = res.items.cpu().numpy(), res.scores.cpu().numpy()
    for b in range(B):
        qa = np.repeat(q[b:b + 1], 20, axis=0)
        pooled = np.concatenate([np.repeat(d_emb[b:b + 1], 20, axis=0), O.esim_pool(qa, cat[got2[b]])], axis=1)
        p = O.activation(O.mlp(pooled, mlp_params(rk.output_mlp), "gelu", "ln") @ Wo + bo, "softmax")[:, 1]
        pmap = {int(i): p[k] for k, i in enumerate(got2[b])}
        np.testing.assert_allclose(s3[b], [pmap[int(i)] for i in got3[b]], atol=1e-2, rtol=0)
        assert min(pmap[int(i)] for i in got3[b]) >= np.sort(p)[::-1][4] - 2e-2, b
    assert torch.all(res.scores[:, :-1] >= res.scores[:, 1:])


def _catalog_recall_batches(N=3000):
    return [synthetic_batch(1000, [False] * 5, seed=50 + i, slot_ids=range(100, 105)) for i in range(N // 1000)]


def _catalog_rank_batches(Ls, N=3000):
    return [synthetic_batch(1000, [False] * Ls, seed=80 + i, slot_ids=range(200, 200 + Ls)) for i in range(N // 1000)]


def test_sharded_cascade_p1_equals_cascade(cuda):
    """ShardedCascade (recall towers on row-sharded tables, collective catalog index; LocalComm at P = 1)
    gives exactly the single-table Cascade's candidates and scores."""
    from recommendflow_amd.backend.encoder.sharded_encoder import LocalComm, ShardedFusedEncoder
    from recommendflow_amd.models.cascade import ShardedCascade

    cas, ur, uk, dense = _build()
    want = cas(ur, uk, dense)
    user = [SlotSpec(f"u{i}", 5000, (2022, 2023)) for i in range(6)]
    ad = [SlotSpec(f"a{i}", 5000, (2022, 2023)) for i in range(5)]
    comm = LocalComm()
    scas = ShardedCascade(cas.recall, cas.ranker, ShardedFusedEncoder(user, 16, 0, 1, comm=comm, seed=1),
                          ShardedFusedEncoder(ad, 16, 0, 1, comm=comm, seed=2), comm, k_recall=100, k_prerank=20,
                          k_final=5, seed=5)
    scas.index_catalog([c.to("cuda") for c in _catalog_recall_batches()],
                       [c.to("cuda") for c in _catalog_rank_batches(cas.ranker.L)])
    assert torch.equal(scas.searcher.index, cas.searcher.index)
    got = scas(ur, uk, dense)
    for f in ("recall_items", "prerank_items", "items", "scores"):
        assert torch.equal(getattr(got, f), getattr(want, f)), f
