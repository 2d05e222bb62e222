"""GPU: the recall -> prerank -> rank cascade (cfg5 wiring, models/cascade.py) against a float64 / explicit
recomposition of each stage."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from recommendflow_amd.backend.encoder.sparse_encoder import FusedSparseEncoder, SlotSpec
from recommendflow_amd.models.cascade import Cascade, gather_rows, topk_rows
from recommendflow_amd.models.matching.dssm import Dssm
from recommendflow_amd.models.ranking.esim import Esim
from recommendflow_amd.runtime.batch import synthetic_batch

pytestmark = pytest.mark.gpu


def _build(N=3000, B=16, Ls=8):
    user = [SlotSpec(f"u{i}", 5000, (2022, 2023)) for i in range(6)]
    ad = [SlotSpec(f"a{i}", 5000, (2022, 2023)) for i in range(5)]
    dssm = Dssm(FusedSparseEncoder(user, 16, seed=1), FusedSparseEncoder(ad, 16, seed=2), units=(128, 64), seed=3)
    esim = Esim([SlotSpec(f"q{i}", 1000, (7, 8)) for i in range(Ls)], [SlotSpec(f"k{i}", 1000, (7, 8)) for i in range(Ls)],
                n_dense=16, dim=64, seed=4)
    cas = Cascade(dssm, esim, k_recall=100, k_prerank=20, k_final=5, seed=5)
    cat_r = [synthetic_batch(1000, [False] * 5, seed=50 + i, slot_ids=range(100, 105)).to("cuda") for i in range(N // 1000)]
    cat_k = [synthetic_batch(1000, [False] * Ls, seed=80 + i, slot_ids=range(200, 200 + Ls)).to("cuda") for i in range(N // 1000)]
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
    cas, ur, uk, dense = _build()
    res = cas(ur, uk, dense)
    B = ur.batch
    items = cas.searcher.index.cpu().numpy()
    with torch.no_grad():
        u = torch.nn.functional.normalize(cas.recall.user_dense(cas.recall.enc_u(ur)), dim=-1, eps=1e-6)
    un = u.cpu().numpy()
    # recall = exact top-100 inner products (ties / fp32-GEMM near-ties excepted)
    want_s, want_i = O.flat_search(un, items, 100)
    got = res.recall_items.cpu().numpy()
    sc = (un.astype(np.float64)[:, None, :] * items[got].astype(np.float64)).sum(-1)
    np.testing.assert_allclose(sc, want_s, rtol=1e-4, atol=1e-5)
    # prerank = top-20 of the light model on exactly those candidates
    with torch.no_grad():
        x = (u[:, None, :] * cas.searcher.index[res.recall_items]).reshape(B * 100, -1)
        s2 = cas.pre2(cas.pre1(x)).view(B, 100).cpu().numpy()
    for b in range(B):
        order = np.argsort(-s2[b], kind="stable")[:20]
        assert set(got[b][order].tolist()) == set(res.prerank_items[b].cpu().tolist()) or \
            np.sort(s2[b])[::-1][19] - np.sort(s2[b])[::-1][20] < 1e-5
    # rank = ESIM p(click) of the (user, candidate) pairs, best 5
    assert res.items.shape == (B, 5) and res.scores.shape == (B, 5)
    assert torch.all(res.scores[:, :-1] >= res.scores[:, 1:])
    for b in range(B):
        assert set(res.items[b].cpu().tolist()) <= set(res.prerank_items[b].cpu().tolist())
    assert torch.all((res.scores >= 0) & (res.scores <= 1))
