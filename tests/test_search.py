"""Recall search: rf_topk_merge exact selection, FaissSearcher Flat ip/cos vs the float64
oracle, recall metrics (eval_utils.py:85-147)."""
import numpy as np
import pytest

from oracle import oracle as O
from recommendflow_amd.backend.utils.eval_utils import MISS, get_click_index


def test_click_index_intended_semantics():
    rec = np.array([[5, 7, 9], [1, 2, 3], [4, 4, 8], [2, 1, 0]])
    lab = np.array([5, 3, 8, 1])
    assert get_click_index(rec, lab).tolist() == [0, 2, 2, 1]
    assert get_click_index(rec, np.array([6, 6, 6, 6])).tolist() == [MISS] * 4


def test_recall_metrics_formula():
    from recommendflow_amd.backend.utils import eval_utils as E

    class Fake:
        def search(self, t, k):
            return (np.array([[1, 2, 3]] * len(t))[:, :k], None)

    hit, mrr, ndcg = E.batch_compute_recall_score(Fake(), np.zeros((4, 2)), np.array([1, 2, 3, 9]), [1, 3], np.ones(4), 2)
    assert np.allclose(hit, [0.25, 0.75])
    assert np.isclose(mrr[0], (1 + 1 / 2 + 1 / 3 + 1 / (MISS + 1)) / 4)
    # click ids [0, 1, 2, MISS]; the reference's simplified idcg = 1 / log2(3) for every hit
    assert np.isclose(ndcg[1], (np.log2(3) + 1 + 0.5 * np.log2(3)) / 4, rtol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("cols,k,k_prev", [(1, 2, 2), (100, 10, 10), (3000, 64, 200), (40, 8, 8)])
def test_topk_merge_unsorted_prev(cuda, cols, k, k_prev):
    """`prev` is any set (rf_api.h): an UNSORTED running list with k_prev >= k must not floor out new keys
    that belong in the top-k (k=2, prev={1,5}, new 3 -> {5,3})."""
    import torch

    from recommendflow_amd.runtime import lib as L

    rng = np.random.default_rng(cols * 7 + k)
    B = 9
    s = rng.standard_normal((B, cols)).astype(np.float32)
    prev_v = rng.standard_normal((B, k_prev)).astype(np.float32)
    prev_i = (rng.permutation(10 ** 6)[: B * k_prev].reshape(B, k_prev) + 10 ** 7).astype(np.int64)
    # rows 0/1: ascending (worst case for a floor read from position k-1); others: shuffled
    prev_v[0] = np.sort(prev_v[0])
    prev_v[1] = np.sort(prev_v[1])
    if cols == 1:  # the advisor's case: prev {1, 5}, new score 3
        prev_v[:, :2] = [1.0, 5.0]
        s[:, 0] = 3.0
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    ov = torch.empty((B, k), device="cuda")
    oi = torch.empty((B, k), dtype=torch.int64, device="cuda")
    # keep the device copies alive until the kernel has run (an inline temporary is freed at once and
    # its block handed to the next argument by the caching allocator)
    ds, pv, pi = dev(s), dev(prev_v), dev(prev_i)
    L.call("rf_topk_merge", L.ptr(ds), cols, B, cols, k, 0, L.ptr(pv), L.ptr(pi), k_prev, k_prev,
           L.ptr(ov), L.ptr(oi), k, L.stream_ptr())
    torch.cuda.synchronize()
    gv, gi = ov.cpu().numpy(), oi.cpu().numpy()
    for b in range(B):
        cand = [(float(s[b, c]), c) for c in range(cols)] + [(float(prev_v[b, j]), int(prev_i[b, j])) for j in range(k_prev)]
        cand.sort(key=lambda x: (-x[0], x[1]))
        assert gi[b].tolist() == [w[1] for w in cand[:k]], b
        assert gv[b].tolist() == [w[0] for w in cand[:k]], b
    if cols == 1:
        assert gv[0].tolist() == [5.0, 3.0]


@pytest.mark.gpu
@pytest.mark.parametrize("cols,k", [(1, 1), (100, 10), (5000, 100), (32768, 1024), (700, 1024)])
def test_topk_merge_exact(cuda, cols, k):
    import torch

    from recommendflow_amd.runtime import lib as L

    rng = np.random.default_rng(cols + k)
    B = 37
    s = (rng.integers(-50, 50, (B, cols)) * 0.25).astype(np.float32)  # many exact ties
    s[3, : min(cols, 5)] = np.nan
    prev_v = np.sort((rng.integers(-50, 50, (B, k)) * 0.25).astype(np.float32), axis=1)[:, ::-1].copy()
    prev_i = rng.permutation(10 ** 6)[: B * k].reshape(B, k).astype(np.int64) + 10 ** 7
    prev_i[5, k // 2:] = -1
    base = 123456
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    ov = torch.empty((B, k), device="cuda")
    oi = torch.empty((B, k), dtype=torch.int64, device="cuda")
    ds, pv, pi = dev(s), dev(prev_v), dev(prev_i)
    L.call("rf_topk_merge", L.ptr(ds), cols, B, cols, k, base, L.ptr(pv), L.ptr(pi), k, k, L.ptr(ov), L.ptr(oi), k, L.stream_ptr())
    gv, gi = ov.cpu().numpy(), oi.cpu().numpy()
    for b in range(B):
        cand = [(float(s[b, c]), base + c) for c in range(cols) if not np.isnan(s[b, c])]
        cand += [(float(prev_v[b, j]), int(prev_i[b, j])) for j in range(k) if prev_i[b, j] >= 0]
        cand.sort(key=lambda x: (-x[0], x[1]))
        want = cand[:k] + [(-np.inf, -1)] * (k - len(cand[:k]))
        assert gi[b].tolist() == [w[1] for w in want], b
        assert gv[b].tolist() == [w[0] for w in want], b


@pytest.mark.gpu
@pytest.mark.parametrize("cols,k", [(100, 10), (5000, 100), (32768, 200), (32768, 1024), (3000, 1024)])
def test_topk_merge_chained(cuda, cols, k):
    """A running top-k written by the kernel itself (sorted keys: the merge-path branch) folded with a
    second block, including a row whose second block holds nothing above the running k-th entry."""
    import torch

    from recommendflow_amd.runtime import lib as L

    rng = np.random.default_rng(cols * 7 + k)
    B = 29
    s1 = (rng.integers(-50, 50, (B, cols)) * 0.25).astype(np.float32)
    s2 = (rng.integers(-60, 50, (B, cols)) * 0.25).astype(np.float32)
    s2[4] = -1e30  # nothing enters
    s2[7, : min(cols, 9)] = np.nan
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    v1 = torch.empty((B, k), device="cuda")
    i1 = torch.empty((B, k), dtype=torch.int64, device="cuda")
    v2, i2 = torch.empty_like(v1), torch.empty_like(i1)
    d1, d2 = dev(s1), dev(s2)
    L.call("rf_topk_merge", L.ptr(d1), cols, B, cols, k, 0, None, None, 0, k, L.ptr(v1), L.ptr(i1), k, L.stream_ptr())
    L.call("rf_topk_merge", L.ptr(d2), cols, B, cols, k, cols, L.ptr(v1), L.ptr(i1), k, k, L.ptr(v2), L.ptr(i2), k,
           L.stream_ptr())
    gv, gi = v2.cpu().numpy(), i2.cpu().numpy()
    for b in range(B):
        cand = [(float(s1[b, c]), c) for c in range(cols)] + \
               [(float(s2[b, c]), cols + c) for c in range(cols) if not np.isnan(s2[b, c])]
        cand.sort(key=lambda x: (-x[0], x[1]))
        want = cand[:k] + [(-np.inf, -1)] * (k - len(cand[:k]))
        assert gi[b].tolist() == [w[1] for w in want], b
        assert gv[b].tolist() == [w[0] for w in want], b


@pytest.mark.gpu
@pytest.mark.parametrize("measurement", ["ip", "cos"])
def test_flat_searcher_vs_oracle(cuda, measurement):
    from recommendflow_amd.backend.third_party_components.faiss_searcher import FaissSearcher

    rng = np.random.default_rng(7)
    N, E, B, k = 70000, 64, 300, 50  # 3 item blocks
    items = rng.normal(size=(N, E)).astype(np.float32)
    q = rng.normal(size=(B, E)).astype(np.float32)
    names = np.array([f"item{i}" for i in range(N)])
    s = FaissSearcher(items=items, item_list=names, index_param="Flat", measurement=measurement).train()
    got_items, got_d = s.search(q, k)
    want_d, want_i = O.flat_search(q, items, k, cos=measurement == "cos")
    np.testing.assert_allclose(got_d, want_d, rtol=1e-4, atol=1e-4)
    # identical lists except where two oracle scores are closer than the fp32 GEMM error
    tol = 1e-4 * np.abs(want_d).max()
    for b in range(B):
        g = [int(x[4:]) for x in got_items[b]]
        if g != want_i[b].tolist():
            gaps = np.diff(want_d[b])
            assert np.abs(gaps).min() < tol or abs(want_d[b, -1] - O.flat_search(q[b:b + 1], items, k + 1)[0][0, -1]) < tol, b
    res = s.search(q, [5, 20], keep_rank_no=True)
    assert res[5][0].shape == (B, 5) and res[20][2].shape == (B, 20)


@pytest.mark.gpu
def test_searcher_fewer_items_than_k(cuda):
    from recommendflow_amd.backend.third_party_components.faiss_searcher import FaissSearcher

    items = np.eye(4, 8, dtype=np.float32)
    s = FaissSearcher(items=items, index_param="Flat", measurement="ip").train()
    d, i = s.search_index(np.ones((2, 8), np.float32), 6)
    assert i.cpu().tolist() == [[0, 1, 2, 3, -1, -1]] * 2
    assert d[0, 4].item() == -np.inf


@pytest.mark.gpu
def test_recall_score_on_gpu_searcher(cuda):
    from recommendflow_amd.backend.third_party_components.faiss_searcher import FaissSearcher
    from recommendflow_amd.backend.utils.eval_utils import batch_compute_recall_score

    rng = np.random.default_rng(3)
    items = rng.normal(size=(5000, 32)).astype(np.float32)
    labels = rng.integers(0, 5000, 400)
    q = items[labels] + 0.5 * rng.normal(size=(400, 32)).astype(np.float32)
    s = FaissSearcher(items=items, index_param="Flat", measurement="cos").train()
    hit, mrr, ndcg = batch_compute_recall_score(s, q, labels, [1, 10, 50], np.ones(400), 128)
    _, idx = O.flat_search(q, items, 50, cos=True)
    ci = get_click_index(idx, labels)
    for j, kk in enumerate([1, 10, 50]):
        assert abs(hit[j] - (ci < kk).mean()) <= 2 / 400
    assert 0 < hit[0] <= hit[1] <= hit[2] <= 1


@pytest.mark.gpu
@pytest.mark.parametrize("C,d,norm", [(1, 8, True), (3, 256, True), (4, 100, False), (16, 64, True)])
def test_attention_fusion_vs_oracle(cuda, C, d, norm):
    import torch

    from recommendflow_amd.backend.layers.fusion_layers import AttentionFusion

    rng = np.random.default_rng(C * d)
    xs = [torch.tensor(rng.normal(size=(333, d)), dtype=torch.float32).cuda() for _ in range(C)]
    af = AttentionFusion(d, C, is_norm=norm, seed=C)
    out = af(xs).cpu().numpy()
    want, att = O.attention_fusion([x.cpu().numpy() for x in xs], af.W.cpu().numpy(), norm)
    np.testing.assert_allclose(out, want, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(af.attention.cpu().numpy(), att, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(af.get_fusion_weights(), att.sum(0, keepdims=True) / att.sum(), rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("cols,k", [(100, 10), (5000, 200), (20000, 1024)])
def test_topk_merge_idx_explicit_indices(cuda, cols, k):
    """rf_topk_merge_idx: the block's item indices come from col_idx (any order, NaN-padded tail), ties by item index."""
    import torch

    from recommendflow_amd.runtime import lib as L

    rng = np.random.default_rng(cols * 3 + k)
    B = 11
    s = (rng.integers(-40, 40, (B, cols)) * 0.5).astype(np.float32)  # many exact ties
    idx = np.stack([rng.permutation(10 ** 7)[:cols] for _ in range(B)]).astype(np.uint32)
    s[2, cols // 3:] = np.nan  # a short candidate list
    prev_v = np.sort((rng.integers(-40, 40, (B, k)) * 0.5).astype(np.float32), axis=1)[:, ::-1].copy()
    prev_i = (rng.permutation(10 ** 6)[: B * k].reshape(B, k) + 2 * 10 ** 7).astype(np.int64)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    ds, di = dev(s), dev(idx.view(np.int32))
    pv, pi = dev(prev_v), dev(prev_i)
    ov = torch.empty((B, k), device="cuda")
    oi = torch.empty((B, k), dtype=torch.int64, device="cuda")
    L.call("rf_topk_merge_idx", L.ptr(ds), L.ptr(di), cols, B, cols, k, L.ptr(pv), L.ptr(pi), k, k, L.ptr(ov), L.ptr(oi), k,
           L.stream_ptr())
    gv, gi = ov.cpu().numpy(), oi.cpu().numpy()
    for b in range(B):
        cand = [(float(s[b, c]), int(idx[b, c])) for c in range(cols) if not np.isnan(s[b, c])]
        cand += [(float(prev_v[b, j]), int(prev_i[b, j])) for j in range(k)]
        cand.sort(key=lambda x: (-x[0], x[1]))
        assert gi[b].tolist() == [w[1] for w in cand[:k]], b
        assert gv[b].tolist() == [w[0] for w in cand[:k]], b


@pytest.mark.gpu
def test_ip_candidates_exact(cuda):
    """rf_ip_candidates_f32 keeps exactly the pairs whose rf_linear_fwd score (the same kernel's bits) is >= the row's
    threshold, with those scores and item indices col_base + n, and counts them."""
    import torch

    from recommendflow_amd.runtime import lib as L

    g = torch.Generator(device="cuda").manual_seed(5)
    B, N, E, base = 200, 50000, 256, 70000
    q = torch.randn((B, E), device="cuda", generator=g)
    items = torch.randn((N, E), device="cuda", generator=g)
    full = torch.empty((B, N), device="cuda")
    L.call("rf_linear_fwd", L.ptr(q), L.DT_F32, B, E, E, L.ptr(items), N, None, 0, L.ptr(full), N, L.stream_ptr())
    thr = torch.quantile(full[:, :4096], 0.995, dim=1).contiguous()
    thr[3] = float("inf")  # nothing passes
    cap = 1024
    count = torch.zeros(B, dtype=torch.int32, device="cuda")
    cval = torch.full((B, cap), float("nan"), device="cuda")
    cidx = torch.empty((B, cap), dtype=torch.int32, device="cuda")
    L.call("rf_ip_candidates_f32", L.ptr(q), E, B, L.ptr(items), N, E, L.ptr(thr), cap, L.ptr(count), L.ptr(cval),
           L.ptr(cidx), base, L.stream_ptr())
    f, t = full.cpu().numpy(), thr.cpu().numpy()
    cnt, cv, ci = count.cpu().numpy(), cval.cpu().numpy(), cidx.cpu().numpy().view(np.uint32)
    for b in range(B):
        want = np.nonzero(f[b] >= t[b])[0]
        assert cnt[b] == len(want), b
        assert cnt[b] <= cap
        got = ci[b, : cnt[b]].astype(np.int64) - base
        order = np.argsort(got)
        np.testing.assert_array_equal(got[order], want)
        np.testing.assert_array_equal(cv[b, : cnt[b]][order].view(np.uint32), f[b, want].view(np.uint32))
        assert np.isnan(cv[b, cnt[b]:]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("K,M,N", [(256, 300, 50000 + 37), (128, 1024, 20000 + 5), (64, 77, 9000 + 1), (256, 300, 100)])
def test_ip_candidates_bf16_screen(cuda, K, M, N):
    """rf_ip_candidates_bf16 (the query-stationary kernel at K = 64 / 128 / 256) keeps every pair whose bf16-operand
    score is >= thr[row] - qbound[row] vnorm[col] and no other: against float64 dot products of the same bf16 values,
    within the fp32 accumulation error of unit rows (1e-4), with each kept pair's score, its index col_base + n, and
    counts equal to the kept entries. Ragged query blocks and item tiles, a row nothing passes, a catalog shorter than
    one tile per workgroup."""
    import torch

    from recommendflow_amd.runtime import lib as L

    g = torch.Generator(device="cuda").manual_seed(K + M)
    q = torch.randn((M, K), device="cuda", generator=g)
    q = q / q.norm(dim=1, keepdim=True)
    items = torch.randn((N, K), device="cuda", generator=g)
    items = items / items.norm(dim=1, keepdim=True)
    qb, ib = q.to(torch.bfloat16).contiguous(), items.to(torch.bfloat16).contiguous()
    ref = qb.double() @ ib.double().t()
    thr = torch.quantile(ref[:, : min(N, 4096)].float(), 0.99, dim=1).contiguous()
    thr[1] = float("inf")  # nothing passes
    qbound = (q.norm(dim=1) * 0.008).contiguous()
    vn = items.norm(dim=1).contiguous()
    cap, base = 2048, 123457
    count = torch.zeros(M, dtype=torch.int32, device="cuda")
    cval = torch.full((M, cap), float("nan"), device="cuda")
    cidx = torch.empty((M, cap), dtype=torch.int32, device="cuda")
    L.call("rf_ip_candidates_bf16", L.ptr(qb), K, M, L.ptr(ib), N, K, L.ptr(thr), L.ptr(qbound), L.ptr(vn), cap,
           L.ptr(count), L.ptr(cval), L.ptr(cidx), base, L.stream_ptr())
    t = (thr.double()[:, None] - qbound.double()[:, None] * vn.double()[None, :]).cpu().numpy()
    r = ref.cpu().numpy()
    cnt, cv, ci = count.cpu().numpy(), cval.cpu().numpy(), cidx.cpu().numpy().view(np.uint32)
    eps = 1e-4
    assert cnt[1] == 0
    for row in range(M):
        assert cnt[row] <= cap, row
        got = ci[row, : cnt[row]].astype(np.int64) - base
        assert len(np.unique(got)) == len(got) and (got >= 0).all() and (got < N).all(), row
        must = np.nonzero(r[row] >= t[row] + eps)[0]
        assert np.isin(must, got).all(), row
        assert (r[row, got] >= t[row, got] - eps).all(), row
        np.testing.assert_allclose(cv[row, : cnt[row]], r[row, got], rtol=0, atol=eps)
        assert np.isnan(cv[row, cnt[row]:]).all()
    assert cnt.sum() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 50, 200, 1024])
@pytest.mark.parametrize("dups", [False, True])
def test_screened_search_equals_block_loop(cuda, k, dups):
    """The screened Flat search returns the block loop's top-k bit for bit (values, indices, tie order): 3 full
    item blocks + a tail, E = 256; with duplicated item rows every score ties with another item's."""
    from recommendflow_amd.backend.third_party_components.faiss_searcher import FaissSearcher

    rng = np.random.default_rng(k + 1000 * dups)
    N, E, B = 3 * 32768 + 5000, 256, 300
    items = rng.normal(size=(N, E)).astype(np.float32)
    if dups:
        items[1::2] = items[0::2][: N // 2]
    q = rng.normal(size=(B, E)).astype(np.float32)
    s = FaissSearcher(items=items, index_param="Flat", measurement="ip").train()
    s.screen = False
    want_v, want_i = [t.cpu().numpy() for t in s.search_index(q, k)]
    s.screen = True
    got_v, got_i = [t.cpu().numpy() for t in s.search_index(q, k)]
    np.testing.assert_array_equal(got_i, want_i)
    np.testing.assert_array_equal(got_v.view(np.uint32), want_v.view(np.uint32))


@pytest.mark.gpu
def test_screened_search_overflow_falls_back(cuda):
    """Every item identical: every candidate list overflows its cap, and the block loop answers."""
    from recommendflow_amd.backend.third_party_components.faiss_searcher import FaissSearcher

    N, E, B, k = 2 * 32768 + 300, 256, 8, 10
    items = np.ones((N, E), np.float32)
    q = np.random.default_rng(2).normal(size=(B, E)).astype(np.float32)
    s = FaissSearcher(items=items, index_param="Flat", measurement="ip").train()
    v, i = [t.cpu().numpy() for t in s.search_index(q, k)]
    assert (i == np.arange(k)[None, :]).all()  # all tie: the smallest item indices
    assert np.allclose(v, q.sum(1, keepdims=True), rtol=1e-5, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("K", [256, 512])
def test_ip_rescore_matches_linear_fwd_bits(cuda, K):
    """rf_ip_rescore_f32 (order 0) reproduces rf_linear_fwd's fp32 scores bit for bit on random candidate pairs."""
    import torch

    from recommendflow_amd.runtime import lib as L

    g = torch.Generator(device="cuda").manual_seed(K)
    B, N, cap = 48, 30000, 1500
    q = torch.randn((B, K), device="cuda", generator=g)
    items = torch.randn((N, K), device="cuda", generator=g)
    full = torch.empty((B, N), device="cuda")
    L.call("rf_linear_fwd", L.ptr(q), L.DT_F32, B, K, K, L.ptr(items), N, None, 0, L.ptr(full), N, L.stream_ptr())
    idx = torch.stack([torch.randperm(N, generator=torch.Generator().manual_seed(r))[:cap] for r in range(B)]).cuda()
    cidx = idx.to(torch.int32).contiguous()
    count = torch.full((B,), cap, dtype=torch.int32, device="cuda")
    count[3] = 7  # short list: entries past it untouched
    cval = torch.full((B, cap), float("nan"), device="cuda")
    L.call("rf_ip_rescore_f32", L.ptr(q), K, B, L.ptr(items), K, L.ptr(count), cap, L.ptr(cval), L.ptr(cidx), 0,
           L.stream_ptr())
    want = torch.gather(full, 1, idx)
    got = cval.clone()
    assert torch.isnan(got[3, 7:]).all()
    got[3, 7:] = want[3, 7:]
    assert torch.equal(got.view(torch.int32), want.view(torch.int32))


@pytest.mark.gpu
@pytest.mark.parametrize("k", [50, 200])
@pytest.mark.parametrize("dups", [False, True])
def test_bf16_screened_search_equals_block_loop(cuda, k, dups):
    """The bf16 screen (9 blocks + a tail: 4 exact blocks, the rest screened on bf16 copies within the bf16 error
    bound, the kept pairs rescored exactly) returns the block loop's top-k bit for bit."""
    from recommendflow_amd.backend.third_party_components.faiss_searcher import FaissSearcher

    rng = np.random.default_rng(k + 7 * dups)
    N, E, B = 9 * 32768 + 3000, 256, 200
    items = rng.normal(size=(N, E)).astype(np.float32)
    if dups:
        items[5::7] = items[0] * 1.0  # many exact duplicates of one item: score ties across the blocks
    q = rng.normal(size=(B, E)).astype(np.float32)
    s = FaissSearcher(items=items, index_param="Flat", measurement="ip").train()
    s.screen = False
    want_v, want_i = [t.cpu().numpy() for t in s.search_index(q, k)]
    s.screen = True
    got_v, got_i = [t.cpu().numpy() for t in s.search_index(q, k)]
    np.testing.assert_array_equal(got_i, want_i)
    np.testing.assert_array_equal(got_v.view(np.uint32), want_v.view(np.uint32))
