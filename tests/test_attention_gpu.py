"""Parity of the reference's generic attention operators against the float64 oracle:

* SelfAttention (attention_layers.py:83-134): PE on q and k, shared relu(xW), query-row mask filled with
  -4294967295, softmax over keys, @ v, mean over the sequence;
* MultiHeadAttention.call (attention_layers.py:137-168): Dense q/k/v with bias (fp32, as the reference),
  split heads, row-masked SDPA, merge, no output projection.

Tolerance (stated): the attention core runs fp16 MFMA operands (cfg5) with fp32 logits,
softmax and accumulation, so outputs match the float64 oracle to |Δ| ≤ 5e-3 absolute for O(1) inputs;
the bf16 option to 3e-2. Projections are exact-fp32 MFMA (rtol 1e-5 vs float64 on their own).
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _mask(B, Ln, seed, full_row_example=0):
    m = (torch.rand(B, Ln, 1, generator=torch.Generator().manual_seed(seed)) > 0.3).float()
    m[full_row_example] = 0.0  # an example whose every query row is masked (uniform over keys)
    return m


@pytest.mark.parametrize("B,Ln,dim,add_pos", [(4, 20, 64, True), (3, 100, 128, True), (5, 7, 32, False)])
def test_self_attention_vs_oracle(cuda, B, Ln, dim, add_pos):
    from recommendflow_amd.backend.layers.attention_layers import SelfAttention

    g = torch.Generator().manual_seed(B * 100 + Ln)
    q, k, v = (torch.randn(B, Ln, dim, generator=g) for _ in range(3))
    mask = _mask(B, Ln, Ln)
    sa = SelfAttention(add_pos=add_pos, seed=3)
    got = sa([q.cuda(), k.cuda(), v.cuda(), mask.cuda()]).cpu().numpy()
    W = sa.W.weight.float().cpu().numpy().T  # [dim_in, dim_out], the Keras kernel layout
    want = O.self_attention(q.numpy(), k.numpy(), v.numpy(), mask.numpy(), W, add_pos=add_pos)
    assert got.shape == (B, dim)
    np.testing.assert_allclose(got, want, atol=5e-3, rtol=0)
    # example 0: every query row masked -> each row is the plain mean of v, so the result is mean(v)
    np.testing.assert_allclose(got[0], v[0].numpy().mean(axis=0), atol=2e-3)


def test_self_attention_projection_is_fp32(cuda):
    """The shared relu(xW) runs in fp32 like the reference's tf.matmul (no bf16 rounding of q, k)."""
    from recommendflow_amd.backend.layers.attention_layers import SelfAttention

    sa = SelfAttention(add_pos=False, seed=1)
    sa.build(64)
    assert sa.W.weight.dtype == torch.float32
    x = torch.randn(50, 64, generator=torch.Generator().manual_seed(2))
    got = sa.W(x.cuda()).cpu().numpy()
    want = np.maximum(x.numpy().astype(np.float64) @ sa.W.weight.cpu().numpy().T.astype(np.float64), 0)
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("B,Ln,d_model,heads,dtype,tol",
                         [(2, 20, 128, 4, torch.float16, 5e-3), (3, 64, 256, 2, torch.float16, 5e-3),
                          (2, 33, 96, 3, torch.float16, 5e-3), (2, 20, 128, 4, torch.bfloat16, 3e-2)])
def test_multi_head_attention_vs_oracle(cuda, B, Ln, d_model, heads, dtype, tol):
    from recommendflow_amd.backend.layers.attention_layers import MultiHeadAttention

    g = torch.Generator().manual_seed(d_model + heads)
    q, k, v = (torch.randn(B, Ln, d_model, generator=g) for _ in range(3))
    mask = _mask(B, Ln, heads)
    mha = MultiHeadAttention(d_model, heads, dtype=dtype, seed=2)
    for dl in (mha.wq, mha.wk, mha.wv):  # non-zero biases exercise the bias path
        dl.bias.copy_(torch.randn(d_model, generator=g).cuda() * 0.1)
    got = mha.call(q.cuda(), k.cuda(), v.cuda(), mask.cuda()).cpu().numpy()
    P = [(dl.weight.cpu().numpy().T, dl.bias.cpu().numpy()) for dl in (mha.wq, mha.wk, mha.wv)]
    want = O.multi_head_attention(q.numpy(), k.numpy(), v.numpy(), mask.numpy(), P[0][0], P[0][1], P[1][0], P[1][1],
                                  P[2][0], P[2][1], heads)
    assert got.shape == (B, Ln, d_model)
    np.testing.assert_allclose(got, want, atol=tol, rtol=0)
    # without a mask
    got = mha.call(q.cuda(), k.cuda(), v.cuda(), None).cpu().numpy()
    want = O.multi_head_attention(q.numpy(), k.numpy(), v.numpy(), None, P[0][0], P[0][1], P[1][0], P[1][1], P[2][0],
                                  P[2][1], heads)
    np.testing.assert_allclose(got, want, atol=tol, rtol=0)


def test_multi_head_attention_projections_fp32(cuda):
    from recommendflow_amd.backend.layers.attention_layers import MultiHeadAttention

    mha = MultiHeadAttention(128, 4, seed=5)
    assert all(dl.weight.dtype == torch.float32 for dl in (mha.wq, mha.wk, mha.wv))


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("L,d", [(100, 128), (37, 64)])
def test_esim_pool_idx_equals_materialised_pairs(cuda, dtype, L, d):
    """rf_esim_soft_attention_idx_fwd (pairs by index: q example e // q_rep, a row a_rows[e]) writes the same pooled
    bits as rf_esim_soft_attention_fwd over the expanded q and the gathered a."""
    from recommendflow_amd.backend.layers.attention_layers import esim_soft_attention_pool, esim_soft_attention_pool_idx

    g = torch.Generator(device="cuda").manual_seed(L + d)
    Bq, rep, N = 23, 7, 300
    q = (torch.randn((Bq, L, d), device="cuda", generator=g) * 0.5).to(dtype)
    cat = (torch.randn((N, L, d), device="cuda", generator=g) * 0.5).to(dtype)
    rows = torch.randint(0, N, (Bq * rep,), device="cuda", generator=g)
    want = esim_soft_attention_pool(q.repeat_interleave(rep, dim=0).contiguous(), cat[rows].contiguous())
    got = torch.empty((Bq * rep, 6 * d + 16), device="cuda")
    esim_soft_attention_pool_idx(q, rep, cat, rows, out=got, out_col=16)
    assert torch.equal(got[:, 16:], want)


def test_esim_pool_idx_rejects_rows_outside_the_catalog(cuda):
    """A pair whose catalog row is outside [0, N) (negative, N, far past the table) reads nothing and gets NaN
    features; every other pair keeps its exact values (the device-side check of rf_esim_soft_attention_idx_fwd)."""
    from recommendflow_amd.backend.layers.attention_layers import esim_soft_attention_pool_idx

    g = torch.Generator(device="cuda").manual_seed(11)
    Bq, rep, N, L, d = 5, 4, 50, 20, 64
    q = (torch.randn((Bq, L, d), device="cuda", generator=g) * 0.5).to(torch.float16)
    cat = (torch.randn((N, L, d), device="cuda", generator=g) * 0.5).to(torch.float16)
    rows = torch.randint(0, N, (Bq * rep,), device="cuda", generator=g)
    want = torch.empty((Bq * rep, 6 * d), device="cuda")
    esim_soft_attention_pool_idx(q, rep, cat, rows, out=want)
    bad = rows.clone()
    bad[[1, 6, 13]] = torch.tensor([-1, N, 1 << 40], device="cuda")
    got = torch.empty_like(want)
    esim_soft_attention_pool_idx(q, rep, cat, bad, out=got)
    torch.cuda.synchronize()
    ok = torch.ones(Bq * rep, dtype=torch.bool)
    ok[[1, 6, 13]] = False
    assert torch.equal(got[ok.cuda()], want[ok.cuda()])
    assert torch.isnan(got[~ok.cuda()]).all()
