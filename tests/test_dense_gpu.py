"""GPU parity of the dense stages (ESIM soft attention + pooling, Dense/LN/BN MLP, masked SDPA) against
the float64 numpy oracle. Tolerances (stated per test) follow from the MFMA operand rounding:
bf16 operands carry 2^-8 relative error, f16 2^-11; exact-fp32 MFMA ~1e-6 relative."""
import numpy as np
import pytest
import torch

from recommendflow_amd.backend.blocks.mlp import create_mlp
from recommendflow_amd.backend.layers.attention_layers import (MultiHeadAttention, SoftAttention,
                                                               esim_soft_attention_pool)
from recommendflow_amd.backend.layers.core import BatchNormalization, Dense, LayerNormalization
from recommendflow_amd.backend.layers.layer_utils import scaled_dot_product_attention

pytestmark = pytest.mark.gpu


def rnd(shape, seed, scale=1.0, dtype=torch.bfloat16):
    g = torch.Generator().manual_seed(seed)
    return ((torch.rand(shape, generator=g) * 2 - 1) * scale).to(dtype)


@pytest.mark.parametrize("L,d", [(1, 64), (7, 64), (16, 128), (33, 128), (100, 128), (128, 64)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_esim_pool_vs_oracle(O, cuda, L, d, dt):
    B = 9
    # embedding-like magnitudes (pooled hash embeddings sum 2 rows of U(-0.05, 0.05)) and a larger case
    for scale in (0.1, 2.0):
        q, a = rnd((B, L, d), L * 7 + d, scale, dt), rnd((B, L, d), L * 11 + d + 1, scale, dt)
        att = torch.empty((B, 2, L, d), device="cuda")
        got = esim_soft_attention_pool(q.cuda(), a.cuda(), att_out=att).cpu().numpy()
        want = O.esim_pool(q.float().numpy(), a.float().numpy())
        aq, aa = O.soft_attention(q.float().numpy(), a.float().numpy())
        # P is rounded once to the MFMA dtype: |d att| <= 2^-8 * max|v| (bf16), sums of 4L terms / 4L
        tol = (2 ** -7 if dt == torch.bfloat16 else 2 ** -10) * scale
        np.testing.assert_allclose(att[:, 0].cpu().numpy(), aq, atol=tol, rtol=0)
        np.testing.assert_allclose(att[:, 1].cpu().numpy(), aa, atol=tol, rtol=0)
        np.testing.assert_allclose(got, want, atol=tol * (scale + 1), rtol=0)


@pytest.mark.parametrize("L", [1, 15, 16, 17, 33, 48, 64, 65, 80, 97, 100, 112, 113, 127, 128])
@pytest.mark.parametrize("d", [64, 128])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_esim_pool_fast_path(O, cuda, L, d, dt):
    """The pooled-only path (no attention output: the 4-wave two-per-CU kernel, one instantiation per
    16-row tile count) against the float64 oracle; B spans more than one persistent pass of the grid."""
    B = 600 if L in (100, 128) else 37
    for scale in (0.1, 2.0):
        q, a = rnd((B, L, d), L * 13 + d, scale, dt), rnd((B, L, d), L * 17 + d + 3, scale, dt)
        got = esim_soft_attention_pool(q.cuda(), a.cuda()).cpu().numpy()
        want = O.esim_pool(q.float().numpy(), a.float().numpy())
        tol = (2 ** -7 if dt == torch.bfloat16 else 2 ** -10) * scale
        np.testing.assert_allclose(got, want, atol=tol * (scale + 1), rtol=0)


@pytest.mark.parametrize("L,d", [(33, 64), (100, 128), (17, 64)])
def test_esim_many_examples_per_workgroup(O, cuda, L, d):
    """The persistent kernel's v6 loop (the next example's images staged beside this example's statistics
    reduction; d = 64 at odd tile counts stages past-the-image chunks into the dummy area): B = 3000 gives
    every workgroup 3 - 6 examples; pooled features against the float64 oracle at the ESIM bar, written at
    an out_col offset with the head columns untouched."""
    B, scale, head = 3000, 0.5, 24
    q, a = rnd((B, L, d), L + 2 * d, scale), rnd((B, L, d), L + 2 * d + 5, scale)
    out = torch.full((B, head + 6 * d), 7.0, device="cuda")
    esim_soft_attention_pool(q.cuda(), a.cuda(), out=out, out_col=head)
    got = out.cpu().numpy()
    assert (got[:, :head] == 7.0).all()
    want = O.esim_pool(q.float().numpy(), a.float().numpy())
    np.testing.assert_allclose(got[:, head:], want, atol=2 ** -7 * scale * (scale + 1), rtol=0)


def test_esim_strided_views(O, cuda):
    """q and a as slices of one [B, 200, 128] token tensor (cfg3: 100 user + 100 ad slots)."""
    x = rnd((6, 200, 128), 5, 0.1).cuda()
    got = esim_soft_attention_pool(x[:, :100], x[:, 100:]).cpu().numpy()
    xf = x.float().cpu().numpy()
    want = O.esim_pool(xf[:, :100], xf[:, 100:])
    np.testing.assert_allclose(got, want, atol=2e-3, rtol=0)


def test_soft_attention_api(O, cuda):
    q, a = rnd((3, 10, 64), 1, 0.5), rnd((3, 10, 64), 2, 0.5)
    aq, aa = SoftAttention()([q.cuda(), a.cuda()])
    wq, wa = O.soft_attention(q.float().numpy(), a.float().numpy())
    np.testing.assert_allclose(aq.cpu().numpy(), wq, atol=4e-3)
    np.testing.assert_allclose(aa.cpu().numpy(), wa, atol=4e-3)


@pytest.mark.parametrize("M,K,N", [(1, 16, 256), (129, 64, 130), (256, 1280, 1024), (300, 512, 2), (64, 8704, 48),
                                   (1000, 1024, 512), (4100, 256, 300), (4096, 1280, 1024)])
@pytest.mark.parametrize("act", [None, "gelu", "relu", "selu", "softmax"])
def test_dense_bf16(O, cuda, M, K, N, act):
    if act == "softmax" and N > 64:
        pytest.skip("softmax head needs N <= 64")
    x = rnd((M, K), M + K, 1.0)
    dense = Dense(K, N, activation=act, dtype=torch.bfloat16, seed=N)
    y = dense(x.cuda()).cpu().numpy()
    W = dense.weight.float().cpu().numpy()
    want = O.activation(x.float().numpy().astype(np.float64) @ W.T.astype(np.float64) + dense.bias.cpu().numpy(), act)
    # operands are exact in bf16; only fp32 accumulation error remains: ~K * 2^-24 * sum|xw|
    bound = 1e-5 * np.abs(x.float().numpy()) @ np.abs(W.T) + 1e-6
    np.testing.assert_array_less(np.abs(y - want), bound * 4 + 1e-5)


@pytest.mark.parametrize("M,K,N", [(1, 4, 1), (300, 512, 2), (4097, 1000, 16), (77, 64, 48)])
@pytest.mark.parametrize("act", [None, "gelu", "softmax"])
@pytest.mark.parametrize("wdt", [torch.bfloat16, torch.float32])
def test_dense_head_fp32_activations(O, cuda, M, K, N, act, wdt):
    """rf_dense_head_fwd (Dense with N <= 16 or a softmax head on fp32 x, e.g. esim.py:53's Dense(2,
    'softmax') after the output MLP): fp32 products of x and the (bf16-stored) weights, fp32 sums."""
    if not (N <= 16 or act == "softmax"):
        pytest.skip("wider non-softmax layers take the MFMA GEMM (bf16 operands)")
    x = (torch.rand((M, K), generator=torch.Generator().manual_seed(M + K)) * 2 - 1).float()
    dense = Dense(K, N, activation=act, dtype=wdt, seed=N + 7, bias=torch.linspace(-0.5, 0.5, N))
    y = dense(x.cuda()).cpu().numpy()
    W = dense.weight.float().cpu().numpy().astype(np.float64)
    want = O.activation(x.numpy().astype(np.float64) @ W.T + dense.bias.cpu().numpy(), act)
    np.testing.assert_allclose(y, want, rtol=1e-5, atol=2e-6 * np.sqrt(K))


@pytest.mark.parametrize("M,K,N", [(100, 32, 64), (257, 8704, 1024), (64, 20480, 256), (4096, 8704, 1024),
                                   (4096, 20480, 1024), (300, 2052, 100)])
@pytest.mark.parametrize("route", ["librf", "blaslt"])
def test_dense_fp32_exact_mfma(O, cuda, M, K, N, route, monkeypatch):
    """cfg2 towers run in fp32 (the reference's dtype): rtol 1e-5 / atol 1e-6 vs float64. route
    "librf" (the default): every shape runs rf_gemm_f32 (asserted: its launch counter moves, torch.addmm / mm are
    never called); "blaslt": the A/B switch (RF_TOWER_BLASLT_WIDE=1) sends K >= 4096 to hipBLASLt."""
    from recommendflow_amd.backend.layers import core
    from recommendflow_amd.runtime import gemm as G

    monkeypatch.setattr(core, "_BLASLT_WIDE", route == "blaslt")
    if route == "librf":
        def refuse(*a, **k):
            raise AssertionError("a vendor GEMM ran on the librf route")
        monkeypatch.setattr(torch, "addmm", refuse)
        monkeypatch.setattr(torch, "mm", refuse)
    x = rnd((M, K), K, 0.5, torch.float32)
    dense = Dense(K, N, activation="selu", dtype=torch.float32, seed=1, bias=torch.linspace(-0.3, 0.3, N))
    n0 = G.calls
    y = dense(x.cuda()).cpu().numpy()
    assert (G.calls - n0 == 1) == (route == "librf" or K < 4096), (route, G.calls - n0)
    W = dense.weight.cpu().numpy().astype(np.float64)
    want = O.activation(x.numpy().astype(np.float64) @ W.T + dense.bias.cpu().numpy(), "selu")
    np.testing.assert_allclose(y, want, rtol=1e-5, atol=1e-6 * np.sqrt(K))
    y2 = dense(x.cuda()).cpu().numpy()
    assert np.array_equal(y, y2)  # fixed partial order: replays are bit-identical


@pytest.mark.parametrize("cols", [16, 200, 256, 1024, 1280, 1400, 1536, 2048, 2050, 3000, 4100, 8704, 20480, 32768, 32772])
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("odt", [torch.float32, torch.bfloat16])
def test_norm_rows(O, cuda, cols, mode, odt):
    """rf_norm_fwd against float64 LayerNorm / BatchNorm-inference: BatchNorm's per-column float4 kernel
    (any width), LayerNorm's one-wave register rows (<= 2048), workgroup-per-row wide rows (<= 32768:
    the DSSM tower inputs 8704 / 20480), and the scalar path (2050, 3000, 32772, a misaligned view)."""
    from recommendflow_amd.backend.layers.core import Norm

    spec = LayerNormalization(epsilon=1e-6) if mode == 0 else BatchNormalization(epsilon=1e-3)
    nm = Norm(spec, cols)
    g = torch.Generator().manual_seed(cols + mode)
    nm.gamma.copy_(torch.rand(cols, generator=g) + 0.5)
    nm.beta.copy_(torch.randn(cols, generator=g))
    if mode == 1:
        nm.mean.copy_(torch.randn(cols, generator=g))
        nm.var.copy_(torch.rand(cols, generator=g) + 0.1)
    base = (torch.randn(67, cols + 4, generator=g) * 3 + 1).cuda()
    for x in (base[:, :cols], base[:, 1: cols + 1]):  # 16-byte aligned rows, then a misaligned view
        y = nm(x, out_dtype=odt).float().cpu().numpy()
        xn = x.cpu().numpy().astype(np.float64)
        if mode == 0:
            want = O.layer_norm(xn, nm.gamma.cpu().numpy(), nm.beta.cpu().numpy(), 1e-6)
        else:
            want = O.batch_norm_infer(xn, nm.gamma.cpu().numpy(), nm.beta.cpu().numpy(), nm.mean.cpu().numpy(),
                                      nm.var.cpu().numpy(), 1e-3)
        tol = 1e-4 if odt == torch.float32 else 2e-2
        np.testing.assert_allclose(y, want, rtol=tol, atol=tol)


@pytest.mark.parametrize("M,K0,H,O_", [(4100, 16, 256, 512), (1, 5, 128, 200), (37, 32, 256, 64), (300, 16, 128, 1024)])
def test_mlp2_small_fused(O, cuda, M, K0, H, O_):
    """rf_mlp2_small_fwd (the ESIM input_mlp in one launch) against the float64 create_mlp oracle, and
    against the layer-by-layer rf_norm_fwd -> rf_linear_fwd chain; written into a strided column slice."""
    from recommendflow_amd.backend.blocks.mlp import create_mlp as cm

    mlp = cm([H, O_], 0.3, "gelu", LayerNormalization(epsilon=1e-6), in_features=K0, dtype=torch.bfloat16, seed=K0 + H)
    g = torch.Generator().manual_seed(M)
    for nm in mlp.norms:
        nm.gamma.copy_(torch.rand(nm.width, generator=g) + 0.5)
        nm.beta.copy_(torch.randn(nm.width, generator=g) * 0.1)
    for dn in mlp.denses:
        dn.bias.copy_(torch.randn(dn.units, generator=g) * 0.1)
    x = (torch.randn(M, K0, generator=g) * 2 + 0.5).cuda()
    assert mlp._fusable(x)
    big = torch.full((M, O_ + 40), float("nan"), device="cuda")
    y = mlp(x, out=big[:, 20: 20 + O_]).cpu().numpy()
    assert torch.isnan(big[:, :20]).all() and torch.isnan(big[:, 20 + O_:]).all()
    h = x if K0 % 8 == 0 else None  # the unfused chain (its bf16 GEMM needs 16-byte rows)
    for nm, dn in zip(mlp.norms, mlp.denses):
        h = dn(nm(h, out_dtype=torch.bfloat16)) if h is not None else None
    params = [{"W": dn.weight.float().cpu().numpy().T, "b": dn.bias.cpu().numpy(), "gamma": nm.gamma.cpu().numpy(),
               "beta": nm.beta.cpu().numpy()} for nm, dn in zip(mlp.norms, mlp.denses)]
    want = O.mlp(x.cpu().numpy(), params, "gelu", "ln")
    np.testing.assert_allclose(y, want, rtol=2e-2, atol=2e-2)
    if h is not None:
        np.testing.assert_allclose(y, h.cpu().numpy(), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("norm", ["ln", "bn"])
def test_create_mlp(O, cuda, norm):
    spec = LayerNormalization(epsilon=1e-6) if norm == "ln" else BatchNormalization(epsilon=1e-6)
    mlp = create_mlp([256, 128], 0.3, "gelu" if norm == "ln" else "selu", spec, in_features=200,
                     dtype=torch.float32, seed=3)
    x = rnd((50, 200), 9, 1.0, torch.float32)
    y = mlp(x.cuda()).cpu().numpy()
    layers = []
    for nm, dn in zip(mlp.norms, mlp.denses):
        layers.append({"W": dn.weight.cpu().numpy().T, "b": dn.bias.cpu().numpy(), "gamma": nm.gamma.cpu().numpy(),
                       "beta": nm.beta.cpu().numpy(), "mean": None if nm.mean is None else nm.mean.cpu().numpy(),
                       "var": None if nm.var is None else nm.var.cpu().numpy()})
    want = O.mlp(x.numpy(), layers, "gelu" if norm == "ln" else "selu", norm)
    np.testing.assert_allclose(y, want, rtol=1e-4, atol=1e-5)


def test_mlp_batchnorm_folded_into_fp32_dense(O, cuda):
    """fp32 layers behind a BatchNormalization run as one GEMM with the normalisation folded into the weights
    (MLP._bn_folded): against float64 BN -> Dense with non-trivial statistics, and again after the BN
    parameters change in place (the fold cache must notice)."""
    mlp = create_mlp([96, 40], 0.3, "selu", BatchNormalization(epsilon=1e-3), in_features=200, dtype=torch.float32, seed=5)
    g = torch.Generator().manual_seed(11)
    x = rnd((70, 200), 12, 2.0, torch.float32)

    def randomise():
        for nm in mlp.norms:
            nm.gamma.copy_(torch.rand(nm.width, generator=g) + 0.5)
            nm.beta.copy_(torch.randn(nm.width, generator=g) * 0.3)
            nm.mean.copy_(torch.randn(nm.width, generator=g) * 0.5)
            nm.var.copy_(torch.rand(nm.width, generator=g) * 2 + 0.1)
        for dn in mlp.denses:
            dn.bias.copy_(torch.randn(dn.units, generator=g) * 0.1)

    for _ in range(2):
        randomise()
        y = mlp(x.cuda()).cpu().numpy()
        layers = [{"W": dn.weight.cpu().numpy().T, "b": dn.bias.cpu().numpy(), "gamma": nm.gamma.cpu().numpy(),
                   "beta": nm.beta.cpu().numpy(), "mean": nm.mean.cpu().numpy(), "var": nm.var.cpu().numpy()}
                  for nm, dn in zip(mlp.norms, mlp.denses)]
        np.testing.assert_allclose(y, O.mlp(x.numpy(), layers, "selu", "bn", eps=1e-3), rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("Lq,Lk,depth,heads", [(10, 10, 64, 2), (100, 100, 32, 4), (37, 200, 128, 1), (1, 5, 64, 3)])
def test_sdpa_masked_rows(O, cuda, Lq, Lk, depth, heads):
    B = 3
    q, k, v = (rnd((B, L_, heads * depth), s, 1.0, torch.float16) for s, L_ in ((1, Lq), (2, Lk), (3, Lk)))
    mask = (torch.rand(B, Lq, generator=torch.Generator().manual_seed(4)) > 0.3).float()
    got = scaled_dot_product_attention(q.cuda(), k.cuda(), v.cuda(), mask.cuda(), heads=heads).cpu().numpy()
    qs = q.float().numpy().reshape(B, Lq, heads, depth).transpose(0, 2, 1, 3)
    ks = k.float().numpy().reshape(B, Lk, heads, depth).transpose(0, 2, 1, 3)
    vs = v.float().numpy().reshape(B, Lk, heads, depth).transpose(0, 2, 1, 3)
    m = np.broadcast_to(mask.numpy()[:, None, :], (B, heads, Lq))
    want = O.sdpa(qs, ks, vs, m).transpose(0, 2, 1, 3).reshape(B, Lq, heads * depth)
    np.testing.assert_allclose(got, want, atol=3e-3, rtol=0)
    # fully masked query rows are uniform over the keys (the -4294967295 fill, A.9)
    b, i = np.argwhere(mask.numpy() == 0)[0]
    np.testing.assert_allclose(got[b, i], vs[b].mean(axis=1).reshape(-1), atol=2e-3)


def test_multi_head_attention_api(O, cuda):
    mha = MultiHeadAttention(128, 4, seed=2)
    x = rnd((2, 20, 128), 8, 1.0, torch.float32).cuda()
    out = mha.call(x, x, x, None)
    assert tuple(out.shape) == (2, 20, 128) and torch.isfinite(out).all()


@pytest.mark.parametrize("mean", [0.0, 40.0, 1000.0])
def test_ln_fold_row_stats_large_mean(cuda, mean):
    """rf_linear_stats_fwd's per-slice (S_p, M2_p) and the Chan combine of rf_linear_lnfold_fwd's prologue
    (restated here in float64 over the kernel's own partials) against the float64 mean / variance of the same
    GEMM's fp32 output (rf_linear_fwd, identical accumulation): rows whose mean is 1000x their spread keep a
    relative variance error <= 1e-4 (fp32 slice sums), where a single sum-of-squares pass (sumsq / K - mu^2)
    would be off by tens of percent."""
    import recommendflow_amd.runtime.lib as L

    M, K, N = 256, 512, 600  # N % 128 != 0: a partial last column tile (slices with n_p < 32 and n_p = 0)
    g = torch.Generator().manual_seed(11)
    x = (torch.randn(M, K, generator=g) * 0.5).to(torch.bfloat16).cuda()
    W = (torch.randn(N, K, generator=g) * 0.04).to(torch.bfloat16).cuda()
    b = (torch.full((N,), mean) + torch.randn(N, generator=g) * 0.1).cuda()
    yb = torch.empty((M, N), dtype=torch.bfloat16, device="cuda")
    P = 4 * ((N + 127) // 128)
    st = torch.empty((M, P, 2), dtype=torch.float32, device="cuda")
    L.call("rf_linear_stats_fwd", L.ptr(x), M, K, x.stride(0), L.ptr(W), N, L.ptr(b), L.ACT["relu"], L.ptr(yb),
           yb.stride(0), L.ptr(st), L.stream_ptr(None))
    y = torch.empty((M, N), dtype=torch.float32, device="cuda")
    L.call("rf_linear_fwd", L.ptr(x), L.DT_BF16, M, K, x.stride(0), L.ptr(W), N, L.ptr(b), L.ACT["relu"], L.ptr(y),
           y.stride(0), L.stream_ptr(None))
    torch.cuda.synchronize()
    y64 = y.cpu().numpy().astype(np.float64)
    S = st[..., 0].cpu().numpy().astype(np.float64)
    M2 = st[..., 1].cpu().numpy().astype(np.float64)
    n = np.clip(N - 32 * np.arange(P), 0, 32).astype(np.float64)
    mu = S.sum(1) / N
    ok = n > 0
    var = (M2[:, ok] + (S[:, ok] - n[ok] * mu[:, None]) ** 2 / n[ok]).sum(1) / N
    np.testing.assert_allclose(mu, y64.mean(1), rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(var, y64.var(1), rtol=1e-4)
    assert (S[:, ~ok] == 0).all() and (M2[:, ~ok] == 0).all()


@pytest.mark.parametrize("M", [300, 4096])
def test_mlp_layernorm_folded_across_gemms(O, cuda, M):
    """A bf16 LayerNorm MLP whose second LayerNorm is folded across the GEMM pair (rf_linear_stats_fwd ->
    rf_linear_lnfold_fwd: row sums from the first GEMM's epilogue, the normalisation applied after the
    second product): against float64 create_mlp at the unfused path's tolerance, and against the unfused
    chain (LN -> bf16 -> GEMM) of the same module; cfg3's output-MLP shapes."""
    mlp = create_mlp([1024, 512], 0.3, "gelu", LayerNormalization(epsilon=1e-6), in_features=1280, dtype=torch.bfloat16,
                     seed=7)
    g = torch.Generator().manual_seed(M)
    for nm in mlp.norms:
        nm.gamma.copy_(torch.rand(nm.width, generator=g) + 0.5)
        nm.beta.copy_(torch.randn(nm.width, generator=g) * 0.2)
    for dn in mlp.denses:
        dn.bias.copy_(torch.randn(dn.units, generator=g) * 0.1)
    x = (torch.randn(M, 1280, generator=g) * 1.5 + 0.3).cuda()
    assert mlp._ln_pair_ok(0, mlp.norms[0](x))
    y = mlp(x).cpu().numpy()
    mlp.fold_ln = False
    y_unfused = mlp(x).cpu().numpy()
    params = [{"W": dn.weight.float().cpu().numpy().T, "b": dn.bias.cpu().numpy(), "gamma": nm.gamma.cpu().numpy(),
               "beta": nm.beta.cpu().numpy()} for nm, dn in zip(mlp.norms, mlp.denses)]
    want = O.mlp(x.cpu().numpy(), params, "gelu", "ln")
    err_fold, err_unfused = np.abs(y - want).max(), np.abs(y_unfused - want).max()
    np.testing.assert_allclose(y, want, rtol=2e-2, atol=2e-2)
    np.testing.assert_allclose(y, y_unfused, rtol=2e-2, atol=2e-2)
    assert err_fold <= 2 * err_unfused + 1e-3, (err_fold, err_unfused)


def _slice_stats(y: np.ndarray) -> np.ndarray:
    """[M, K] fp32 -> [M, K / 32, 2]: per 32-column slice its sum and squared deviations from the slice mean."""
    M, K = y.shape
    s = y.reshape(M, K // 32, 32).astype(np.float64)
    S = s.sum(2)
    M2 = ((s - S[..., None] / 32) ** 2).sum(2)
    return np.stack([S, M2], axis=2)


def _bf16_bits(t: torch.Tensor) -> np.ndarray:
    return t.contiguous().view(torch.int16).cpu().numpy()


@pytest.mark.parametrize("M", [100, 4096])
def test_mlp2_small_stats_output(cuda, M):
    """rf_mlp2_small_stats_fwd: the same values as rf_mlp2_small_fwd, stored as bf16 (round-to-nearest-even of the
    fp32 output, bit for bit), and per 32-column slice the (sum, squared deviations) pair of those fp32 values
    at columns [p0, p0 + O / 32) of a wider stats row."""
    mlp = create_mlp([256, 512], 0.3, "gelu", LayerNormalization(epsilon=1e-6), in_features=16, dtype=torch.bfloat16,
                     seed=3)
    x = torch.randn(M, 16, generator=torch.Generator().manual_seed(M)).cuda()
    y = mlp(x)
    pb = torch.zeros((M, 1280), dtype=torch.bfloat16, device="cuda")
    st = torch.full((M, 40, 2), -7.0, device="cuda")
    mlp.forward_stats(x, pb[:, :512], st, 0)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_bf16_bits(pb[:, :512]), _bf16_bits(y.to(torch.bfloat16)))
    got = st.cpu().numpy()
    np.testing.assert_allclose(got[:, :16], _slice_stats(y.cpu().numpy()), rtol=1e-5, atol=1e-4)
    assert (got[:, 16:] == -7.0).all()  # slots past the producer's columns untouched


@pytest.mark.parametrize("M", [300, 4096])
def test_mlp_prenormed_head(O, cuda, M):
    """forward_prenormed_head (LN0 folded from producer partials -> rf_linear_lnfold_stats_fwd -> LN1 folded with the
    Dense(2, softmax) head in the epilogue -> rf_linear_lnfold_head_fwd) against float64 LN -> Dense(gelu) x 2 ->
    Dense(2, softmax) of the same parameters (cfg3's output MLP + head shapes); x is given to it as bf16 values +
    slice partials of the fp32 row, as the input MLP and the attention write them."""
    mlp = create_mlp([1024, 512], 0.3, "gelu", LayerNormalization(epsilon=1e-6), in_features=1280, dtype=torch.bfloat16,
                     seed=9)
    head = Dense(512, 2, activation="softmax", dtype=torch.bfloat16, seed=31)
    g = torch.Generator().manual_seed(M + 1)
    for nm in mlp.norms:
        nm.gamma.copy_(torch.rand(nm.width, generator=g) + 0.5)
        nm.beta.copy_(torch.randn(nm.width, generator=g) * 0.2)
    for dn in mlp.denses:
        dn.bias.copy_(torch.randn(dn.units, generator=g) * 0.1)
    head.bias.copy_(torch.randn(2, generator=g) * 0.1)
    x = torch.randn(M, 1280, generator=g) * 1.5 + 0.3
    xb = x.to(torch.bfloat16).cuda()
    xs = torch.from_numpy(_slice_stats(x.numpy()).astype(np.float32)).cuda()
    assert mlp.prenormed_head_ok(1280, head)
    pt = mlp.forward_prenormed_head(xb, xs, head)
    # the last tile of each row block finishes the softmax and resets its counter: a second call gives the same bits
    assert torch.equal(mlp.forward_prenormed_head(xb, xs, head), pt)
    p = pt.cpu().numpy()
    params = [{"W": dn.weight.float().cpu().numpy().T, "b": dn.bias.cpu().numpy(), "gamma": nm.gamma.cpu().numpy(),
               "beta": nm.beta.cpu().numpy()} for nm, dn in zip(mlp.norms, mlp.denses)]
    h = O.mlp(x.numpy(), params, "gelu", "ln")
    want = O.activation(h @ head.weight.float().cpu().numpy().T.astype(np.float64) + head.bias.cpu().numpy(), "softmax")
    np.testing.assert_allclose(p.sum(1), 1.0, atol=1e-5)
    # the unfused chain of the same module (fp32 x -> LN pass -> stats GEMM -> LN-fold GEMM -> head kernel)
    p_unfused = head(mlp(x.cuda())).cpu().numpy()
    err_f, err_u = np.abs(p - want).max(), np.abs(p_unfused - want).max()
    flips_f = int((p.argmax(1) != want.argmax(1)).sum())
    flips_u = int((p_unfused.argmax(1) != want.argmax(1)).sum())
    assert err_f <= 1e-2, (err_f, err_u, flips_f, flips_u)
    # the same error class as the unfused chain (bf16 operands either way; here uncentered ones)
    assert err_f <= 2 * err_u + 2e-3, (err_f, err_u, flips_f, flips_u)
    # arg-max: random head weights leave many rows near p = 0.5, where any rounding flips it
    assert flips_f <= max(2 * flips_u, 0.002 * M), (err_f, err_u, flips_f, flips_u)


def test_mlp_prenormed_head_varying_batch(cuda):
    """One module called at M = 4096, then a tail batch M = 300, then 4096 again: the head's workspace
    keeps its per-64-row counters at a fixed offset and its partial logits at the far end, so the smaller call's
    partials never land on counters a later call reads. Every row must come out as the full-batch call gives it."""
    mlp = create_mlp([1024, 512], 0.3, "gelu", LayerNormalization(epsilon=1e-6), in_features=1280, dtype=torch.bfloat16,
                     seed=9)
    head = Dense(512, 2, activation="softmax", dtype=torch.bfloat16, seed=31)
    g = torch.Generator().manual_seed(77)
    x = torch.randn(4096, 1280, generator=g) * 1.5 + 0.3
    xb = x.to(torch.bfloat16).cuda()
    xs = torch.from_numpy(_slice_stats(x.numpy()).astype(np.float32)).cuda()
    full = mlp.forward_prenormed_head(xb, xs, head).clone()
    for m in (300, 64, 4000, 1):
        tail = mlp.forward_prenormed_head(xb[:m].contiguous(), xs[:m].contiguous(), head)
        torch.testing.assert_close(tail, full[:m], rtol=0, atol=1e-6)
    torch.testing.assert_close(mlp.forward_prenormed_head(xb, xs, head), full, rtol=0, atol=0)
