"""GPU: rf_gemm_f32 (recommendflow_amd/csrc/rf_gemm32.hip), the exact-fp32 stream-K GEMM of the DSSM towers'
forward and training step (models/matching/dssm.py:25-26; example/ranking_search/train.py:96-104), against a float64
torch GEMM of the same operands. It is a floating-point kernel, so the oracle is a float64 product: the bound is on
|C - ref| / (|A| |B| + |bias|) elementwise, 2e-6 (fp32 products and K-term fp32 accumulation; K <= 20480), and the
result must be the same bits on every launch (tiles cut between workgroups are summed in k order)."""
import pytest
import torch

from recommendflow_amd.runtime import gemm as G

pytestmark = pytest.mark.gpu

ACT = {"none": lambda t: t, "selu": torch.selu, "relu": torch.relu, "gelu": torch.nn.functional.gelu}


def _operands(M, N, K, ta, tb, seed, bias=True):
    g = torch.Generator(device="cuda").manual_seed(seed)
    a = torch.randn((K, M) if ta else (M, K), device="cuda", generator=g)
    b = torch.randn((N, K) if tb else (K, N), device="cuda", generator=g)
    bi = torch.randn(N, device="cuda", generator=g) if bias else None
    return a, b, bi


def _check(c, a, b, ta, tb, bias, act):
    A = (a.t() if ta else a).double()
    B = (b.t() if tb else b).double()
    ref = A @ B
    scale = A.abs() @ B.abs()
    if bias is not None:
        ref = ref + bias.double()
        scale = scale + bias.double().abs()
    ref = ACT[act](ref)
    err = ((c.double() - ref).abs() / (scale + 1e-30)).max().item() if c.numel() else 0.0
    assert not torch.isnan(c).any()
    assert err < 2e-6, err


# the cfg2 towers' GEMMs at full size: forward (x W^T, 8704 / 20480 wide inputs), weight gradient (dpre^T h),
# input gradient (dpre W)
TOWER = [("fwd_user", 4096, 1024, 8704, False, True, "selu"), ("fwd_ad", 4096, 1024, 20480, False, True, "selu"),
         ("fwd_l2", 4096, 512, 1024, False, True, "selu"), ("fwd_l3", 4096, 256, 512, False, True, "selu"),
         ("dw_user", 1024, 8704, 4096, True, False, "none"), ("dw_ad", 1024, 20480, 4096, True, False, "none"),
         ("dw_l2", 512, 1024, 4096, True, False, "none"), ("dz_user", 4096, 8704, 1024, False, False, "none"),
         ("dz_ad", 4096, 20480, 1024, False, False, "none"), ("dz_l3", 4096, 512, 256, False, False, "none")]


@pytest.mark.parametrize("name,M,N,K,ta,tb,act", TOWER, ids=[t[0] for t in TOWER])
def test_tower_shapes_vs_float64(cuda, name, M, N, K, ta, tb, act):
    a, b, bias = _operands(M, N, K, ta, tb, seed=M + N + K, bias=act != "none")
    c = G.gemm_f32(a, b, trans_a=ta, trans_b=tb, bias=bias, act=act)
    _check(c, a, b, ta, tb, bias, act)
    c2 = G.gemm_f32(a, b, trans_a=ta, trans_b=tb, bias=bias, act=act)
    assert torch.equal(c, c2)  # fixed combine order: replays are bit-identical


EDGE = [(300, 200, 100), (132, 260, 36), (257, 132, 1028), (132, 127, 68), (1000, 700, 4100), (1, 4, 4), (129, 1, 132),
        (64, 64, 0), (4096, 300, 12)]


@pytest.mark.parametrize("M,N,K", EDGE)
@pytest.mark.parametrize("ta,tb", [(False, True), (True, False), (False, False), (True, True)])
def test_ragged_shapes_every_layout(cuda, M, N, K, ta, tb):
    """Ragged M / N (partial tiles), K tails (K % 32 != 0), K = 0 (bias + activation only), tiny grids, every
    operand layout; the m/n-contiguous layouts need their leading dimension % 4 == 0, so M and N are padded in
    storage there (the operand is a column slice of a wider tensor)."""
    g = torch.Generator(device="cuda").manual_seed(M * 31 + N * 7 + K)
    pad = lambda n: (n + 3) // 4 * 4
    a_full = torch.randn((K, pad(M)) if ta else (M, pad(K)), device="cuda", generator=g)
    b_full = torch.randn((N, pad(K)) if tb else (K, pad(N)), device="cuda", generator=g)
    a = a_full[:, :M] if ta else a_full[:, :K]
    b = b_full[:, :K] if tb else b_full[:, :N]
    bias = torch.randn(N, device="cuda", generator=g)
    c = torch.full((M, N), float("nan"), device="cuda")
    G.gemm_f32(a, b, trans_a=ta, trans_b=tb, bias=bias, act="relu", out=c)
    _check(c, a, b, ta, tb, bias, "relu")


# few 64-k steps per tile and many tiles per workgroup: every segment boundary hands the next tile's first two
# k-steps over from the previous segment's last two (RF_G32_XTILE), single-step tails and cut tiles included
SHORT_K = [(4096, 2048, 128), (2048, 4096, 192), (3000, 1000, 320), (4096, 1024, 64), (1500, 3000, 100)]


@pytest.mark.parametrize("M,N,K", SHORT_K)
@pytest.mark.parametrize("ta,tb", [(False, True), (True, False), (False, False)])
def test_short_k_many_tiles(cuda, M, N, K, ta, tb):
    a, b, bias = _operands(M, N, K, ta, tb, seed=7 * M + N + K)
    c = G.gemm_f32(a, b, trans_a=ta, trans_b=tb, bias=bias, act="selu")
    _check(c, a, b, ta, tb, bias, "selu")
    assert torch.equal(c, G.gemm_f32(a, b, trans_a=ta, trans_b=tb, bias=bias, act="selu"))


# few tiles over a long K (the ESIM training step's small weight gradients and head): every tile is cut into many
# segments, which gemm32_fixup_kernel combines in a launch of its own (GemmArgs::defer), ragged edges and bias / act
FEW_TILES_LONG_K = [(4, 512, 4096, True, False, "none"), (256, 16, 4096, True, False, "none"),
                    (512, 256, 4096, True, False, "none"), (130, 200, 8192, False, True, "selu"),
                    (4, 4, 2048, False, False, "relu"), (1, 129, 4100, True, True, "none")]


@pytest.mark.parametrize("M,N,K,ta,tb,act", FEW_TILES_LONG_K)
def test_few_tiles_long_k_deferred_combine(cuda, M, N, K, ta, tb, act):
    g = torch.Generator(device="cuda").manual_seed(M + 3 * N + K)
    pad = lambda n: (n + 3) // 4 * 4
    a_full = torch.randn((K, pad(M)) if ta else (M, pad(K)), device="cuda", generator=g)
    b_full = torch.randn((N, pad(K)) if tb else (K, pad(N)), device="cuda", generator=g)
    a = a_full[:, :M] if ta else a_full[:, :K]
    b = b_full[:, :K] if tb else b_full[:, :N]
    bias = torch.randn(N, device="cuda", generator=g) if act != "none" else None
    c = G.gemm_f32(a, b, trans_a=ta, trans_b=tb, bias=bias, act=act)
    _check(c, a, b, ta, tb, bias, act)
    assert torch.equal(c, G.gemm_f32(a, b, trans_a=ta, trans_b=tb, bias=bias, act=act))


def test_workspace_shared_across_shapes(cuda):
    """One zeroed workspace per stream serves every shape: a small call after a large one, a large one after a small
    one (the per-tile counters sit at the start, the partial tiles at the far end), the results unchanged."""
    shapes = [(4096, 1024, 8704, False, True), (256, 512, 4096, True, False), (4096, 8704, 1024, False, False),
              (300, 200, 100, False, True), (1024, 20480, 4096, True, False)]
    first = []
    for i, (M, N, K, ta, tb) in enumerate(shapes):
        a, b, _ = _operands(M, N, K, ta, tb, seed=i, bias=False)
        first.append((a, b, ta, tb, G.gemm_f32(a, b, trans_a=ta, trans_b=tb)))
    for a, b, ta, tb, c in reversed(first):
        assert torch.equal(G.gemm_f32(a, b, trans_a=ta, trans_b=tb), c)
    for a, b, ta, tb, c in first:
        _check(c, a, b, ta, tb, None, "none")


def test_output_row_stride_and_views(cuda):
    """Operands and output as column blocks of wider tensors (the towers read their blocks of the fused encoder
    output in place): leading dimensions larger than the logical widths."""
    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(512, 8704 + 20480, device="cuda", generator=g)
    W = torch.randn(1024, 20480, device="cuda", generator=g) * 0.01
    out = torch.full((512, 2048), float("nan"), device="cuda")
    G.gemm_f32(x[:, 8704:], W, trans_b=True, out=out[:, 1024:])
    _check(out[:, 1024:], x[:, 8704:], W, False, True, None, "none")
    assert torch.isnan(out[:, :1024]).all()  # nothing written outside the view


@pytest.mark.parametrize("ta,tb", [(False, True), (True, False), (False, False)])
def test_grouped_problems_vs_float64(cuda, ta, tb):
    """rf_gemm_f32_grouped: the same layer of the two DSSM towers in one launch (their tiles share the stream-K grid)
    plus a ragged third and fourth problem; every output vs float64, replays bit-identical."""
    shapes = [(4096, 512, 1024), (4096, 512, 1024), (300, 200, 100), (132, 68, 4100)] if not ta else \
        [(512, 1024, 4096), (512, 1024, 4096), (300, 200, 100), (132, 68, 4100)]
    probs = []
    for i, (M, N, K) in enumerate(shapes):
        a, b, bias = _operands(M, N, K, ta, tb, seed=50 + i)
        probs.append((a, b, bias, "selu" if i % 2 else "none", None))
    outs = G.gemm_f32_grouped(probs, trans_a=ta, trans_b=tb)
    for (a, b, bias, act, _), c in zip(probs, outs):
        _check(c, a, b, ta, tb, bias, act)
    outs2 = G.gemm_f32_grouped(probs, trans_a=ta, trans_b=tb)
    assert all(torch.equal(x, y) for x, y in zip(outs, outs2))


def test_forward_towers_matches_each_tower(cuda):
    """backend.blocks.mlp.forward_towers (the DSSM inference towers layer by layer, one grouped launch per layer)
    against each MLP's own forward: the same folded weights and epilogue, so equal within fp32 summation order."""
    from recommendflow_amd.backend.blocks.mlp import create_mlp, forward_towers
    from recommendflow_amd.backend.layers.core import BatchNormalization

    bn = BatchNormalization(epsilon=1e-6)
    mu = create_mlp([1024, 512, 256], 0.3, "selu", bn, in_features=8704, dtype=torch.float32, seed=1)
    ma = create_mlp([1024, 512, 256], 0.3, "selu", bn, in_features=20480, dtype=torch.float32, seed=2)
    g = torch.Generator(device="cuda").manual_seed(9)
    x = torch.randn(1024, 8704 + 20480, device="cuda", generator=g) * 0.05
    xu, xa = x[:, :8704], x[:, 8704:]
    n0 = G.calls
    u, a = forward_towers([mu, ma], [xu, xa])
    want = sum(1 if G.group_pays([(1024, u), (1024, u)]) else 2 for u in (1024, 512, 256))
    assert G.calls - n0 == want  # grouped where it pays (layers without a tile per CU), else one launch each
    u1, a1 = mu(xu), ma(xa)
    torch.testing.assert_close(u, u1, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(a, a1, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("width", [300, 1000, 132])
def test_trailing_column_view_operand(cuda, width):
    """The weight-gradient layout dpre^T h with h the LAST `width` columns of a wider tensor (the towers' layer-0 view
    of the fused encoder output), width % 128 != 0: the n-contiguous operand's buffer extent ends at the view's last
    column, not at the parent's row end, and the result is exact."""
    g = torch.Generator(device="cuda").manual_seed(width)
    K, M, ld = 1000, 64, 1024 + width
    dpre = torch.randn(K, M, device="cuda", generator=g)
    x = torch.randn(K, ld, device="cuda", generator=g)
    h = x[:, ld - width:]
    c = G.gemm_f32(dpre, h, trans_a=True)
    _check(c, dpre, h, True, False, None, "none")


def test_oversized_operand_block_goes_to_the_fallback(cuda):
    """An m/n-contiguous operand whose (K + 192) k-rows span >= 2 GiB is outside rf_gemm_f32's 32-bit offsets:
    supported_gemm says so, the tower layer routes it to torch (counted), and the result is the product."""
    from recommendflow_amd.backend.blocks.train_mlp import _gemm_layer

    K, M, N = 4100, 64, 131072  # (4100 + 192) * 131072 * 4 B = 2.25 GB
    g = torch.Generator(device="cuda").manual_seed(5)
    a = torch.randn(K, M, device="cuda", generator=g)
    b = torch.randn(K, N, device="cuda", generator=g)
    assert not G.supported_gemm(a, b, trans_a=True, trans_b=False)
    fb0 = G.torch_fallbacks
    with pytest.warns(RuntimeWarning) if not G._warned[0] else _nowarn():
        (c,) = _gemm_layer([(a, b, None, "none", None)], True, False, torch.cuda.current_stream().cuda_stream)
    assert G.torch_fallbacks == fb0 + 1
    A, B = a.t().double(), b[:, :2048].double()
    err = ((c[:, :2048].double() - A @ B).abs() / (A.abs() @ B.abs())).max().item()
    assert err < 1e-5, err
    del b, c


class _nowarn:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False
