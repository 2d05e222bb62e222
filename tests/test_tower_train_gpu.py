"""GPU: the DSSM towers under training on librf.so (backend.blocks.train_mlp.TrainTower: BatchNormalization with
batch statistics folded into the fp32 MFMA GEMM, SELU + dropout + BatchNormalization backward kernels) against
the float64 oracle (oracle.tower_train_fwd / tower_train_bwd, itself pinned by finite differences in
tests/test_tower_oracle_cpu.py). Tolerance: rtol 1e-4 with an absolute floor of 1e-4 x the largest magnitude
(fp32 accumulation; the BatchNormalization backward subtracts column means)."""
import numpy as np
import pytest
import torch

from recommendflow_amd.backend.blocks.train_mlp import TrainTower, layer_seed
import recommendflow_amd.runtime.lib as L

pytestmark = pytest.mark.gpu


def close(got, want, rtol=1e-4):
    want = np.asarray(want, np.float64)
    np.testing.assert_allclose(np.asarray(got, np.float64), want, rtol=rtol, atol=rtol * max(np.abs(want).max(), 1e-30))


def _tower(in_f, units, rate, seed=5):
    t = TrainTower(in_f, units, rate=rate, seed=seed)
    g = torch.Generator().manual_seed(seed + 100)
    with torch.no_grad():
        for l in range(len(units)):
            t.b[l].copy_(torch.randn(t.b[l].shape, generator=g) * 0.1)
            t.gamma[l].copy_(torch.rand(t.gamma[l].shape, generator=g) + 0.5)
            t.beta[l].copy_(torch.randn(t.beta[l].shape, generator=g) * 0.1)
    return t


def _oracle_layers(t):
    return [{"W": t.W[l].detach().cpu().numpy().astype(np.float64), "b": t.b[l].detach().cpu().numpy().astype(np.float64),
             "gamma": t.gamma[l].detach().cpu().numpy().astype(np.float64),
             "beta": t.beta[l].detach().cpu().numpy().astype(np.float64)} for l in range(len(t.units))]


@pytest.mark.parametrize("M,in_f,units,rate,off", [(512, 384, (128, 64, 32), 0.3, 4), (300, 2048, (256, 64), 0.0, 4),
                                                   (1024, 8704, (1024, 512, 256), 0.3, 4),
                                                   (512, 20480, (1024, 512, 256), 0.3, 8)])
@pytest.mark.parametrize("route", ["librf", "blas"])
def test_tower_forward_backward_vs_oracle(O, cuda, M, in_f, units, rate, off, route, monkeypatch):
    """Output, input gradient and every parameter gradient vs float64; the last shapes are cfg2's user and ad towers
    (K = 8704 / 20480). route "librf" (the default): every forward and backward GEMM runs rf_gemm_f32 (asserted:
    3 launches per layer, torch.mm / addmm never called); "blas": the A/B switches (hipBLASLt forward for K >= 4096,
    torch.mm backward)."""
    from recommendflow_amd.backend.blocks import train_mlp
    from recommendflow_amd.runtime import gemm as G

    monkeypatch.setattr(train_mlp, "_BLASLT_WIDE", route == "blas")
    monkeypatch.setattr(train_mlp, "_BWD_BLAS", route == "blas")
    if route == "librf":
        def refuse(*a, **k):
            raise AssertionError("a vendor GEMM ran on the librf route")
        monkeypatch.setattr(torch, "addmm", refuse)
        monkeypatch.setattr(torch, "mm", refuse)
    n0, fb0 = G.calls, G.torch_fallbacks
    t = _tower(in_f, units, rate)
    g = torch.Generator().manual_seed(M + in_f)
    xfull = (torch.randn(M, in_f + 8, generator=g) * 0.05 + 0.01).cuda()
    x = xfull[:, off: off + in_f].detach().requires_grad_(True)  # a strided view, as the DSSM column blocks
    step = t.steps
    out = t(x)
    dout = torch.randn(out.shape, generator=g).cuda()
    out.backward(dout)
    if route == "librf":
        assert G.calls - n0 == 3 * len(units), G.calls - n0
        assert G.torch_fallbacks == fb0  # no GEMM of the tower left librf
    layers = _oracle_layers(t)
    seeds = [layer_seed(t.seed, step, l) for l in range(len(units))]
    want, cache = O.tower_train_fwd(x.detach().cpu().numpy(), layers, rate, seeds)
    close(out.detach().cpu().numpy(), want)
    dx, grads = O.tower_train_bwd(dout.cpu().numpy(), layers, cache, rate)
    close(x.grad.cpu().numpy(), dx)
    for l in range(len(units)):
        close(t.W[l].grad.cpu().numpy(), grads[l]["W"])
        close(t.b[l].grad.cpu().numpy(), grads[l]["b"])
        close(t.gamma[l].grad.cpu().numpy(), grads[l]["gamma"])
        close(t.beta[l].grad.cpu().numpy(), grads[l]["beta"])
    # Keras moving statistics: moving = 0.99 moving + 0.01 batch (biased variance), from (0, 1)
    for l in range(len(units)):
        close(t.moving_mean[l].cpu().numpy(), 0.01 * cache[l]["mean"], rtol=1e-4)
        close(t.moving_var[l].cpu().numpy(), 0.99 + 0.01 * cache[l]["var"], rtol=1e-4)


@pytest.mark.parametrize("fused", [False, True])
def test_two_tower_loss_and_gradients_vs_oracle(O, cuda, fused):
    """The DSSM training graph on two towers: u, v = l2norm(tower(x)), cosent loss on <u, v> (match_losses.py
    :42-56); loss and the gradients reaching the towers' inputs and parameters vs float64 at rtol 1e-4. fused: the
    train step's form (cosine_cosent_loss on the raw tower outputs: rf_cosine_rows_fwd / _bwd around cosent)."""
    from recommendflow_amd.backend.losses.match_losses import cosent_loss, cosine_cosent_loss

    M, ku, ka, units, rate = 256, 320, 448, (96, 48), 0.3
    tu, ta = _tower(ku, units, rate, seed=7), _tower(ka, units, rate, seed=8)
    g = torch.Generator().manual_seed(1)
    xu = (torch.randn(M, ku, generator=g) * 0.05).cuda().requires_grad_(True)
    xa = (torch.randn(M, ka, generator=g) * 0.05).cuda().requires_grad_(True)
    y = (torch.arange(M) % 3 == 0).float().cuda()
    su, sa = tu.steps, ta.steps
    if fused:
        loss = cosine_cosent_loss(y, tu(xu), ta(xa), eps=1e-6)
    else:
        u = torch.nn.functional.normalize(tu(xu), dim=-1, eps=1e-6)
        v = torch.nn.functional.normalize(ta(xa), dim=-1, eps=1e-6)
        loss = cosent_loss(y, u, v)
    loss.backward()

    lu, la = _oracle_layers(tu), _oracle_layers(ta)
    ou, cu = O.tower_train_fwd(xu.detach().cpu().numpy(), lu, rate, [layer_seed(tu.seed, su, l) for l in range(2)])
    oa, ca = O.tower_train_fwd(xa.detach().cpu().numpy(), la, rate, [layer_seed(ta.seed, sa, l) for l in range(2)])
    nu, na = np.linalg.norm(ou, axis=1, keepdims=True), np.linalg.norm(oa, axis=1, keepdims=True)
    uu, vv = ou / nu, oa / na
    want_loss, ds = O.cosent_loss(y.cpu().numpy(), (uu * vv).sum(1))
    assert abs(float(loss.detach()) - want_loss) <= 1e-4 * max(1.0, abs(want_loss))
    du, dv = ds[:, None] * vv, ds[:, None] * uu
    dou = (du - uu * (uu * du).sum(1, keepdims=True)) / nu
    doa = (dv - vv * (vv * dv).sum(1, keepdims=True)) / na
    dxu, gu = O.tower_train_bwd(dou, lu, cu, rate)
    dxa, ga = O.tower_train_bwd(doa, la, ca, rate)
    close(xu.grad.cpu().numpy(), dxu)
    close(xa.grad.cpu().numpy(), dxa)
    for t, gs in ((tu, gu), (ta, ga)):
        for l in range(2):
            close(t.W[l].grad.cpu().numpy(), gs[l]["W"])
            close(t.b[l].grad.cpu().numpy(), gs[l]["b"])
            close(t.gamma[l].grad.cpu().numpy(), gs[l]["gamma"])
            close(t.beta[l].grad.cpu().numpy(), gs[l]["beta"])


@pytest.mark.parametrize("M,K,off", [(3000, 700, 0), (3000, 701, 1), (37, 5, 0), (4096, 256, 0), (5, 2048, 4)])
def test_col_stats_large_mean_and_dropout_mask(O, cuda, M, K, off):
    """rf_col_stats on columns whose mean is 1000x their spread (pivoted chunks + Chan combine) and
    rf_dropout_fwd's mask bit-exact against oracle.dropout_keep; the float4 path (16-byte aligned rows) and
    the scalar one (odd K, a view starting one float in), tiny and cfg2-shaped chunkings."""
    g = torch.Generator().manual_seed(4)
    ld = K + 4
    xfull = (torch.randn(M, ld, generator=g) + 1000.0).cuda()
    x = xfull[:, off: off + K]
    mean, var = torch.empty(K, device="cuda"), torch.empty(K, device="cuda")
    ws = torch.empty(int(L.load().rf_tower_ws_bytes(M, K)), dtype=torch.uint8, device="cuda")
    L.call("rf_col_stats", L.ptr(x), M, K, ld, L.ptr(mean), L.ptr(var), L.ptr(ws), ws.numel(), L.stream_ptr(None))
    x64 = x.cpu().numpy().astype(np.float64)
    close(mean.cpu().numpy(), x64.mean(0), rtol=1e-6)
    close(var.cpu().numpy(), x64.var(0), rtol=2e-4)
    y = torch.ones(M, K, device="cuda")
    L.call("rf_dropout_fwd", L.ptr(y), M, K, K, 0.3, 987654321, L.ptr(y), K, L.stream_ptr(None))
    keep = O.dropout_keep(987654321, M, K, 0.3)
    assert np.array_equal(y.cpu().numpy() != 0, keep)


@pytest.mark.parametrize("M,K", [(4096, 256), (333, 520)])
def test_column_kernels_float4_equals_scalar(cuda, M, K):
    """The column kernels pick float4 lanes when every row is 16-byte aligned and scalar lanes otherwise; both
    walk the same row chunks in the same order, so the results are bit-identical (a view one float in forces the
    scalar path)."""
    g = torch.Generator().manual_seed(M)
    st = L.stream_ptr(None)
    ws = torch.empty(int(L.load().rf_tower_ws_bytes(M, K)), dtype=torch.uint8, device="cuda")

    def views(t):  # the same values, aligned and one float in
        a = torch.zeros(M, K + 4, device="cuda")
        b = torch.zeros(M, K + 4, device="cuda")
        a[:, :K] = t
        b[:, 1:K + 1] = t
        return a[:, :K], b[:, 1:K + 1]

    x = torch.randn(M, K, generator=g).cuda() * 0.3 + 0.1
    dz = torch.randn(M, K, generator=g).cuda()
    gamma, var = torch.rand(K).cuda() + 0.5, torch.rand(K).cuda() + 0.1
    mean = torch.randn(K).cuda() * 0.1
    outs = []
    for xv, dv in zip(views(x), views(dz)):
        ld = K + 4
        mu, va = torch.empty(K, device="cuda"), torch.empty(K, device="cuda")
        L.call("rf_col_stats", L.ptr(xv), M, K, ld, L.ptr(mu), L.ptr(va), L.ptr(ws), ws.numel(), st)
        dpre, db = torch.zeros(M, K + 4, device="cuda"), torch.empty(K, device="cuda")
        dp = dpre[:, 1:K + 1] if xv.data_ptr() % 16 else dpre[:, :K]
        L.call("rf_selu_dropout_bwd", L.ptr(dv), ld, L.ptr(xv), ld, M, K, 0.3, 77, L.ptr(dp), ld, L.ptr(db), L.ptr(ws),
               ws.numel(), st)
        dx, dg, dbe = torch.zeros(M, K + 4, device="cuda"), torch.empty(K, device="cuda"), torch.empty(K, device="cuda")
        dxv = dx[:, 1:K + 1] if xv.data_ptr() % 16 else dx[:, :K]
        L.call("rf_bn_bwd", L.ptr(dv), ld, L.ptr(xv), ld, M, K, L.ptr(mean), L.ptr(var), L.ptr(gamma), 1e-6, L.ptr(dxv), ld,
               L.ptr(dg), L.ptr(dbe), L.ptr(ws), ws.numel(), st)
        outs.append([t.clone() for t in (mu, va, dp, db, dxv, dg, dbe)])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_eval_mode_folds_moving_statistics(O, cuda):
    t = _tower(256, (64, 32), 0.3)
    g = torch.Generator().manual_seed(9)
    with torch.no_grad():
        for l in range(2):
            t.moving_mean[l].copy_(torch.randn(t.moving_mean[l].shape, generator=g) * 0.1)
            t.moving_var[l].copy_(torch.rand(t.moving_var[l].shape, generator=g) + 0.5)
    t.eval()
    x = (torch.randn(200, 256, generator=g) * 0.1).cuda()
    got = t(x).cpu().numpy()
    h = x.cpu().numpy().astype(np.float64)
    for l, p in enumerate(_oracle_layers(t)):
        h = O.batch_norm_infer(h, p["gamma"], p["beta"], t.moving_mean[l].cpu().numpy(), t.moving_var[l].cpu().numpy(),
                               1e-6)
        h = O.selu(h @ p["W"].T + p["b"])
    close(got, h)


def test_cosine_rows_vs_float64(cuda):
    """rf_cosine_rows_fwd / _bwd: the score and both input gradients vs float64 (rtol 1e-5 / 1e-4), including a
    zero row (clamped norm: u = a / eps), a row below eps, strided inputs, and the upstream scale folded in."""
    from recommendflow_amd.runtime import lib as L

    B, N, eps = 37, 200, 1e-6
    g = torch.Generator().manual_seed(5)
    base = torch.randn(B, N + 8, generator=g, dtype=torch.float64)
    base[3] = 0.0
    base[7] *= 1e-9
    b64 = torch.randn(B, N, generator=g, dtype=torch.float64)
    a = base.float().cuda()[:, :N]  # row stride N + 8
    b = b64.float().cuda()
    s = torch.empty(B, device="cuda")
    nrm = torch.empty(2 * B, device="cuda")
    L.call("rf_cosine_rows_fwd", L.ptr(a), a.stride(0), L.ptr(b), b.stride(0), B, N, eps, L.ptr(s), L.ptr(nrm),
           L.stream_ptr())
    A, Bm = a.double().cpu(), b.double().cpu()
    na = A.norm(dim=1, keepdim=True).clamp_min(eps)
    nb = Bm.norm(dim=1, keepdim=True).clamp_min(eps)
    want = ((A / na) * (Bm / nb)).sum(1)
    np.testing.assert_allclose(s.double().cpu().numpy(), want.numpy(), rtol=1e-5, atol=1e-6)
    ds = torch.randn(B, generator=g).cuda()
    gs = torch.tensor(0.25, device="cuda")
    da = torch.empty(B, N, device="cuda")
    db = torch.empty(B, N, device="cuda")
    L.call("rf_cosine_rows_bwd", L.ptr(a), a.stride(0), L.ptr(b), b.stride(0), B, N, eps, L.ptr(s), L.ptr(nrm), L.ptr(ds),
           L.ptr(gs), L.ptr(da), N, L.ptr(db), N, L.stream_ptr())
    Ar = A.clone().requires_grad_(True)
    Br = Bm.clone().requires_grad_(True)
    sc = ((Ar / Ar.norm(dim=1, keepdim=True).clamp_min(eps)) * (Br / Br.norm(dim=1, keepdim=True).clamp_min(eps))).sum(1)
    (sc * ds.double().cpu() * 0.25).sum().backward()
    np.testing.assert_allclose(da.double().cpu().numpy(), Ar.grad.numpy(), rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(db.double().cpu().numpy(), Br.grad.numpy(), rtol=1e-4, atol=1e-6)
