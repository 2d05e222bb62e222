"""GPU: the ESIM ranking-model training path (models/ranking/esim_train.py; esim.py:45-53,69-89 under model.fit,
example/ranking_search/train.py:96-104) against the float64 oracle (oracle.esim_train_loss / esim_pool_bwd /
ln_mlp_train_bwd, whose analytic gradients tests/test_esim_train_oracle_cpu.py pins by finite differences).

Floating-point bars (fp32 kernels vs float64): every tensor within 1e-4 of its largest reference magnitude
(|got - want| <= 1e-4 max|want| + 1e-7), the loss within 1e-5 relative; dropout masks are the same counter hash on
both sides (oracle.dropout_keep)."""
import numpy as np
import pytest
import torch

from oracle import oracle as O
from recommendflow_amd.runtime import lib as L

pytestmark = pytest.mark.gpu


def close(got, want, rel=1e-4, what=""):
    got = np.asarray(got, np.float64)
    want = np.asarray(want, np.float64)
    assert got.shape == want.shape, (what, got.shape, want.shape)
    assert np.isfinite(got).all(), what
    err = np.abs(got - want).max() if got.size else 0.0
    assert err <= rel * np.abs(want).max() + 1e-7, (what, err, np.abs(want).max())


def _qa(B, Lq, d, seed, dup=True):
    g = torch.Generator().manual_seed(seed)
    q = torch.randn((B, Lq, d), generator=g)
    a = torch.randn((B, Lq, d), generator=g) * 0.7
    if dup and Lq >= 3:
        q[:, 2] = q[:, 1]  # duplicate rows: ties in max_q (two slots on the same table row, e.g. both empty)
        a[:, Lq - 1] = a[:, 0]
    return q, a


@pytest.mark.parametrize("B,Lq,d", [(37, 100, 128), (16, 37, 64), (9, 1, 64), (5, 128, 128), (6, 16, 128), (3, 113, 64)])
def test_esim_attention_train_fwd_bwd_vs_oracle(cuda, B, Lq, d):
    q, a = _qa(B, Lq, d, seed=B * 1000 + Lq)
    # q and a as column blocks of one [B, 2 L d] row (the fused encoder's output), as TrainableEsim passes them
    x = torch.cat([q.reshape(B, -1), a.reshape(B, -1)], dim=1).contiguous().cuda()
    Ld = Lq * d
    W = 16 + 6 * d  # pooled columns start at out_off 16
    pooled = torch.full((B, W), float("nan"), device="cuda")
    aux = torch.empty((B, 2 * d), device="cuda")
    L.call("rf_esim_train_fwd_f32", L.ptr(x), L.ptr(x) + 4 * Ld, B, Lq, d, x.stride(0), d, L.ptr(pooled), W, 16, L.ptr(aux),
           L.stream_ptr())
    want = O.esim_pool(q.numpy(), a.numpy())
    close(pooled[:, 16:].cpu().numpy(), want, 1e-5, "pooled")
    assert torch.isnan(pooled[:, :16]).all()  # nothing written outside the block
    # tie counts: how many of the 4L candidates equal each max (the float64 oracle's sets on exact-duplicate rows)
    qd, ad = q.double().numpy(), a.double().numpy()
    g = torch.Generator().manual_seed(5)
    dp = torch.randn((B, W), generator=g)
    dpd = dp.cuda()
    dx = torch.full_like(x, float("nan"))
    ws = torch.empty(int(L.load().rf_esim_train_ws_bytes(B, Lq, d)), dtype=torch.uint8, device="cuda")
    L.call("rf_esim_train_bwd_f32", L.ptr(x), L.ptr(x) + 4 * Ld, B, Lq, d, x.stride(0), d, L.ptr(pooled), W, 16, L.ptr(dpd), W,
           16, L.ptr(aux), L.ptr(dx), L.ptr(dx) + 4 * Ld, dx.stride(0), d, L.ptr(ws), ws.numel(), L.stream_ptr())
    dq, da = O.esim_pool_bwd(qd, ad, dp[:, 16:].double().numpy())
    got = dx.cpu().numpy()
    close(got[:, :Ld].reshape(B, Lq, d), dq, 1e-4, "dq")
    close(got[:, Ld:].reshape(B, Lq, d), da, 1e-4, "da")
    # replay: the same bits (no atomics)
    dx2 = torch.empty_like(dx)
    L.call("rf_esim_train_bwd_f32", L.ptr(x), L.ptr(x) + 4 * Ld, B, Lq, d, x.stride(0), d, L.ptr(pooled), W, 16, L.ptr(dpd), W,
           16, L.ptr(aux), L.ptr(dx2), L.ptr(dx2) + 4 * Ld, dx2.stride(0), d, L.ptr(ws), ws.numel(), L.stream_ptr())
    assert torch.equal(dx, dx2)


def test_esim_train_tie_counts(cuda):
    """aux = the number of candidates equal to each max: a column where two duplicate q rows hold the max of the
    q candidates counts both."""
    B, Lq, d = 4, 8, 64
    q = torch.full((B, Lq, d), -1.0)
    q[:, 3] = 0.5
    q[:, 5] = 0.5  # rows 3 and 5 hold the max 0.5 of candidate q; att = S q < 0.5, q - att < 0.5 + 1, ...
    a = torch.zeros((B, Lq, d))
    x = torch.cat([q.reshape(B, -1), a.reshape(B, -1)], dim=1).contiguous().cuda()
    pooled = torch.empty((B, 6 * d), device="cuda")
    aux = torch.empty((B, 2 * d), device="cuda")
    L.call("rf_esim_train_fwd_f32", L.ptr(x), L.ptr(x) + 4 * Lq * d, B, Lq, d, x.stride(0), d, L.ptr(pooled), 6 * d, 0,
           L.ptr(aux), L.stream_ptr())
    want = O.esim_pool(q.numpy(), a.numpy())
    close(pooled.cpu().numpy(), want, 1e-6, "pooled")
    # oracle count of the candidates equal to the max, side q
    qd = q.double().numpy()
    att_q, att_a = O.soft_attention(qd, a.double().numpy())
    cands = [qd, att_q, qd - att_q, qd * att_q]
    M = np.max([c.max(axis=1) for c in cands], axis=0)
    cnt = sum((c == M[:, None, :]).sum(axis=1) for c in cands)
    np.testing.assert_array_equal(aux[:, :d].cpu().numpy(), cnt)


def test_ln_mlp_train_vs_oracle(cuda):
    from recommendflow_amd.backend.blocks.train_ln_mlp import TrainLNMLP

    M, K = 300, 48
    mlp = TrainLNMLP(K, (64, 32), rate=0.3, activation="gelu", seed=3)
    for p in mlp.gamma + mlp.beta:  # non-trivial LayerNorm parameters
        p.add_(torch.randn(p.shape, generator=torch.Generator().manual_seed(p.numel())).cuda() * 0.1)
    g = torch.Generator().manual_seed(1)
    x = torch.randn((M, K), generator=g) * 2 + 0.5
    h = mlp.forward(x.cuda(), step=7)
    layers = [{"W": mlp.W[i].cpu().double().numpy(), "b": mlp.b[i].cpu().double().numpy(),
               "gamma": mlp.gamma[i].cpu().double().numpy(), "beta": mlp.beta[i].cpu().double().numpy()} for i in range(2)]
    want, cache = O.ln_mlp_train_fwd(x.double().numpy(), layers, 0.3, mlp.layer_seeds(7))
    close(h.cpu().numpy(), want, 1e-5, "h")
    dh = torch.randn(h.shape, generator=g)
    dx = mlp.backward(dh.cuda())
    wdx, grads = O.ln_mlp_train_bwd(dh.double().numpy(), layers, cache, 0.3)
    close(dx.cpu().numpy(), wdx, 1e-4, "dx")
    for i in range(2):
        close(mlp.W[i].grad.cpu().numpy(), grads[i]["W"], 1e-4, f"W{i}")
        close(mlp.b[i].grad.cpu().numpy(), grads[i]["b"], 1e-4, f"b{i}")
        close(mlp.gamma[i].grad.cpu().numpy(), grads[i]["gamma"], 1e-4, f"gamma{i}")
        close(mlp.beta[i].grad.cpu().numpy(), grads[i]["beta"], 1e-4, f"beta{i}")


def test_softmax_ce_loss(cuda):
    B = 1000
    g = torch.Generator().manual_seed(2)
    z = torch.randn((B, 2), generator=g) * 3
    y = torch.randint(0, 2, (B,), generator=g).to(torch.int32)
    zc, yc = z.cuda(), y.cuda()
    loss = torch.empty(1, device="cuda")
    prob, dz = torch.empty_like(zc), torch.empty_like(zc)
    ws = torch.empty(int(L.load().rf_loss_ws_bytes(B)), dtype=torch.uint8, device="cuda")
    L.call("rf_softmax_ce_loss", L.ptr(zc), 2, L.ptr(yc), B, 2, L.ptr(loss), L.ptr(prob), 2, L.ptr(dz), 2, L.ptr(ws), ws.numel(),
           L.stream_ptr())
    zd = z.double().numpy()
    lse = np.log(np.exp(zd).sum(1))
    want = (lse - zd[np.arange(B), y.numpy()]).mean()
    assert abs(loss.item() - want) <= 1e-6 * abs(want)
    p = np.exp(zd - lse[:, None])
    close(prob.cpu().numpy(), p, 1e-6, "prob")
    oh = np.zeros_like(p)
    oh[np.arange(B), y.numpy()] = 1
    close(dz.cpu().numpy(), (p - oh) / B, 1e-5, "dz")
    # a label out of range: that row NaN, the others unchanged
    y[3] = 5
    yc = y.cuda()
    L.call("rf_softmax_ce_loss", L.ptr(zc), 2, L.ptr(yc), B, 2, L.ptr(loss), None, 0, L.ptr(dz), 2, L.ptr(ws), ws.numel(),
           L.stream_ptr())
    assert np.isnan(loss.item()) and torch.isnan(dz[3]).all() and not torch.isnan(dz[4]).any()


def _esim_model(L_=8, dim=32, B=64, n_dense=16, rate=0.3, seed=0, multi=False):
    from recommendflow_amd.backend.encoder.sparse_encoder import SlotSpec
    from recommendflow_amd.models.ranking.esim_train import TrainableEsim
    from recommendflow_amd.runtime.batch import synthetic_batch

    user = [SlotSpec(f"q{i}", 1000, (7, 8)) for i in range(L_)]
    ad = [SlotSpec(f"k{i}", 1000, (7, 8)) for i in range(L_)]
    m = TrainableEsim(user, ad, n_dense, dim=dim, input_units=(32, 48), output_units=(64, 32), dropout=rate, seed=seed)
    batch = synthetic_batch(B, [multi and i % 3 == 0 for i in range(2 * L_)], seed=seed + 3,
                            slot_ids=range(400, 400 + 2 * L_)).to("cuda")
    g = torch.Generator().manual_seed(seed + 9)
    dense = torch.randn((B, n_dense), generator=g).cuda()
    labels = torch.randint(0, 2, (B,), generator=g).cuda()
    return m, batch, dense, labels


def _oracle_layers(mlp):
    return [{"W": mlp.W[i].cpu().double().numpy(), "b": mlp.b[i].cpu().double().numpy(),
             "gamma": mlp.gamma[i].cpu().double().numpy(), "beta": mlp.beta[i].cpu().double().numpy()}
            for i in range(len(mlp.units))]


@pytest.mark.parametrize("rate,multi", [(0.0, False), (0.3, False), (0.3, True)])
def test_trainable_esim_grads_vs_oracle(cuda, rate, multi):
    """The whole training graph: loss, every dense gradient and the fused encoder output's gradient (dq, da) vs
    oracle.esim_train_loss on the GPU encoder's q, a (the encoder itself is bit-exact, tests/test_embed_gpu.py);
    multi: every third slot multi-valued (its token sequence sum-pooled into the slot's row)."""
    m, batch, dense, labels = _esim_model(rate=rate, multi=multi)
    step = 4
    loss, prob = m.loss_and_grads(batch, dense, labels, step=step)
    x = m.enc(batch).cpu().double().numpy()
    B, Ld = x.shape[0], m.L * m.d
    q, a = x[:, :Ld].reshape(B, m.L, m.d), x[:, Ld:].reshape(B, m.L, m.d)
    seeds = (m.input_mlp.layer_seeds(step), m.pooled_dropout_seed(step), m.output_mlp.layer_seeds(step))
    wl, wp, g = O.esim_train_loss(q, a, dense.cpu().double().numpy(), labels.cpu().numpy(), _oracle_layers(m.input_mlp),
                                  _oracle_layers(m.output_mlp), m.W_out.cpu().double().numpy(), m.b_out.cpu().double().numpy(),
                                  rate=rate, seeds=seeds, grads=True)
    assert abs(loss.item() - wl) <= 1e-5 * abs(wl), (loss.item(), wl)
    close(prob.cpu().numpy(), wp, 1e-5, "prob")
    close(m.W_out.grad.cpu().numpy(), g["W_out"], 1e-4, "W_out")
    close(m.b_out.grad.cpu().numpy(), g["b_out"], 1e-4, "b_out")
    for name, mlp in (("input", m.input_mlp), ("output", m.output_mlp)):
        for i in range(len(mlp.units)):
            for k, t in (("W", mlp.W[i]), ("b", mlp.b[i]), ("gamma", mlp.gamma[i]), ("beta", mlp.beta[i])):
                close(t.grad.cpu().numpy(), g[name][i][k], 1e-4, f"{name}[{i}].{k}")
    d = m.dout.cpu().numpy()
    close(d[:, :Ld].reshape(B, m.L, m.d), g["q"], 1e-4, "dq")
    close(d[:, Ld:].reshape(B, m.L, m.d), g["a"], 1e-4, "da")


def test_trainable_esim_steps_reduce_the_loss(cuda):
    """model.fit on one fixed batch: Adam on the table and the dense parameters drives the loss down; predict()
    afterwards reads every table row current."""
    m, batch, dense, labels = _esim_model(rate=0.0, B=128)
    losses = [m.step(batch, dense, labels).item() for _ in range(12)]
    assert all(np.isfinite(losses))
    assert losses[-1] < 0.7 * losses[0], losses
    p = m.predict(batch, dense)
    assert torch.allclose(p.sum(1), torch.ones(128, device="cuda"), atol=1e-6)


def test_trainable_esim_data_parallel_world1_matches_single(cuda):
    """TrainableEsim.step(dp=DataParallel) over RCCL with one rank (the bucketed dense all-reduce and the rank-ordered
    sparse all-gather are identities at P = 1): three steps give bit-identical tables and dense parameters."""
    import socket

    import torch.distributed as dist

    from recommendflow_amd.runtime.dist import DataParallel

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        dp = DataParallel(bucket_bytes=1 << 16)
        (m0, batch, dense, labels), (m1, _, _, _) = _esim_model(rate=0.3), _esim_model(rate=0.3)
        for _ in range(3):
            m0.step(batch, dense, labels)
            m1.step(batch, dense, labels, dp=dp)
        torch.cuda.synchronize()
        m0.sparse_opt.materialize()
        m1.sparse_opt.materialize()
        assert torch.equal(m0.enc.table, m1.enc.table)
        for a, b in zip(m0.dense_parameters(), m1.dense_parameters()):
            assert torch.equal(a, b)
    finally:
        dist.destroy_process_group()
