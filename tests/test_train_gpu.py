"""GPU parity of the sparse training backward (rf_fused_hash_embed_bwd) and the Keras Adam step
(rf_adam_apply) against the C oracle, through the C ABI. Bar: bit-exact (same order of fp32 additions
as Keras' unsorted_segment_sum on CPU; same fp32 Adam expression)."""
import numpy as np
import pytest
import torch

from recommendflow_amd.backend.encoder.sparse_encoder import FusedSparseEncoder, SlotSpec
from recommendflow_amd.backend.optim import SparseAdam
from recommendflow_amd.runtime.batch import from_lists, synthetic_batch

pytestmark = pytest.mark.gpu
COMBS = ["sum", "avg", "max", "min", "first", "last"]


def bits(x):
    return np.ascontiguousarray(x).view(np.uint32)


def run_bwd(O, enc, hb, seed=0):
    dev = hb.to("cuda")
    out = enc(dev)
    g = torch.Generator(device="cpu").manual_seed(seed)
    dout = torch.randn(out.shape, generator=g).cuda()
    sg = enc.backward(dev, dout, out=out)
    n = sg.count()
    got_rows = sg.rows[:n].cpu().numpy()
    got_grad = sg.grad[:n].cpu().numpy()
    flags = O.FLAG_MASK_PADDING if enc.mask_padding else 0
    want_rows, want_grad = O.fused_hash_embed_bwd(enc.host_desc, hb.tok_bytes, hb.tok_off, hb.bag_off, hb.lmax,
                                                  hb.batch, enc.table.cpu().numpy(), enc.dim, out.cpu().numpy(),
                                                  dout.cpu().numpy(), flags)
    return sg, got_rows, got_grad, want_rows, want_grad


@pytest.mark.parametrize("dim", [4, 16, 64, 128])
@pytest.mark.parametrize("masked", [False, True])
def test_bwd_every_combiner(O, cuda, dim, masked):
    S, B = 12, 96
    specs = [SlotSpec(f"f{s}", 50 + 7 * s, (2022 + s, 2023), COMBS[s % 6]) for s in range(S)]
    enc = FusedSparseEncoder(specs, dim, seed=3, mask_padding=masked)
    hb = synthetic_batch(B, [s % 2 == 0 for s in range(S)], seed=11, id_max=40)  # small vocab: many collisions
    _, gr, gg, wr, wg = run_bwd(O, enc, hb, seed=1)
    np.testing.assert_array_equal(gr, wr)
    assert np.array_equal(bits(gg), bits(wg)), np.abs(gg - wg).max()


@pytest.mark.parametrize("dim", [4, 40, 64, 128, 256])
def test_bwd_long_segments(O, cuda, dim):
    """Rows with thousands of positions (a 5-id vocabulary over 1,024 examples, pad rows of multi-valued slots)
    take the long-segment kernel: its in-order adds bit-exact at every dim the lane mapping handles."""
    S, B = 4, 1024
    specs = [SlotSpec(f"f{s}", 3 + s, (2022 + s, 2023), COMBS[s % 6]) for s in range(S)]
    enc = FusedSparseEncoder(specs, dim, seed=9)
    hb = synthetic_batch(B, [True, False, True, False], seed=5, id_max=5)
    _, gr, gg, wr, wg = run_bwd(O, enc, hb, seed=4)
    np.testing.assert_array_equal(gr, wr)
    assert np.array_equal(bits(gg), bits(wg)), np.abs(gg - wg).max()


def test_bwd_ties_empty_tokens_and_empty_bags(O, cuda):
    # duplicate tokens in one bag (max/min ties), b"" tokens (= the pad row), empty bags, lmax padding
    rows = []
    rng = np.random.default_rng(4)
    for b in range(40):
        r = []
        for s in range(6):
            n = int(rng.integers(0, 5))
            r.append([rng.choice([b"", b"a", b"b", b"a", b"zz"]) for _ in range(n)])
        rows.append(r)
    hb = from_lists(rows, lmax=[6, 4, 5, 4, 4, 7])
    specs = [SlotSpec(f"f{s}", 3 + s, (7, 9), c) for s, c in enumerate(["max", "min", "sum", "avg", "first", "last"])]
    for masked in (False, True):
        enc = FusedSparseEncoder(specs, 8, seed=5, mask_padding=masked)
        _, gr, gg, wr, wg = run_bwd(O, enc, hb, seed=2)
        np.testing.assert_array_equal(gr, wr)
        assert np.array_equal(bits(gg), bits(wg))


def test_bwd_cfg2_full_size(O, cuda):
    """base_recall_sdpa.yaml: 229 slots, 10M x 64 fp32 fused table, B = 4096 — bit-exact."""
    import os

    from recommendflow_amd.config_parser.configuration import Configuration

    conf = Configuration(os.path.join(os.path.dirname(__file__), "golden", "conf", "base_recall_sdpa.yaml"))
    feats = conf.features.hashing_features
    nb = 10_000_000 // (2 * len(feats))
    specs = [SlotSpec(f.name, nb, tuple(f.hash_seeds), f.pooling.value) for f in feats]
    enc = FusedSparseEncoder(specs, 64, seed=2023)
    hb = synthetic_batch(4096, [bool(f.multivalued) for f in feats], seed=1234)
    sg, gr, gg, wr, wg = run_bwd(O, enc, hb, seed=3)
    np.testing.assert_array_equal(gr, wr)
    assert np.array_equal(bits(gg), bits(wg))
    assert len(gr) > 100_000


@pytest.mark.parametrize("lazy", [False, True])
def test_adam_matches_keras_restatement(O, cuda, lazy):
    S, B, D = 8, 64, 16
    specs = [SlotSpec(f"f{s}", 97, (2022, 2023), COMBS[s % 4]) for s in range(S)]
    enc = FusedSparseEncoder(specs, D, seed=9)
    opt = SparseAdam(enc.table, learning_rate=0.01, lazy=lazy)
    t_ref = enc.table.cpu().numpy().copy()
    m_ref = np.zeros_like(t_ref)
    v_ref = np.zeros_like(t_ref)
    for step in range(3):
        hb = synthetic_batch(B, [s % 3 == 0 for s in range(S)], seed=100 + step, id_max=200)
        dev = hb.to("cuda")
        out = enc(dev)
        dout = torch.randn(out.shape, generator=torch.Generator().manual_seed(step)).cuda()
        sg = enc.backward(dev, dout, out=out)
        n = sg.count()
        wr, wg = O.fused_hash_embed_bwd(enc.host_desc, hb.tok_bytes, hb.tok_off, hb.bag_off, hb.lmax, B, t_ref, D,
                                        out.cpu().numpy(), dout.cpu().numpy())
        np.testing.assert_array_equal(sg.rows[:n].cpu().numpy(), wr)
        lr = O.keras_adam_lr(0.01, 0.9, 0.999, step + 1)
        assert lr == opt.step_lr()
        opt.apply(sg)
        O.adam_apply(t_ref, m_ref, v_ref, wr, wg, lr, 0.9, 0.999, 1e-7, lazy=lazy)
        assert np.array_equal(bits(enc.table.cpu().numpy()), bits(t_ref)), step
        assert np.array_equal(bits(opt.m.cpu().numpy()), bits(m_ref))
        assert np.array_equal(bits(opt.v.cpu().numpy()), bits(v_ref))


def test_bwd_rejects_wrong_positions(O, cuda):
    specs = [SlotSpec("a", 10, (1, 2))]
    enc = FusedSparseEncoder(specs, 8, seed=1)
    hb = synthetic_batch(8, [True], seed=1)
    dev = hb.to("cuda")
    dev.host_lmax = np.array([int(hb.lmax[0]) + 1], np.int32)  # inconsistent host lmax -> n_positions wrong
    out = enc(dev)
    sg = enc.backward(dev, torch.ones_like(out))
    with pytest.raises(ValueError, match="error bits 2"):
        sg.count()


@pytest.mark.parametrize("n", [1, 7, 4096, 1000003])
def test_keras_adam_dense_matches_oracle(O, cuda, n):
    """backend.optim.KerasAdam (rf_adam_dense) vs oracle.adam_dense over three steps: bit-exact (the float4 path
    for n % 4 == 0, the scalar one otherwise)."""
    from recommendflow_amd.backend.optim import KerasAdam

    g = torch.Generator().manual_seed(n)
    w0 = torch.randn(n, generator=g)
    p = torch.nn.Parameter(w0.clone().cuda())
    opt = KerasAdam([p], learning_rate=0.01)
    w, m, v = w0.numpy().copy(), np.zeros(n, np.float32), np.zeros(n, np.float32)
    for step in range(1, 4):
        grad = torch.randn(n, generator=g) * (10.0 ** -step)
        opt.zero_grad()
        p.grad = grad.cuda()
        opt.step()
        O.adam_dense(w, grad.numpy(), m, v, O.keras_adam_lr(0.01, 0.9, 0.999, step), 0.9, 0.999, 1e-7)
    torch.cuda.synchronize()
    assert np.array_equal(bits(p.detach().cpu().numpy()), bits(w))
    assert np.array_equal(bits(opt.m[0].cpu().numpy()), bits(m))
    assert np.array_equal(bits(opt.v[0].cpu().numpy()), bits(v))


def test_keras_adam_multi_tensor_list(O, cuda):
    """One rf_adam_dense_multi launch over parameters of mixed sizes (scalar and float4 paths) and a parameter
    without a gradient (skipped, as Keras skips None gradients): each bit-exact vs oracle.adam_dense."""
    from recommendflow_amd.backend.optim import KerasAdam

    g = torch.Generator().manual_seed(3)
    sizes = [7, 4096, 1000003, 64]
    ps = [torch.nn.Parameter(torch.randn(n, generator=g).cuda()) for n in sizes]
    ref = [(p.detach().cpu().numpy().copy(), np.zeros(p.numel(), np.float32), np.zeros(p.numel(), np.float32)) for p in ps]
    opt = KerasAdam(ps, learning_rate=0.003)
    for step in range(1, 4):
        opt.zero_grad()
        for i, p in enumerate(ps):
            if i == 3 and step == 2:
                continue  # no gradient this step
            gr = torch.randn(p.numel(), generator=g)
            p.grad = gr.cuda()
            w, m, v = ref[i]
            O.adam_dense(w, gr.numpy(), m, v, O.keras_adam_lr(0.003, 0.9, 0.999, step), 0.9, 0.999, 1e-7)
        opt.step()
    torch.cuda.synchronize()
    for p, (w, m, v), om, ov in zip(ps, ref, opt.m, opt.v):
        assert np.array_equal(bits(p.detach().cpu().numpy()), bits(w))
        assert np.array_equal(bits(om.cpu().numpy()), bits(m))
        assert np.array_equal(bits(ov.cpu().numpy()), bits(v))


def _positions_per_row(O, enc, hb):
    """Number of gradient positions of every fused-table row (the reference's padded [B, Lmax] id tensor per slot
    and table: tokens at their bucket row, pad positions at the slot's pad row)."""
    _, idx = O.fused_hash_embed(enc.host_desc, hb.tok_bytes, hb.tok_off, hb.bag_off, hb.lmax, hb.batch,
                                enc.table.cpu().numpy(), enc.dim, enc.out_width, emit_idx=True)
    S = len(enc.slots)
    empty = from_lists([[[b""] for _ in range(S)]])
    _, pidx = O.fused_hash_embed(enc.host_desc, empty.tok_bytes, empty.tok_off, empty.bag_off, empty.lmax, 1,
                                 enc.table.cpu().numpy(), enc.dim, enc.out_width, emit_idx=True)
    rb = np.asarray(enc.host_desc["row_base"], np.int64)  # [S][2]
    lens = np.diff(hb.bag_off).reshape(hb.batch, S)
    slot_of_tok = np.repeat(np.tile(np.arange(S), hb.batch), lens.reshape(-1))
    cnt = np.zeros(enc.table.shape[0], np.int64)
    for k in range(2):
        np.add.at(cnt, rb[slot_of_tok, k] + idx[: len(slot_of_tok), k], 1)
        pads = (np.asarray(hb.lmax)[None, :] - lens).sum(axis=0)  # pad positions per slot
        np.add.at(cnt, rb[:, k] + pidx[:S, k], pads)
    return cnt


@pytest.mark.parametrize("dim", [16, 64, 128])
def test_bwd_tree_reduce_within_bound(O, cuda, dim):
    """RF_FLAG_TREE_REDUCE (FusedSparseEncoder.tree_reduce): rows with more than 256 positions are summed as
    fixed-order partials + a pairwise tree. Against the oracle's CPU-order sums every element must satisfy SURVEY
    §8d's bar |d| <= L 2^-23 sum|x| (L = the row's positions, sum|x| = the oracle on |dout|); rows and short
    segments are bit-exact, and the result replays bit-identically."""
    S, B = 4, 2048
    specs = [SlotSpec(f"f{s}", 3 + s, (2022 + s, 2023), COMBS[s % 6]) for s in range(S)]
    enc = FusedSparseEncoder(specs, dim, seed=9)
    enc.tree_reduce = True
    hb = synthetic_batch(B, [True, False, True, False], seed=5, id_max=5)
    dev = hb.to("cuda")
    out = enc(dev)
    dout = torch.randn(out.shape, generator=torch.Generator().manual_seed(4)).cuda()
    sg = enc.backward(dev, dout, out=out)
    n = sg.count()
    gr, gg = sg.rows[:n].cpu().numpy(), sg.grad[:n].cpu().numpy()
    sg2 = enc.backward(dev, dout, out=out)
    assert np.array_equal(bits(sg2.grad[:n].cpu().numpy()), bits(gg))  # replay-deterministic
    args = (enc.host_desc, hb.tok_bytes, hb.tok_off, hb.bag_off, hb.lmax, hb.batch, enc.table.cpu().numpy(), enc.dim,
            out.cpu().numpy())
    wr, wg = O.fused_hash_embed_bwd(*args, dout.cpu().numpy())
    _, wabs = O.fused_hash_embed_bwd(*args, np.abs(dout.cpu().numpy()))
    np.testing.assert_array_equal(gr, wr)
    L = _positions_per_row(O, enc, hb)[gr].astype(np.float64)
    assert L.max() > 256  # the long-segment kernel ran
    bound = L[:, None] * 2.0 ** -23 * wabs.astype(np.float64)
    err = np.abs(gg.astype(np.float64) - wg.astype(np.float64))
    assert (err <= bound).all(), float((err - bound).max())
    short = L <= 256
    assert np.array_equal(bits(gg[short]), bits(wg[short]))


@pytest.mark.parametrize("dim", [4, 40, 64, 128])
def test_adam_deferred_replay_matches_dense(cuda, dim):
    """SparseAdam(deferred=True) against the one-launch dense Adam over seven steps whose row sets differ (rows
    untouched for up to six steps): after prepare() / prepare_ids() (repeated and out-of-table ids) the listed
    rows equal the dense table's rows; after
    materialize() table, m and v are bit-identical; an invalid batch (n_uniq < 0) moves nothing."""
    from recommendflow_amd.backend.encoder.sparse_encoder import SparseGrad

    R = 3000
    g0 = torch.Generator().manual_seed(dim)
    base = torch.randn((R, dim), generator=g0).cuda()
    dense = SparseAdam(base.clone(), learning_rate=0.01)
    defer = SparseAdam(base.clone(), learning_rate=0.01, deferred=True)
    for k in range(7):
        n = [900, 40, 2500, 7, 1200, 300, 2999][k]
        rows = torch.sort(torch.randperm(R, generator=g0)[:n]).values.cuda()
        grad = torch.randn((n, dim), generator=g0).cuda()
        nu = torch.tensor([n], dtype=torch.int32, device="cuda")
        g = SparseGrad(rows, grad, nu, n)
        if k % 2:  # an id list with repeats and out-of-table ids (a shard's served requests): each row replayed once
            ids = torch.cat([rows, torch.tensor([-1, R, R + 5], device="cuda"), rows.flip(0)])
            defer.prepare_ids(ids)
        else:
            defer.prepare(rows, nu, n)
        assert torch.equal(defer.table[rows], dense.table[rows])
        dense.apply(g)
        defer.apply(g)
        assert torch.equal(defer.table[rows], dense.table[rows])
    bad = torch.tensor([-1], dtype=torch.int32, device="cuda")
    before = defer.table.clone()
    defer.prepare(rows, bad, n)
    assert torch.equal(before, defer.table)
    defer.materialize()
    torch.cuda.synchronize()
    for a, b in ((defer.table, dense.table), (defer.m, dense.m), (defer.v, dense.v)):
        assert np.array_equal(bits(a.cpu().numpy()), bits(b.cpu().numpy()))
    assert int(defer.last.min()) == defer.iterations == 7


def test_adam_invalid_batch_same_rule_every_mode(cuda):
    """one rule for an invalid batch (n_uniq < 0, the backward plan's error flag) in every table-Adam mode:
    the step counts, no row takes a gradient, every row takes that step's untouched update. The one-launch dense
    Adam, the split form (untouched rows, then the listed rows) and the deferred form (replayed at materialize) stay
    bit-identical over valid, invalid, valid steps."""
    from recommendflow_amd.backend.encoder.sparse_encoder import SparseGrad

    R, dim = 2000, 32
    g0 = torch.Generator().manual_seed(5)
    base = torch.randn((R, dim), generator=g0).cuda()
    dense = SparseAdam(base.clone(), learning_rate=0.01)
    split = SparseAdam(base.clone(), learning_rate=0.01)
    defer = SparseAdam(base.clone(), learning_rate=0.01, deferred=True)
    for k, valid in enumerate((True, False, True)):
        n = 700
        rows = torch.sort(torch.randperm(R, generator=g0)[:n]).values.cuda()
        grad = torch.randn((n, dim), generator=g0).cuda()
        nu = torch.tensor([n if valid else -4], dtype=torch.int32, device="cuda")
        g = SparseGrad(rows, grad, nu, n)
        dense.apply(g)
        split.apply_untouched(rows, nu, n)
        split.apply_touched(g)
        defer.prepare(rows, nu, n)
        defer.apply(g)
    defer.materialize()
    torch.cuda.synchronize()
    assert dense.iterations == split.iterations == defer.iterations == 3
    for x in (split, defer):
        for a, b in ((x.table, dense.table), (x.m, dense.m), (x.v, dense.v)):
            assert np.array_equal(bits(a.cpu().numpy()), bits(b.cpu().numpy()))
    assert not torch.equal(dense.table, base)
