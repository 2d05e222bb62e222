"""Row-sharded lookup on the GPU: rf_hash_rows, rf_bucketize_owner, rf_gather_rows,
rf_pool_rows_fwd through the C ABI, composed by ShardedFusedEncoder.

Bar: bit-exact. P shards are simulated in one process (the exchange done by slicing; one GPU per box);
the torch.distributed exchange itself is covered by the gloo test in tests/test_sharded_cpu.py.
"""
import numpy as np
import pytest
import torch

from recommendflow_amd.backend.encoder.sharded_encoder import (GpuShardOps, ShardedFusedEncoder,
                                                               simulate_sharded_forward)
from recommendflow_amd.backend.encoder.sparse_encoder import FusedSparseEncoder, SlotSpec
from recommendflow_amd.runtime.batch import synthetic_batch

pytestmark = pytest.mark.gpu
COMBS = ["sum", "avg", "max", "min", "first", "last"]


def slots(n=40, seed=0):
    rng = np.random.default_rng(seed)
    return [SlotSpec(f"s{i}", int(rng.integers(100, 200000)), (2022 + i, 2029 + i), COMBS[i % 6],
                     mask_empty=(i % 7 != 3)) for i in range(n)]


def bits(t):
    t = t.cpu()
    return t.view(torch.int16).numpy() if t.dtype == torch.bfloat16 else t.numpy().view(np.uint32)


def test_hash_rows_matches_oracle(O, cuda):
    sp = slots()
    enc = FusedSparseEncoder(sp, 16, seed=3)
    hb = synthetic_batch(300, [i % 3 == 0 for i in range(len(sp))], seed=5)
    got = GpuShardOps().hash_rows(enc.desc, len(sp), hb.to("cuda")).cpu().numpy()
    want = O.hash_rows(enc.host_desc, hb.tok_bytes, hb.tok_off, hb.bag_off, hb.batch)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("P", [1, 2, 3, 8, 64, 1000])
@pytest.mark.parametrize("n", [0, 1, 63, 2047, 2048, 2049, 300001])
def test_bucketize_matches_oracle(O, cuda, P, n):
    rng = np.random.default_rng(n * 7 + P)
    rows = rng.integers(0, 10 ** 9, n).astype(np.int64)
    rows[: n // 3] = rng.integers(0, 50, n // 3)  # hot rows: many equal owners in a round
    c, p, l, inv = GpuShardOps().bucketize(torch.from_numpy(rows).cuda(), P)
    wc, wp, wl, winv = O.bucketize_owner(rows, P)
    np.testing.assert_array_equal(c.cpu().numpy(), wc)
    np.testing.assert_array_equal(p.cpu().numpy(), wp)
    np.testing.assert_array_equal(l.cpu().numpy(), wl)
    np.testing.assert_array_equal(inv.cpu().numpy(), winv)


@pytest.mark.parametrize("tdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("mask_padding", [False, True])
@pytest.mark.parametrize("dim", [16, 64, 128])
def test_pool_rows_equals_fused(O, cuda, tdt, mask_padding, dim):
    sp = slots(24, seed=dim)
    enc = FusedSparseEncoder(sp, dim, table_dtype=tdt, seed=9, mask_padding=mask_padding)
    hb = synthetic_batch(257, [i % 4 == 0 for i in range(len(sp))], seed=dim)
    db = hb.to("cuda")
    want = enc(db)
    ops = GpuShardOps()
    sh = ShardedFusedEncoder(sp, dim, 0, 1, ops=ops, table_dtype=tdt, seed=9, mask_padding=mask_padding)
    assert torch.equal(sh.shard.view(torch.int16) if tdt == torch.bfloat16 else sh.shard,
                       enc.table.view(torch.int16) if tdt == torch.bfloat16 else enc.table)
    req = torch.cat([ops.hash_rows(enc.desc, len(sp), db), sh.pad_rows])
    gathered = ops.gather(enc.table, req)
    got = ops.pool(enc.desc, len(sp), db, gathered, torch.empty_like(want), 1 if mask_padding else 0)
    np.testing.assert_array_equal(bits(got), bits(want))
    # through a row map: gathered rows stored permuted, read back at row_map[j]
    perm = torch.randperm(req.numel(), generator=torch.Generator().manual_seed(dim)).cuda()
    shuffled = torch.empty_like(gathered)
    shuffled[perm] = gathered
    got = ops.pool(enc.desc, len(sp), db, shuffled, torch.empty_like(want), 1 if mask_padding else 0,
                   row_map=perm.to(torch.int32))
    np.testing.assert_array_equal(bits(got), bits(want))


@pytest.mark.parametrize("P", [1, 2, 8, 1000])
@pytest.mark.parametrize("n", [0, 1, 1000, 300001])
def test_route_rows_matches_oracle(O, cuda, P, n):
    rng = np.random.default_rng(n + P)
    R = 50_000_000
    rows = (rng.zipf(1.2, n) * 7919 % R).astype(np.int64)
    if n > 10:
        rows[3] = -5          # invalid rows: local -1 (gathered as NaN)
        rows[7] = R + 11
    c, l, m = GpuShardOps().route(torch.from_numpy(rows).cuda(), P, R)
    wc, wl, wm = O.route_rows(rows, P, R)
    np.testing.assert_array_equal(c.cpu().numpy(), wc)
    np.testing.assert_array_equal(l.cpu().numpy()[: int(wc.sum())], wl)
    np.testing.assert_array_equal(m.cpu().numpy(), wm)


@pytest.mark.parametrize("P", [1, 2, 3, 8, 1000])
@pytest.mark.parametrize("rank", [-1, 0, "last"])
@pytest.mark.parametrize("n", [0, 1, 1000, 300001])
def test_route_hash_matches_oracle(O, cuda, P, rank, n):
    """rf_route_hash_build/finish (hash-table dedup; rows of `rank` left in place) == oracle.route_rows_local."""
    rank = P - 1 if rank == "last" else rank
    rng = np.random.default_rng(n + 3 * P)
    R = 50_000_000
    rows = (rng.zipf(1.2, n) * 7919 % R).astype(np.int64)
    if n > 10:
        rows[3] = -5          # invalid rows: routed to the last owner, local -1 (gathered as NaN)
        rows[7] = R + 11
    ops = GpuShardOps()
    c, state = ops.route_hash_build(torch.from_numpy(rows).cuda(), P, rank, R)
    _check_route_hash(O, ops, rows, P, rank, R, c, state)


def _check_route_hash(O, ops, rows, P, rank, R, c, state):
    wc, wl, wm = O.route_rows_local(rows, P, rank, R)
    np.testing.assert_array_equal(c.cpu().numpy(), wc)
    l, m = ops.route_hash_finish(state, int(wc.sum()))
    l, m = l.cpu().numpy(), m.cpu().numpy()
    if P > 64:  # compacted keys radix-sorted: the oracle's order exactly
        np.testing.assert_array_equal(l, wl)
        np.testing.assert_array_equal(m, wm)
        return
    # P <= 64: owner-major without the sort (rh_scatter_owner_kernel): within an owner the distinct rows come in
    # table-slot order, so each owner's segment is the oracle's as a set and every request maps to its own row
    ends = np.cumsum(wc)
    for p in range(P):
        seg = slice(int(ends[p] - wc[p]), int(ends[p]))
        got = l[seg]
        got = got[np.lexsort((got, got < 0))]  # key order: the invalid-row sentinel (-1) sorts last
        np.testing.assert_array_equal(got, wl[seg])
    loc = wm < 0  # rank-local rows: 0x80000000 | local, exact
    np.testing.assert_array_equal(m[loc], wm[loc])
    np.testing.assert_array_equal(l[m[~loc]], wl[wm[~loc]])


@pytest.mark.parametrize("P", [1, 2, 8, 1000])
@pytest.mark.parametrize("rank", [-1, 0])
@pytest.mark.parametrize("B", [0, 1, 300])
def test_route_hash_tokens_matches_oracle(O, cuda, P, rank, B):
    """rf_route_hash_build_tokens (rf_hash_rows fused into the insert) == oracle.route_rows_local over the oracle's
    hashed request list [2 n_tok token rows | the slots' pad rows]: the counts, the distinct rows per owner and every
    request's row."""
    sp = slots(30, seed=P + 1)
    enc = FusedSparseEncoder(sp, 16, seed=1)
    hb = synthetic_batch(B, [i % 3 == 0 for i in range(len(sp))], seed=P + B)
    ops = GpuShardOps()
    sh = ShardedFusedEncoder(sp, 16, 0, P, ops=ops, seed=1)
    R = sh.table_rows
    rows = np.concatenate([O.hash_rows(enc.host_desc, hb.tok_bytes, hb.tok_off, hb.bag_off, hb.batch).reshape(-1),
                           sh.pad_rows.cpu().numpy()]).astype(np.int64)
    c, state, n = ops.route_hash_build_tokens(enc.desc, len(sp), hb.to("cuda"), sh.pad_rows, P, rank, R)
    assert n == rows.size
    if P <= 64:  # the device-count finish (n_uniq = -1, enqueued before the host read) writes the same ids and map
        l_dev, m_dev = ops.route_hash_finish(state, -1)
        l_dev, m_dev = l_dev.clone(), m_dev.clone()
        l_host, m_host = ops.route_hash_finish(state, int(c.sum()))
        assert torch.equal(l_dev[: l_host.numel()], l_host) and torch.equal(m_dev, m_host)
    _check_route_hash(O, ops, rows, P, rank, R, c, state)


@pytest.mark.parametrize("P", [1, 2, 4, 8])
@pytest.mark.parametrize("tdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("mode", ["bucketize", "radix", "hash", "hash_local"])
def test_simulated_shards_bit_exact(cuda, P, tdt, mode):
    sp = slots(48, seed=P)
    full = FusedSparseEncoder(sp, 64, table_dtype=tdt, seed=21)
    encs = [ShardedFusedEncoder(sp, 64, r, P, table_dtype=tdt, seed=21, dedup=mode != "bucketize",
                                route="radix" if mode == "radix" else "hash") for r in range(P)]
    batches = [synthetic_batch(200 + 17 * r, [i % 3 == 0 for i in range(len(sp))], seed=40 + r) for r in range(P)]
    outs = simulate_sharded_forward(encs, batches, local_fast=mode == "hash_local")
    for r in range(P):
        want = full(batches[r].to("cuda"))
        np.testing.assert_array_equal(bits(outs[r]), bits(want))


def _oracle_pooled(O, enc, host_batch, seed, dtype_code, lo=-0.05, hi=0.05):
    """The pooled output of host_batch from the oracle alone: token rows by the oracle's hash (orf_hash_rows), pad
    rows by its bucket of b"" (bin 0 under mask_value ""), each needed row by the oracle's table init (the same
    counter-based rows rf_table_init_uniform writes), then orf_pool_rows_fwd over that compact row set."""
    desc = enc.host_desc
    h = host_batch
    tok_rows = O.hash_rows(desc, h.tok_bytes, h.tok_off, h.bag_off, h.batch)
    pad = np.zeros(2 * len(desc), np.int64)
    for s, d in enumerate(desc):
        for k in range(2):
            salt = int(d["salt"][k])
            b = 0 if d["mask_empty"] else int(O.hash_tokens(np.zeros(1, np.uint8), np.zeros(2, np.int32), salt, salt,
                                                          int(d["num_bins"]), False)[0])
            pad[2 * s + k] = int(d["row_base"][k]) + b
    logical = np.concatenate([tok_rows, pad])
    uniq, inv = np.unique(logical, return_inverse=True)
    rows = np.stack([O.table_init_uniform(1, enc.dim, dtype_code, seed=seed, row0=int(r), row_stride=1, lo=lo, hi=hi)[0]
                     for r in uniq])
    if dtype_code != O.DT_F32:  # bf16 rows widen exactly
        rows = (rows.astype(np.uint32) << 16).view(np.float32)
    return O.pool_rows(desc, h.bag_off, h.lmax, h.batch, h.n_tokens, rows, enc.dim, enc.out_width,
                       row_map=inv.astype(np.int32))


@pytest.mark.parametrize("P", [2, 8])
@pytest.mark.parametrize("tdt", [torch.float32, torch.bfloat16])
def test_simulated_shards_vs_oracle(O, cuda, P, tdt):
    """The simulated P-rank forward against the oracle alone (test_simulated_shards_bit_exact compares
    with this repo's unsharded kernel): every rank's pooled output bit-exact with orf_pool_rows_fwd over rows from
    the oracle's hash and table init (bf16 tables: the oracle's fp32 result rounded to nearest even)."""
    sp = slots(48, seed=P)
    encs = [ShardedFusedEncoder(sp, 64, r, P, table_dtype=tdt, seed=21, dedup=True, route="hash") for r in range(P)]
    batches = [synthetic_batch(120 + 17 * r, [i % 3 == 0 for i in range(len(sp))], seed=60 + r) for r in range(P)]
    outs = simulate_sharded_forward(encs, batches, local_fast=True)
    ref = FusedSparseEncoder(sp, 64, table_dtype=tdt, seed=21)  # descriptors only (the oracle builds the rows)
    code = O.DT_F32 if tdt == torch.float32 else O.DT_BF16
    for r in range(P):
        want = torch.from_numpy(_oracle_pooled(O, ref, batches[r], 21, code))
        if tdt == torch.bfloat16:
            want = want.to(torch.bfloat16)
        np.testing.assert_array_equal(bits(outs[r]), bits(want))


def test_sharded_cfg2_layout(cuda):
    """The 229-slot base_recall_sdpa layout, 10M x 64 fp32 fused table, 4 simulated shards, B=1024 per rank."""
    import os

    from recommendflow_amd.config_parser.configuration import Configuration

    conf = Configuration(os.path.join(os.path.dirname(__file__), "golden", "conf", "base_recall_sdpa.yaml"))
    feats = conf.features.hashing_features
    n_bins = 10_000_000 // (2 * len(feats))
    sp = [SlotSpec(f.name, n_bins, tuple(f.hash_seeds), f.pooling.value) for f in feats]
    full = FusedSparseEncoder(sp, 64, seed=2023)
    P = 4
    encs = [ShardedFusedEncoder(sp, 64, r, P, seed=2023) for r in range(P)]
    batches = [synthetic_batch(1024, [bool(f.multivalued) for f in feats], seed=7 + r) for r in range(P)]
    for lf in (False, True):
        outs = simulate_sharded_forward(encs, batches, local_fast=lf)
        for r in range(P):
            np.testing.assert_array_equal(bits(outs[r]), bits(full(batches[r].to("cuda"))))


@pytest.mark.parametrize("P", [1, 3])
def test_partial_pool_stages_vs_numpy(O, cuda, P):
    """Each rf_pp_* stage against the numpy restatement in tests/shard_helpers.py (plan entries, owner-major order,
    segment counts, seg_of; the owner's segments and partials; the combine)."""
    import sys
    import os

    sys.path.insert(0, os.path.dirname(__file__))
    from shard_helpers import OracleShardOps

    sp = slots(10, seed=P + 3)
    enc = ShardedFusedEncoder(sp, 32, 0, P, seed=4)
    hb = synthetic_batch(40, [i % 3 == 0 for i in range(len(sp))], seed=9, id_max=4000, max_len=7)
    db = hb.to("cuda")
    ops, ref = GpuShardOps(), OracleShardOps()
    rows = torch.cat([ops.hash_rows(enc.desc, len(sp), db), enc.pad_rows])
    got = ops.pp_plan(enc.desc, len(sp), db, rows, 0, P)
    want = ref.pp_plan(enc.host_desc, len(sp), hb, rows.cpu(), 0, P)
    for name, g, w in zip(("ent", "counts", "seg_counts", "seg_of"), got, want):
        np.testing.assert_array_equal(g.cpu().numpy(), w.numpy(), err_msg=name)
    ent = got[0]
    counts = [int(c) for c in got[1].cpu().tolist()]
    chunk = ent[: counts[0]]  # owner 0's entries from this requester
    sc, ss = ops.pp_owner_pool(enc.desc, len(sp), chunk, [counts[0]], enc.shard)
    wsc, wss = ref.pp_owner_pool(enc.host_desc, len(sp), chunk.cpu(), [counts[0]], enc.shard.cpu())
    np.testing.assert_array_equal(sc.cpu().numpy(), wsc.numpy())
    n_seg = int(wsc.sum())
    np.testing.assert_array_equal(ss.cpu().numpy()[:n_seg], wss.numpy())
    part = ops.pp_owner_partials(enc.desc, len(sp), chunk, ss, n_seg, enc.shard)
    wpart = ref.pp_owner_partials(enc.host_desc, len(sp), chunk.cpu(), wss, n_seg, enc.shard.cpu())
    np.testing.assert_array_equal(bits(part), wpart.numpy().view(np.uint32))


@pytest.mark.parametrize("P", [1, 2, 3, 8])
@pytest.mark.parametrize("mask_padding", [False, True])
def test_partial_pool_vs_oracle(O, cuda, P, mask_padding):
    """Owner-side partial pooling (rf_partial.hip, simulated P ranks): bit-exact vs oracle.partial_pool (the
    owner-ordered sum), bit-identical to the unsharded kernel at P = 1 and for max / min / first / last at any P."""
    from recommendflow_amd.backend.encoder.sharded_encoder import simulate_partial_forward

    sp = slots(18, seed=P + 11)
    full = FusedSparseEncoder(sp, 32, seed=4, mask_padding=mask_padding)
    encs = [ShardedFusedEncoder(sp, 32, r, P, seed=4, mask_padding=mask_padding) for r in range(P)]
    batches = [synthetic_batch(90 + 7 * r, [i % 3 == 0 for i in range(len(sp))], seed=60 + r, id_max=4000, max_len=9)
               for r in range(P)]
    outs = simulate_partial_forward(encs, batches)
    table = full.table.cpu().numpy()
    for r in range(P):
        hb = batches[r]
        want = O.partial_pool(full.host_desc, hb.tok_bytes, hb.tok_off, hb.bag_off, hb.lmax, hb.batch, table, 32,
                              full.out_width, P, 1 if mask_padding else 0)
        np.testing.assert_array_equal(bits(outs[r]), want.view(np.uint32))
        ref = bits(full(hb.to("cuda")))
        for i, spc in enumerate(sp):
            cols = slice(i * 64, (i + 1) * 64)
            if P == 1 or spc.combiner in ("max", "min", "first", "last"):
                np.testing.assert_array_equal(bits(outs[r])[:, cols], ref[:, cols], err_msg=f"P={P} {spc.combiner}")


def test_local_comm_forward_pools_in_place(cuda):
    """P = 1 through forward() (LocalComm): every row is rank-local, nothing routed, nothing exchanged; the
    output equals the unsharded kernel's bit for bit."""
    from recommendflow_amd.backend.encoder.sharded_encoder import LocalComm

    sp = slots(30, seed=5)
    full = FusedSparseEncoder(sp, 128, seed=8)
    enc = ShardedFusedEncoder(sp, 128, 0, 1, comm=LocalComm(), seed=8)
    hb = synthetic_batch(640, [i % 3 == 0 for i in range(len(sp))], seed=2).to("cuda")
    st, recv = enc.route_exchange(hb, local_fast=True)
    assert st.counts == [0] and st.n_requests == 0 and recv == [0]
    np.testing.assert_array_equal(bits(enc(hb)), bits(full(hb)))


def full_table(encs):
    P = len(encs)
    rows = encs[0].table_rows
    t = np.zeros((rows, encs[0].dim), np.float32)
    for r, e in enumerate(encs):
        t[r::P] = e.shard.cpu().numpy()
    return t


@pytest.mark.parametrize("P", [1, 2, 4])
@pytest.mark.parametrize("mask_padding", [False, True])
def test_simulated_backward_and_adam(O, cuda, P, mask_padding):
    """Sharded training step (DESIGN D-sharded-grad-order): rf_pool_rows_bwd on every requester, the reverse
    exchange, rf_segment_sum_rows on every owner, SparseAdam on every shard — bit-exact vs the oracle's
    per-rank unsharded backward summed in rank order, and the dense Keras Adam on the logical table."""
    from shard_helpers import sharded_grad_oracle

    from recommendflow_amd.backend.encoder.sharded_encoder import simulate_sharded_backward
    from recommendflow_amd.backend.optim import SparseAdam

    sp = slots(18, seed=10 + P)
    encs = [ShardedFusedEncoder(sp, 16, r, P, seed=5, mask_padding=mask_padding) for r in range(P)]
    batches = [synthetic_batch(64 + 9 * r, [i % 3 == 0 for i in range(len(sp))], seed=70 + r, id_max=300)
               for r in range(P)]
    table0 = full_table(encs)
    g = torch.Generator().manual_seed(P)
    douts = [torch.randn((b.batch, encs[0].out_width), generator=g).cuda() for b in batches]
    outs, grads = simulate_sharded_backward(encs, batches, douts)
    flags = O.FLAG_MASK_PADDING if mask_padding else 0
    want = sharded_grad_oracle(O, encs[0].host_desc, table0, 16, batches, [o.cpu().numpy() for o in outs],
                               [d.cpu().numpy() for d in douts], P, flags)
    for o in range(P):
        n = grads[o].count()
        np.testing.assert_array_equal(grads[o].rows[:n].cpu().numpy(), want[o][0])
        assert np.array_equal(bits(grads[o].grad[:n]), want[o][1].view(np.uint32))
    # Adam on every shard == dense Keras Adam on the logical table with the summed gradient
    for o in range(P):
        SparseAdam(encs[o].shard, learning_rate=0.01).apply(grads[o])
    t, m, v = table0.copy(), np.zeros_like(table0), np.zeros_like(table0)
    rows = np.concatenate([want[o][0] * P + o for o in range(P)])
    gr = np.concatenate([want[o][1] for o in range(P)])
    order = np.argsort(rows)
    O.adam_apply(t, m, v, rows[order], gr[order], O.keras_adam_lr(0.01, 0.9, 0.999, 1), 0.9, 0.999, 1e-7)
    assert np.array_equal(full_table(encs).view(np.uint32), t.view(np.uint32))


def test_sharded_deferred_adam_equals_dense(cuda):
    """The cfg4 training step's optimizer: SparseAdam(deferred=True) on the shard with serve_hook replaying the
    served rows (ids repeat: the forward_train path serves every request) against the dense Keras Adam on a twin
    encoder, four steps over batches with different row sets: the pooled outputs of every step and, after
    materialize(), the shard, m and v bit-identical."""
    from recommendflow_amd.backend.encoder.sharded_encoder import LocalComm
    from recommendflow_amd.backend.optim import SparseAdam

    sp = slots(14, seed=31)
    encs = [ShardedFusedEncoder(sp, 32, 0, 1, comm=LocalComm(), seed=6) for _ in range(2)]
    dense = SparseAdam(encs[0].shard, learning_rate=0.01)
    defer = SparseAdam(encs[1].shard, learning_rate=0.01, deferred=True)
    encs[1].serve_hook = defer.prepare_ids
    hbs = [synthetic_batch(96, [i % 3 == 0 for i in range(len(sp))], seed=90 + k, id_max=150 + 100 * k).to("cuda")
           for k in range(3)]
    g = torch.Generator().manual_seed(3)
    for k in (0, 1, 2, 0):
        dout = torch.randn((96, encs[0].out_width), generator=g).cuda()
        outs = []
        for e, opt in zip(encs, (dense, defer)):
            ctx = e.forward_train(hbs[k])
            outs.append(ctx.out.clone())
            sg = e.backward(ctx, dout)
            if opt.deferred:
                opt.apply(sg, rows_current=True)  # the bench's form: the gradient's rows were served, so replayed
            else:
                opt.apply(sg)
        assert torch.equal(outs[0], outs[1])
    defer.materialize()
    torch.cuda.synchronize()
    for a, b in ((dense.table, defer.table), (dense.m, defer.m), (dense.v, defer.v)):
        assert np.array_equal(bits(a), bits(b))
