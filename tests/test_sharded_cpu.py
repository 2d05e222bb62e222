"""Row-sharded lookup on CPU ranks: routing, all-to-all exchange and un-permute.

The sharded result must equal the unsharded fused lookup bit for bit (same logical table for any P,
same pooling order). Stage kernels are the oracle's (tests/shard_helpers.py); the GPU stages are
checked against the same property in tests/test_sharded_gpu.py.
"""
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from recommendflow_amd.backend.encoder.sharded_encoder import (ShardedFusedEncoder, build_slot_desc, shard_rows,
                                                               simulate_sharded_backward, simulate_sharded_forward)
from shard_helpers import OracleShardOps, dist_worker, rank_batch, sharded_grad_oracle, small_slots

DIM, SEED = 8, 11


def unsharded(O, rank):
    desc, rows = build_slot_desc(small_slots(), DIM)
    table = O.table_init_uniform(rows, DIM, seed=SEED)
    b = rank_batch(rank)
    out, _ = O.fused_hash_embed(desc, b.tok_bytes, b.tok_off, b.bag_off, b.lmax, b.batch, table, DIM,
                                2 * DIM * len(desc))
    return out


def partial_desc():
    return build_slot_desc(small_slots(), DIM)[0]


def full_table():
    from oracle import oracle as O

    desc, rows = build_slot_desc(small_slots(), DIM)
    return O.table_init_uniform(rows, DIM, seed=SEED)


def test_shard_rows_partition():
    for R in (0, 1, 7, 100, 101):
        for P in (1, 2, 3, 8):
            assert sum(shard_rows(R, r, P) for r in range(P)) == R
            assert all(shard_rows(R, r, P) == len(range(r, R, P)) for r in range(P))


def test_pool_rows_equals_fused(O):
    desc, rows = build_slot_desc(small_slots(), DIM)
    table = O.table_init_uniform(rows, DIM, seed=SEED)
    b = rank_batch(0)
    want = unsharded(O, 0)
    req = np.concatenate([O.hash_rows(desc, b.tok_bytes, b.tok_off, b.bag_off, b.batch),
                          O.hash_rows(desc, np.zeros(0, np.uint8), np.zeros(len(desc) + 1, np.int32),
                                      np.arange(len(desc) + 1, dtype=np.int32), 1)])
    got = O.pool_rows(desc, b.bag_off, b.lmax, b.batch, b.n_tokens, table[req], DIM, want.shape[1])
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("P", [1, 2, 3, 8])
@pytest.mark.parametrize("dedup", [False, True])
def test_simulated_shards_bit_exact(O, P, dedup):
    encs = [ShardedFusedEncoder(small_slots(), DIM, r, P, ops=OracleShardOps(), seed=SEED, device="cpu", dedup=dedup)
            for r in range(P)]
    assert sum(e.local_rows for e in encs) == encs[0].table_rows
    outs = simulate_sharded_forward(encs, [rank_batch(r) for r in range(P)])
    for r in range(P):
        np.testing.assert_array_equal(outs[r].numpy(), unsharded(O, r))


def expected_grads(O, P, douts, mask_padding=False):
    desc, rows = build_slot_desc(small_slots(), DIM)
    table = O.table_init_uniform(rows, DIM, seed=SEED)
    flags = O.FLAG_MASK_PADDING if mask_padding else 0
    batches = [rank_batch(r) for r in range(P)]
    outs = []
    for b in batches:
        out, _ = O.fused_hash_embed(desc, b.tok_bytes, b.tok_off, b.bag_off, b.lmax, b.batch, table, DIM,
                                    2 * DIM * len(desc), flags=flags)
        outs.append(out)
    return sharded_grad_oracle(O, desc, table, DIM, batches, outs, douts, P, flags)


@pytest.mark.parametrize("P", [1, 2, 3])
@pytest.mark.parametrize("mask_padding", [False, True])
def test_simulated_backward(O, P, mask_padding):
    """Sharded training gradient: requester pool_rows_bwd + reverse exchange + owner segment sum equals each
    rank's unsharded backward summed over ranks in rank order (DESIGN D-sharded-grad-order)."""
    encs = [ShardedFusedEncoder(small_slots(), DIM, r, P, ops=OracleShardOps(), seed=SEED, device="cpu",
                                mask_padding=mask_padding) for r in range(P)]
    rng = np.random.default_rng(7)
    douts = [torch.from_numpy(rng.standard_normal((24, 2 * DIM * 12)).astype(np.float32)) for _ in range(P)]
    outs, grads = simulate_sharded_backward(encs, [rank_batch(r) for r in range(P)], douts)
    want = expected_grads(O, P, [d.numpy() for d in douts], mask_padding)
    for o in range(P):
        n = grads[o].count()
        np.testing.assert_array_equal(grads[o].rows[:n].numpy(), want[o][0])
        assert np.array_equal(grads[o].grad[:n].numpy().view(np.uint32), want[o][1].view(np.uint32))


def test_gloo_world2_bit_exact(O, tmp_path):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(dist_worker, args=(2, port, DIM, SEED, str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        np.testing.assert_array_equal(np.load(tmp_path / f"out{r}.npy"), unsharded(O, r))
        np.testing.assert_array_equal(np.load(tmp_path / f"pipe{r}.npy"), unsharded(O, r))  # pipelined, 3 micro
        np.testing.assert_array_equal(np.load(tmp_path / f"radix{r}.npy"), unsharded(O, r))
        b = rank_batch(r)  # owner-side partial pooling over gloo: the oracle's owner-ordered restatement, bit-exact
        d = partial_desc()
        want_pp = O.partial_pool(d, b.tok_bytes, b.tok_off, b.bag_off, b.lmax, b.batch, full_table(), DIM,
                                 2 * DIM * len(d), 2)
        np.testing.assert_array_equal(np.load(tmp_path / f"pp{r}.npy").view(np.uint32), want_pp.view(np.uint32))
    want = expected_grads(O, 2, [np.load(tmp_path / f"dout{r}.npy") for r in range(2)])
    for o in range(2):
        np.testing.assert_array_equal(np.load(tmp_path / f"gid{o}.npy"), want[o][0])
        np.testing.assert_array_equal(np.load(tmp_path / f"gval{o}.npy").view(np.uint32), want[o][1].view(np.uint32))
