"""Data-parallel gradient sync (runtime/dist.py; SURVEY §8f.1 "the dense all-reduce") on CPU ranks over gloo.

Dense: bucketed SUM all-reduce == the elementwise sum of the ranks' gradients (bit-exact for 2 ranks:
one fp32 add). Sparse: all-gather of deduplicated (row, grad) pairs + rf_segment_sum_rows in rank order
== the oracle's rank-ordered sum (tests/shard_helpers.OracleShardOps stands in for the GPU segment sum).
"""
import os
import socket

import numpy as np
import torch
import torch.multiprocessing as mp

from shard_helpers import OracleShardOps


def rank_tensors(rank):
    g = torch.Generator().manual_seed(100 + rank)
    dense = [torch.randn(37, 5, generator=g), torch.randn(3000, generator=g), torch.randn(1, generator=g)]
    rows = torch.unique(torch.randint(0, 500, (80 + 17 * rank,), generator=g))  # ascending, distinct
    grad = torch.randn(rows.numel(), 8, generator=g)
    return dense, rows, grad


def worker(rank, world, port, out_dir):
    import torch.distributed as dist

    from recommendflow_amd.backend.encoder.sparse_encoder import SparseGrad
    from recommendflow_amd.runtime.dist import DataParallel

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        dp = DataParallel(bucket_bytes=4096, ops=OracleShardOps())
        dense, rows, grad = rank_tensors(rank)
        params = [torch.nn.Parameter(torch.zeros_like(d)) for d in dense]
        for p, d in zip(params, dense):
            p.grad = d.clone()
        nb = dp.allreduce_dense(params)
        sg = dp.allgather_sparse(SparseGrad(rows, grad, torch.tensor([rows.numel()], dtype=torch.int32), rows.numel()), 500)
        n = sg.count()
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), *[p.grad.numpy() for p in params], rows=sg.rows[:n].numpy(),
                 grad=sg.grad[:n].numpy(), nb=np.array(nb), scale=np.array(dp.loss_scale()))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_dense_and_sparse(O, tmp_path):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    world = 2
    mp.spawn(worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    ranks = [rank_tensors(r) for r in range(world)]
    want_dense = [sum(ranks[r][0][i] for r in range(world)) for i in range(3)]
    ids = torch.cat([ranks[r][1] for r in range(world)]).numpy()
    vals = torch.cat([ranks[r][2] for r in range(world)]).numpy()
    want_rows, want_grad = O.segment_sum_rows(ids, vals)
    for r in range(world):
        z = np.load(tmp_path / f"r{r}.npz")
        for i in range(3):
            np.testing.assert_array_equal(z[f"arr_{i}"], want_dense[i].numpy())
        assert int(z["nb"]) >= 2  # 4 KB buckets: the 12 KB tensor gets its own bucket
        assert float(z["scale"]) == 0.5
        np.testing.assert_array_equal(z["rows"], want_rows)
        np.testing.assert_array_equal(z["grad"].view(np.uint32), want_grad.view(np.uint32))


def buffer_worker(rank, world, port, out_dir):
    import torch.distributed as dist

    from recommendflow_amd.runtime.dist import DataParallel

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        dp = DataParallel(ops=OracleShardOps())
        bn = torch.nn.BatchNorm1d(6, eps=1e-6, momentum=0.01).train()
        x = torch.randn(32, 6, generator=torch.Generator().manual_seed(7 + rank)) * (1 + rank)
        bn(x)  # rank-local moving statistics
        local = [bn.running_mean.clone(), bn.running_var.clone()]
        n = dp.sync_buffers([bn])
        np.savez(os.path.join(out_dir, f"b{rank}.npz"), lm=local[0].numpy(), lv=local[1].numpy(),
                 m=bn.running_mean.numpy(), v=bn.running_var.numpy(), n=np.array(n),
                 t=np.array(int(bn.num_batches_tracked)))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_bn_buffers_mean(tmp_path):
    """BatchNorm moving statistics are MEAN-aggregated over replicas (MirroredStrategy ON_READ/MEAN):
    after sync every rank holds the same buffers, equal to the mean of the rank-local ones."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(buffer_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    z = [np.load(tmp_path / f"b{r}.npz") for r in range(2)]
    assert not np.array_equal(z[0]["lm"], z[1]["lm"])  # the ranks really diverged before the sync
    for r in range(2):
        assert int(z[r]["n"]) == 2 and int(z[r]["t"]) == 1
        np.testing.assert_allclose(z[r]["m"], (z[0]["lm"] + z[1]["lm"]) / 2, rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(z[r]["v"], (z[0]["lv"] + z[1]["lv"]) / 2, rtol=1e-6, atol=1e-7)
    np.testing.assert_array_equal(z[0]["m"], z[1]["m"])
    np.testing.assert_array_equal(z[0]["v"], z[1]["v"])
