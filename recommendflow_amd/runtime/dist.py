"""Data-parallel gradient sync for replicated models ("the dense ncclAllReduce").

The reference trains under `tf.distribute.MirroredStrategy` (run/train.py): every replica
holds all variables, each replica's loss is scaled by 1 / global batch, and the gradients of all
replicas are SUMMED before one optimizer step per replica. The MI355X build keeps that contract with
one process per GPU over torch.distributed (RCCL over xGMI on the GPU box, gloo in the CPU tests):

* dense parameters (towers): gradients flattened into buckets of `bucket_bytes` and all-reduced with
  SUM — a few large collectives instead of one per tensor (xGMI rings are per-link bound, so the
  bucket is sized for bandwidth, not latency);
* the fused embedding table: each rank's deduplicated `SparseGrad` (rows ascending) is all-gathered
  (counts first, then rows and gradients padded to the largest count) and summed per row in rank order
  0..P-1 with rf_segment_sum_rows — the IndexedSlices all-gather + sum of MirroredStrategy with a
  defined order (deviation D-sharded-grad-order). Every rank then applies the same Adam
  step to its replica, so the replicas' PARAMETERS stay bit-identical;
* non-trainable state (BatchNorm moving mean / variance): MirroredStrategy keeps these as ON_READ
  variables with MEAN aggregation, so `sync_buffers` all-reduces every floating buffer and divides by
  P after each step. Without it each replica's moving statistics would follow its own local batches.

`loss_scale()` = 1 / P turns the per-replica mean loss into the reference's per-replica
sum / global_batch (equal per-replica batches).
"""
from __future__ import annotations

from typing import Iterable, List, Optional

import torch

from ..backend.encoder.sparse_encoder import SparseGrad


class DataParallel:
    def __init__(self, group=None, bucket_bytes: int = 64 << 20, ops=None):
        import torch.distributed as dist

        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.bucket_bytes = int(bucket_bytes)
        self._ops = ops  # segment-sum provider (GpuShardOps by default; the CPU tests pass oracle ops)

    @property
    def ops(self):
        if self._ops is None:
            from ..backend.encoder.sharded_encoder import GpuShardOps

            self._ops = GpuShardOps()
        return self._ops

    def loss_scale(self) -> float:
        return 1.0 / self.world

    # -- dense ------------------------------------------------------------------------------------
    def allreduce_dense(self, params: Iterable[torch.nn.Parameter]) -> int:
        """SUM-all-reduce the .grad of every parameter, bucketed by dtype/device; returns the bucket count."""
        grads = [p.grad for p in params if p.grad is not None]
        buckets: List[List[torch.Tensor]] = []
        cur: List[torch.Tensor] = []
        size = 0
        for g in grads:
            nb = g.numel() * g.element_size()
            if cur and (size + nb > self.bucket_bytes or g.dtype != cur[0].dtype or g.device != cur[0].device):
                buckets.append(cur)
                cur, size = [], 0
            cur.append(g)
            size += nb
        if cur:
            buckets.append(cur)
        for b in buckets:
            flat = torch.cat([g.reshape(-1) for g in b])
            self.dist.all_reduce(flat, op=self.dist.ReduceOp.SUM, group=self.group)
            off = 0
            for g in b:
                n = g.numel()
                g.copy_(flat[off: off + n].view_as(g))
                off += n
        return len(buckets)

    def sync_buffers(self, modules: Iterable[torch.nn.Module]) -> int:
        """MEAN-all-reduce every floating-point buffer (BatchNorm running_mean / running_var) so rank-local
        eval and checkpoints agree; integer buffers (num_batches_tracked) advance identically on every rank
        and are left alone. Returns the number of buffers synced."""
        bufs = [b for m in modules for b in m.buffers() if b.is_floating_point()]
        if not bufs or self.world == 1:
            return len(bufs)
        flat = torch.cat([b.reshape(-1).float() for b in bufs])
        self.dist.all_reduce(flat, op=self.dist.ReduceOp.SUM, group=self.group)
        flat /= self.world
        off = 0
        for b in bufs:
            n = b.numel()
            b.copy_(flat[off: off + n].view_as(b))
            off += n
        return len(bufs)

    # -- sparse -----------------------------------------------------------------------------------
    def allgather_sparse(self, sg: SparseGrad, table_rows: int) -> SparseGrad:
        """Sum of every rank's SparseGrad (rows of a replicated table), rank order 0..P-1."""
        n = sg.count()
        dev = sg.rows.device
        D = sg.grad.shape[1]
        cnt = torch.tensor([n], dtype=torch.int64, device=dev)
        cnts = [torch.zeros_like(cnt) for _ in range(self.world)]
        self.dist.all_gather(cnts, cnt, group=self.group)
        counts = [int(c.item()) for c in cnts]
        m = max(max(counts), 1)
        rows = torch.full((m,), -1, dtype=torch.int64, device=dev)
        grad = torch.zeros((m, D), dtype=torch.float32, device=dev)
        rows[:n] = sg.rows[:n]
        grad[:n] = sg.grad[:n]
        all_rows = [torch.empty_like(rows) for _ in range(self.world)]
        all_grad = [torch.empty_like(grad) for _ in range(self.world)]
        self.dist.all_gather(all_rows, rows, group=self.group)
        self.dist.all_gather(all_grad, grad, group=self.group)
        ids = torch.cat([r[:c] for r, c in zip(all_rows, counts)])
        vals = torch.cat([g[:c] for g, c in zip(all_grad, counts)])
        uid, uval, n_uniq, cap = self.ops.segment_sum(ids, vals, int(table_rows))
        return SparseGrad(uid, uval, n_uniq, cap)


def data_parallel_step(model, batch, labels, dp: Optional[DataParallel]):
    """One TrainableDssm step under data parallelism (dp=None: single replica)."""
    return model.step(batch, labels, dp=dp)
