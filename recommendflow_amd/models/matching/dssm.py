"""Two-tower DSSM recall scorer on the MI355X hot path (reference: models/matching/dssm.py:11-64).

The reference builds the towers `create_mlp([1024, 512, 256], 0.3, "selu", BatchNormalization(1e-6))`
(dssm.py:25-26) and `K.l2_normalize` (:35-36) but its `call` never wires them (:38-60); deviation
D-dssm-wiring defines the forward the class intends:
  u = l2norm(user_tower([pool_s]_{s in user}))  v = l2norm(ad_tower([pool_s]_{s in ad}))  score = <u, v>
(the dot-product score of que2search.py:137 / match_losses.py:46). Towers run in fp32 (the reference
dtype) on the exact-fp32 MFMA path; the sparse part is one fused encoder launch per tower.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from ...backend.blocks.mlp import create_mlp, forward_towers
from ...backend.encoder.sparse_encoder import FusedSparseEncoder
from ...backend.layers.core import BatchNormalization
from ...runtime.batch import SparseBatch


class Dssm(torch.nn.Module):
    def __init__(self, user_encoder: FusedSparseEncoder, ad_encoder: FusedSparseEncoder, units=(1024, 512, 256),
                 tower_dtype=torch.float32, seed: int = 0, device="cuda"):
        super().__init__()
        self.enc_u, self.enc_a = user_encoder, ad_encoder
        bn = BatchNormalization(epsilon=1e-6)
        self.user_dense = create_mlp(list(units), 0.3, "selu", bn, name="user_dense_tower",
                                     in_features=user_encoder.out_width, dtype=tower_dtype, seed=seed + 1, device=device)
        self.ad_dense = create_mlp(list(units), 0.3, "selu", bn, name="ad_dense_tower",
                                   in_features=ad_encoder.out_width, dtype=tower_dtype, seed=seed + 2, device=device)

    def towers(self, xu: torch.Tensor, xa: torch.Tensor):
        """l2norm(user_tower(xu)), l2norm(ad_tower(xa)) from the pooled encoder outputs: both towers layer by layer
        (backend.blocks.mlp.forward_towers: the small layers of both towers share one launch)."""
        u, a = forward_towers([self.user_dense, self.ad_dense], [xu, xa])
        return torch.nn.functional.normalize(u, dim=-1, eps=1e-6), torch.nn.functional.normalize(a, dim=-1, eps=1e-6)

    def embed(self, user: SparseBatch, ad: SparseBatch):
        return self.towers(self.enc_u(user), self.enc_a(ad))

    def forward(self, user: SparseBatch, ad: SparseBatch) -> torch.Tensor:
        u, a = self.embed(user, ad)
        return (u * a).sum(dim=-1)

    def graphed(self, user: SparseBatch, ad: SparseBatch, **kw):
        """forward() as one hipGraph on static copies of (user, ad) (runtime.graphs.GraphedForward)."""
        from ...runtime.graphs import GraphedForward

        return GraphedForward(self.forward, user, ad, **kw)

    def flops_per_example(self) -> float:
        f = 0
        for m in (self.user_dense, self.ad_dense):
            for dn in m.denses:
                f += 2 * dn.in_features * dn.units
        return float(f)


class TrainableDssm(torch.nn.Module):
    """DSSM training graph (deviation D-dssm-wiring as above): ONE fused encoder over the user slots then
    the ad slots (one forward and one backward launch for both towers), towers
    [BatchNormalization(eps 1e-6, Keras momentum 0.99) -> Dense(selu) -> Dropout(0.3)] x [1024, 512, 256]
    (dssm.py:25-26, mlp.py:4-15) on librf.so (backend.blocks.train_mlp.TrainTower: batch statistics folded
    into the fp32 MFMA GEMM, SELU / dropout / BatchNormalization backward kernels, library GEMMs for the two
    backward products), l2 normalisation (dssm.py:35-36), and the configured loss (cosent_loss for
    base_recall_sdpa.yaml). step() = forward, backward, SparseAdam on the table (rf_adam_apply) and KerasAdam
    on the towers (rf_adam_dense), Keras defaults (lr 1e-3, 0.9, 0.999, 1e-7)."""

    def __init__(self, encoder: FusedSparseEncoder, n_user_slots: int, units=(1024, 512, 256), dropout=0.3,
                 learning_rate=1e-3, loss="cosent", lazy_adam=False, seed=0, deferred_adam=None):
        super().__init__()
        from ...backend.blocks.train_mlp import TrainTower
        from ...backend.losses import match_losses
        from ...backend.optim import KerasAdam, SparseAdam

        self.enc = encoder
        self.wu = 2 * encoder.dim * n_user_slots
        self.wa = encoder.out_width - self.wu
        g = torch.Generator().manual_seed(seed)
        dev = encoder.table.device
        self.user_tower = TrainTower(self.wu, units, rate=dropout, eps=1e-6, seed=2 * seed + 1, generator=g, device=dev)
        self.ad_tower = TrainTower(self.wa, units, rate=dropout, eps=1e-6, seed=2 * seed + 2, generator=g, device=dev)
        self.loss_fn = {"cosent": match_losses.cosent_loss,
                        "inbatch_ce": match_losses.batch_neg_sample_scaled_multi_class_ce_loss}[loss]
        # cosent on the raw tower outputs: normalisation, row dot, loss and their backward in 3 + 4 launches
        self._fused_loss = match_losses.cosine_cosent_loss if loss == "cosent" else None
        if deferred_adam is None:
            deferred_adam = self.deferred_table_adam and not lazy_adam
        self.sparse_opt = SparseAdam(encoder.table, learning_rate=learning_rate, lazy=lazy_adam, deferred=deferred_adam)
        self.dense_opt = KerasAdam(list(self.user_tower.parameters()) + list(self.ad_tower.parameters()),
                                   learning_rate=learning_rate)

    overlap_table_adam = True  # False: the table's dense Adam runs after the backward in one launch (A/B)
    # True: the table's dense Adam is deferred per row (SparseAdam(deferred=True): a row's missed untouched steps are
    # replayed when the row is next read; bit-identical rows, no whole-table pass per step). Default for new models.
    deferred_table_adam = True
    fused_loss = os.environ.get("RF_FUSED_LOSS", "1") != "0"  # cosent: match_losses.cosine_cosent_loss on the raw tower outputs (False: torch normalize + loss)

    def materialize(self):
        """Bring every table row current (deferred Adam) before anything outside step() reads the table."""
        self.sparse_opt.materialize()

    def embedding_table(self) -> torch.Tensor:
        """The fused table with every row current: the accessor for readers outside step() / the eval forward
        (export, search index builds). enc.table itself may hold rows behind by deferred steps."""
        self.materialize()
        return self.enc.table

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        # the fused table is a plain attribute of the encoder, not a parameter: a checkpoint gets it here, with the
        # table optimizer's m, v and step count, every row current (the dense step's values bit for bit)
        super()._save_to_state_dict(destination, prefix, keep_vars)
        st = self.sparse_opt.state()
        for k in ("table", "m", "v"):
            t = st[k]
            destination[prefix + "sparse_" + k] = t if keep_vars else t.detach()
        destination[prefix + "sparse_iterations"] = torch.tensor(st["iterations"], dtype=torch.int64)

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                              error_msgs):
        keys = [prefix + "sparse_" + k for k in ("table", "m", "v", "iterations")]
        present = [k in state_dict for k in keys]
        if all(present):
            t, m, v, it = (state_dict[k] for k in keys)
            # rows loaded are current through the checkpoint's step: the deferred replay starts from there
            self.sparse_opt.load_state(t, m, v, int(it))
        elif strict:
            missing_keys.extend(k for k, p in zip(keys, present) if not p)
        rest = {k: v for k, v in state_dict.items() if k not in keys}
        super()._load_from_state_dict(rest, prefix, local_metadata, strict, missing_keys, unexpected_keys, error_msgs)

    def _side_stream(self):
        s = getattr(self, "_side", None)
        if s is None:
            s = self._side = torch.cuda.Stream(device=self.enc.table.device)
        return s

    def forward(self, batch: SparseBatch, after_embed=None, raw: bool = False):
        from ...backend.blocks.train_mlp import towers_forward
        from ...runtime.train import embed

        if not self.training:
            self.sparse_opt.materialize()
        x = embed(self.enc, batch)
        if after_embed is not None:
            after_embed()
        if self.training:
            # both towers read their column blocks of x in place (row stride = the full width); the backward
            # writes both input gradients into one full-width buffer
            tu, ta = towers_forward(x, [(self.user_tower, 0, self.wu), (self.ad_tower, self.wu, self.wa)])
        else:
            tu, ta = self.user_tower(x[:, : self.wu]), self.ad_tower(x[:, self.wu:])
        if raw:
            return tu, ta
        u = torch.nn.functional.normalize(tu, dim=-1, eps=1e-6)
        v = torch.nn.functional.normalize(ta, dim=-1, eps=1e-6)
        return u, v

    def step(self, batch: SparseBatch, labels: torch.Tensor, dp=None) -> torch.Tensor:
        """One training step; `dp` (runtime.dist.DataParallel) = MirroredStrategy-style replicas: the
        loss is scaled by 1/P, dense gradients are SUM-all-reduced in buckets and the table's sparse
        gradients all-gathered and summed in rank order before the (identical) optimizer steps; the
        BatchNorm moving statistics are then averaged over the replicas (DataParallel.sync_buffers)."""
        self.train()
        self.dense_opt.zero_grad(set_to_none=True)
        # single replica, dense (exact Keras) Adam: the table rows NOT in this batch's gradient take their update
        # on a side stream while the towers run (their Keras step needs no gradient); the gradient's rows get
        # theirs after the backward (SparseAdam.apply_untouched / apply_touched == apply, bit for bit)
        deferred = self.sparse_opt.deferred
        split = dp is None and not self.sparse_opt.lazy and not deferred and self.overlap_table_adam
        if deferred:
            # the batch's rows current before the forward reads them; the backward's reduce reuses the plan
            plan = self.enc.backward_plan(batch)
            self.sparse_opt.prepare(plan.rows, plan.n_uniq, plan.cap)
            self.enc._plan, self.enc._plan_batch, self.enc._plan_stream = plan, batch, None

        def launch_untouched():
            main = torch.cuda.current_stream()
            side = self._side_stream()
            side.wait_stream(main)
            with torch.cuda.stream(side):
                plan = self.enc.backward_plan(batch)
                planned = torch.cuda.Event()
                planned.record(side)
                self.sparse_opt.apply_untouched(plan.rows, plan.n_uniq, plan.cap)
            # plan.batch is a device copy made on the side stream when `batch` was a host batch: the main stream's
            # reduce reads it too
            pb = plan.batch
            for t in (plan.rows, plan.n_uniq, plan.ws, pb.tok_bytes, pb.tok_off, pb.bag_off, pb.lmax):
                if isinstance(t, torch.Tensor) and t.is_cuda:
                    t.record_stream(main)
            # the backward's reduce waits for the plan only: the untouched rows' update keeps running through the
            # towers' backward, the reduce and the touched rows' update (disjoint rows), and the step joins it last
            self.enc._plan, self.enc._plan_batch, self.enc._plan_stream = plan, batch, planned

        fused = self._fused_loss is not None and self.fused_loss
        u, v = self(batch, after_embed=launch_untouched if split else None, raw=fused)
        loss = self._fused_loss(labels, u, v, eps=1e-6) if fused else self.loss_fn(labels, u, v)
        from ...backend.blocks.train_mlp import join_input_wgrad, overlap_input_wgrad

        with overlap_input_wgrad():  # the towers' input-layer weight gradients run beside the sparse reduce / Adam
            (loss * dp.loss_scale() if dp is not None else loss).backward()
        sg = self.enc.grad
        if dp is not None:
            join_input_wgrad()
            dp.allreduce_dense(list(self.user_tower.parameters()) + list(self.ad_tower.parameters()))
            sg = dp.allgather_sparse(sg, self.enc.table_rows)
        if split:
            self.sparse_opt.apply_touched(sg)
        else:
            self.sparse_opt.apply(sg)
        join_input_wgrad()
        self.dense_opt.step()
        if split:  # the next step's lookup reads every row
            torch.cuda.current_stream().wait_stream(self._side_stream())
        if dp is not None:  # BN moving statistics: ON_READ / MEAN across replicas (MirroredStrategy)
            dp.sync_buffers([self.user_tower, self.ad_tower])
        return loss.detach()
