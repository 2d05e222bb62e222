"""ESIM ranking-model training step (reference: models/ranking/esim.py:13-93 under model.fit with
tf.keras.optimizers.Adam, example/ranking_search/train.py:96-104).

Keras builds the model in float32, so the training path computes in fp32 end to end (the inference path,
models/ranking/esim.py, runs bf16 MFMA):

  x       = ONE fused encoder over the user slots then the ad slots  [B, 2 L d]   rf_fused_hash_embed_fwd (fp32 table)
  d_emb   = input_mlp(dense)                                          TrainLNMLP  (esim.py:45-48, 73-75)
  pooled  = [d_emb, ESIM(q = x[:, :Ld], a = x[:, Ld:])]               rf_esim_train_fwd_f32 (esim.py:78-84)
  h       = output_mlp(Dropout(0.3)(pooled))                          rf_dropout_fwd + TrainLNMLP (esim.py:85-86)
  z       = h W_o^T + b_o;  loss = SparseCategoricalCE(softmax(z), y) rf_gemm_f32 + rf_softmax_ce_loss (esim.py:53,88)
backward in reverse (rf_esim_train_bwd_f32 for the attention block, rf_fused_hash_embed_bwd_reduce for the table),
then Keras Adam: SparseAdam (deferred, exact dense semantics) on the fused table, KerasAdam on every dense parameter.
Explicit forward / backward through librf; no torch autograd, no vendor GEMM.

Deviations: D-esim-inputs (each slot is one token = its DoubleHashingEmbedding output, as the inference model),
D-shared-norm (one LayerNormalization per layer), the loss is the sparse categorical cross-entropy of the click
head (the reference passes `loss` to the constructor but never wires it: esim.py:17,21).
"""
from __future__ import annotations

from typing import Optional, Sequence

import math

import torch

from ...backend.blocks.train_ln_mlp import TrainLNMLP
from ...backend.blocks.train_mlp import layer_seed
from ...backend.encoder.sparse_encoder import FusedSparseEncoder, SlotSpec
from ...backend.optim import KerasAdam, SparseAdam
from ...runtime import gemm as GM
from ...runtime import lib as L
from ...runtime.batch import SparseBatch


class TrainableEsim:
    def __init__(self, user_slots: Sequence[SlotSpec], ad_slots: Sequence[SlotSpec], n_dense: int, dim: int = 64,
                 input_units=(256, 512), output_units=(1024, 512), dropout: float = 0.3, learning_rate: float = 1e-3,
                 seed: int = 0, device="cuda", encoder: Optional[FusedSparseEncoder] = None):
        if len(user_slots) != len(ad_slots):
            raise ValueError("SoftAttention needs equal q / a lengths (attention_layers.py:74)")
        self.L = len(user_slots)
        self.d = 2 * dim
        if self.d not in (64, 128) or not 1 <= self.L <= 128:
            raise ValueError("the fp32 ESIM training kernels need 2 * dim in {64, 128} and 1 <= L <= 128")
        self.enc = encoder if encoder is not None else FusedSparseEncoder(list(user_slots) + list(ad_slots), dim,
                                                                          table_dtype=torch.float32, seed=seed + 1,
                                                                          device=device)
        if self.enc.table.dtype != torch.float32 or self.enc.out_width != 2 * self.L * self.d:
            raise ValueError("TrainableEsim needs one fp32 fused encoder over the user slots then the ad slots")
        g = torch.Generator().manual_seed(seed)
        self.rate = float(dropout)
        self.seed = int(seed)
        self.input_mlp = TrainLNMLP(n_dense, input_units, dropout, "gelu", seed=2 * seed + 11, generator=g, device=device)
        self.d_emb = self.input_mlp.out_features
        self.pooled_width = self.d_emb + 6 * self.d
        self.output_mlp = TrainLNMLP(self.pooled_width, output_units, dropout, "gelu", seed=2 * seed + 12, generator=g,
                                     device=device)
        k = self.output_mlp.out_features
        lim = math.sqrt(6.0 / (k + 2))
        # Dense(2, softmax): the parameters W_out [2][k], b_out [2] are the first rows of zero-padded [4][k] / [4] buffers
        # (rf_gemm_f32 takes K and leading dimensions in multiples of 4; the padded logits are never read, their
        # gradients stay zero)
        self._W4 = torch.zeros((4, k), device=device)
        self._b4 = torch.zeros(4, device=device)
        self._W4[:2] = ((torch.rand((2, k), generator=g) * 2 - 1) * lim).to(device)
        self.W_out, self.b_out = self._W4[:2], self._b4[:2]
        self.sparse_opt = SparseAdam(self.enc.table, learning_rate=learning_rate, deferred=True)
        self.dense_opt = KerasAdam(self.dense_parameters(), learning_rate=learning_rate)
        self.steps = 0
        self._ws = {}

    def dense_parameters(self):
        return self.input_mlp.parameters() + self.output_mlp.parameters() + [self.W_out, self.b_out]

    def _buf(self, name: str, nbytes: int, device) -> torch.Tensor:
        t = self._ws.get(name)
        if t is None or t.numel() < nbytes:
            t = self._ws[name] = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=device)
        return t

    def pooled_dropout_seed(self, step: int) -> int:
        return layer_seed(3 * self.seed + 5, step, 0)

    def forward(self, batch: SparseBatch, dense: torch.Tensor, training: bool = True, step: Optional[int] = None):
        """(logits [B, 2], caches) of one batch (batch: the user slots then the ad slots of each example)."""
        if batch.n_slots != 2 * self.L:
            raise ValueError(f"batch has {batch.n_slots} slots, the model {2 * self.L} (user then ad)")
        step = self.steps if step is None else step
        B, dev = batch.batch, self.enc.table.device
        st = L.stream_ptr(None)
        x = self.enc(batch)  # [B, 2 L d] fp32
        pooled = torch.empty((B, self.pooled_width), dtype=torch.float32, device=dev)
        self.input_mlp.forward(dense.float(), step, out=pooled[:, : self.d_emb], training=training)
        aux = torch.empty((B, 2 * self.d), dtype=torch.float32, device=dev)
        Ld = self.L * self.d
        L.call("rf_esim_train_fwd_f32", L.ptr(x), L.ptr(x) + 4 * Ld, B, self.L, self.d, x.stride(0), self.d, L.ptr(pooled),
               pooled.stride(0), self.d_emb, L.ptr(aux), st)
        rate = self.rate if training else 0.0
        xd = pooled
        if rate > 0:
            xd = torch.empty_like(pooled)
            L.call("rf_dropout_fwd", L.ptr(pooled), B, self.pooled_width, pooled.stride(0), rate, self.pooled_dropout_seed(step),
                   L.ptr(xd), xd.stride(0), st)
        h = self.output_mlp.forward(xd, step, training=training)
        z = GM.gemm_f32(h, self._W4, trans_b=True, bias=self._b4, stream=st)  # [B, 4]: logits in columns 0, 1
        return z, (batch, x, pooled, aux, h, rate, step)

    def predict(self, batch: SparseBatch, dense: torch.Tensor) -> torch.Tensor:
        """p(click) [B, 2] without dropout (every table row current first)."""
        self.sparse_opt.materialize()
        z, _ = self.forward(batch, dense, training=False)
        B = z.shape[0]
        prob = torch.empty((B, 2), device=z.device)
        ws = self._buf("loss", int(L.load().rf_loss_ws_bytes(B)), z.device)
        loss = torch.empty(1, device=z.device)
        lab = torch.zeros(B, dtype=torch.int32, device=z.device)
        L.call("rf_softmax_ce_loss", L.ptr(z), z.stride(0), L.ptr(lab), B, 2, L.ptr(loss), L.ptr(prob), prob.stride(0), None, 0,
               L.ptr(ws), ws.numel(), L.stream_ptr(None))
        return prob

    def loss_and_grads(self, batch: SparseBatch, dense: torch.Tensor, labels: torch.Tensor, step: Optional[int] = None,
                       training: bool = True, plan=None, loss_scale: float = 1.0):
        """Forward + backward without the optimizer: (loss, prob); dense parameters get .grad, the table's sparse
        gradient lands in self.enc.grad, the fused encoder output's gradient in self.dout. plan: the batch's
        backward plan when the caller made it already (step())."""
        lib = L.load()
        st = L.stream_ptr(None)
        z, (batch, x, pooled, aux, h, rate, step) = self.forward(batch, dense, training=training, step=step)
        B, dev = z.shape[0], z.device
        lab = labels.to(device=dev, dtype=torch.int32).contiguous()
        loss = torch.empty(1, device=dev)
        prob = torch.empty((B, 2), device=dev)
        dz = torch.zeros_like(z)  # [B, 4]: columns 2, 3 stay zero
        ws = self._buf("loss", int(lib.rf_loss_ws_bytes(B)), dev)
        L.call("rf_softmax_ce_loss", L.ptr(z), z.stride(0), L.ptr(lab), B, 2, L.ptr(loss), L.ptr(prob), prob.stride(0),
               L.ptr(dz), dz.stride(0), L.ptr(ws), ws.numel(), st)
        if loss_scale != 1.0:  # data parallel: the global loss is the mean over the replicas
            dz.mul_(loss_scale)
        # head: dW_o = dz^T h, db_o = column sums of dz, dh = dz W_o (on the padded [B, 4] / [4, k] operands)
        self.W_out.grad = GM.gemm_f32(dz, h, trans_a=True, stream=st)[:2]
        db = torch.empty(4, device=dev)
        dzc = torch.empty_like(dz)
        wst = self._buf("tower", int(lib.rf_tower_ws_bytes(B, 4)), dev)
        L.call("rf_act_dropout_bwd", L.ptr(dz), dz.stride(0), L.ptr(dz), dz.stride(0), B, 4, L.ACT["none"], 0.0, 0, L.ptr(dzc),
               dzc.stride(0), L.ptr(db), L.ptr(wst), wst.numel(), st)
        self.b_out.grad = db[:2]
        dh = GM.gemm_f32(dz, self._W4, stream=st)
        dxd = self.output_mlp.backward(dh)
        dpooled = dxd
        if rate > 0:
            dpooled = torch.empty_like(dxd)
            L.call("rf_dropout_fwd", L.ptr(dxd), B, self.pooled_width, dxd.stride(0), rate, self.pooled_dropout_seed(step),
                   L.ptr(dpooled), dpooled.stride(0), st)
        self.input_mlp.backward(dpooled[:, : self.d_emb], need_dx=False)
        # the attention block's gradient straight into the fused encoder's output gradient
        dout = torch.empty_like(x)
        Ld = self.L * self.d
        wse = self._buf("esim", int(lib.rf_esim_train_ws_bytes(B, self.L, self.d)), dev)
        L.call("rf_esim_train_bwd_f32", L.ptr(x), L.ptr(x) + 4 * Ld, B, self.L, self.d, x.stride(0), self.d, L.ptr(pooled),
               pooled.stride(0), self.d_emb, L.ptr(dpooled), dpooled.stride(0), self.d_emb, L.ptr(aux), L.ptr(dout),
               L.ptr(dout) + 4 * Ld, dout.stride(0), self.d, L.ptr(wse), wse.numel(), st)
        self.dout = dout
        self.enc.grad = self.enc.backward(batch, dout, out=x) if plan is None else self.enc.backward_reduce(plan, dout, out=x)
        return loss, prob

    def step(self, batch: SparseBatch, dense: torch.Tensor, labels: torch.Tensor, dp=None) -> torch.Tensor:
        """One training step (model.fit's train_step): forward, backward, Adam on the table and the dense parameters.
        `dp` (runtime.dist.DataParallel) = MirroredStrategy-style replicas, as TrainableDssm.step: the loss scaled by
        1/P, dense gradients SUM-all-reduced in buckets, the table's sparse gradients all-gathered and summed in rank
        order before the (identical) optimizer steps."""
        plan = self.enc.backward_plan(batch)
        self.sparse_opt.prepare(plan.rows, plan.n_uniq, plan.cap)  # the batch's rows current before the forward
        self.dense_opt.zero_grad(set_to_none=True)
        scale = dp.loss_scale() if dp is not None else 1.0
        loss, _ = self.loss_and_grads(batch, dense, labels, plan=plan, loss_scale=scale)
        sg = self.enc.grad
        if dp is not None:
            dp.allreduce_dense(self.dense_parameters())
            sg = dp.allgather_sparse(sg, self.enc.table_rows)
        self.sparse_opt.apply(sg)
        self.dense_opt.step()
        self.steps += 1
        return loss
