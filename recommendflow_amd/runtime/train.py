"""Training step plumbing for the sparse hot path.

The fused encoder joins torch autograd through `embed()`: forward = rf_fused_hash_embed_fwd, backward =
rf_fused_hash_embed_bwd, whose deduplicated row gradient is parked on the encoder (`enc.grad`) for
SparseAdam (rf_adam_apply) — the table is never a dense torch gradient. Dense parameters (towers) train
with torch autograd + backend.optim.KerasAdam (rf_adam_dense: Keras' dense Adam update, Keras defaults;
reference: model.fit with tf.keras.optimizers.Adam, example/recall_search/train.py:96-104).
"""
from __future__ import annotations

from typing import Optional

import torch

from ..backend.encoder.sparse_encoder import FusedSparseEncoder, SparseGrad
from .batch import SparseBatch


class _EmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, enc: FusedSparseEncoder, batch: SparseBatch):
        out = enc(batch)
        ctx.enc, ctx.batch = enc, batch
        ctx.save_for_backward(out)
        return out

    @staticmethod
    def backward(ctx, dout):
        (out,) = ctx.saved_tensors
        enc = ctx.enc
        plan = getattr(enc, "_plan", None)
        if plan is not None and getattr(enc, "_plan_batch", None) is ctx.batch:
            # the batch-only half already ran (possibly on a side stream: _plan_stream is then that stream or an
            # event recorded on it after the plan): join it, reduce dout on this stream
            side = getattr(enc, "_plan_stream", None)
            if isinstance(side, torch.cuda.Event):
                torch.cuda.current_stream().wait_event(side)
            elif side is not None:
                torch.cuda.current_stream().wait_stream(side)
            enc.grad = enc.backward_reduce(plan, dout.float().contiguous(), out=out)
            enc._plan = enc._plan_batch = enc._plan_stream = None
        else:
            enc.grad = enc.backward(ctx.batch, dout.float().contiguous(), out=out)
        return None, None, None


def embed(enc: FusedSparseEncoder, batch: SparseBatch) -> torch.Tensor:
    """enc(batch) with a sparse backward: after loss.backward(), enc.grad holds the SparseGrad."""
    if not hasattr(enc, "_anchor"):
        enc._anchor = torch.zeros(1, device=enc.table.device, requires_grad=True)
    enc.grad: Optional[SparseGrad] = None
    return _EmbedFn.apply(enc._anchor, enc, batch)
