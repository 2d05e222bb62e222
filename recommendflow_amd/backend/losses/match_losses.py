"""Two-tower training losses (reference: backend/losses/match_losses.py), forward + gradient in one HIP
call each (rf_cosent_loss, rf_inbatch_ce_loss). Same names and (y_true, query, doc, scale) signatures as
the reference; they are torch autograd functions so the towers' backward flows through them.

* cosent_loss (match_losses.py:42-56) — the loss of base_recall_sdpa.yaml (Networks.loss).
* batch_neg_sample_scaled_multi_class_ce_loss (match_losses.py:150-165) — Que2Search in-batch softmax;
  the [B, B] logits are one library GEMM (query . doc^T), the softmax/CE and its gradient are ours.
"""
from __future__ import annotations

import torch

from ...runtime import lib as L


def _ws(batch: int, device) -> torch.Tensor:
    return torch.empty(max(int(L.load().rf_loss_ws_bytes(batch)), 256), dtype=torch.uint8, device=device)


class _Cosent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, score, label, scale):
        score = score.float().contiguous()
        label = label.float().contiguous()
        B = score.shape[0]
        loss = torch.empty((), dtype=torch.float32, device=score.device)
        ds = torch.empty_like(score)
        ws = _ws(B, score.device)
        L.call("rf_cosent_loss", L.ptr(score), L.ptr(label), B, float(scale), L.ptr(loss), L.ptr(ds), L.ptr(ws),
               ws.numel(), L.stream_ptr())
        ctx.save_for_backward(ds)
        return loss

    @staticmethod
    def backward(ctx, g):
        (ds,) = ctx.saved_tensors
        return ds * g, None, None


class _InBatchCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, label, scale):
        logits = logits.float().contiguous()
        label = label.float().contiguous()
        B = logits.shape[0]
        loss = torch.empty((), dtype=torch.float32, device=logits.device)
        dl = torch.empty_like(logits)
        ws = _ws(B, logits.device)
        L.call("rf_inbatch_ce_loss", L.ptr(logits), logits.stride(0), L.ptr(label), B, float(scale), L.ptr(loss),
               L.ptr(dl), dl.stride(0), L.ptr(ws), ws.numel(), L.stream_ptr())
        ctx.save_for_backward(dl)
        return loss

    @staticmethod
    def backward(ctx, g):
        (dl,) = ctx.saved_tensors
        return dl * g, None, None


class _CosineCosent(torch.autograd.Function):
    """cosent_loss(y, l2norm(a), l2norm(b)) from the raw tower outputs a, b in 2 + 4 launches: rf_cosine_rows_fwd
    (both normalisations and the row dot product), rf_cosent_loss (loss and dscore), and one backward launch
    (rf_cosine_rows_bwd: the normalisations' Jacobians with dscore and the upstream gradient folded in)."""

    @staticmethod
    def forward(ctx, a, b, label, scale, eps):
        a, b = a.float(), b.float()
        if a.stride(1) != 1 or b.stride(1) != 1:
            a, b = a.contiguous(), b.contiguous()
        B, N = a.shape
        s = torch.empty(B, dtype=torch.float32, device=a.device)
        nrm = torch.empty(2 * B, dtype=torch.float32, device=a.device)
        L.call("rf_cosine_rows_fwd", L.ptr(a), a.stride(0), L.ptr(b), b.stride(0), B, N, float(eps), L.ptr(s), L.ptr(nrm),
               L.stream_ptr())
        label = label.float().contiguous()
        loss = torch.empty((), dtype=torch.float32, device=a.device)
        ds = torch.empty_like(s)
        ws = _ws(B, a.device)
        L.call("rf_cosent_loss", L.ptr(s), L.ptr(label), B, float(scale), L.ptr(loss), L.ptr(ds), L.ptr(ws), ws.numel(),
               L.stream_ptr())
        ctx.save_for_backward(a, b, s, nrm, ds)
        ctx.eps = float(eps)
        return loss

    @staticmethod
    def backward(ctx, g):
        a, b, s, nrm, ds = ctx.saved_tensors
        B, N = a.shape
        g = g.float().contiguous()
        da = torch.empty((B, N), dtype=torch.float32, device=a.device)
        db = torch.empty((B, N), dtype=torch.float32, device=a.device)
        L.call("rf_cosine_rows_bwd", L.ptr(a), a.stride(0), L.ptr(b), b.stride(0), B, N, ctx.eps, L.ptr(s), L.ptr(nrm),
               L.ptr(ds), L.ptr(g), L.ptr(da), N, L.ptr(db), N, L.stream_ptr())
        return da, db, None, None, None


def cosine_cosent_loss(y_true, a, b, scale=20, eps=1e-6):
    """cosent_loss(y_true, normalize(a), normalize(b)) (the DSSM training loss, dssm.py:35-36 + match_losses.py:42-56)
    on the towers' raw outputs, fused (_CosineCosent)."""
    L.require_gpu()
    return _CosineCosent.apply(a, b, y_true.reshape(-1), scale, eps)


def cosent_loss(y_true, query, doc, scale=20):
    """logsumexp([0] ++ [scale*(s_i - s_j) : y_i < y_j]), s = <query_i, doc_i> (match_losses.py:42-56)."""
    L.require_gpu()
    return _Cosent.apply((query * doc).sum(dim=1), y_true.reshape(-1), scale)


def _mm_nt(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """x [M, K] @ w[N, K]^T in fp32 on librf (rf_linear_fwd: exact-fp32 MFMA, LDS-DMA ring when K % 32 == 0 and
    K >= 256). Shapes whose rows are not 16-byte multiples (K % 4 != 0: odd in-batch sizes in the backward) stay on
    torch's GPU GEMM."""
    x, w = x.float().contiguous(), w.float().contiguous()
    M, K = x.shape
    N = w.shape[0]
    if K % 4 or x.data_ptr() % 16 or w.data_ptr() % 16 or M == 0:
        return x @ w.t()
    y = torch.empty((M, N), dtype=torch.float32, device=x.device)
    L.call("rf_linear_fwd", L.ptr(x), L.DT_F32, M, K, x.stride(0), L.ptr(w), N, None, 0, L.ptr(y), y.stride(0),
           L.stream_ptr())
    return y


class _InBatchLogits(torch.autograd.Function):
    """logits = query @ doc^T (match_losses.py:160, tf.matmul(query, doc, transpose_b=True)) and its two backward
    products on librf: dq = g @ doc, dd = g^T @ query (each as x @ w^T with w the transposed operand)."""

    @staticmethod
    def forward(ctx, q, d):
        q, d = q.float().contiguous(), d.float().contiguous()
        ctx.save_for_backward(q, d)
        return _mm_nt(q, d)

    @staticmethod
    def backward(ctx, g):
        q, d = ctx.saved_tensors
        g = g.float().contiguous()
        dq = _mm_nt(g, d.t()) if ctx.needs_input_grad[0] else None
        dd = _mm_nt(g.t(), q.t()) if ctx.needs_input_grad[1] else None
        return dq, dd


def batch_neg_sample_scaled_multi_class_ce_loss(y_true, query, doc, scale=20):
    """mean_i(-log(exp(s<q_i,d_i>) / sum_j exp(s<q_i,d_j>)) * y_i) (match_losses.py:150-165)."""
    L.require_gpu()
    return _InBatchCE.apply(_InBatchLogits.apply(query, doc), y_true.reshape(-1), scale)
