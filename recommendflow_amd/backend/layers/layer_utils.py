"""Attention helpers (reference: backend/layers/layer_utils.py)."""
from __future__ import annotations

from typing import Optional

import torch

from ...runtime import lib as L


def scaled_dot_product_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, mask: Optional[torch.Tensor] = None,
                                 heads: int = 1, dtype=torch.float16) -> torch.Tensor:
    """softmax(where(mask == 0, -4294967295, q k^T / sqrt(depth))) @ v   (layer_utils.py:4-24).

    q: [B, Lq, heads*depth], k, v: [B, Lk, heads*depth]; head h = columns [h*depth, (h+1)*depth)
    (split_heads, :27-38). mask: [B, Lq] or [B, Lq, 1] — zero marks a QUERY row whose logits are all
    replaced (the reference's [..., Lq, 1] mask broadcasts over keys). Returns fp32 [B, Lq, heads*depth]
    (the merged-heads layout of MultiHeadAttention.call, attention_layers.py:167). Logits and softmax
    are fp32 inside the kernel; operands are rounded to `dtype` (fp16 for cfg5) for the MFMA.
    """
    L.require_gpu()
    B, Lq, width = q.shape
    Lk = k.shape[1]
    if width % heads:
        raise ValueError("width must be divisible by heads")
    depth = width // heads
    qh, kh, vh = (t.to(dtype).contiguous() for t in (q, k, v))
    m = None
    if mask is not None:
        m = mask.reshape(B, Lq).to(device=q.device, dtype=torch.float32).contiguous()
    out = torch.empty((B, Lq, width), dtype=torch.float32, device=q.device)
    L.call("rf_sdpa_fwd", L.ptr(qh), L.ptr(kh), L.ptr(vh), L.torch_dtype_code(dtype), B, heads, Lq, Lk, depth, L.ptr(m),
           L.ptr(out), L.stream_ptr())
    return out


def split_heads(x: torch.Tensor, seq_len: int, num_heads: int, depth: int) -> torch.Tensor:
    """[B, L, H*depth] -> [B, H, L, depth] (layer_utils.py:27-38); a view-level helper."""
    return x.reshape(-1, seq_len, num_heads, depth).permute(0, 2, 1, 3)
