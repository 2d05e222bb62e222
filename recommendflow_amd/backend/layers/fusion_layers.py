"""AttentionFusion (reference: backend/layers/fusion_layers.py:6-61, Que2Search), forward on
rf_attention_fusion_fwd: att = softmax(concat(inputs) @ W), out = sum_c att_c * x_c, l2-normalised.

The inference statistics of the reference (infer_weights += sum over the batch of att, :44;
init_attention :48-50; get_fusion_weights :52-53) are kept on the device.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch

from ...runtime import lib as L


class AttentionFusion(torch.nn.Module):
    def __init__(self, input_dim: int, channel_num: int, initializer="glorot_uniform", regularizer=None, constraint=None,
                 is_norm: bool = True, name: Optional[str] = None, seed: int = 0, device="cuda"):
        super().__init__()
        if initializer != "glorot_uniform":
            raise NotImplementedError("only the glorot_uniform initializer is implemented")
        L.load()
        L.require_gpu()
        self.input_dim, self.channel_num, self.is_norm, self.name = int(input_dim), int(channel_num), bool(is_norm), name
        fan_in, fan_out = self.input_dim * self.channel_num, self.channel_num
        lim = (6.0 / (fan_in + fan_out)) ** 0.5
        g = torch.Generator().manual_seed(seed)
        self.W = (torch.rand(fan_in, fan_out, generator=g) * 2 * lim - lim).to(device)  # [C*d][C], Keras layout
        self.infer_weights = torch.zeros(1, self.channel_num, device=device)
        self.attention = None

    def forward(self, inputs: Sequence[torch.Tensor], training: bool = False) -> torch.Tensor:
        x = torch.cat([t.float() for t in inputs], dim=1).contiguous() if not isinstance(inputs, torch.Tensor) else inputs.float().contiguous()
        B = x.shape[0]
        assert x.dim() == 2 and x.shape[1] == self.input_dim * self.channel_num, \
            f"get shape(?, {x.shape[-1]}), expect(?, {self.input_dim * self.channel_num})"
        out = torch.empty((B, self.input_dim), dtype=torch.float32, device=x.device)
        att = torch.empty((B, self.channel_num), dtype=torch.float32, device=x.device)
        L.call("rf_attention_fusion_fwd", L.ptr(x), B, self.channel_num, self.input_dim, x.stride(0), L.ptr(self.W),
               int(self.is_norm), L.ptr(out), out.stride(0), L.ptr(att), L.stream_ptr())
        self.attention = att
        self.infer_weights += att.sum(dim=0, keepdim=True)
        return out

    def init_attention(self):
        self.infer_weights.zero_()

    def get_fusion_weights(self):
        w = self.infer_weights.cpu().numpy()
        return w / w.sum(axis=1)

    def get_config(self):
        return {"channel_num": self.channel_num}
