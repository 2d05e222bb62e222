"""recall -> prerank -> rank cascade (BASELINE.json configs[4]).

The reference has the three stages as separate model families (models/matching = recall,
models/preranking/cold.py = prerank — an empty file, models/ranking = ESIM) glued by offline scripts
(FaissSearcher + eval_utils). The build wires them into one serving step on the MI355X path:

  offline (catalog of N items):
    v_item  = l2norm(ad tower(ad slots))           [N, E]  fp32, resident      (Dssm, dssm.py:25-36)
    a_item  = ESIM ad-side slot sequence           [N, L, d] fp16, resident    (esim.py; fp16 MFMA attention)
  online (a batch of B users):
    u       = l2norm(user tower(user slots))                                   (Dssm)
    recall  : top-K1 items by <u, v_item>        FaissSearcher Flat (rf_linear_fwd blocks + rf_topk_merge)
    prerank : s = Dense(1)(relu(Dense(64)(u * v_cand)))  on B x K1 pairs -> top-K2 (rf_topk_merge)
              (build-defined: cold.py is empty; a COLD-style light interaction model)
    rank    : ESIM(q = user sequence, a = a_item[cand], dense) on B x K2 pairs -> p(click) -> top-K3

Row gathers use rf_gather_rows (fp16 rows are moved as 2-byte elements). Everything stays on the GPU;
the only host traffic is the final [B, K3] ids and scores.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Sequence

import torch

from ..backend.encoder.sparse_encoder import FusedSparseEncoder, SlotSpec
from ..backend.layers.attention_layers import esim_soft_attention_pool
from ..backend.layers.core import Dense
from ..backend.third_party_components.faiss_searcher import FaissSearcher
from ..runtime import lib as L
from ..runtime.batch import SparseBatch
from .matching.dssm import Dssm
from .ranking.esim import Esim


def gather_rows(src: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """src[idx] for a 2-D row-major tensor (rf_gather_rows; 16-byte rows)."""
    idx = idx.reshape(-1).to(torch.int64).contiguous()
    rows, width = src.shape
    esz = src.element_size()
    code = L.DT_F32 if esz == 4 else L.DT_BF16  # a row copy: only the element size matters
    out = torch.empty((max(idx.numel(), 1), width), dtype=src.dtype, device=src.device)
    if idx.numel():
        L.call("rf_gather_rows", L.ptr(idx), idx.numel(), L.ptr(src), code, rows, width, L.ptr(out), L.stream_ptr())
    return out[: idx.numel()]


def topk_rows(scores: torch.Tensor, k: int):
    """(values, positions) of the k best columns of every row (rf_topk_merge, one block)."""
    B, n = scores.shape
    v = torch.empty((B, k), dtype=torch.float32, device=scores.device)
    i = torch.empty((B, k), dtype=torch.int64, device=scores.device)
    s = scores.float().contiguous()
    L.call("rf_topk_merge", L.ptr(s), s.stride(0), B, n, k, 0, None, None, 0, k, L.ptr(v), L.ptr(i), k, L.stream_ptr())
    return v, i


@dataclass
class CascadeResult:
    items: torch.Tensor       # [B, K3] int64 item ids
    scores: torch.Tensor      # [B, K3] fp32 p(click)
    recall_items: torch.Tensor
    prerank_items: torch.Tensor


class Cascade(torch.nn.Module):
    def __init__(self, recall: Dssm, ranker: Esim, k_recall: int = 200, k_prerank: int = 50, k_final: int = 10,
                 prerank_units: int = 64, rank_dtype=torch.float16, seed: int = 0, device="cuda"):
        super().__init__()
        if not (k_final <= k_prerank <= k_recall <= 1024):
            raise ValueError("need k_final <= k_prerank <= k_recall <= 1024")
        self.recall, self.ranker = recall, ranker
        self.k1, self.k2, self.k3 = k_recall, k_prerank, k_final
        self.rank_dtype = rank_dtype
        E = recall.user_dense.out_features
        self.pre1 = Dense(E, prerank_units, "relu", dtype=torch.float32, seed=seed + 1, device=device)
        self.pre2 = Dense(prerank_units, 1, None, dtype=torch.float32, seed=seed + 2, device=device)
        self.searcher: Optional[FaissSearcher] = None
        self.a_item: Optional[torch.Tensor] = None

    @torch.no_grad()
    def index_catalog(self, recall_ad: Sequence[SparseBatch], rank_ad: Sequence[SparseBatch]):
        """Offline: item vectors for recall and ESIM ad sequences for ranking, batch by batch."""
        vs, as_ = [], []
        for rb, kb in zip(recall_ad, rank_ad):
            v = torch.nn.functional.normalize(self.recall.ad_dense(self.recall.enc_a(rb)), dim=-1, eps=1e-6)
            vs.append(v)
            as_.append(self.ranker.enc_a(kb).to(self.rank_dtype))
        items = torch.cat(vs)
        self.searcher = FaissSearcher(items=items, index_param="Flat", measurement="ip").train()
        self.a_item = torch.cat(as_).contiguous()  # [N, L * d]
        return self

    @torch.no_grad()
    def forward(self, recall_user: SparseBatch, rank_user: SparseBatch, dense: torch.Tensor) -> CascadeResult:
        B = recall_user.batch
        u = torch.nn.functional.normalize(self.recall.user_dense(self.recall.enc_u(recall_user)), dim=-1, eps=1e-6)
        # recall
        _, cand1 = self.searcher.search_index(u, self.k1)                                   # [B, K1] item ids
        v = gather_rows(self.searcher.index, cand1)                                         # [B*K1, E]
        x = (u[:, None, :] * v.view(B, self.k1, -1)).reshape(B * self.k1, -1).contiguous()
        # prerank
        s2 = self.pre2(self.pre1(x)).view(B, self.k1)
        _, pos2 = topk_rows(s2, self.k2)
        cand2 = torch.gather(cand1, 1, pos2)                                                # [B, K2]
        # rank: ESIM over (user sequence, candidate item sequence) pairs, fp16 MFMA attention
        Lq, d = self.ranker.L, self.ranker.d
        q = self.ranker.enc_q(rank_user).to(self.rank_dtype).view(B, 1, Lq * d).expand(B, self.k2, Lq * d)
        q = q.reshape(B * self.k2, Lq, d)
        a = gather_rows(self.a_item, cand2).view(B * self.k2, Lq, d)
        pooled = torch.empty((B * self.k2, self.ranker.pooled_width), dtype=torch.float32, device=u.device)
        xd = dense.repeat_interleave(self.k2, dim=0) if dense.shape[0] == B else dense
        self.ranker.input_mlp(xd, out=pooled[:, : self.ranker.d_emb])
        esim_soft_attention_pool(q, a, out=pooled, out_col=self.ranker.d_emb)
        p = self.ranker.dense_output(self.ranker.output_mlp(pooled))[:, 1].view(B, self.k2)
        s3, pos3 = topk_rows(p, self.k3)
        return CascadeResult(torch.gather(cand2, 1, pos3), s3, cand1, cand2)
