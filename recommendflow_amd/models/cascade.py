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
from ..backend.layers.attention_layers import esim_soft_attention_pool, esim_soft_attention_pool_idx
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
        u = torch.nn.functional.normalize(self.recall.user_dense(self.recall.enc_u(recall_user)), dim=-1, eps=1e-6)
        _, cand1 = self.searcher.search_index(u, self.k1)                                   # [B, K1] item ids
        return self._prerank_rank(u, cand1, rank_user, dense)

    def _prerank_rank(self, u: torch.Tensor, cand1: torch.Tensor, rank_user: SparseBatch, dense: torch.Tensor):
        B = u.shape[0]
        v = gather_rows(self.searcher.index, cand1)                                         # [B*K1, E]
        x = (u[:, None, :] * v.view(B, self.k1, -1)).reshape(B * self.k1, -1).contiguous()
        # prerank
        s2 = self.pre2(self.pre1(x)).view(B, self.k1)
        _, pos2 = topk_rows(s2, self.k2)
        cand2 = torch.gather(cand1, 1, pos2)                                                # [B, K2]
        # rank: ESIM over (user sequence, candidate item sequence) pairs, fp16 MFMA attention
        Lq, d = self.ranker.L, self.ranker.d
        # the (user, candidate) pairs by index: user b's sequence for its k2 candidates, the candidates' rows of the
        # encoded catalog (rf_esim_soft_attention_idx_fwd; nothing expanded or gathered)
        q = self.ranker.enc_q(rank_user).to(self.rank_dtype).view(B, Lq, d).contiguous()
        pooled = torch.empty((B * self.k2, self.ranker.pooled_width), dtype=torch.float32, device=u.device)
        xd = dense.repeat_interleave(self.k2, dim=0) if dense.shape[0] == B else dense
        self.ranker.input_mlp(xd, out=pooled[:, : self.ranker.d_emb])
        esim_soft_attention_pool_idx(q, self.k2, self.a_item.view(-1, Lq, d), cand2, out=pooled, out_col=self.ranker.d_emb)
        p = self.ranker.dense_output(self.ranker.output_mlp(pooled))[:, 1].view(B, self.k2)
        s3, pos3 = topk_rows(p, self.k3)
        return CascadeResult(torch.gather(cand2, 1, pos3), s3, cand1, cand2)


# ------------------------------------------------------------------------------------------------
# cfg5 over P ranks (BASELINE.json configs[4]: "8-GPU data-parallel + sharded tables")
# ------------------------------------------------------------------------------------------------
class ShardedRecall:
    """The recall stage over P ranks, the only stage of the cascade with collectives:

      * request batches are data-parallel (each rank its own users);
      * both towers' sparse lookups read row-sharded fused tables (ShardedFusedEncoder: one all-to-all
        pair per lookup, bit-identical to the single-table kernel for any P);
      * the catalog index is built collectively: rank r encodes its contiguous slice of the catalog, then an
        all-gather assembles the full [N, E] index on every rank (rank order = catalog order);
      * the search is local (exact inner-product top-k over the replicated index).

    The dense parts are callables so the orchestration runs on CPU ranks in the tests with oracle ops:
    user_tower / ad_tower: pooled [B, W] -> l2-normalised [B, E]; search(u, index, k) -> (scores, ids).
    """

    def __init__(self, enc_u, enc_a, user_tower, ad_tower, search, comm, k: int):
        self.enc_u, self.enc_a = enc_u, enc_a
        self.user_tower, self.ad_tower, self.search = user_tower, ad_tower, search
        self.comm, self.k = comm, int(k)
        self.index: Optional[torch.Tensor] = None
        self.offsets = None  # catalog id of each rank's first item

    @torch.no_grad()
    def index_catalog(self, local_batches: Sequence[SparseBatch]) -> torch.Tensor:
        """Collective: every rank passes ITS slice of the catalog (the same number of batches on every rank:
        each batch is one sharded lookup, a collective)."""
        counts = self.comm.all_gather_ints(len(local_batches))
        if len(set(counts)) != 1:
            raise ValueError(f"every rank must encode the same number of catalog batches, got {counts}")
        vs = [self.ad_tower(self.enc_a(b)) for b in local_batches]
        local = torch.cat(vs) if vs else torch.zeros((0, 1))
        sizes = self.comm.all_gather_ints(local.shape[0])
        self.offsets = [sum(sizes[:r]) for r in range(len(sizes))]
        self.index = self.comm.all_gather_rows(local.contiguous())
        return self.index

    @torch.no_grad()
    def forward(self, user_batch: SparseBatch):
        """Collective (the sharded user lookup): (u [B, E], scores [B, k], catalog ids [B, k])."""
        u = self.user_tower(self.enc_u(user_batch))
        scores, ids = self.search(u, self.index, self.k)
        return u, scores, ids


class ShardedCascade(Cascade):
    """Cascade with a ShardedRecall (recall towers on row-sharded tables, collective catalog index) and the
    prerank / rank stages of Cascade, data-parallel (each rank ranks its own users' candidates against the
    replicated ESIM catalog)."""

    def __init__(self, recall: Dssm, ranker: Esim, enc_u, enc_a, comm, **kw):
        super().__init__(recall, ranker, **kw)
        self.srecall = ShardedRecall(enc_u, enc_a, self._tower(recall.user_dense), self._tower(recall.ad_dense),
                                     self._search, comm, self.k1)

    @staticmethod
    def _tower(mlp):
        return lambda x: torch.nn.functional.normalize(mlp(x), dim=-1, eps=1e-6)

    def _search(self, u, index, k):
        d, i = self.searcher.search_index(u, k)
        return d, i

    @torch.no_grad()
    def index_catalog(self, recall_ad_local: Sequence[SparseBatch], rank_ad: Sequence[SparseBatch]):
        """Collective. recall_ad_local: this rank's slice of the catalog (ad slots of the recall tables);
        rank_ad: the whole catalog's ESIM ad sequences (replicated ranker tables: every rank encodes all)."""
        items = self.srecall.index_catalog(recall_ad_local)
        self.searcher = FaissSearcher(items=items, index_param="Flat", measurement="ip").train()
        self.a_item = torch.cat([self.ranker.enc_a(kb).to(self.rank_dtype) for kb in rank_ad]).contiguous()
        return self

    @torch.no_grad()
    def forward(self, recall_user: SparseBatch, rank_user: SparseBatch, dense: torch.Tensor) -> CascadeResult:
        u, _, cand1 = self.srecall.forward(recall_user)
        return self._prerank_rank(u, cand1, rank_user, dense)
