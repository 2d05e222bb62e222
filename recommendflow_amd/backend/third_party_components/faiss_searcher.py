"""FaissSearcher on the GPU: exact (Flat) inner-product / cosine search (reference:
backend/third_party_components/faiss_searcher.py:23-225, which wraps faiss.index_factory).

Only the exact index is rebuilt (index_param "Flat", measurement "ip" | "cos"): the item matrix stays
resident in HBM (fp32, l2-normalised for "cos" like __normvec__ :104-105), each query batch is scored
block by block with the MFMA GEMM (rf_linear_fwd: queries . items_block^T, 32768 items per block) and
the running top-k is merged after every block (rf_topk_merge: radix select + bitonic merge, ties by
smaller item index). Approximate faiss indexes (IVF / HNSW / PQ) are out of scope.

Screened form (round 5; fp32 index, E >= 256, E % 32 == 0, more than one block, not inside a graph capture): the
first block is scored and merged as above, its k-th best score per query is a threshold no item of the exact top-k
falls below (the k-th best over all items is at least the k-th best of any subset), and ONE launch over the other
N - 32768 items (rf_ip_candidates_f32: the same fp32 MFMA scores, no score matrix written) keeps every item at or
above it; one rf_topk_merge_idx over those candidates and the first block's top-k gives the result. Same scores,
same ties (item index), same top-k as the block loop; a query whose candidate list overflows `cap` sends the whole
batch back to the block loop (one host read of the counts). It removes the [B, N] score matrix's write and re-read
(2 x 4.3 GB at the cfg5 shapes). On long catalogs (more than 8 blocks, E % 64 == 0) the first 4 blocks are scored
exactly for the threshold (blocks 2-4 screened by block 1's k-th score) and the rest is screened on bf16 copies (rf_ip_candidates_bf16: a pair is kept when its
bf16 score is within the bf16 error bound C ||q|| ||v|| of the threshold), the kept pairs rescored exactly in
rf_linear_fwd's k order (rf_ip_rescore_f32: the same bits) before the merge: the result is still the block loop's,
bit for bit.

search() returns what the reference returns without an encoder: (item_list[indexes], directories) for
an int topK, {k: (items, sims)} for a list of topK (:178-204).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Union

import numpy as np
import torch

from ...runtime import lib as L

BLOCK = 32768
SCREEN_CAP_MAX = 32768  # rf_topk_merge_idx's column limit
# bf16 screen: |<q~, v~> - <q, v>| <= (2u + u^2 + 2 gamma_K (1 + u)^2) sum |q_i v_i| <= C ||q|| ||v|| with u = 2^-8 (bf16
# round to nearest), gamma_K = K 2^-24 / (1 - K 2^-24) for the fp32 sums of both (K <= 1024): 0.00791 at K = 1024;
# C = 0.008 also covers the rounding of the two norms
SCREEN_BF16_C = 0.008
SCREEN_EXACT_BLOCKS = 4  # leading blocks scored exactly for the threshold before a bf16 screen


class FaissSearcher:
    def __init__(self, encoder=None, items=None, item_list: Optional[Sequence] = None, index_param: str = None,
                 measurement: Union[str, int] = None, norm_vec: bool = False, use_gpu: bool = True,
                 dtype=torch.float32, device="cuda", **kwargs):
        if encoder is not None:
            raise NotImplementedError("FaissSearcher(encoder=...) (text encoders) is outside the hot path; pass vectors")
        if items is None or index_param is None or measurement is None:
            raise AssertionError("Args 'items' 'index_param' 'measurement' must be given.")
        items = items.detach().cpu().numpy() if isinstance(items, torch.Tensor) else items
        if not isinstance(items, np.ndarray):
            raise ReferenceError("如果不传入encoder，则item只能输入numpy.array类型")
        if len(items.shape) != 2:
            raise AssertionError(f"encoder=None, 输入只能是二维矩阵[(n, dim)]，当前维度为[{items.shape}]")
        if item_list is not None:
            assert len(item_list) == len(items), f"len(item_list)={len(item_list)} != len(items)={len(items)}"
        if str(index_param).lower() != "flat":
            raise NotImplementedError(f"index_param {index_param!r}: only the exact 'Flat' index is implemented")
        if measurement not in ("ip", "cos"):
            raise NotImplementedError(f"measurement {measurement!r}: only 'ip' and 'cos' are implemented")
        L.load()
        L.require_gpu()
        self.index_param, self.measurement = index_param, measurement
        self.norm_vec = True if measurement == "cos" else norm_vec
        self.items = items
        self.item_list = np.array(item_list if item_list is not None else np.arange(len(items)))
        self.vec_dim = items.shape[1]
        self.dtype = dtype
        self.device = torch.device(device)
        self.index = None

    def get_vecs(self, items) -> torch.Tensor:
        x = items if isinstance(items, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(items))
        x = x.to(self.device, torch.float32)
        if self.norm_vec:
            x = x / (x * x).sum(dim=1, keepdim=True).sqrt()
        return x.to(self.dtype).contiguous()

    def train(self):
        self.index = self.get_vecs(self.items)  # [N, E] resident in HBM
        return self

    @property
    def index(self):
        return self._index

    @index.setter
    def index(self, value):
        # assigning an index drops the bf16 screen's copy and the item norms derived from the old one
        self._index = value
        self._screen_key = None
        self.index_bf16 = self.index_norm = None

    def _bf16_screen_index(self):
        # keyed on the index tensor's identity and version as well: an in-place write to the index rebuilds them
        key = (self._index.data_ptr(), tuple(self._index.shape), self._index._version)
        if self.index_bf16 is None or self._screen_key != key:
            self.index_bf16 = self._index.to(torch.bfloat16).contiguous()
            self.index_norm = self._index.norm(dim=1).contiguous()
            self._screen_key = key
        return self.index_bf16, self.index_norm

    screen = True  # the screened search where it applies (A/B: False keeps the block loop)

    screen_bf16 = True  # the bf16 screen + exact rescoring where the catalog is long enough (A/B: False)

    def _screened(self, q: torch.Tensor, k: int):
        """The screened search (module docstring), or None when a candidate list overflowed."""
        B, E = q.shape
        N = self.index.shape[0]
        dev = self.device
        st = L.stream_ptr()
        bf = self.screen_bf16 and N > 2 * SCREEN_EXACT_BLOCKS * BLOCK and E % 64 == 0 and E <= 1024
        n0 = SCREEN_EXACT_BLOCKS * BLOCK if bf else BLOCK
        # the first block exactly (the block loop's scores and merge)
        scores = torch.empty((B, BLOCK), dtype=torch.float32, device=dev)
        v0 = torch.empty((B, k), dtype=torch.float32, device=dev)
        i0 = torch.empty((B, k), dtype=torch.int64, device=dev)
        L.call("rf_linear_fwd", L.ptr(q), L.DT_F32, B, E, q.stride(0), L.ptr(self.index), BLOCK, None, 0, L.ptr(scores),
               scores.stride(0), st)
        L.call("rf_topk_merge", L.ptr(scores), scores.stride(0), B, BLOCK, k, 0, None, None, 0, k, L.ptr(v0), L.ptr(i0), k, st)
        del scores
        lead_counts = []
        if n0 > BLOCK:
            # the next leading blocks exactly as well, but screened by the first block's k-th score (one fp32
            # compaction launch, one merge of its few candidates) instead of a score block and a merge each
            t0 = v0[:, k - 1].contiguous()
            cap0 = int(min(SCREEN_CAP_MAX, max(1024, 3 * k * (n0 - BLOCK) // BLOCK + k)))  # ~3x the expected count
            cnt0 = torch.zeros(B, dtype=torch.int32, device=dev)
            cv0 = torch.full((B, cap0), float("nan"), dtype=torch.float32, device=dev)
            ci0 = torch.empty((B, cap0), dtype=torch.int32, device=dev)
            L.call("rf_ip_candidates_f32", L.ptr(q), q.stride(0), B, L.ptr(self.index[BLOCK:]), n0 - BLOCK, E, L.ptr(t0),
                   cap0, L.ptr(cnt0), L.ptr(cv0), L.ptr(ci0), BLOCK, st)
            v1 = torch.empty_like(v0)
            i1 = torch.empty_like(i0)
            L.call("rf_topk_merge_idx", L.ptr(cv0), L.ptr(ci0), cap0, B, cap0, k, L.ptr(v0), L.ptr(i0), k, k, L.ptr(v1),
                   L.ptr(i1), k, st)
            v0, i0 = v1, i1
            lead_counts.append((cnt0, cap0))  # checked with the later counts (one host read)
        thr = v0[:, k - 1].contiguous()  # -inf where the blocks held fewer than k scores (then every item passes)
        # room for ~3x the candidates a uniform score distribution gives (k per n0 items; x1.5 for the bf16 margin)
        per = 3 * k * (N - n0) // n0 * (3 if bf else 2) // 2 + k
        cap = int(min(SCREEN_CAP_MAX, max(1024, per)))
        count = torch.zeros(B, dtype=torch.int32, device=dev)
        cval = torch.full((B, cap), float("nan"), dtype=torch.float32, device=dev)
        cidx = torch.empty((B, cap), dtype=torch.int32, device=dev)
        if bf:
            # candidates by bf16 scores within their error bound of the threshold, then their exact fp32 scores in
            # rf_linear_fwd's k order (rf_ip_rescore_f32: the same bits)
            ib, vn = self._bf16_screen_index()
            qb = q.to(torch.bfloat16).contiguous()
            qbound = (q.norm(dim=1) * SCREEN_BF16_C).contiguous()
            L.call("rf_ip_candidates_bf16", L.ptr(qb), qb.stride(0), B, L.ptr(ib[n0:]), N - n0, E, L.ptr(thr),
                   L.ptr(qbound), L.ptr(vn[n0:]), cap, L.ptr(count), L.ptr(cval), L.ptr(cidx), n0, st)
            if int(count.max().item()) > cap or any(int(c.max().item()) > cp for c, cp in lead_counts):
                return None
            L.call("rf_ip_rescore_f32", L.ptr(q), q.stride(0), B, L.ptr(self.index), E, L.ptr(count), cap, L.ptr(cval),
                   L.ptr(cidx), 0, st)
        else:
            L.call("rf_ip_candidates_f32", L.ptr(q), q.stride(0), B, L.ptr(self.index[n0:]), N - n0, E, L.ptr(thr), cap,
                   L.ptr(count), L.ptr(cval), L.ptr(cidx), n0, st)
            if int(count.max().item()) > cap:
                return None
        out_v = torch.empty((B, k), dtype=torch.float32, device=dev)
        out_i = torch.empty((B, k), dtype=torch.int64, device=dev)
        L.call("rf_topk_merge_idx", L.ptr(cval), L.ptr(cidx), cap, B, cap, k, L.ptr(v0), L.ptr(i0), k, k, L.ptr(out_v),
               L.ptr(out_i), k, st)
        return out_v, out_i

    def search_index(self, target, k: int):
        """(directories [B, k] fp32, indexes [B, k] int64) on the device — faiss index.search."""
        if self.index is None:
            raise Exception("Faiss dose not train, please use train method before search or load a trained index...")
        if not 1 <= k <= 1024:
            raise ValueError("topK must be in [1, 1024]")
        q = self.get_vecs(target)
        B, E = q.shape
        N = self.index.shape[0]
        if (self.screen and self.dtype == torch.float32 and N > BLOCK and E >= 256 and E % 32 == 0 and B > 0
                and not torch.cuda.is_current_stream_capturing()):
            res = self._screened(q, k)
            if res is not None:
                return res
        dev = self.device
        vals = [torch.empty((B, k), dtype=torch.float32, device=dev) for _ in range(2)]
        idxs = [torch.empty((B, k), dtype=torch.int64, device=dev) for _ in range(2)]
        scores = torch.empty((B, min(BLOCK, max(N, 1))), dtype=torch.float32, device=dev)
        st = L.stream_ptr()
        dt = L.torch_dtype_code(self.dtype)
        cur, k_prev = 0, 0
        for c0 in range(0, N, BLOCK):
            n = min(BLOCK, N - c0)
            blk = self.index[c0:c0 + n]
            L.call("rf_linear_fwd", L.ptr(q), dt, B, E, q.stride(0), L.ptr(blk), n, None, 0, L.ptr(scores), scores.stride(0), st)
            nxt = 1 - cur
            L.call("rf_topk_merge", L.ptr(scores), scores.stride(0), B, n, k, c0, L.ptr(vals[cur]), L.ptr(idxs[cur]), k_prev,
                   k, L.ptr(vals[nxt]), L.ptr(idxs[nxt]), k, st)
            cur, k_prev = nxt, k
        if k_prev == 0:
            vals[cur].fill_(-float("inf"))
            idxs[cur].fill_(-1)
        return vals[cur], idxs[cur]

    def search(self, target, topK: Union[int, List[int]], keep_rank_no=False):
        if isinstance(topK, int):
            d, i = self.search_index(target, topK)
            i = i.cpu().numpy()
            return (self.item_list[i], d.cpu().numpy(), i) if keep_rank_no else (self.item_list[i], d.cpu().numpy())
        if isinstance(topK, list):
            d, i = self.search_index(target, max(topK))
            d, i = d.cpu().numpy(), i.cpu().numpy()
            res = {}
            for k in topK:
                res[k] = (self.item_list[i[:, :k]], d[:, :k], i[:, :k]) if keep_rank_no else (self.item_list[i[:, :k]], d[:, :k])
            return res
        raise TypeError(f"TopK dose not support type: {type(topK)}")
