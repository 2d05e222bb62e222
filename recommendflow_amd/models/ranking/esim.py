"""ESIM ranker on the MI355X hot path (reference: models/ranking/esim.py:13-93).

Forward (reference lines in brackets):
  d_emb  = input_mlp(dense)                                   [esim.py:70-75; create_mlp gelu + LayerNorm]
  q, a   = user / ad sparse-slot token sequences [B, L, 2D]   (deviation D-esim-inputs: the reference takes
           BERT token sequences; here each slot is one token = its DoubleHashingEmbedding output, so the
           sequence comes straight out of one fused encoder launch per tower)
  pooled = [d_emb, avg_q, max_q, avg_a, max_a, avg_q-avg_a, max_q-max_a]   [esim.py:78-84; one fused kernel
           (rf_esim_gather_fwd: the q / a token rows gathered from the tables by id)]
  p      = softmax(output_mlp(pooled) W + b)                  [esim.py:85-88; Dropout = identity]
Buffers: the ESIM kernel and the input MLP write straight into column ranges of one [B, 512 + 6d] tensor.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import torch

from ...backend.blocks.mlp import create_mlp
from ...backend.encoder.sparse_encoder import FusedSparseEncoder, SlotSpec
from ...backend.layers.attention_layers import esim_soft_attention_pool
from ...backend.layers.core import Dense, LayerNormalization
from ...runtime.batch import SparseBatch


class Esim(torch.nn.Module):
    def __init__(self, user_slots: Sequence[SlotSpec], ad_slots: Sequence[SlotSpec], n_dense: int, dim: int = 64,
                 table_dtype=torch.bfloat16, mlp_dtype=torch.bfloat16, input_units=(256, 512), output_units=(1024, 512),
                 seed: int = 0, device="cuda", encoders: Optional[tuple] = None):
        super().__init__()
        if len(user_slots) != len(ad_slots):
            raise ValueError("SoftAttention needs equal q / a lengths (attention_layers.py:74)")
        self.L = len(user_slots)
        self.d = 2 * dim
        if encoders is None:
            encoders = (FusedSparseEncoder(user_slots, dim, table_dtype=table_dtype, seed=seed + 1, device=device,
                                           spec_rows=True),
                        FusedSparseEncoder(ad_slots, dim, table_dtype=table_dtype, seed=seed + 2, device=device,
                                           spec_rows=True))
        self.enc_q, self.enc_a = encoders
        ln = LayerNormalization(epsilon=1e-6)
        self.input_mlp = create_mlp(list(input_units), 0.3, "gelu", ln, in_features=n_dense, dtype=mlp_dtype,
                                    seed=seed + 10, device=device)
        self.d_emb = self.input_mlp.out_features
        self.pooled_width = self.d_emb + 6 * self.d
        self.output_mlp = create_mlp(list(output_units), 0.3, "gelu", ln, in_features=self.pooled_width,
                                     dtype=mlp_dtype, seed=seed + 20, device=device)
        self.dense_output = Dense(self.output_mlp.out_features, 2, activation="softmax", dtype=mlp_dtype,
                                  seed=seed + 30, device=device)

    def forward(self, user: SparseBatch, ad: SparseBatch, dense: torch.Tensor) -> torch.Tensor:
        """The input MLP (dense features only) writes pooled[:, :d_emb], the attention pooled[:, d_emb:]. By
        default it runs first on the current stream; concurrent_input_mlp = True puts it on a side stream
        beside the two encoders (the output MLP waits for both; inside a hipGraph capture the fork/join
        become graph edges)."""
        B = user.batch
        cur = torch.cuda.current_stream(dense.device)
        pooled = torch.empty((B, self.pooled_width), dtype=torch.float32, device=dense.device)
        if not self.concurrent_input_mlp:
            if self._gather_ok(user, ad) and self._fused_scorer_ok(dense):
                return self._forward_fused_scorer(user, ad, dense)
            self.input_mlp(dense, out=pooled[:, : self.d_emb])
            if self._gather_ok(user, ad):
                self._esim_gather(user, ad, pooled)
            else:
                q = self.enc_q(user).view(B, self.L, self.d)
                a = self.enc_a(ad).view(B, self.L, self.d)
                esim_soft_attention_pool(q, a, out=pooled, out_col=self.d_emb)
            return self.dense_output(self.output_mlp(pooled))
        side = self._side_stream(dense.device)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            self.input_mlp(dense, out=pooled[:, : self.d_emb])
        pooled.record_stream(side)
        dense.record_stream(side)
        if self._gather_ok(user, ad):
            self._esim_gather(user, ad, pooled)
        else:
            q = self.enc_q(user).view(B, self.L, self.d)
            a = self.enc_a(ad).view(B, self.L, self.d)
            esim_soft_attention_pool(q, a, out=pooled, out_col=self.d_emb)
        cur.wait_stream(side)
        return self.dense_output(self.output_mlp(pooled))

    # True: the input MLP on a side stream beside the encoders / the id pass. Measured (tools/cfg3_gaps.py,
    # graph-replayed forward): serial is faster in both forms — encoders 0.2601-0.2604 vs 0.2638-0.2665 ms
    # (profiles/r03/r03b6_*: the side launch slowed both encoder launches by ~2.4 us each), gather path
    # 0.1802-0.1815 vs 0.1883 ms (r03b9: the id launches 12.7 -> 15.5 us beside it, plus the fork/join)
    concurrent_input_mlp = False

    # True: the attention gathers its q / a token rows from the tables by id (rf_single_token_ids_fwd ->
    # rf_esim_gather_fwd) when every slot of both batches is single-valued, bf16 tables; the encoders'
    # [B, L, 2D] outputs are then never written. Bit-identical to the encoder path
    # (test_esim_gather_equals_encoders_plus_attention); cfg3 forward 0.2616 -> 0.1843 ms
    # (profiles/r03/r03b7_cfg3_gather_trace.txt). False: encoders + rf_esim_soft_attention_fwd.
    gather = True

    # True (gather path): the pooled row is never normalised by its own pass nor stored as fp32 — the input MLP and
    # the attention write it as bf16 with per-32-column-slice partials, the output MLP folds both LayerNorms into
    # its GEMMs and the Dense(2, softmax) head's partial logits ride the last GEMM's epilogue.
    # False: pooled fp32 -> rf_norm_fwd -> stats GEMM -> LN-fold GEMM -> rf_dense_head_fwd.
    fused_scorer = True

    def _fused_scorer_ok(self, dense: torch.Tensor) -> bool:
        return (self.fused_scorer and self.d_emb % 32 == 0 and (6 * self.d) % 32 == 0
                and self.input_mlp.denses and self.input_mlp._fusable(dense)
                and self.output_mlp.prenormed_head_ok(self.pooled_width, self.dense_output))

    def _forward_fused_scorer(self, user: SparseBatch, ad: SparseBatch, dense: torch.Tensor) -> torch.Tensor:
        """input MLP -> pooled[:, :d_emb] (bf16 + slice partials, rf_mlp2_small_stats_fwd); id pass; attention ->
        pooled[:, d_emb:] (rf_esim_gather_stats_fwd); output MLP + head on the folded chain (forward_prenormed_head)."""
        from ...runtime import lib as L

        B, W = user.batch, self.pooled_width
        pb = torch.empty((B, W), dtype=torch.bfloat16, device=dense.device)
        pst = torch.empty((B, W // 32, 2), dtype=torch.float32, device=dense.device)
        self.input_mlp.forward_stats(dense, pb[:, : self.d_emb], pst, 0)
        q_ids, a_ids = self.token_ids(user, ad)
        self._check_ids(q_ids, a_ids)
        eq, ea = self.enc_q, self.enc_a
        L.call("rf_esim_gather_stats_fwd", L.ptr(q_ids), L.ptr(a_ids), L.ptr(eq.table), eq.table.shape[0], L.ptr(ea.table),
               ea.table.shape[0], L.DT_BF16, B, self.L, self.d, L.ptr(pb), pb.stride(0), self.d_emb, L.ptr(pst), W // 32,
               self.d_emb // 32, L.stream_ptr(None))
        return self.output_mlp.forward_prenormed_head(pb, pst, self.dense_output)

    def _check_batches(self, user: SparseBatch, ad: SparseBatch):
        """The shapes both ESIM paths rely on: the gather path sizes its id buffers [B, L, 2] from these, so a
        mismatch must raise before any launch (the encoder path raises the same errors)."""
        if user.batch != ad.batch:
            raise ValueError(f"user batch {user.batch} != ad batch {ad.batch}")
        for name, b, enc in (("user", user, self.enc_q), ("ad", ad, self.enc_a)):
            if len(enc.slots) != self.L:
                raise ValueError(f"{name} encoder has {len(enc.slots)} slots, the attention L = {self.L}")
            if b.n_slots != len(enc.slots):
                raise ValueError(f"batch has {b.n_slots} slots, encoder {len(enc.slots)}")

    def _gather_ok(self, user: SparseBatch, ad: SparseBatch) -> bool:
        self._check_batches(user, ad)
        eq, ea = self.enc_q, self.enc_a
        return (self.gather and isinstance(eq, FusedSparseEncoder) and isinstance(ea, FusedSparseEncoder)
                and eq.table.dtype == torch.bfloat16 and ea.table.dtype == torch.bfloat16
                and 2 * eq.dim == self.d and 2 * ea.dim == self.d and self.d in (64, 128) and self.L <= 128
                and not eq.extra_flags and not ea.extra_flags and eq.spec_rows and ea.spec_rows
                and eq._single_token_batch(user) and ea._single_token_batch(ad))

    def token_ids(self, user: SparseBatch, ad: SparseBatch):
        """(q_ids, a_ids) [B, L, 2] int32: each token's two fused-table rows (rf_single_token_ids_fwd)."""
        from ...runtime import lib as L

        self._check_batches(user, ad)
        B, dev = user.batch, self.enc_q.table.device
        ids, tasks, keep = [], (L.IdsTask * 2)(), []
        for k, (enc, b) in enumerate(((self.enc_q, user), (self.enc_a, ad))):
            if not b.is_device():
                b = b.to(dev)
                keep.append(b)
            t = torch.empty((B, self.L, 2), dtype=torch.int32, device=dev)
            tasks[k] = L.IdsTask(L.ptr(enc.desc), L.ptr(b.tok_bytes), L.ptr(b.tok_off), L.ptr(b.bag_off), L.ptr(b.lmax),
                                 L.ptr(t), enc.table.shape[0], len(enc.slots), B,
                                 (L.FLAG_MASK_PADDING if enc.mask_padding else 0) | L.FLAG_SPEC_ROWS, 0)
            ids.append(t)
        # both towers' index passes in one launch (rf_single_token_ids_multi_fwd; the host task array is read at the
        # call, so it need not outlive it)
        L.call("rf_single_token_ids_multi_fwd", ctypes.addressof(tasks), 2, L.stream_ptr(None))
        return ids[0], ids[1]

    def _check_ids(self, q_ids: torch.Tensor, a_ids: torch.Tensor):
        B = q_ids.shape[0]
        if (q_ids.shape != (B, self.L, 2) or a_ids.shape != (B, self.L, 2) or q_ids.dtype != torch.int32
                or a_ids.dtype != torch.int32 or not q_ids.is_contiguous() or not a_ids.is_contiguous()):
            raise ValueError(f"token ids must be int32 [B, {self.L}, 2] on both sides, got {tuple(q_ids.shape)} / "
                             f"{tuple(a_ids.shape)}")

    def attention_gather(self, q_ids: torch.Tensor, a_ids: torch.Tensor, pooled: torch.Tensor):
        """The ESIM attention + pooling into pooled[:, d_emb:], its q / a images gathered by id (rf_esim_gather_fwd)."""
        from ...runtime import lib as L

        B = q_ids.shape[0]
        self._check_ids(q_ids, a_ids)
        if pooled.dtype != torch.float32 or pooled.dim() != 2 or pooled.shape[0] != B or pooled.shape[1] < self.d_emb + 6 * self.d or pooled.stride(1) != 1:
            raise ValueError(f"pooled must be a row-major [{B}, >= {self.d_emb + 6 * self.d}] fp32 tensor")
        eq, ea = self.enc_q, self.enc_a
        if not (eq.spec_rows and ea.spec_rows):
            raise ValueError("the gather path needs encoders built with spec_rows=True")
        L.call("rf_esim_gather_fwd", L.ptr(q_ids), L.ptr(a_ids), L.ptr(eq.table), eq.table.shape[0], L.ptr(ea.table),
               ea.table.shape[0], L.DT_BF16, q_ids.shape[0], self.L, self.d, L.ptr(pooled), pooled.stride(0),
               self.d_emb, L.stream_ptr(None))

    def _esim_gather(self, user: SparseBatch, ad: SparseBatch, pooled: torch.Tensor):
        self.attention_gather(*self.token_ids(user, ad), pooled)

    def _side_stream(self, device):
        s = getattr(self, "_side", None)
        if s is None or s.device != device:
            s = self._side = torch.cuda.Stream(device=device)
        return s

    def graphed(self, user: SparseBatch, ad: SparseBatch, dense: torch.Tensor, **kw):
        """This forward captured as one hipGraph on static copies of (user, ad, dense) (runtime.graphs):
        the returned callable takes batches of the same B / slot counts and replays the launches without
        the per-launch host path. Its output buffer is reused by the next call."""
        from ...runtime.graphs import GraphedForward

        return GraphedForward(self.forward, user, ad, dense, **kw)

    def flops_per_example(self) -> float:
        """Dense FLOPs per example: ESIM products (2 L^2 d for E + 2 * 2 L^2 d for the alignments) + MLP GEMMs."""
        att = 2 * self.L * self.L * self.d * 3
        mlp = 0
        for m in (self.input_mlp, self.output_mlp):
            for dn in m.denses:
                mlp += 2 * dn.in_features * dn.units
        mlp += 2 * self.dense_output.in_features * 2
        return float(att + mlp)
