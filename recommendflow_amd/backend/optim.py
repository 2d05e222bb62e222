"""Optimizers for the fused embedding tables.

Reference: ``tf.keras.optimizers.Adam(learning_rate=args.learning_rate)`` compiled into every training
script (example/ranking_search/train.py:97, example/recall_search/train.py:97, finetune.py:78); Keras'
defaults beta_1 = 0.9, beta_2 = 0.999, epsilon = 1e-7. For an Embedding variable Keras applies
Adam._resource_apply_sparse to the deduplicated IndexedSlices gradient: m and v decay over the whole
variable, the scaled gradient is scatter-added, and every row moves (dense semantics). ``lazy=True``
touches only the rows in the gradient (TF-Addons LazyAdam; deviation D-lazy-adam, opt-in).
``deferred=True`` keeps the dense semantics but moves an untouched row only when it is next listed: each row
carries the step it is current through, and rf_adam_replay applies the missed steps' untouched updates (same
fp32 expressions, same order, each step's own lr) before a forward reads the row or its gradient update runs.
Every row read is bit-identical to the dense step's; ``materialize()`` brings the whole table current before
anything else reads it (evaluation, checkpoints, tests).

Dense variables (the towers) take Keras' Adam._resource_apply_dense (TF ResourceApplyAdam) through
``KerasAdam`` (rf_adam_dense, one launch per variable).
"""
from __future__ import annotations

import numpy as np
import torch

from ..runtime import lib as L
from .encoder.sparse_encoder import SparseGrad


class SparseAdam:
    """tf.keras.optimizers.Adam for an fp32 fused embedding table, driven by SparseGrad (rf_adam_apply)."""

    def __init__(self, table: torch.Tensor, learning_rate: float = 0.001, beta_1: float = 0.9, beta_2: float = 0.999,
                 epsilon: float = 1e-7, lazy: bool = False, deferred: bool = False):
        if table.dtype != torch.float32 or table.dim() != 2 or not table.is_contiguous():
            raise ValueError("SparseAdam needs a contiguous fp32 [rows, dim] table")
        if lazy and deferred:
            raise ValueError("SparseAdam: lazy and deferred are exclusive (deferred keeps the dense semantics)")
        self.table = table
        self.learning_rate, self.beta_1, self.beta_2, self.epsilon = learning_rate, beta_1, beta_2, epsilon
        self.lazy = bool(lazy)
        self.deferred = bool(deferred)
        self.m = torch.zeros_like(table)
        self.v = torch.zeros_like(table)
        self.iterations = 0
        wsb = int(L.load().rf_adam_ws_bytes(table.shape[0], int(self.lazy or self.deferred)))
        self._ws = torch.empty(max(wsb, 256), dtype=torch.uint8, device=table.device)
        if self.deferred:
            self.last = torch.zeros(table.shape[0], dtype=torch.int32, device=table.device)
            self._lr_host = np.zeros(1, np.float32)  # index = step (entry 0 unused)
            self._lr_dev = None

    def _lr_at(self, t: int) -> np.float32:
        f = np.float32
        tt = f(t)
        b1p, b2p = np.power(f(self.beta_1), tt), np.power(f(self.beta_2), tt)
        return f(self.learning_rate) * (np.sqrt(f(1) - b2p) / (f(1) - b1p))

    def step_lr(self) -> float:
        """lr_t * sqrt(1 - beta_2^t) / (1 - beta_1^t) in float32, t = iterations + 1 (Keras local_step)."""
        return float(self._lr_at(self.iterations + 1))

    def _lr_log(self, t: int) -> torch.Tensor:
        """Device f32 [>= t + 1]: entry s = step s's lr (the scalar step_lr() computes, element by element)."""
        if self._lr_dev is None or len(self._lr_host) <= t:
            n = max(4096, 2 * len(self._lr_host), t + 1)
            host = np.zeros(n, np.float32)
            host[: len(self._lr_host)] = self._lr_host
            for s in range(max(1, len(self._lr_host)), n):
                host[s] = self._lr_at(s)
            self._lr_host = host
            self._lr_dev = torch.from_numpy(host).to(self.table.device)
        return self._lr_dev

    def _replay(self, rows, n_uniq, cap: int, t_set: int, stream=None):
        t = self.iterations
        L.call("rf_adam_replay", L.ptr(self.table), L.ptr(self.m), L.ptr(self.v), self.table.shape[0],
               self.table.shape[1], L.ptr(rows) if rows is not None else None, L.ptr(n_uniq) if n_uniq is not None else None,
               cap, L.ptr(self.last), t, t_set, L.ptr(self._lr_log(t)), self.beta_1, self.beta_2, self.epsilon,
               L.stream_ptr(stream))

    def prepare_ids(self, ids: torch.Tensor, stream=None):
        """deferred: prepare() for a plain int64 id list that may repeat ids (the rows a shard serves to every
        requester; each listed row is replayed once, ids outside the table are skipped)."""
        if self.deferred and ids.numel():
            if ids.dtype != torch.int64 or not ids.is_contiguous():
                ids = ids.to(torch.int64).contiguous()
            self._replay(ids, None, ids.numel(), self.iterations, stream)

    def prepare(self, rows: torch.Tensor, n_uniq: torch.Tensor, cap: int, stream=None):
        """deferred: bring rows[:n_uniq] current through the last completed step before a forward reads them."""
        if self.deferred:
            self._replay(rows, n_uniq, cap, self.iterations, stream)
            self._prepared = (rows, n_uniq, self.iterations)

    def materialize(self, stream=None):
        """deferred: every row current (the table, m and v then equal the dense step's, bit for bit)."""
        if self.deferred:
            self._replay(None, None, 0, self.iterations, stream)

    def state(self) -> dict:
        """The table, m, v and the step count, every row current (materialize() first): what a checkpoint holds."""
        self.materialize()
        return {"table": self.table, "m": self.m, "v": self.v, "iterations": int(self.iterations)}

    def load_state(self, table: torch.Tensor, m: torch.Tensor, v: torch.Tensor, iterations: int, stream=None):
        """Overwrite the table, m and v in place with a checkpoint's values taken after `iterations` steps. Every row
        is then current through that step (deferred: `last` is reset, so no missed step is replayed onto the loaded
        values)."""
        for dst, src, nm in ((self.table, table, "table"), (self.m, m, "m"), (self.v, v, "v")):
            if tuple(src.shape) != tuple(dst.shape):
                raise ValueError(f"SparseAdam.load_state: {nm} shape {tuple(src.shape)} != {tuple(dst.shape)}")
            dst.copy_(src)
        self.iterations = int(iterations)
        self._prepared = None
        if self.deferred:
            self.last.fill_(self.iterations)

    def apply_untouched(self, rows: torch.Tensor, n_uniq: torch.Tensor, cap: int, stream=None):
        """The first half of this iteration's dense step: every row not in rows[:n_uniq] (rf_adam_untouched). The
        second half is apply_touched() with the gradient over exactly those rows; together they equal apply()."""
        L.call("rf_adam_untouched", L.ptr(self.table), L.ptr(self.m), L.ptr(self.v), self.table.shape[0],
               self.table.shape[1], L.ptr(rows), L.ptr(n_uniq), cap, self.step_lr(), self.beta_1, self.beta_2,
               self.epsilon, L.ptr(self._ws), self._ws.numel(), L.stream_ptr(stream))

    def apply_touched(self, g: SparseGrad, stream=None):
        """The second half (after apply_untouched on g's row set): the listed rows with their gradient."""
        L.call("rf_adam_apply", L.ptr(self.table), L.ptr(self.m), L.ptr(self.v), self.table.shape[0], self.table.shape[1],
               L.ptr(g.rows), L.ptr(g.grad), L.ptr(g.n_uniq), g.cap, self.step_lr(), self.beta_1, self.beta_2,
               self.epsilon, 1, L.ptr(self._ws), self._ws.numel(), L.stream_ptr(stream))
        self.iterations += 1

    def apply(self, g: SparseGrad, stream=None, rows_current: bool = False):
        """One Keras Adam step with g. rows_current (deferred only): the caller guarantees every row of g was
        replayed for this step (prepare / prepare_ids), so the marking rides on the touched update."""
        if self.deferred:
            prep = getattr(self, "_prepared", None)
            self._prepared = None
            if (rows_current or (prep is not None and prep[0] is g.rows and prep[1] is g.n_uniq
                                 and prep[2] == self.iterations)):
                # every gradient row was replayed for this step (the plan's own rows, or the caller says so): the
                # touched update marks them in the same pass
                L.call("rf_adam_apply_current", L.ptr(self.table), L.ptr(self.m), L.ptr(self.v), self.table.shape[0],
                       self.table.shape[1], L.ptr(g.rows), L.ptr(g.grad), L.ptr(g.n_uniq), g.cap, self.step_lr(),
                       self.beta_1, self.beta_2, self.epsilon, L.ptr(self.last), self.iterations + 1,
                       L.stream_ptr(stream))
                self.iterations += 1
                return
            # the gradient's rows current through the last step (a no-op for rows prepare() already moved), marked
            # current through this one, then their touched update
            self._replay(g.rows, g.n_uniq, g.cap, self.iterations + 1, stream)
            L.call("rf_adam_apply", L.ptr(self.table), L.ptr(self.m), L.ptr(self.v), self.table.shape[0],
                   self.table.shape[1], L.ptr(g.rows), L.ptr(g.grad), L.ptr(g.n_uniq), g.cap, self.step_lr(), self.beta_1,
                   self.beta_2, self.epsilon, 1, L.ptr(self._ws), self._ws.numel(), L.stream_ptr(stream))
            self.iterations += 1
            return
        L.call("rf_adam_apply", L.ptr(self.table), L.ptr(self.m), L.ptr(self.v), self.table.shape[0], self.table.shape[1],
               L.ptr(g.rows), L.ptr(g.grad), L.ptr(g.n_uniq), g.cap, self.step_lr(), self.beta_1, self.beta_2,
               self.epsilon, int(self.lazy), L.ptr(self._ws), self._ws.numel(), L.stream_ptr(stream))
        self.iterations += 1


class KerasAdam:
    """tf.keras.optimizers.Adam on dense fp32 parameters (Adam._resource_apply_dense -> ResourceApplyAdam):
    m += (g - m)(1 - beta_1); v += (g^2 - v)(1 - beta_2); var -= m lr_t / (sqrt(v) + epsilon) with Keras'
    bias-corrected lr_t in float32. The torch.optim-style surface (zero_grad, step, param_groups) the
    training loops use; parameters without a gradient are skipped, as Keras skips None gradients."""

    def __init__(self, params, learning_rate: float = 0.001, beta_1: float = 0.9, beta_2: float = 0.999,
                 epsilon: float = 1e-7):
        self.params = [p for p in params]
        for p in self.params:
            if p.dtype != torch.float32 or not p.is_contiguous():
                raise ValueError("KerasAdam needs contiguous fp32 parameters")
        self.learning_rate, self.beta_1, self.beta_2, self.epsilon = learning_rate, beta_1, beta_2, epsilon
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]
        self.iterations = 0
        self.param_groups = [{"params": self.params, "lr": learning_rate}]

    def zero_grad(self, set_to_none: bool = True):
        for p in self.params:
            if set_to_none:
                p.grad = None
            elif p.grad is not None:
                p.grad.zero_()

    def step_lr(self) -> float:
        f = np.float32
        t = f(self.iterations + 1)
        b1p, b2p = np.power(f(self.beta_1), t), np.power(f(self.beta_2), t)
        return float(f(self.learning_rate) * (np.sqrt(f(1) - b2p) / (f(1) - b1p)))

    @torch.no_grad()
    def step(self, stream=None):
        """One launch for every parameter with a gradient (rf_adam_dense_multi): descriptors (w, g, m, v, n)
        written into a pinned ring slot and copied to the device on the step's stream."""
        lr = self.step_lr()
        rows, grads = [], []
        for p, m, v in zip(self.params, self.m, self.v):
            g = p.grad
            if g is None:
                continue
            if g.dtype != torch.float32 or not g.is_contiguous():
                g = g.float().contiguous()
            grads.append(g)
            rows.append((p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel()))
        if rows:
            dev = self.params[0].device
            if not hasattr(self, "_ring"):
                self._ring = [torch.empty((len(self.params), 5), dtype=torch.int64).pin_memory() for _ in range(2)]
                self._ring_ev = [None, None]
                self._desc = torch.empty((len(self.params), 5), dtype=torch.int64, device=dev)
            k = self.iterations % 2
            if self._ring_ev[k] is not None:
                self._ring_ev[k].synchronize()  # the copy that last read this slot is done
            host = self._ring[k]
            host[: len(rows)].copy_(torch.tensor(rows, dtype=torch.int64))
            cur = torch.cuda.current_stream(dev) if stream is None else stream
            with torch.cuda.stream(cur):
                self._desc[: len(rows)].copy_(host[: len(rows)], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(cur)
            self._ring_ev[k] = ev
            L.call("rf_adam_dense_multi", L.ptr(self._desc), len(rows), max(r[4] for r in rows), lr, self.beta_1,
                   self.beta_2, self.epsilon, L.stream_ptr(cur))
            for g in grads:  # the kernel reads them on `cur`
                g.record_stream(cur)
        self.iterations += 1
