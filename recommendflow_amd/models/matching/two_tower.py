"""Two-tower matching model assembled from a parsed configuration (BASELINE configs[0]: conf/demo_conf.yaml).

Reference surface: the matching models take ``self.preprocessor = get_preprocess_layers(conf)``
(models/matching/dssm.py:16, que2search.py:16, siamese_bert.py:17) and call ``self.preprocessor[name](x)``
per feature (que2search.py:76-79) on the dict that ``parse_example`` returns (backend/core/dataloader.py:77-89);
the towers are ``create_mlp(units, 0.3, "selu", BatchNormalization(1e-6))`` (dssm.py:25-26), l2-normalised
(dssm.py:35-36), and the score is the dot product (que2search.py:137, match_losses.py:46).

What each tower concatenates, in configuration order (deviation D-dssm-wiring: the reference's Dssm.call never
wires features to towers, dssm.py:38-60):
  * hashing features      -> the tower's fused encoder (one launch; [B, 2D] per feature)
  * lookup / discrete     -> LookupEmbedding / DiscreteEmbedding ([B, D])
  * token_id features     -> deviation D-token-id: demo_conf's token ids feed BERT towers in the reference
                             (siamese_bert.BertModel, out of scope); here an EmbeddingBag over the ids
                             with the configured pooling (cls = first, D-cls) stands in for the encoder
  * numeric features      -> the raw float column ([B, 1])
Input: a ``runtime.tfrecord.FeatureBatch`` on the device (FeaturePipe's output).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ...backend.blocks.mlp import create_mlp
from ...backend.layers.core import BatchNormalization
from ...backend.layers.preprocess_layers import EmbeddingBag
from ...backend.utils.preprocess_utils import get_preprocess_layers
from ...runtime import lib as L


def padded_ids(rc, name: str, B: int) -> torch.Tensor:
    """Padded [B, Lmax] int64 ids of one int-list feature of a device RaggedColumns, padding 0 (the
    FixedLenSequenceFeature default of dataloader.py:32-33)."""
    S = len(rc.names)
    s = rc.names.index(name)
    lm = rc.lmax
    lmax = int(lm[s]) if isinstance(lm, np.ndarray) else int(lm[s].item())
    dev = rc.values.device if isinstance(rc.values, torch.Tensor) else torch.device("cuda")
    vals = rc.values if isinstance(rc.values, torch.Tensor) else torch.from_numpy(np.asarray(rc.values)).to(dev)
    bo = rc.bag_off if isinstance(rc.bag_off, torch.Tensor) else torch.from_numpy(np.asarray(rc.bag_off)).to(dev)
    bo = bo.long()
    starts, ends = bo[s:-1:S][:B], bo[s + 1::S][:B]
    if lmax == 0:
        return torch.zeros((B, 1), dtype=torch.int64, device=dev)
    idx = starts[:, None] + torch.arange(lmax, device=dev)[None, :]
    ok = idx < ends[:, None]
    n = max(int(vals.numel()), 1)
    src = vals.long() if vals.numel() else torch.zeros(1, dtype=torch.int64, device=dev)
    return torch.where(ok, src[idx.clamp(max=n - 1)], torch.zeros((), dtype=torch.int64, device=dev))


class ConfTwoTower(torch.nn.Module):
    TOWERS = ("user", "ad")

    def __init__(self, conf, layers=None, units=(64, 32), token_vocab: int = 21128, token_dim: int = 16,
                 seed: int = 0, device="cuda"):
        super().__init__()
        L.require_gpu()
        self.conf = conf
        self.device = torch.device(device)
        self.layers = layers if layers is not None else get_preprocess_layers(conf, device=device, seed=seed)
        self.token_ops: Dict[str, EmbeddingBag] = {}
        self.parts: Dict[str, List[Tuple[str, str, int]]] = {}  # tower -> [(kind, name, width)]
        self.mlps = {}
        for ti, tower in enumerate(self.TOWERS):
            parts = []
            for f in conf.train_features:
                if f.tower.value != tower:
                    continue
                if f.is_hashing():
                    if f.pooling.value == "null":
                        raise NotImplementedError(f"{f.name}: a 'null' pooled hashing feature has no fixed tower width")
                    parts.append(("hashing", f.name, 2 * self.layers[f.name].output_dim))
                elif f.is_lookup() or f.is_discrete():
                    parts.append(("lookup" if f.is_lookup() else "discrete", f.name, f.embedding_dim))
                elif f.is_token_id():
                    op = EmbeddingBag(token_vocab, token_dim, combiner=f.pooling.value, name=f"token_{f.name}",
                                      seed=seed * 131 + len(self.token_ops) + 1, device=device)
                    self.token_ops[f.name] = op
                    parts.append(("token", f.name, token_dim))
                elif f.is_numeric():
                    parts.append(("numeric", f.name, 1))
            if not parts:
                raise ValueError(f"tower {tower!r} has no working feature")
            self.parts[tower] = parts
            width = sum(p[2] for p in parts)
            self.mlps[tower] = create_mlp(list(units), 0.3, "selu", BatchNormalization(epsilon=1e-6),
                                          name=f"{tower}_dense_tower", in_features=width, dtype=torch.float32,
                                          seed=seed * 7 + ti + 1, device=device)
        self.user_dense, self.ad_dense = self.mlps["user"], self.mlps["ad"]

    # ---- per-tower input -------------------------------------------------------------------------
    def _hashing_block(self, fb, tower: str, names: List[str]) -> Dict[str, torch.Tensor]:
        """{name: [B, 2D]} of the tower's hashing features: ONE fused launch when the batch's bytes slots are
        exactly the tower's hashing features, else the per-feature operators (views of the same table)."""
        enc_key = tower if tower in self.layers.encoders else None
        if enc_key is not None and list(fb.sparse_names) == self.layers.slots[enc_key] == names:
            out = self.layers.encoders[enc_key](fb.sparse)
            D2 = 2 * self.layers.encoders[enc_key].dim
            return {n: out[:, i * D2:(i + 1) * D2] for i, n in enumerate(names)}
        return {n: self.layers[n](fb.sparse.slot(fb.sparse_names.index(n)).to(self.device)) for n in names}

    def tower_input(self, fb, tower: str) -> torch.Tensor:
        """[B, width] fp32: the tower's feature blocks in configuration order."""
        B = fb.batch
        parts = self.parts[tower]
        hashed = self._hashing_block(fb, tower, [n for k, n, _ in parts if k == "hashing"])
        cols = []
        for kind, name, _w in parts:
            if kind == "hashing":
                cols.append(hashed[name].float())
            elif kind == "token":
                cols.append(self.token_ops[name](padded_ids(fb.int_seq, name, B)).float())
            elif kind == "lookup":
                op = self.layers[name]
                if op.kind == 0:
                    cols.append(op(fb.sparse, slot=fb.sparse_names.index(name)).float())
                else:
                    cols.append(op(fb.int_seq, slot=fb.int_seq.names.index(name)).float())
            elif kind == "discrete":
                op = self.layers[name]
                cols.append(op(fb.float_seq, slot=fb.float_seq.names.index(name)).float())
            else:
                col = fb.scalar(name)
                col = col if isinstance(col, torch.Tensor) else torch.from_numpy(np.asarray(col))
                cols.append(col.to(self.device, torch.float32).reshape(B, 1))
        return torch.cat(cols, dim=1).contiguous()

    def embed(self, fb):
        u = self.user_dense(self.tower_input(fb, "user"))
        v = self.ad_dense(self.tower_input(fb, "ad"))
        return torch.nn.functional.normalize(u, dim=-1, eps=1e-6), torch.nn.functional.normalize(v, dim=-1, eps=1e-6)

    def forward(self, fb) -> torch.Tensor:
        u, v = self.embed(fb)
        return (u * v).sum(dim=-1)
