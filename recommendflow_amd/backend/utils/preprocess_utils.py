"""Operator factory — the drop-in boundary (reference: backend/utils/preprocess_utils.py:7-47).

``get_preprocess_layers(conf)`` returns {feature name: operator} for every working feature, exactly as
the reference does (hashing -> DoubleHashingEmbedding(mask_value="", mask_zero=True), lookup ->
LookupEmbedding, discrete -> DiscreteEmbedding, bert_encode -> BertEncode, other deals -> nothing).

MI355X addition: the hashing features of each tower share ONE fused table and ONE fused encoder
(``layers.encoders[tower]``) so a model runs a whole tower in one kernel launch; the per-feature
DoubleHashingEmbedding entries are views into that table (same rows, same results). A tower whose
hashing features mix embedding dims gets one fused encoder per dim, keyed ``"tower:dim"``.
"""
from __future__ import annotations

from typing import Dict, List

import torch

from ...config_parser.configuration import Configuration
from ..encoder.sparse_encoder import FusedSparseEncoder, SlotSpec, normalize_seeds
from ..layers.preprocess_layers import BertEncode, DiscreteEmbedding, DoubleHashingEmbedding, LookupEmbedding


class PreprocessLayers(dict):
    """dict name -> operator, plus ``encoders`` (tower, or "tower:dim" for a mixed-dim tower -> FusedSparseEncoder)
    and ``slots`` (same key -> feature names in the tower's column order)."""

    def __init__(self):
        super().__init__()
        self.encoders: Dict[str, FusedSparseEncoder] = {}
        self.slots: Dict[str, List[str]] = {}


def get_preprocess_layers(conf: Configuration, table_dtype=torch.float32, out_dtype=None, device="cuda", seed: int = 0,
                          fused: bool = True, mask_padding: bool = False, dim_override: int = None,
                          num_bins_override=None) -> PreprocessLayers:
    layers = PreprocessLayers()
    built = {}
    hashing = [f for f in conf.train_features if f.is_hashing()]
    groups: Dict[str, list] = {}
    for f in hashing:
        if fused and f.pooling.value != "null":
            groups.setdefault(f.tower.value, []).append(f)
    ti = 0
    for tower, tfeats in groups.items():
        # one fused launch per (tower, embedding_dim): a tower whose features mix dims gets one encoder per
        # dim, keyed "tower:dim" (a single-dim tower keeps the key "tower")
        dims = sorted({dim_override or f.embedding_dim for f in tfeats})
        for dim in dims:
            feats = [f for f in tfeats if (dim_override or f.embedding_dim) == dim]
            key = tower if len(dims) == 1 else f"{tower}:{dim}"
            specs = [SlotSpec(f.name, num_bins_override or f.vocab_size, normalize_seeds(f.hash_seeds), f.pooling.value,
                              True) for f in feats]
            enc = FusedSparseEncoder(specs, dim, table_dtype=table_dtype, out_dtype=out_dtype, seed=seed + 7919 * ti,
                                     mask_padding=mask_padding, device=device)
            ti += 1
            layers.encoders[key] = enc
            layers.slots[key] = [f.name for f in feats]
            for i, f in enumerate(feats):
                built[f.name] = DoubleHashingEmbedding(
                    num_bins=specs[i].num_bins, output_dim=dim, seeds=f.hash_seeds, mask_value="", mask_zero=True,
                    combiner=f.pooling.value, name=f"hashing_{f.name}", dtype=table_dtype, out_dtype=out_dtype,
                    mask_padding=mask_padding, device=device, table=enc.table,
                    row_base=int(enc.host_desc[i]["row_base"][0]))
    for f in conf.train_features:  # reference order (preprocess_utils.py:9)
        if f.name in built:
            layers[f.name] = built[f.name]
        elif f.is_hashing():
            layers[f.name] = DoubleHashingEmbedding(
                num_bins=num_bins_override or f.vocab_size, output_dim=dim_override or f.embedding_dim,
                seeds=f.hash_seeds, mask_value="", mask_zero=True, combiner=f.pooling.value, name=f"hashing_{f.name}",
                dtype=table_dtype, out_dtype=out_dtype, mask_padding=mask_padding, device=device)
        elif f.is_lookup():
            layers[f.name] = LookupEmbedding(embedding_dim=f.embedding_dim, dtype=f.type, vocabs=f.vocabs,
                                             vocab_size=f.vocab_size, pooling=f.pooling.value, name=f"lookup_{f.name}",
                                             device=device, table_dtype=table_dtype)
        elif f.is_discrete():
            layers[f.name] = DiscreteEmbedding(embedding_dim=f.embedding_dim, vocabs=f.vocabs, vocab_size=f.vocab_size,
                                               pooling=f.pooling.value, name=f"discrete_{f.name}", device=device,
                                               table_dtype=table_dtype)
        elif f.is_bert_encode():
            layers[f.name] = BertEncode(dict_path=f.vocabs, name=f"bert_encode_{f.name}")
    return layers
