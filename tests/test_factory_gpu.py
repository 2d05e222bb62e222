"""The drop-in factory get_preprocess_layers (backend/utils/preprocess_utils.py:7-47) on the GPU.

Checks, for the reference's own configs (tests/golden/conf):
* the returned dict has one operator per working hashing/lookup/discrete/bert feature, in the reference's
  feature order (preprocess_utils.py:9), and a DoubleHashingEmbedding for each hashing feature;
* the hashing features of each tower share one fused encoder, slots in config order;
* every fused tower output equals the C oracle bit for bit, and every per-feature DoubleHashingEmbedding
  (a view into the tower's table at its row_base) equals the oracle for that feature AND its column slice
  of the fused output, bit for bit;
* a tower whose features mix embedding dims gets one fused encoder per dim (the reference builds one
  layer per feature, so mixed dims are legal there).
"""
import os

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu
CONF = os.path.join(os.path.dirname(__file__), "golden", "conf")


def _expected_names(conf):
    return [f.name for f in conf.train_features if f.is_hashing() or f.is_lookup() or f.is_discrete()
            or f.is_bert_encode()]


def _check_tower(layers, conf, key, B, seed):
    from recommendflow_amd.backend.layers.preprocess_layers import DoubleHashingEmbedding
    from recommendflow_amd.runtime.batch import synthetic_batch

    enc = layers.encoders[key]
    feats = {f.name: f for f in conf.train_features}
    names = layers.slots[key]
    # multivalued comes from the slot map (base_recall_sdpa); configs without one alternate single/multi
    multi = [bool(feats[n].multivalued) if feats[n].multivalued is not None else s % 2 == 1 for s, n in enumerate(names)]
    hb = synthetic_batch(B, multi, seed=seed)
    fused = enc(hb.to("cuda")).cpu().numpy()
    table = enc.table.cpu().numpy()
    want, _ = O.fused_hash_embed(enc.host_desc, hb.tok_bytes, hb.tok_off, hb.bag_off, hb.lmax, B, table, enc.dim,
                                 enc.out_width)
    np.testing.assert_array_equal(fused.view(np.uint32), want.view(np.uint32))
    D2 = 2 * enc.dim
    for s, n in enumerate(names):
        op = layers[n]
        assert isinstance(op, DoubleHashingEmbedding)
        assert op.table.data_ptr() == enc.table.data_ptr() and op.row_base == int(enc.host_desc[s]["row_base"][0])
        sb = hb.slot(s)
        got = op(sb).cpu().numpy()
        np.testing.assert_array_equal(got.view(np.uint32), fused[:, s * D2:(s + 1) * D2].view(np.uint32), err_msg=n)
        one = enc.host_desc[s:s + 1].copy()
        one[0]["out_off"] = 0
        ref1, _ = O.fused_hash_embed(one, sb.tok_bytes, sb.tok_off, sb.bag_off, sb.lmax, B, table, enc.dim, D2)
        np.testing.assert_array_equal(got.view(np.uint32), ref1.view(np.uint32), err_msg=n)


def test_factory_base_recall_sdpa(cuda):
    from recommendflow_amd.backend.utils.preprocess_utils import get_preprocess_layers
    from recommendflow_amd.config_parser.configuration import Configuration

    conf = Configuration(os.path.join(CONF, "base_recall_sdpa.yaml"))
    layers = get_preprocess_layers(conf)
    assert list(layers.keys()) == _expected_names(conf)
    hashing = [f for f in conf.train_features if f.is_hashing()]
    assert set(layers.encoders) == {"user", "ad"}
    for tower in ("user", "ad"):
        assert layers.slots[tower] == [f.name for f in hashing if f.tower.value == tower]
        enc = layers.encoders[tower]
        assert enc.dim == 8 and all(s.num_bins == 100000 for s in enc.slots)
        assert all(tuple(s.seeds) == (2022, 2023) for s in enc.slots)
    assert len(layers.slots["user"]) + len(layers.slots["ad"]) == len(hashing) == 229
    _check_tower(layers, conf, "user", 384, 31)
    _check_tower(layers, conf, "ad", 384, 32)


def test_factory_base_conf(cuda):
    from recommendflow_amd.backend.utils.preprocess_utils import get_preprocess_layers
    from recommendflow_amd.config_parser.configuration import Configuration

    conf = Configuration(os.path.join(CONF, "base_conf.yaml"))
    layers = get_preprocess_layers(conf)
    assert list(layers.keys()) == ["app_id"] == _expected_names(conf)
    assert layers.slots == {"ad": ["app_id"]}
    op = layers["app_id"]
    assert (op.num_bins, op.output_dim, op.combiner, op.seeds) == (3000, 16, "sum", [2022, 2023])
    _check_tower(layers, conf, "ad", 300, 33)


def test_factory_mixed_dim_tower(cuda, tmp_path):
    """A tower with 16- and 8-dim hashing features: one fused encoder per dim ("user:8", "user:16")."""
    from recommendflow_amd.backend.utils.preprocess_utils import get_preprocess_layers
    from recommendflow_amd.config_parser.configuration import Configuration

    text = open(os.path.join(CONF, "base_conf.yaml")).read()
    text = text.replace("query_nlp_token,str,user,hashing,5000,16,sum,false", "query_nlp_token,str,user,hashing,5000,8,sum,true")
    text = text.replace("clk_app_ids,str,user,hashing,3000,16,sum,false", "clk_app_ids,str,user,hashing,3000,16,max,true")
    text = text.replace("clk_app_kws,str,user,hashing,5000,16,sum,false", "clk_app_kws,str,user,hashing,5000,8,avg,true")
    p = tmp_path / "mixed.yaml"
    p.write_text(text)
    conf = Configuration(str(p))
    layers = get_preprocess_layers(conf)
    assert list(layers.keys()) == _expected_names(conf)
    assert layers.slots["user:8"] == ["query_2gram", "query_3gram", "query_token", "clk_app_kws"]
    assert layers.slots["user:16"] == ["clk_app_ids"]
    assert layers.slots["ad"] == ["app_id"]
    for key in ("user:8", "user:16", "ad"):
        _check_tower(layers, conf, key, 200, hash(key) % 1000)
