"""cfg1 end to end (BASELINE.json configs[0]: demo_conf.yaml two-tower matching, tiny synthetic TFRecord).

Path under test, as the reference runs it:
  conf/demo_conf.yaml -> Configuration (config_parser/configuration.py:25-45; D-cls: pooling cls = first)
  -> synthetic rows of its working features written as GZIP TFRecord Examples by the build's writer
     (utils/make_tfrecord.py:26-41,139-144: "-1" -> b"", GZIP)
  -> FeaturePipe(parse host | device) (backend/core/dataloader.py:23-44,541-578)
  -> get_preprocess_layers operators (backend/utils/preprocess_utils.py:7-47) + a two-tower scorer
     (models/matching/dssm.py:25-36; models/matching/two_tower.py for the wiring and deviations).

Synthetic input: 256 examples; app_id tokens "app{id}" with id ~ Zipf(1.1) over 5,000 (5 %
missing -> "-1" -> b""); query/app_name token and segment ids: int lists of length 8 (tokens ~ U[1, 21128),
segments in {0, 1}); label ~ Bernoulli(0.1); down ~ U(0, 1).

Bars: app_id's pooled [B, 32] bit-exact vs oracle.fused_hash_embed on the written CSR; token-id blocks
bit-exact vs oracle.embedding_bag; score vs float64 (oracle.mlp BN/selu, l2_normalize) at rtol 1e-4;
labels and every other column round-trip exactly.
"""
import os

import numpy as np
import pytest
import torch

from recommendflow_amd.config_parser.configuration import Configuration
from recommendflow_amd.runtime import tfrecord as T
from model_helpers import mlp_params

pytestmark = pytest.mark.gpu
CONF = os.path.join(os.path.dirname(__file__), "golden", "conf", "demo_conf.yaml")
N_EX, BS = 256, 128


def cfg1_rows(n=N_EX, seed=1234):
    from recommendflow_amd.runtime.batch import synthetic_demo_rows

    return synthetic_demo_rows(n, seed)


def write_cfg1(path, conf, rows):
    specs = T.build_feature_description(conf)
    fb = T.columns_from_rows(specs, rows)
    data, off = T.encode_examples(specs, fb)
    with T.TFRecordWriter(str(path), "GZIP") as w:
        w.write_many(data, off)
    return specs


def _randomize_bn(model, seed):
    g = torch.Generator().manual_seed(seed)
    for m in (model.user_dense, model.ad_dense):
        for nm in m.norms:
            w = nm.width
            nm.gamma.copy_(torch.rand(w, generator=g) + 0.5)
            nm.beta.copy_(torch.rand(w, generator=g) * 0.2 - 0.1)
            nm.mean.copy_(torch.rand(w, generator=g) * 0.1 - 0.05)
            nm.var.copy_(torch.rand(w, generator=g) + 0.5)


def _oracle_scores(O, model, conf, rows):
    specs = T.build_feature_description(conf)
    hfb = T.columns_from_rows(specs, rows)
    B = len(rows)
    blocks = {}
    enc = model.layers.encoders["ad"]
    sb = hfb.sparse
    app, _ = O.fused_hash_embed(enc.host_desc, sb.tok_bytes, sb.tok_off, sb.bag_off, sb.lmax, B,
                                enc.table.cpu().numpy(), enc.dim, enc.out_width)
    blocks["app_id"] = app
    for name, op in model.token_ops.items():
        ids = hfb.int_seq.dense(name, 0)
        blocks[name] = O.embedding_bag(ids, op.table.cpu().numpy(), op.combiner)
    towers = {}
    for tower in model.TOWERS:
        x = np.concatenate([blocks[n] if k != "numeric" else hfb.scalar(n).reshape(B, 1)
                            for k, n, _w in model.parts[tower]], axis=1)
        towers[tower] = O.l2_normalize(O.mlp(x, mlp_params(model.mlps[tower]), "selu", "bn"))
    return (towers["user"] * towers["ad"]).sum(1), blocks


@pytest.mark.parametrize("parse", ["host", "device"])
def test_cfg1_tfrecord_two_tower(O, cuda, tmp_path, parse):
    from recommendflow_amd.models.matching.two_tower import ConfTwoTower

    conf = Configuration(CONF)
    rows = cfg1_rows()
    path = tmp_path / "demo-part-0.tfrecord.gz"
    specs = write_cfg1(path, conf, rows)
    with open(path, "rb") as f:
        assert f.read(2) == b"\x1f\x8b"  # GZIP (make_tfrecord.py:142)
    model = ConfTwoTower(conf, seed=3)
    _randomize_bn(model, 9)
    assert [n for _k, n, _w in model.parts["user"]] == ["query_tok_id", "query_seg_id"]
    assert [n for _k, n, _w in model.parts["ad"]] == ["app_name_tok_id", "app_name_seg_id", "app_id"]
    pipe = T.FeaturePipe([str(path)], specs, BS, thread_num=2, compression_type="GZIP", parse=parse)
    seen = 0
    for fb in pipe:
        chunk = rows[seen:seen + fb.batch]
        want, blocks = _oracle_scores(O, model, conf, chunk)
        got_ad = model.tower_input(fb, "ad").cpu().numpy()
        got_user = model.tower_input(fb, "user").cpu().numpy()
        np.testing.assert_array_equal(got_ad[:, 32:64].view(np.uint32), blocks["app_id"].view(np.uint32))
        np.testing.assert_array_equal(got_ad[:, :16].view(np.uint32), blocks["app_name_tok_id"].view(np.uint32))
        np.testing.assert_array_equal(got_user[:, 16:32].view(np.uint32), blocks["query_seg_id"].view(np.uint32))
        score = model(fb).cpu().numpy()
        np.testing.assert_allclose(score, want, rtol=1e-4, atol=1e-6)
        labels = fb.labels(conf.features.label_names)["label"].cpu().numpy()
        assert labels.tolist() == [r["label"] for r in chunk]
        assert fb.scalar("down").cpu().numpy().tolist() == [r["down"] for r in chunk]
        assert fb.tokens("app_id") == [[r["app_id"][0].encode()] for r in chunk]
        seen += fb.batch
    assert seen == N_EX
    pipe.close()
