"""cfg1 plumbing on the CPU (BASELINE.json configs[0]): demo_conf.yaml's working features written as a GZIP
TFRecord by the build's writer (utils/make_tfrecord.py:26-41,142) and read back by the C++ reader
(backend/core/dataloader.py:23-44,541-578, host parse): every column round-trips, the app_id tokens hash
to the oracle's bins, and the padded token-id view matches the written lists. The GPU half (FeaturePipe
into the two-tower scorer) is tests/test_cfg1_gpu.py."""
import os

import numpy as np

from recommendflow_amd.config_parser.configuration import Configuration
from recommendflow_amd.runtime import tfrecord as T
from test_cfg1_gpu import CONF, cfg1_rows, write_cfg1


def test_cfg1_gzip_roundtrip(O, tmp_path):
    conf = Configuration(CONF)
    rows = cfg1_rows()
    path = tmp_path / "demo.tfrecord.gz"
    specs = write_cfg1(path, conf, rows)
    assert [s.name for s in specs] == ["query_tok_id", "query_seg_id", "app_name_tok_id", "app_name_seg_id",
                                       "app_id", "label", "down"]
    seen = 0
    for fb in T.TFRecordReader([str(path)], specs, 100, thread_num=2, compression_type="GZIP"):
        chunk = rows[seen:seen + fb.batch]
        for n in ("query_tok_id", "query_seg_id", "app_name_tok_id", "app_name_seg_id"):
            assert fb.int_seq.dense(n).tolist() == [r[n] for r in chunk]
        assert fb.tokens("app_id") == [[r["app_id"][0].encode()] for r in chunk]
        assert fb.scalar("label").tolist() == [r["label"] for r in chunk]
        assert fb.scalar("down").tolist() == [r["down"] for r in chunk]
        sb = fb.sparse
        bins = O.hash_tokens(sb.tok_bytes, sb.tok_off, 2022, 2022, 3000, True)
        want = [0 if r["app_id"][0] == "" else O.hash_bucket(r["app_id"][0].encode(), 3000, 2022) for r in chunk]
        assert bins.tolist() == want
        assert (bins[[r["app_id"][0] == "" for r in chunk]] == 0).all()
        seen += fb.batch
    assert seen == len(rows)
    assert os.path.getsize(path) < 64 * len(rows)  # compressed
