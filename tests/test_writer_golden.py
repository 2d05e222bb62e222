"""The TSV -> TFRecord writer (recommendflow_amd.utils.make_tfrecord) against the REFERENCE's own writer path run on
the same committed TSV (tests/golden/make_writer_golden.py: the reference's read_csv and
build_tfrecord / _build_*_feature with a recording tf.train stand-in; fixture tests/golden/writer/writer_golden.json).
Pins row SURVEY §8 a.2 (missing -> "-1" -> b"", split on ",") and f.2's writer by reference output. CPU only: the
Example encoding and the TFRecord reader are librf.so's host code."""
import json
import os

import numpy as np
import pytest

from recommendflow_amd.config_parser.configuration import Configuration
from recommendflow_amd.runtime import tfrecord as T
from recommendflow_amd.utils import make_tfrecord as W

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "writer")
GOLD = json.load(open(os.path.join(HERE, "writer_golden.json")))
CONF = os.path.join(HERE, "writer_conf.yaml")
TSV = os.path.join(HERE, "writer_input.tsv")


def _want(r):
    return {f["feature"]: f for f in r["features"]}


def test_read_csv_matches_reference():
    df = W.read_csv(TSV, sep="\t")
    assert len(df) == len(GOLD["rows"])
    for (_, row), g in zip(df.iterrows(), GOLD["rows"]):
        assert {k: str(v) for k, v in row.items()} == g["tsv_row"]


def test_example_values_match_reference():
    conf = Configuration(CONF)
    df = W.read_csv(TSV, sep="\t")
    for (_, row), g in zip(df.iterrows(), GOLD["rows"]):
        got = W.build_tfrecord(row, conf)
        want = _want(g)
        assert list(got) == [f["feature"] for f in g["features"]]  # same features, same order
        for name, w in want.items():
            v = got[name]
            if w["kind"] == "bytes":
                assert [t.decode() for t in v] == w["values"], name
            elif w["kind"] == "int64":
                assert v == w["values"], name
            else:  # FloatList stores float32
                assert np.array_equal(np.float32(v), np.float32(w["values"])), name


@pytest.mark.parametrize("compression", ["GZIP", None])
def test_written_file_reads_back_as_reference_values(tmp_path, compression):
    """dump_tfrecord_data through librf's Example encoder and TFRecord writer, then librf's reader with the
    feature description (dataloader.py:23-44): every value as the reference writer produced it (numeric features are
    FixedLenFeature scalars: their one value)."""
    conf = Configuration(CONF)
    p = str(tmp_path / "w.tfr")
    assert W.dump_tfrecord_data(TSV, p, conf, compression_type=compression) == len(GOLD["rows"])
    specs = T.build_feature_description(conf)
    fb = next(iter(T.TFRecordReader(p, specs, 64, thread_num=1, compression_type=compression)))
    assert fb.batch == len(GOLD["rows"])
    for s in specs:
        want = [_want(g)[s.name] for g in GOLD["rows"]]
        if s.kind == T.BYTES:
            assert [[t.decode() for t in row] for row in fb.tokens(s.name)] == [w["values"] for w in want], s.name
        elif s.shape == T.SCALAR:
            got = fb.scalar(s.name).tolist()
            assert np.array_equal(np.float32(got), np.float32([w["values"][0] for w in want])), s.name
        else:
            rc = fb.int_seq if s.kind == T.INT64 else fb.float_seq
            i, S = rc.names.index(s.name), len(rc.names)
            vals, bo = np.asarray(rc.values), np.asarray(rc.bag_off)
            got = [vals[bo[b * S + i]: bo[b * S + i + 1]].tolist() for b in range(fb.batch)]
            if s.kind == T.INT64:
                assert got == [w["values"] for w in want], s.name
            else:
                assert all(np.array_equal(np.float32(a), np.float32(w["values"])) for a, w in zip(got, want)), s.name
