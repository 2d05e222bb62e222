"""GPU: tf.train.Example parsing on the device (rf_tfr_parse_device, runtime/tfrecord.DeviceParser) gives
the same columns, byte for byte, as the host reader's C++ parse (rf_tfr_next_batch) on the same records —
which test_tfrecord.py pins against Google's protobuf library and oracle/tfrecord_oracle.py — and the
same errors with the same messages. Also the FeaturePipe(parse="device") path into the fused encoder."""
import numpy as np
import pytest
import torch

from oracle import tfrecord_oracle as TO
from recommendflow_amd.runtime import tfrecord as T
from recommendflow_amd.runtime.batch import synthetic_batch
from tests import tf_example_pb as PB
from tests.test_tfrecord import SPECS, pb_record, random_rows

pytestmark = pytest.mark.gpu

COLS = ["tok_bytes", "tok_off", "bag_off", "lmax", "ival", "ibag_off", "ilmax", "fval", "fbag_off", "flmax",
        "iscalar", "fscalar"]


def _host_batches(paths, specs, B, compression):
    rd = T.TFRecordReader(paths, specs, B, thread_num=3, compression_type=compression)
    cols, out = rd.new_columns(), []
    while True:
        r = rd.read_into(cols)
        if r is None:
            break
        cols, c = r
        out.append({k: np.array(v) for k, v in cols.views(c).items()})
    rd.close()
    return out


def _device_batches(paths, specs, B, compression, slack=64):
    """read_records (host half) -> H2D -> DeviceParser, synchronously."""
    rd = T.TFRecordReader(paths, specs, B, thread_num=3, compression_type=compression)
    P = T.DeviceParser(specs, "cuda")
    buf, off = np.empty(1024, np.uint8), np.empty(B + 1, np.int64)
    out = []
    s = torch.cuda.current_stream()
    while True:
        buf, n, nb = rd.read_records(buf, off)
        if n == 0:
            break
        first = rd.records_read - n
        rec = torch.zeros(nb + slack, dtype=torch.uint8, device="cuda")
        rec[:nb] = torch.from_numpy(buf[:nb].copy()).cuda()
        offd = torch.from_numpy(off[: n + 1].copy()).cuda()
        bufs, small = P.parse(rec, offd, n, nb, int(np.diff(off[: n + 1]).max()), s)
        torch.cuda.synchronize()
        sm = small.cpu().numpy()
        st = P.check(sm, first)
        v = P.views(bufs, st, n)
        d = {k: x.cpu().numpy() for k, x in v.items()}
        if st.n_tok_bytes == 0 and "tok_bytes" in d:
            d["tok_bytes"] = d["tok_bytes"][:0]
        out.append(d)
    rd.close()
    return out


def _assert_same(host, dev):
    assert len(host) == len(dev)
    for h, d in zip(host, dev):
        for k in COLS:
            if k not in d:
                assert h[k].size == 0 or k in ("lmax", "ilmax", "flmax", "bag_off", "ibag_off", "fbag_off"), k
                continue
            a, b = h[k], d[k]
            assert a.shape == b.shape, (k, a.shape, b.shape)
            assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), k


def _write(tmp_path, recs, compression, name="a.tfr"):
    p = str(tmp_path / name)
    TO.write_file(p, recs, compression or "NONE")
    return p


@pytest.mark.parametrize("compression", ["GZIP", None])
@pytest.mark.parametrize("packed", [True, False])
@pytest.mark.parametrize("B", [1, 64, 1000])
def test_device_parse_equals_host_parse(tmp_path, compression, packed, B):
    rows = random_rows(700, 11 + B, missing=0.2)
    recs = [pb_record(r, packed=packed) for r in rows]
    p = _write(tmp_path, recs, compression)
    _assert_same(_host_batches([p], SPECS, B, compression), _device_batches([p], SPECS, B, compression))


def test_device_parse_interleaved_files_and_empty_examples(tmp_path):
    paths = []
    for f, n in enumerate([40, 0, 13, 77]):
        rows = random_rows(n, 100 + f, missing=0.5)
        recs = [pb_record(r) for r in rows] + [b""]  # an empty Example: every key missing
        paths.append(_write(tmp_path, recs, None, f"f{f}"))
    _assert_same(_host_batches(paths, SPECS, 32, None), _device_batches(paths, SPECS, 32, None))


def test_device_parse_duplicates_kindless_unknown_keys(tmp_path):
    e1 = PB.make_example({"tags": ("none", []), "cnt": ("int64", [3]), "zzz": ("bytes", [b"ignored"])})
    e2 = PB.make_example({"cnt": ("int64", [4]), "tags": ("bytes", [b"a"])}) + \
        PB.make_example({"cnt": ("int64", [5]), "tags": ("bytes", [b"b", b"cc"])})  # concatenated = merged, last wins
    e3 = PB.make_example({"tags": ("bytes", [b"x"] * 3)}) + PB.make_example({"tags": ("none", [])})
    p = _write(tmp_path, [e1, e2, e3, e1], None)
    spec = [T.FeatureSpec("tags", T.BYTES, T.SEQ, ""), T.FeatureSpec("cnt", T.INT64, T.SCALAR, -9)]
    h, d = _host_batches([p], spec, 8, None), _device_batches([p], spec, 8, None)
    _assert_same(h, d)
    assert d[0]["iscalar"].tolist() == [3, 5, -9, 3]


def test_device_parse_long_records_from_hbm(tmp_path):
    """Records larger than the LDS staging slot (64 KiB workgroup budget) are parsed from HBM."""
    rows = random_rows(24, 5, missing=0.0)
    for i, r in enumerate(rows):
        if i % 3 == 0:
            r["tags"] = [f"long-token-{k:06d}-" * 4 for k in range(1500 + i)]  # ~ 70-100 KB records
            r["tok"] = list(range(-3000, 3000 + i))
    recs = [pb_record(r, packed=bool(i % 2)) for i, r in enumerate(rows)]
    p = _write(tmp_path, recs, None)
    _assert_same(_host_batches([p], SPECS, 10, None), _device_batches([p], SPECS, 10, None))


def test_device_parse_cfg2_shape(tmp_path):
    from recommendflow_amd.config_parser.configuration import Configuration
    import os

    root = os.path.dirname(os.path.abspath(__file__))
    feats = Configuration(os.path.join(root, "golden", "conf", "base_recall_sdpa.yaml")).features.hashing_features
    specs = [T.FeatureSpec(f.name, T.BYTES, T.SEQ, "") for f in feats] + [T.FeatureSpec("label", T.FLOAT, T.SCALAR, 0.0)]
    B = 2048
    hb = synthetic_batch(B, [bool(f.multivalued) for f in feats], seed=17)
    fb = T.FeatureBatch(B, hb, [f.name for f in feats], None, None, np.zeros((B, 0), np.int64), [],
                        np.arange(B, dtype=np.float32).reshape(B, 1), ["label"])
    data, off = T.encode_examples(specs, fb)
    p = str(tmp_path / "cfg2.tfr")
    with T.TFRecordWriter(p, None) as w:
        w.write_many(data, off)
    d = _device_batches([p], specs, B, None)
    _assert_same(_host_batches([p], specs, B, None), d)
    assert np.array_equal(d[0]["bag_off"], hb.bag_off) and np.array_equal(d[0]["tok_off"], hb.tok_off)
    assert np.array_equal(d[0]["tok_bytes"], hb.tok_bytes) and np.array_equal(d[0]["lmax"], hb.lmax)


def _errors(tmp_path, recs, spec, B=4):
    """(host message, device message) for the same records."""
    p = _write(tmp_path, recs, None, "err")
    msgs = []
    for fn in (_host_batches, _device_batches):
        with pytest.raises(T.DataLossError) as ei:
            fn([p], spec, B, None)
        msgs.append(str(ei.value))
    return msgs


def test_device_parse_errors_match_host(tmp_path):
    spec = [T.FeatureSpec("tags", T.BYTES, T.SEQ, ""), T.FeatureSpec("cnt", T.INT64, T.SCALAR, 0),
            T.FeatureSpec("f", T.FLOAT, T.SEQ, 0.0)]
    good = PB.make_example({"cnt": ("int64", [1]), "tags": ("bytes", [b"q"])})
    cases = [
        [good, PB.make_example({"cnt": ("float", [1.0])})],                              # kind mismatch
        [good, good, PB.make_example({"cnt": ("int64", [1, 2])})],                       # SCALAR with 2 values
        [good, PB.make_example({"tags": ("bytes", [b"a"])})] + [good],                   # SCALAR missing: default, fine
        [b"\x0a\xff\xff", good],                                                         # malformed Example
        [good, PB.make_example({"cnt": ("int64", [1]), "f": ("float", [1.0])})[:-2] + b"\x15\x00", good],
        [good, PB.make_example({"cnt": ("int64", [2]), "tags": ("int64", [5])}),         # two bad records:
         PB.make_example({"cnt": ("float", [2.0])})],                                    # the first is reported
        [PB.make_example({"cnt": ("int64", [1, 1]), "tags": ("float", [1.0])})],         # first key in schema order
    ]
    for recs in cases:
        p = _write(tmp_path, recs, None, "err")
        try:
            _host_batches([p], spec, 4, None)
        except T.DataLossError as e:
            host = str(e)
        else:
            _assert_same(_host_batches([p], spec, 4, None), _device_batches([p], spec, 4, None))
            continue
        with pytest.raises(T.DataLossError) as ei:
            _device_batches([p], spec, 4, None)
        assert str(ei.value) == host


def test_device_parse_errors_report_record_numbers_across_batches(tmp_path):
    spec = [T.FeatureSpec("cnt", T.INT64, T.SCALAR, 0)]
    recs = [PB.make_example({"cnt": ("int64", [i])}) for i in range(10)] + [PB.make_example({"cnt": ("int64", [])})]
    h, d = _errors(tmp_path, recs, spec, B=4)
    assert h == d and "record 10" in d


@pytest.mark.parametrize("compression", ["GZIP", None])
def test_pipe_device_parse_feeds_encoder(O, cuda, tmp_path, compression):
    from recommendflow_amd.backend.encoder.sparse_encoder import FusedSparseEncoder, SlotSpec

    S, B, D = 12, 700, 16
    multi = [s % 3 == 0 for s in range(S)]
    specs = [T.FeatureSpec(f"f{s}", T.BYTES, T.SEQ, "") for s in range(S)] + [T.FeatureSpec("label", T.FLOAT, T.SCALAR, 0.0)]
    slots = [SlotSpec(f"f{s}", 2000 + 31 * s, (2022, 2023), ["sum", "avg", "max", "min"][s % 4]) for s in range(S)]
    enc = FusedSparseEncoder(slots, D, seed=5)
    hb = synthetic_batch(B, multi, seed=21)
    fb = T.FeatureBatch(B, hb, [s.name for s in specs[:S]], None, None, np.zeros((B, 0), np.int64), [],
                        np.arange(B, dtype=np.float32).reshape(B, 1), ["label"])
    data, off = T.encode_examples(specs, fb)
    paths = []
    for f in range(3):
        p = str(tmp_path / f"part-{f}.tfr")
        with T.TFRecordWriter(p, compression) as w:
            lo, hi = f * 250, min(B, (f + 1) * 250)
            w.write_many(data, off[lo:hi + 1])
        paths.append(p)
    host = T.FeaturePipe(paths, specs, 128, thread_num=3, compression_type=compression, prefetch=2)
    devp = T.FeaturePipe(paths, specs, 128, thread_num=3, compression_type=compression, prefetch=2, parse="device")
    n = 0
    for a, b in zip(host, devp):
        assert a.batch == b.batch
        for x, y in ((a.sparse.tok_bytes, b.sparse.tok_bytes), (a.sparse.tok_off, b.sparse.tok_off),
                     (a.sparse.bag_off, b.sparse.bag_off), (a.sparse.lmax, b.sparse.lmax)):
            assert torch.equal(x, y)
        assert np.array_equal(a.sparse.host_lmax, b.sparse.host_lmax)
        assert torch.equal(a.scalar("label"), b.scalar("label"))
        ya, yb = enc(a.sparse), enc(b.sparse)
        assert torch.equal(ya.view(torch.int32), yb.view(torch.int32))
        n += b.batch
    assert n == B
    host.close()
    devp.close()
