"""TFRecord(GZIP) <-> batched-CSR pipe (include/rf_io.h, runtime/tfrecord.py) — CPU, no GPU.

Pins: CRC-32C check vectors (RFC 3720 §B.4 + "123456789"); Google's protobuf library as an
independent tf.train.Example encoder/decoder (tests/tf_example_pb.py); the Python restatement in
oracle/tfrecord_oracle.py for framing, parse_example semantics and the interleave order.
"""
import gzip
import os
import struct

import numpy as np
import pytest

from oracle import tfrecord_oracle as TO
from recommendflow_amd.runtime import tfrecord as T
from recommendflow_amd.runtime.batch import synthetic_batch
from tests import tf_example_pb as PB

CRC_VECTORS = [  # RFC 3720 §B.4 (iSCSI CRC-32C examples) and the standard check value
    (bytes(32), 0x8A9136AA),
    (bytes([0xFF] * 32), 0x62A8AB43),
    (bytes(range(32)), 0x46DD794E),
    (bytes(range(31, -1, -1)), 0x113FDB5C),
    (b"123456789", 0xE3069283),
    (b"", 0x0),
]


@pytest.mark.parametrize("data,want", CRC_VECTORS)
def test_crc32c_vectors(data, want):
    assert T.crc32c(data) == want
    assert TO.crc32c(data) == want


def test_crc32c_long_and_incremental():
    rng = np.random.default_rng(0)
    for n in (1, 7, 8, 9, 63, 64, 65, 1000, 4099):
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        want = TO.crc32c(d)
        assert T.crc32c(d) == want
        k = n // 3
        assert T.crc32c(d[k:], T.crc32c(d[:k])) == want
        assert T.masked_crc32c(d) == TO.masked_crc32c(d)


SPECS = [
    T.FeatureSpec("app_id", T.BYTES, T.SEQ, ""),
    T.FeatureSpec("tags", T.BYTES, T.SEQ, ""),
    T.FeatureSpec("tok", T.INT64, T.SEQ, 0),
    T.FeatureSpec("disc", T.FLOAT, T.SEQ, 0.0),
    T.FeatureSpec("label", T.FLOAT, T.SCALAR, 0.0),
    T.FeatureSpec("cnt", T.INT64, T.SCALAR, 7),
    T.FeatureSpec("sc", T.BYTES, T.SCALAR, ""),
]
PB_KIND = {T.BYTES: "bytes", T.INT64: "int64", T.FLOAT: "float"}


def random_rows(n, seed, missing=0.15):
    rng = np.random.default_rng(seed)
    rows = []
    for _ in range(n):
        r = {}
        if rng.random() > missing:
            r["app_id"] = [f"app{int(rng.integers(0, 5000))}"]
        if rng.random() > missing:
            r["tags"] = [("" if rng.random() < 0.1 else f"t{int(rng.integers(0, 99))}") for _ in range(int(rng.integers(0, 9)))]
        if rng.random() > missing:
            r["tok"] = [int(x) for x in rng.integers(-(1 << 40), 1 << 40, int(rng.integers(0, 12)))]
        if rng.random() > missing:
            r["disc"] = [float(np.float32(x)) for x in rng.normal(size=int(rng.integers(0, 5)))]
        if rng.random() > missing:
            r["label"] = float(np.float32(rng.random()))
        if rng.random() > missing:
            r["cnt"] = int(rng.integers(-5, 1 << 62))
        if rng.random() > missing:
            r["sc"] = "x" * int(rng.integers(0, 4))
        rows.append(r)
    return rows


def pb_record(row, packed=True):
    vals = {}
    for s in SPECS:
        if s.name in row:
            v = row[s.name]
            vals[s.name] = (PB_KIND[s.kind], v if isinstance(v, list) else [v])
    return PB.make_example(vals, packed=packed)


def expected(rows):
    return TO.parse_examples([pb_record(r) for r in rows], SPECS)


def check_batch(fb, want, lo, hi):
    B = hi - lo
    assert fb.batch == B
    for s in SPECS:
        w = want[s.name][lo:hi]
        if s.kind == T.BYTES:
            got = fb.tokens(s.name)
            if s.shape == T.SCALAR:
                w = [[x] for x in w]
            assert got == [[x if isinstance(x, bytes) else x.encode() for x in e] for e in w], s.name
            k = fb.sparse_names.index(s.name)
            assert int(fb.sparse.lmax[k]) == max([len(e) for e in w] or [0])
        elif s.shape == T.SEQ:
            rc = fb.int_seq if s.kind == T.INT64 else fb.float_seq
            k = rc.names.index(s.name)
            S = len(rc.names)
            got = [list(rc.values[rc.bag_off[b * S + k]:rc.bag_off[b * S + k + 1]]) for b in range(B)]
            if s.kind == T.FLOAT:
                assert [np.float32(x).tolist() for e in got for x in e] == [np.float32(x).tolist() for e in w for x in e]
                assert [len(e) for e in got] == [len(e) for e in w]
            else:
                assert got == w, s.name
            assert int(rc.lmax[k]) == max([len(e) for e in w] or [0])
            dense = rc.dense(s.name)
            assert dense.shape == (B, int(rc.lmax[k]))
        else:
            got = fb.scalar(s.name).tolist()
            if s.kind == T.FLOAT:
                assert np.array_equal(np.float32(got), np.float32(w)), s.name
            else:
                assert got == w, s.name


def test_encoder_matches_protobuf():
    rows = random_rows(200, 1)
    fb = T.columns_from_rows(SPECS, rows)
    data, off = T.encode_examples(SPECS, fb)
    assert len(off) == 201
    for i, r in enumerate(rows):
        mine = PB.parse_example(bytes(data[off[i]:off[i + 1]]))
        ref = PB.parse_example(pb_record(r))
        for s in SPECS:
            mk, mv = mine[s.name]
            if s.name in ref:
                rk, rv = ref[s.name]
                assert mv == rv and (mk == rk or not rv), (s.name, mine[s.name], ref[s.name])
            else:  # missing key: the encoder writes an empty list (SEQ) or the default (SCALAR)
                assert (mv == []) if s.shape == T.SEQ else len(mv) == 1


@pytest.mark.parametrize("compression", ["GZIP", None])
@pytest.mark.parametrize("packed", [True, False])
def test_reader_matches_oracle(tmp_path, compression, packed):
    rows = random_rows(300, 2)
    recs = [pb_record(r, packed=packed) for r in rows]
    p = str(tmp_path / "a.tfr")
    TO.write_file(p, recs, compression or "NONE")
    want = TO.parse_examples(recs, SPECS)
    rd = T.TFRecordReader([p], SPECS, 64, thread_num=3, compression_type=compression)
    lo = 0
    for fb in rd:
        check_batch(fb, want, lo, lo + fb.batch)
        lo += fb.batch
    assert lo == 300 and rd.records_read == 300


def test_writer_roundtrip_and_oracle_reads_it(tmp_path):
    rows = random_rows(150, 3)
    fb = T.columns_from_rows(SPECS, rows)
    data, off = T.encode_examples(SPECS, fb)
    p = str(tmp_path / "w.tfrecord.gz")
    with T.TFRecordWriter(p, "GZIP") as w:
        w.write_many(data, off)
    recs = TO.read_file(p, "GZIP")  # the writer's framing + gzip read by Python's gzip and the oracle CRC
    assert recs == [bytes(data[off[i]:off[i + 1]]) for i in range(150)]
    want = TO.parse_examples(recs, SPECS)
    got = list(T.TFRecordReader(p, SPECS, 1000, thread_num=2))
    assert len(got) == 1
    check_batch(got[0], want, 0, 150)


def test_interleave_order(tmp_path):
    counts = [5, 0, 3, 9, 1, 4]
    paths = []
    for f, n in enumerate(counts):
        p = str(tmp_path / f"f{f}.gz")
        TO.write_file(p, [PB.make_example({"cnt": ("int64", [f * 100 + i])}) for i in range(n)])
        paths.append(p)
    spec = [T.FeatureSpec("cnt", T.INT64, T.SCALAR, -1)]
    for threads in (1, 2, 3, 4, 8):
        order = [int(x) for fb in T.TFRecordReader(paths, spec, 4, thread_num=threads) for x in fb.scalar("cnt")]
        want = [f * 100 + i for f, i in TO.interleave_order(counts, threads)]
        assert order == want, threads


def test_drop_remainder_and_small_capacity_growth(tmp_path):
    rows = random_rows(100, 4, missing=0.0)
    for r in rows:  # long lists force the ENOSPC -> grow -> retry path
        r["tags"] = [f"tag-{i:05d}-" * 3 for i in range(40)]
    p = str(tmp_path / "g.gz")
    TO.write_file(p, [pb_record(r) for r in rows])
    want = expected(rows)
    rd = T.TFRecordReader(p, SPECS, 32, thread_num=2, drop_remainder=True)
    rd.caps = {"tok": 8, "tok_bytes": 8, "ival": 1, "fval": 1}
    got = list(rd)
    assert [fb.batch for fb in got] == [32, 32, 32]
    for i, fb in enumerate(got):
        check_batch(fb, want, 32 * i, 32 * i + 32)


def test_errors(tmp_path):
    good = PB.make_example({"cnt": ("int64", [1])})
    blob = TO.frame([good, good])
    # corrupt data crc
    bad = bytearray(blob)
    bad[-1] ^= 1
    p = str(tmp_path / "crc")
    open(p, "wb").write(bytes(bad))
    spec = [T.FeatureSpec("cnt", T.INT64, T.SCALAR, 0)]
    with pytest.raises(T.DataLossError, match="crc"):
        list(T.TFRecordReader(p, spec, 4, compression_type=None))
    # truncated record
    open(p, "wb").write(blob[:-3])
    with pytest.raises(T.DataLossError, match="truncated"):
        list(T.TFRecordReader(p, spec, 4, compression_type=None))
    # truncated gzip stream
    open(p, "wb").write(gzip.compress(blob)[:-12])
    with pytest.raises(T.DataLossError):
        list(T.TFRecordReader(p, spec, 4))
    # type mismatch (parse_example: "Data types don't match")
    TO.write_file(p, [PB.make_example({"cnt": ("float", [1.0])})])
    with pytest.raises(T.DataLossError, match="Data types"):
        list(T.TFRecordReader(p, spec, 4))
    # FixedLenFeature(()) with 2 values
    TO.write_file(p, [PB.make_example({"cnt": ("int64", [1, 2])})])
    with pytest.raises(T.DataLossError, match="Number of values"):
        list(T.TFRecordReader(p, spec, 4))
    # malformed protobuf
    TO.write_file(p, [b"\x0a\xff\xff"])
    with pytest.raises(T.DataLossError, match="malformed"):
        list(T.TFRecordReader(p, spec, 4))
    # missing file
    with pytest.raises(OSError):
        T.TFRecordReader(str(tmp_path / "nope"), spec, 4)


def test_feature_without_kind_and_duplicate_keys(tmp_path):
    # a Feature with no kind set reads as an empty list; a repeated map key: the last entry wins
    C = PB.classes(True)
    e1 = PB.make_example({"tags": ("none", []), "cnt": ("int64", [3])})
    e2 = PB.make_example({"cnt": ("int64", [4])}) + PB.make_example({"cnt": ("int64", [5])})  # concatenated = merged
    p = str(tmp_path / "k.gz")
    TO.write_file(p, [e1, e2])
    spec = [T.FeatureSpec("tags", T.BYTES, T.SEQ, ""), T.FeatureSpec("cnt", T.INT64, T.SCALAR, 0)]
    fb = next(iter(T.TFRecordReader(p, spec, 8)))
    assert fb.tokens("tags") == [[], []]
    assert fb.scalar("cnt").tolist() == [3, 5]
    assert C  # schema classes build


def test_cfg2_synthetic_batch_roundtrip(tmp_path):
    """A cfg2-shaped SparseBatch survives encode -> GZIP file -> parse byte for byte."""
    from recommendflow_amd.config_parser.configuration import Configuration

    root = os.path.dirname(os.path.abspath(__file__))
    conf = Configuration(os.path.join(root, "golden", "conf", "base_recall_sdpa.yaml"))
    feats = conf.features.hashing_features
    specs = [T.FeatureSpec(f.name, T.BYTES, T.SEQ, "") for f in feats]
    hb = synthetic_batch(256, [bool(f.multivalued) for f in feats], seed=9)
    fb = T.FeatureBatch(256, hb, [s.name for s in specs], None, None, np.zeros((256, 0), np.int64), [],
                        np.zeros((256, 0), np.float32), [])
    data, off = T.encode_examples(specs, fb)
    p = str(tmp_path / "cfg2.tfrecord.gz")
    with T.TFRecordWriter(p) as w:
        w.write_many(data, off)
    got = list(T.TFRecordReader([p], specs, 100, thread_num=4))
    assert [g.batch for g in got] == [100, 100, 56]
    # concatenate and compare CSR exactly
    S = len(specs)
    b0 = 0
    for g in got:
        sb = g.sparse
        for b in range(g.batch):
            for s in range(S):
                a, e = hb.bag_off[(b0 + b) * S + s], hb.bag_off[(b0 + b) * S + s + 1]
                ga, ge = sb.bag_off[b * S + s], sb.bag_off[b * S + s + 1]
                assert e - a == ge - ga
                for t in range(e - a):
                    assert bytes(hb.tok_bytes[hb.tok_off[a + t]:hb.tok_off[a + t + 1]]) == \
                        bytes(sb.tok_bytes[sb.tok_off[ga + t]:sb.tok_off[ga + t + 1]])
        b0 += g.batch


def test_build_feature_description_matches_reference_rules():
    from recommendflow_amd.config_parser.configuration import Configuration

    root = os.path.dirname(os.path.abspath(__file__))
    conf = Configuration(os.path.join(root, "golden", "conf", "base_conf.yaml"))
    desc = {s.name: s for s in T.build_feature_description(conf)}
    assert [s for s in desc] == conf.train_feature_names
    assert desc["app_id"].kind == T.BYTES and desc["app_id"].shape == T.SEQ  # hashing -> FixedLenSequenceFeature
    assert desc["query_tok_id"].kind == T.INT64 and desc["query_tok_id"].shape == T.SEQ  # token_id
    assert desc["label"].kind == T.FLOAT and desc["label"].shape == T.SCALAR and desc["label"].default == 0.0


def test_library_exports_io_symbols():
    import re

    from recommendflow_amd.runtime import lib as L

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = re.sub(r"/\*.*?\*/", "", open(os.path.join(root, "include", "rf_io.h")).read(), flags=re.S)
    syms = sorted(set(re.findall(r"\b(rf_[a-z0-9_]+)\s*\(", src)))
    assert set(syms) == set(T.IO_SIGS), set(syms) ^ set(T.IO_SIGS)
    lib = L.load()
    for s in syms:
        assert hasattr(lib, s), s
    assert struct.calcsize("<qiiqd") == 32


@pytest.mark.parametrize("compression", ["GZIP", None])
def test_next_records_packs_the_interleaved_records(tmp_path, compression):
    """The device-parse host half (rf_tfr_next_records): same records, same order as the host parse."""
    counts = [7, 0, 12, 5]
    paths, recs = [], []
    for f, n in enumerate(counts):
        r = [pb_record(x) for x in random_rows(n, 30 + f)]
        p = str(tmp_path / f"n{f}")
        TO.write_file(p, r, compression or "NONE")
        paths.append(p)
        recs.append(r)
    want = [recs[f][i] for f, i in TO.interleave_order(counts, 3)]
    rd = T.TFRecordReader(paths, SPECS, 5, thread_num=3, compression_type=compression)
    buf, off, got = np.empty(8, np.uint8), np.empty(6, np.int64), []  # 8 bytes: forces the ENOSPC -> grow path
    while True:
        buf, n, nb = rd.read_records(buf, off)
        if n == 0:
            break
        assert off[0] == 0 and off[n] == nb
        got += [bytes(buf[off[i]:off[i + 1]]) for i in range(n)]
    assert got == want and rd.records_read == len(want)


def test_schema_blob_and_device_check_messages():
    """The device schema blob (rf_tfr_blob.h) and the host-side error text for device parse errors."""
    import ctypes

    L = T._lib()
    feats, _keep = T._feats_array(SPECS)
    need = ctypes.c_int64(0)
    assert L.rf_tfr_schema_blob(feats, len(SPECS), None, 0, ctypes.byref(need)) == T.RF_ENOSPC
    blob = np.zeros(int(need.value), np.uint8)
    assert L.rf_tfr_schema_blob(feats, len(SPECS), blob.ctypes.data, blob.size, ctypes.byref(need)) == 0
    F, Sb, Si, Sf, Ni, Nf, hmask, names_off = (int(x) for x in np.frombuffer(blob[:32].tobytes(), np.int32))
    assert (F, Sb, Si, Sf, Ni, Nf) == (7, 3, 1, 1, 1, 1) and hmask + 1 >= 2 * F and (hmask + 1) & hmask == 0
    fe = blob[40:40 + 40 * F].reshape(F, 40)
    ht = np.frombuffer(blob[40 + 40 * F:40 + 40 * F + 4 * (hmask + 1)].tobytes(), np.int32)
    for j, s in enumerate(SPECS):
        kind, shape, gpos, no, nl = np.frombuffer(fe[j, :20].tobytes(), np.int32)
        assert (kind, shape) == (s.kind, s.shape)
        assert bytes(blob[names_off + no:names_off + no + nl]) == s.name.encode()
        h = 2166136261
        for ch in s.name.encode():
            h = ((h ^ ch) * 16777619) & 0xFFFFFFFF
        slot = h & hmask
        while ht[slot] != j:  # linear probing reaches the key before an empty slot
            assert ht[slot] >= 0
            slot = (slot + 1) & hmask
    assert int(L.rf_tfr_device_workspace_bytes(blob.ctypes.data, 100)) > 16 * 100 * F

    def msg(**kw):
        st = T._DevStats(err_b=kw.pop("b", 2147483647), **kw)
        rc = L.rf_tfr_device_check(ctypes.addressof(st), feats, len(SPECS), 40)
        return rc, L.rf_last_error().decode()

    assert msg()[0] == 0
    assert msg(b=3, err_type=1) == (T.RF_EDATA, "rf_tfr_next_batch: malformed tf.train.Example at batch position 3 (record 43)")
    assert msg(b=0, err_type=2, err_feat=5, err_kind=T.FLOAT)[1] == \
        "rf_tfr_next_batch: Key: cnt. Data types don't match. Expected int64, got float (record 40)"
    assert msg(b=1, err_type=3, err_feat=3)[1] == "rf_tfr_next_batch: Key: disc. malformed float list (record 41)"
    assert msg(b=1, err_type=4, err_feat=4, err_count=2)[1] == \
        "rf_tfr_next_batch: Key: label. Number of values != expected. Values size: 2 but output shape: [] (record 41)"


@pytest.mark.parametrize("compression", [None, "GZIP"])
def test_writer_crc_every_length_class(tmp_path, compression):
    """The build's CRC-32C (three interleaved streams over 1024- and 128-byte blocks, then single steps) against
    the oracle's bitwise CRC on payloads around every block boundary."""
    rng = np.random.default_rng(8)
    sizes = [0, 1, 7, 8, 9, 383, 384, 385, 1000, 3071, 3072, 3073, 3456, 3457, 4000, 20000, 65537]
    recs = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in sizes]
    data = np.frombuffer(b"".join(recs), np.uint8)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    p = str(tmp_path / ("c.gz" if compression else "c"))
    with T.TFRecordWriter(p, compression) as w:
        w.write_many(data, off)
    assert TO.read_file(p, compression or "NONE") == recs
