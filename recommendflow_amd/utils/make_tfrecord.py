"""TSV -> TFRecord(GZIP) of tf.train.Example, the writer side of the feature pipe, through librf.so's
Example encoder and TFRecord writer (include/rf_io.h).

Mirrors, with the reference's names:
  * read_csv(path, sep="\\t", na="-1")      utils/util.py:220-232: pandas, every column as str, missing -> "-1"
  * build_tfrecord(row, conf)               utils/make_tfrecord.py:92-125: one Example's value lists, per feature:
        numeric / discrete        _build_float_feature   float(i) for i in data.split(",")
        hashing / bert_encode     _build_str_feature     ("" if data == "-1" else data).split(","), UTF-8
        lookup (str)              _build_str_feature
        lookup (int) / token_id   _build_int_feature     int(i) for i in data.split(",")
        a column missing from the row: "-1" (get_or_ignore_row_data, make_tfrecord.py:88-90)
  * dump_tfrecord_data(input_file, out_file, conf)   make_tfrecord.py:139-144 (GZIP)
Deviations: D-writer-loop (the reference loop iterates Configuration.features, a non-iterable
Features object, make_tfrecord.py:95; here the train features, as its comment says), D-writer-lookup (the
reference's lookup branch compares a tf dtype with "int"/"str" and never matches, so it raises for lookup features;
here lookup features are written), D-writer-kind (every feature is stored with the kind the reader's feature
description expects; the reference stores numeric / discrete as float lists even when typed int). Embedding and
image features are out of scope (NotImplementedError). Pinned by tests/golden/writer (the reference's own
_build_*_feature and read_csv run on a committed TSV).
"""
from __future__ import annotations

from typing import Dict, List, Sequence

from ..runtime import tfrecord as T


def read_csv(path: str, sep: str = "\t", na: str = "-1", nrows: int = None):
    """utils/util.py:220-232 for a local path: a header row, every column read as str, missing cells -> na."""
    import pandas as pd

    nrows = None if nrows and nrows < 0 else nrows
    return pd.read_csv(path, sep=sep, dtype=str, nrows=nrows).fillna(na)


def _cell(row, name: str, na: str = "-1") -> str:
    return str(row[name]) if name in row else na


def build_tfrecord(row, conf) -> Dict[str, List]:
    """The value lists one Example holds for this row (make_tfrecord.py:92-125's rules, above), keyed by feature
    name, over conf's train features; bytes values as UTF-8 bytes."""
    from ..config_parser.config_proto import FeatureDeal

    feats = conf.features.train_features if hasattr(conf, "features") else list(conf)
    out: Dict[str, List] = {}
    for f in feats:
        data = _cell(row, f.name)
        if f.deal in (FeatureDeal.Numeric, FeatureDeal.Discrete):
            vals = [float(i) for i in data.split(",")]
            out[f.name] = [int(v) for v in vals] if f.type == "int" else vals  # D-writer-kind
        elif f.deal in (FeatureDeal.Hashing, FeatureDeal.BertEncode) or (f.deal == FeatureDeal.Lookup and f.type == "str"):
            out[f.name] = [t.encode() for t in ("" if data == "-1" else data).split(",")]
        elif f.deal == FeatureDeal.TokenId or (f.deal == FeatureDeal.Lookup and f.type == "int"):
            out[f.name] = [int(i) for i in data.split(",")]
        elif f.deal == FeatureDeal.Lookup and f.type == "float":
            out[f.name] = [float(i) for i in data.split(",")]
        elif f.deal in (FeatureDeal.Embedding, FeatureDeal.Image):
            raise NotImplementedError(f"{f.deal.value} features are out of scope (SURVEY §2): {f.name}")
        else:
            raise ValueError(f"Unsupported deal method feature: {f.name}")
    return out


def encode_rows(rows: Sequence[Dict[str, List]], conf):
    """Examples of build_tfrecord's value dicts, serialised by librf (rf_tfr_encode_examples): (bytes, rec_off)."""
    specs = T.build_feature_description(conf)
    by = {s.name: s for s in specs}
    norm = []
    for r in rows:
        d = {}
        for n, v in r.items():
            if n not in by:
                continue
            d[n] = v[0] if by[n].shape == T.SCALAR and len(v) == 1 else v
        norm.append(d)
    fb = T.columns_from_rows(specs, norm)
    return T.encode_examples(specs, fb)


def dump_tfrecord_data(input_file: str, out_file: str, conf, compression_type: str = "GZIP", batch: int = 4096) -> int:
    """make_tfrecord.py:139-144: every row of a TSV as one Example in a GZIP TFRecord file. Returns the row count."""
    df = read_csv(input_file, sep="\t")
    n = 0
    with T.TFRecordWriter(out_file, compression_type) as w:
        for s in range(0, len(df), batch):
            rows = [build_tfrecord(row, conf) for _, row in df.iloc[s: s + batch].iterrows()]
            data, rec_off = encode_rows(rows, conf)
            w.write_many(data, rec_off)
            n += len(rows)
    return n
