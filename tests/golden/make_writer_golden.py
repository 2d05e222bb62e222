"""Generate tests/golden/writer/writer_golden.json by running the REFERENCE's own TFRecord writer path on a committed
TSV: utils.util.read_csv (pandas, dtype=str, fillna("-1"), util.py:232) and
utils.make_tfrecord.build_tfrecord with its _build_str_feature / _build_int_feature / _build_float_feature
(make_tfrecord.py:26-41, 92-125), over a Configuration the reference parses itself.

Runs only in the development container (it reads /root/reference; the tests read the committed JSON). The reference
modules import tensorflow / tensorflow_io / case_class at module level, absent here; they are supplied as inert
stand-ins, and tf.train.{Feature, BytesList, Int64List, FloatList, Features, Example} as RECORDING stand-ins: the
reference code builds its Example objects unmodified, and Example.SerializeToString returns the recorded structure
instead of protobuf bytes (the byte encoding itself is pinned separately by Google's protobuf library,
tests/test_tfrecord.py). pandas, numpy, tqdm, sklearn and psutil are the real libraries.

The reference writer is broken as written (make_tfrecord.py:95 iterates a non-iterable Features object); its
per-feature loop body runs here over Features.train_features (see main()); recorded in DESIGN.md §5 as D-writer-loop.
Lookup features are not working in writer_conf.yaml: build_tfrecord compares Feature.type (a tf dtype after
config_proto.TYPE_MAP) with the strings TYPE_INT / TYPE_STR (make_tfrecord.py:103-106), which never match, so the
reference raises "Unsupported deal method feature" for every lookup feature.

Output: per TSV row, per feature in build_tfrecord's order, {"kind": "bytes" | "int64" | "float", "values": [...]}
(bytes as latin-1 text; float values as the Python floats the reference passes to FloatList, which stores them
as float32).

Usage: python tests/golden/make_writer_golden.py
"""
import json
import os
import sys
import types

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "writer", "writer_golden.json")


class _List:
    def __init__(self, value=()):
        self.value = list(value)


class _Feature:
    def __init__(self, bytes_list=None, int64_list=None, float_list=None):
        if bytes_list is not None:
            self.kind, self.values = "bytes", [v.decode("latin-1") for v in bytes_list.value]
        elif int64_list is not None:
            self.kind, self.values = "int64", [int(v) for v in int64_list.value]
        else:
            self.kind, self.values = "float", [float(v) for v in float_list.value]


class _Features:
    def __init__(self, feature):
        self.feature = feature


class _Example:
    def __init__(self, features):
        self.features = features

    def SerializeToString(self):  # noqa: N802 — the tf.train.Example method name
        return [{"feature": getattr(k, "name", str(k)), "kind": f.kind, "values": f.values}
                for k, f in self.features.feature.items()]


def _install_stubs():
    tf = types.ModuleType("tensorflow")
    tf.int64, tf.float32, tf.string = "tf.int64", "tf.float32", "tf.string"
    tf.train = types.SimpleNamespace(Feature=_Feature, BytesList=_List, Int64List=_List, FloatList=_List,
                                     Features=_Features, Example=_Example)
    sys.modules["tensorflow"] = tf
    tfio = types.ModuleType("tensorflow_io")
    tfio.version = "stub"
    sys.modules["tensorflow_io"] = tfio
    cc_pkg = types.ModuleType("case_class")
    cc_mod = types.ModuleType("case_class.case_class")

    class CaseClass:
        pass

    cc_mod.CaseClass = CaseClass
    cc_pkg.case_class = cc_mod
    sys.modules["case_class"] = cc_pkg
    sys.modules["case_class.case_class"] = cc_mod


def main():
    _install_stubs()
    sys.path.insert(0, REF)
    cwd = os.getcwd()
    os.chdir(REF)  # the reference resolves some paths relative to its root
    try:
        from config_parser.configuration import Configuration
        from utils.make_tfrecord import build_tfrecord
        from utils.util import read_csv

        conf = Configuration(os.path.join(HERE, "writer", "writer_conf.yaml"))
        # build_tfrecord loops `for feature in conf.features` (make_tfrecord.py:95), but Configuration.features is a
        # Features object, which is not iterable (TypeError): the reference writer cannot run as written. Its loop
        # body runs unmodified here over the list its comment names ("only train_cols are stored",
        # make_tfrecord.py:96): a view of the Configuration whose .features is Features.train_features.
        view = types.SimpleNamespace(features=conf.features.train_features)
        df = read_csv(os.path.join(HERE, "writer", "writer_input.tsv"), sep="\t")
        rows = []
        for _, row in df.iterrows():
            rows.append({"tsv_row": {k: str(v) for k, v in row.items()}, "features": build_tfrecord(row, view)})
    finally:
        os.chdir(cwd)
    res = {"generator": "tests/golden/make_writer_golden.py",
           "reference": ["utils/util.py:220-232 read_csv", "utils/make_tfrecord.py:26-41 _build_*_feature",
                         "utils/make_tfrecord.py:92-125 build_tfrecord"],
           "conf": "tests/golden/writer/writer_conf.yaml", "input": "tests/golden/writer/writer_input.tsv",
           "rows": rows}
    with open(OUT, "w") as fh:
        json.dump(res, fh, indent=1)
    print(f"wrote {OUT}: {len(rows)} rows")


if __name__ == "__main__":
    main()
