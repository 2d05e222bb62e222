"""Generate tests/golden/config_golden.json from the REFERENCE's own config parser.

Runs only in the development container (it reads /root/reference, which does not exist on the GPU
box; the tests read the committed JSON). The reference parser (config_parser/*.py, utils/*.py) is
pure Python except for module-level imports of tensorflow / tensorflow_io / case_class, which are
absent here; it only uses tf.int64/float32/string as opaque dtype constants (config_proto.py:41) and
CaseClass as a base class (features.py:17). Those three names are supplied as inert stand-in
modules in sys.modules — the reference's parsing code itself runs unmodified.

Outputs, per config:
  * base_conf.yaml        parsed by reference Configuration (parses: 7 train features);
  * demo_conf.yaml        the reference's error (pooling `cls`, deviation D-cls);
  * base_recall_sdpa.yaml the reference's error through Configuration (no slot map, D-slotmap), and
                          the reference `Features` parse of the same YAML given a slot map whose
                          Spark type names are translated to str/int/float (the D-slotmap mapping),
                          which pins the reference's ellipsis behaviour ([0, 4, ..., 71] drops 0).

Usage: python tests/golden/make_config_golden.py   (writes tests/golden/config_golden.json)
"""
import enum
import json
import os
import sys
import tempfile
import types

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def _install_stubs():
    tf = types.ModuleType("tensorflow")
    tf.int64, tf.float32, tf.string = "tf.int64", "tf.float32", "tf.string"
    sys.modules["tensorflow"] = tf
    tfio = types.ModuleType("tensorflow_io")
    tfio.version = "stub"
    sys.modules["tensorflow_io"] = tfio
    cc_pkg = types.ModuleType("case_class")
    cc_mod = types.ModuleType("case_class.case_class")

    class CaseClass:  # plain base class; Feature defines its own __eq__/__hash__
        pass

    cc_mod.CaseClass = CaseClass
    cc_pkg.case_class = cc_mod
    sys.modules["case_class"] = cc_pkg
    sys.modules["case_class.case_class"] = cc_mod


def _jsonable(v):
    if isinstance(v, enum.Enum):
        return v.value
    if isinstance(v, (list, tuple)):
        return [_jsonable(i) for i in v]
    if isinstance(v, dict):
        return {str(k): _jsonable(x) for k, x in v.items()}
    if isinstance(v, (str, int, float, bool)) or v is None:
        return v
    return str(v)


def _try(fn, *a):
    try:
        return {"ok": True, "value": _jsonable(fn(*a))}
    except Exception as e:  # noqa: BLE001
        return {"ok": False, "error_type": type(e).__name__}


TYPE_BACK = {"tf.int64": "int", "tf.float32": "float", "tf.string": "str"}


def _feature_dict(f):
    return {
        "name": f.name,
        "field_name": f.field_name,
        "type": TYPE_BACK[f.type],
        "tower": f.tower.value,
        "deal": f.deal.value,
        "vocab_size": f.vocab_size,
        "embedding_dim": f.embedding_dim,
        "pooling": f.pooling.value,
        "working": f.working,
        "vocabs": _jsonable(f.vocabs),
        "hash_seeds": _jsonable(f.hash_seeds),
        "default": f.default,
    }


SPARK = {"stringtype": "str", "integertype": "int", "longtype": "int", "floattype": "float", "doubletype": "float"}


def _translate_slot_map(src, dst):
    with open(src) as fi, open(dst, "w") as fo:
        for line in fi:
            line = line.strip()
            if not line:
                continue
            name, rest = line.split(":", 1)
            slot = rest.rsplit(":", 1)[1]
            tname = rest.rsplit(":", 1)[0].lower()
            t = "str" if tname.startswith("arraytype") else SPARK[tname]
            fo.write(f"{name}:{t}:{slot}\n")


def main():
    _install_stubs()
    sys.path.insert(0, REF)
    cwd = os.getcwd()
    tmp = tempfile.mkdtemp()
    os.chdir(tmp)  # read_csv creates ./__datacache__ (utils/util.py:181-185)
    try:
        from config_parser.configuration import Configuration
        from config_parser.features import Features
        import yaml

        out = {"generator": "tests/golden/make_config_golden.py", "reference": "mechsihao/RecommendFlow @ /root/reference"}
        # 1. base_conf.yaml
        c = Configuration(os.path.join(REF, "conf/base_conf.yaml"))
        out["base_conf"] = {
            "ok": True,
            "all_features": [_feature_dict(f) for f in c.features.features],
            "train_feature_names": c.train_feature_names,
            "hashing_feature_names": c.features.hashing_feature_names,
            "label_names": c.features.label_names,
            "experiment_ids": [int(i) for i in c.experiments.index],
            "experiment_fields": c.experiment_field,
            "experiments": [_jsonable(r) for r in c.experiments.reset_index().values.tolist()],
            "networks": _jsonable(c.networks),
            "conf_values": {k: _jsonable(c.get_conf_value(k)) for k in ["seeds", "task", "dayno", "data", "train_data1", "7days", "del_sug_and_desc", "max_len", "vocab_path"]},
            "set_str": {s: _try(c._set_str, s) for s in ["$dayno-7", "a/$task/b", "$task.$dayno", "x_$task_y", "$seeds"]},
        }
        # 2. demo_conf.yaml
        try:
            Configuration(os.path.join(REF, "conf/demo_conf.yaml"))
            out["demo_conf"] = {"ok": True}
        except Exception as e:  # noqa: BLE001
            out["demo_conf"] = {"ok": False, "error_type": type(e).__name__, "error": str(e)}
        # 3. base_recall_sdpa.yaml
        try:
            Configuration(os.path.join(REF, "conf/base_recall_sdpa.yaml"))
            out["base_recall_sdpa"] = {"ok": True}
        except BaseException as e:  # noqa: BLE001  (AssertionError)
            out["base_recall_sdpa"] = {"ok": False, "error_type": type(e).__name__, "error": str(e)}
        smap = os.path.join(tmp, "sdpa.translated.map")
        _translate_slot_map(os.path.join(REF, "conf/base_recall_sdpa.feature.map"), smap)
        conf = yaml.load(open(os.path.join(REF, "conf/base_recall_sdpa.yaml")).read(), Loader=yaml.FullLoader)
        conf["Features"]["features"] = [[i for i in line.split(",")] for line in conf["Features"]["features"].split()]
        feats = Features(conf, {}, [2022, 2023], slot_map_path=smap)
        out["base_recall_sdpa_features_with_translated_map"] = {
            "note": "reference Features(...) with slot map types translated per D-slotmap; shows the "
                    "reference ellipsis rule ([0, 4, ..., 71] -> 4..71, slot 0 dropped)",
            "features": [_feature_dict(f) for f in feats.features],
            "n_hashing": len(feats.hashing_feature_names),
            "user": feats.user_feature_names,
            "ad": feats.ad_feature_names,
        }
    finally:
        os.chdir(cwd)
    path = os.path.join(HERE, "config_golden.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, ensure_ascii=False)
    print("wrote", path)


if __name__ == "__main__":
    main()
