"""tf.train.Example message classes built with Google's protobuf library from the public schema of
tensorflow/core/example/{example,feature}.proto (field numbers only; TensorFlow itself is absent).
Used as an independent encoder/decoder to pin the C++ wire codec (rf_io.cpp).

    message BytesList { repeated bytes value = 1; }
    message FloatList { repeated float value = 1 [packed = true]; }
    message Int64List { repeated int64 value = 1 [packed = true]; }
    message Feature   { oneof kind { BytesList bytes_list = 1; FloatList float_list = 2; Int64List int64_list = 3; } }
    message Features  { map<string, Feature> feature = 1; }
    message Example   { Features features = 1; }

`packed=False` builds a proto2 variant whose repeated scalars go on the wire unpacked (legal input
that a reader must also accept).
"""
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

_T = descriptor_pb2.FieldDescriptorProto
_cache = {}


def classes(packed: bool = True):
    if packed in _cache:
        return _cache[packed]
    pkg = "tfpin" if packed else "tfpin2"
    fdp = descriptor_pb2.FileDescriptorProto(name=f"{pkg}/example.proto", package=pkg,
                                             syntax="proto3" if packed else "proto2")
    rep = _T.LABEL_REPEATED
    opt = _T.LABEL_OPTIONAL

    def msg(name):
        return fdp.message_type.add(name=name)

    m = msg("BytesList")
    m.field.add(name="value", number=1, type=_T.TYPE_BYTES, label=rep)
    for name, ty in (("FloatList", _T.TYPE_FLOAT), ("Int64List", _T.TYPE_INT64)):
        m = msg(name)
        f = m.field.add(name="value", number=1, type=ty, label=rep)
        f.options.packed = packed
    m = msg("Feature")
    m.oneof_decl.add(name="kind")
    for i, (n, t) in enumerate((("bytes_list", "BytesList"), ("float_list", "FloatList"), ("int64_list", "Int64List"))):
        m.field.add(name=n, number=i + 1, type=_T.TYPE_MESSAGE, type_name=f".{pkg}.{t}", label=opt, oneof_index=0)
    m = msg("Features")
    e = m.nested_type.add(name="FeatureEntry")
    e.options.map_entry = True
    e.field.add(name="key", number=1, type=_T.TYPE_STRING, label=opt)
    e.field.add(name="value", number=2, type=_T.TYPE_MESSAGE, type_name=f".{pkg}.Feature", label=opt)
    m.field.add(name="feature", number=1, type=_T.TYPE_MESSAGE, type_name=f".{pkg}.Features.FeatureEntry", label=rep)
    m = msg("Example")
    m.field.add(name="features", number=1, type=_T.TYPE_MESSAGE, type_name=f".{pkg}.Features", label=opt)
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    out = {n: message_factory.GetMessageClass(pool.FindMessageTypeByName(f"{pkg}.{n}"))
           for n in ("BytesList", "FloatList", "Int64List", "Feature", "Features", "Example")}
    _cache[packed] = out
    return out


def make_example(values: dict, packed: bool = True) -> bytes:
    """values: {name: ("bytes"|"float"|"int64", list)} -> serialized Example."""
    C = classes(packed)
    ex = C["Example"]()
    for name, (kind, vals) in values.items():
        f = ex.features.feature[name]
        if kind == "bytes":
            f.bytes_list.value.extend([v.encode() if isinstance(v, str) else v for v in vals])
        elif kind == "float":
            f.float_list.value.extend(vals)
        elif kind == "int64":
            f.int64_list.value.extend(vals)
        elif kind == "none":
            f.SetInParent()
        else:
            raise ValueError(kind)
    return ex.SerializeToString()


def parse_example(data: bytes) -> dict:
    C = classes(True)
    ex = C["Example"]()
    ex.ParseFromString(data)
    out = {}
    for k, f in ex.features.feature.items():
        w = f.WhichOneof("kind")
        out[k] = (w, list(getattr(f, w).value) if w else [])
    return out
