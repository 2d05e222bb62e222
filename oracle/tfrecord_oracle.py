"""CPU oracle for the TFRecord -> batched-CSR pipe (TEST INFRASTRUCTURE ONLY — never imported by the
product; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it).

Restates, in plain Python, what the reference gets from TensorFlow for this path:
  * tf.io.TFRecordWriter / TFRecordDataset framing (TF core/lib/io/record_writer.cc format:
    u64 length, masked crc32c(length), payload, masked crc32c(payload); mask = rot15 + 0xa282ead8),
    GZIP = a gzip stream (zlib windowBits 16+15) over the framed bytes
    (utils/make_tfrecord.py:142; backend/core/dataloader.py:567-570);
  * tf.io.parse_example with the feature description of build_feature_description
    (dataloader.py:23-44): FixedLenSequenceFeature(allow_missing) -> list (missing -> []), padded
    to the batch max; FixedLenFeature(()) -> exactly one value or the default;
  * the deterministic interleave of TFRecordDataset(num_parallel_reads=n)
    (tf.data InterleaveDataset, cycle_length n, block_length 1).

TensorFlow is absent here, so this is pinned by: the CRC-32C check vectors of RFC 3720 §B.4 and the
standard "123456789" check value, and Google's protobuf library (an independent tf.train.Example
encoder/decoder built from the public example.proto / feature.proto schema in tests/tf_example_pb.py).
"""
from __future__ import annotations

import gzip
import struct
from typing import Dict, List, Sequence, Tuple

BYTES, INT64, FLOAT = 0, 1, 2
SEQ, SCALAR = 0, 1


def crc32c(data: bytes) -> int:
    """Bitwise CRC-32C (Castagnoli, reflected polynomial 0x82F63B78)."""
    c = 0xFFFFFFFF
    for b in data:
        c ^= b
        for _ in range(8):
            c = (c >> 1) ^ (0x82F63B78 if c & 1 else 0)
    return c ^ 0xFFFFFFFF


def masked_crc32c(data: bytes) -> int:
    c = crc32c(data)
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def frame(records: Sequence[bytes]) -> bytes:
    out = bytearray()
    for r in records:
        ln = struct.pack("<Q", len(r))
        out += ln + struct.pack("<I", masked_crc32c(ln)) + r + struct.pack("<I", masked_crc32c(r))
    return bytes(out)


def write_file(path: str, records: Sequence[bytes], compression: str = "GZIP"):
    blob = frame(records)
    with open(path, "wb") as f:
        f.write(gzip.compress(blob) if compression == "GZIP" else blob)


def read_file(path: str, compression: str = "GZIP") -> List[bytes]:
    with open(path, "rb") as f:
        blob = f.read()
    if compression == "GZIP":
        blob = gzip.decompress(blob)
    out, p = [], 0
    while p < len(blob):
        if len(blob) - p < 12:
            raise ValueError("truncated record header")
        (n,) = struct.unpack_from("<Q", blob, p)
        if struct.unpack_from("<I", blob, p + 8)[0] != masked_crc32c(blob[p:p + 8]):
            raise ValueError("length crc")
        p += 12
        if len(blob) - p < n + 4:
            raise ValueError("truncated record")
        rec = blob[p:p + n]
        if struct.unpack_from("<I", blob, p + n)[0] != masked_crc32c(rec):
            raise ValueError("data crc")
        out.append(rec)
        p += n + 4
    return out


# ---- protobuf wire format ------------------------------------------------------------------------
def _varint(b: bytes, p: int) -> Tuple[int, int]:
    r, s = 0, 0
    while True:
        x = b[p]
        p += 1
        r |= (x & 0x7F) << s
        if not x & 0x80:
            return r, p
        s += 7


def _fields(b: bytes):
    p = 0
    while p < len(b):
        tag, p = _varint(b, p)
        f, wt = tag >> 3, tag & 7
        if wt == 0:
            v, p = _varint(b, p)
        elif wt == 1:
            v, p = b[p:p + 8], p + 8
        elif wt == 2:
            n, p = _varint(b, p)
            v, p = b[p:p + n], p + n
        elif wt == 5:
            v, p = b[p:p + 4], p + 4
        else:
            raise ValueError("bad wire type")
        yield f, wt, v


def decode_example(rec: bytes) -> Dict[str, Tuple[int, list]]:
    """tf.train.Example -> {key: (kind, values)}; the last map entry of a key wins."""
    out = {}
    for f, wt, feats in _fields(rec):
        if f != 1 or wt != 2:
            continue
        for f2, wt2, entry in _fields(feats):
            if f2 != 1 or wt2 != 2:
                continue
            key, val = b"", None
            for f3, wt3, v in _fields(entry):
                if f3 == 1 and wt3 == 2:
                    key = v
                elif f3 == 2 and wt3 == 2:
                    val = v
            kind, lst = None, b""
            for f4, wt4, v in _fields(val or b""):
                if wt4 == 2 and f4 in (1, 2, 3):
                    kind, lst = {1: BYTES, 2: FLOAT, 3: INT64}[f4], v
            vals = []
            if kind is not None:
                for f5, wt5, v in _fields(lst):
                    if f5 != 1:
                        continue
                    if kind == BYTES:
                        vals.append(bytes(v))
                    elif kind == FLOAT:
                        vals.extend(struct.unpack(f"<{len(v) // 4}f", v) if wt5 == 2 else struct.unpack("<f", v))
                    else:
                        if wt5 == 0:
                            vals.append(v - (1 << 64) if v >= 1 << 63 else v)
                        else:
                            q = 0
                            while q < len(v):
                                x, q = _varint(v, q)
                                vals.append(x - (1 << 64) if x >= 1 << 63 else x)
            out[key.decode()] = (kind, vals)
    return out


def parse_examples(records: Sequence[bytes], specs) -> Dict[str, list]:
    """parse_example restated: {name: per-example value lists (SEQ) or values (SCALAR)}; raises
    ValueError where tf.io.parse_example raises InvalidArgument/DataLoss."""
    out = {s.name: [] for s in specs}
    for rec in records:
        ex = decode_example(rec)
        for s in specs:
            kind, vals = ex.get(s.name, (None, None))
            if vals is not None and kind is not None and kind != s.kind:
                raise ValueError(f"Key: {s.name}. Data types don't match")
            if vals is None:
                vals = None if s.shape == SCALAR else []
            if s.shape == SEQ:
                out[s.name].append(list(vals))
            else:
                if vals is None:
                    out[s.name].append(b"" if s.kind == BYTES else s.default)
                elif len(vals) != 1:
                    raise ValueError(f"Key: {s.name}. Number of values != expected")
                else:
                    out[s.name].append(vals[0])
    return out


def interleave_order(counts: Sequence[int], cycle: int) -> List[Tuple[int, int]]:
    """(file, record) order of tf.data InterleaveDataset(cycle_length=cycle, block_length=1) over files
    with the given record counts: an empty cycle slot opens the next file and produces from it; an
    exhausted file frees its slot and the cursor moves on."""
    cycle = max(1, min(cycle, len(counts)))
    slots: List = [None] * cycle
    nxt, cur, out = 0, 0, []
    while nxt < len(counts) or any(s is not None for s in slots):
        s = slots[cur]
        if s is None:
            if nxt < len(counts):
                slots[cur] = [nxt, 0]
                nxt += 1
                continue
            cur = (cur + 1) % cycle
            continue
        f, i = s
        if i < counts[f]:
            out.append((f, i))
            s[1] += 1
            cur = (cur + 1) % cycle
        else:
            slots[cur] = None
            cur = (cur + 1) % cycle
    return out
