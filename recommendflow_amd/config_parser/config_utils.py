"""Config helpers (reference: config_parser/config_utils.py).

* ``is_punctuation``  — the `$`-substitution tokeniser's separator test (config_utils.py:85-95).
* ``load_slot_map``   — `name:type:slot` lines (config_utils.py:21-33). Deviation D-slotmap
  (SURVEY A.10): Spark SQL type names are accepted — StringType / ArrayType(StringType,..) -> str,
  IntegerType / LongType -> int, FloatType / DoubleType -> float — because the reference's own
  conf/base_recall_sdpa.feature.map uses them and its assert (:31) rejects them.
* ``load_vocab``      — BERT vocab file -> {token: id} (config_utils.py:98-107).
"""
from __future__ import annotations

import os
import unicodedata
from typing import Dict, List

from .config_proto import SUPPORT_TYPE

_SPARK_TYPES = {
    "stringtype": "str",
    "integertype": "int",
    "longtype": "int",
    "shorttype": "int",
    "bytetype": "int",
    "floattype": "float",
    "doubletype": "float",
}


def is_punctuation(ch: str, except_char: str = "") -> bool:
    if ch in except_char:
        return False
    c = ord(ch)
    if 33 <= c <= 47 or 58 <= c <= 64 or 91 <= c <= 96 or 123 <= c <= 126:
        return True
    return unicodedata.category(ch).startswith("P")


def normalize_type_name(type_name: str) -> str:
    t = str(type_name).strip().lower()
    if t in SUPPORT_TYPE:
        return t
    if t.startswith("arraytype"):
        inner = t[len("arraytype"):].strip("()").split(",")[0].strip()
        return normalize_type_name(inner or "stringtype")
    if t in _SPARK_TYPES:
        return _SPARK_TYPES[t]
    raise ValueError(f"Unsupported type {type_name}")


def slot_map_multivalued(type_name: str) -> bool:
    return str(type_name).strip().lower().startswith("arraytype")


def load_slot_map(path: str) -> Dict[int, List]:
    """slot id -> [name, type] where type in {int, float, str}; `name:type:slot` per line.

    The type may itself contain ':'-free commas and parentheses (ArrayType(StringType,true)), so the
    line is split at its FIRST and LAST ':'.
    """
    out: Dict[int, List] = {}
    with open(path, encoding="utf-8") as f:
        for raw in f:
            line = raw.strip()
            if not line:
                continue
            first, last = line.find(":"), line.rfind(":")
            if first < 0 or first == last:
                raise ValueError(f"bad slot-map line: {line!r}")
            name, tname, slot = line[:first], line[first + 1:last], line[last + 1:]
            out[int(slot)] = [name, normalize_type_name(tname), slot_map_multivalued(tname)]
    return out


def side_car_slot_map(config_path: str) -> str:
    """`conf/x.yaml` -> `conf/x.feature.map` when that file exists, else ''."""
    stem, _ = os.path.splitext(config_path)
    cand = stem + ".feature.map"
    return cand if os.path.isfile(cand) else ""


def load_vocab(dict_path: str, encoding: str = "utf-8") -> Dict[str, int]:
    vocab: Dict[str, int] = {}
    with open(dict_path, encoding=encoding) as f:
        for line in f:
            parts = line.split()
            tok = parts[0] if parts else line.strip()
            vocab[tok] = len(vocab)
    return vocab
