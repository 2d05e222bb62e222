"""Enumerations of the feature-config grammar (reference: config_parser/config_proto.py:5-42).

The reference maps element types to TensorFlow dtypes (TYPE_MAP :41); the build maps them to the
numpy dtype of the parsed column instead (no TensorFlow). Deviation D-cls: the
documented pooling `cls` (conf/README.md) is accepted as an alias of `first`.
"""
from __future__ import annotations

from enum import Enum

import numpy as np


class FeatureTower(Enum):
    Null = "null"
    User = "user"
    Ad = "ad"
    Context = "context"
    Label = "label"


class FeatureDeal(Enum):
    Null = "null"
    Numeric = "numeric"
    Discrete = "discrete"
    Hashing = "hashing"
    Lookup = "lookup"
    Image = "image"
    Embedding = "embedding"
    TokenId = "token_id"
    BertEncode = "bert_encode"


class FeaturePooling(Enum):
    Null = "null"
    Avg = "avg"
    Min = "min"
    Max = "max"
    Sum = "sum"
    First = "first"
    Last = "last"

    @classmethod
    def _missing_(cls, value):
        # D-cls: `cls` (take the first element) is documented in conf/README.md but absent from the enum
        if isinstance(value, str) and value.lower() == "cls":
            return cls.First
        return None


TYPE_INT = "int"
TYPE_FLOAT = "float"
TYPE_STR = "str"
SUPPORT_TYPE = [TYPE_INT, TYPE_FLOAT, TYPE_STR]
TYPE_MAP = {TYPE_INT: np.dtype(np.int64), TYPE_FLOAT: np.dtype(np.float32), TYPE_STR: np.dtype(object)}
DEFAULT_MAP = {TYPE_INT: 0, TYPE_FLOAT: 0.0, TYPE_STR: ""}
TYPE_NAME = {v: k for k, v in TYPE_MAP.items()}
