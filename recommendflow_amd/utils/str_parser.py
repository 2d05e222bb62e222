"""String helpers of the config surface.

Mirrors utils/str_parser.py of the reference (str2list :30-31, str2dict :34-44) for the subset the
config parser uses; tensorflow-typed conversions are dropped (no TF here).
"""
from __future__ import annotations

from typing import Any, Callable, Dict, List, Union

import numpy as np


def _convert(kind: Union[str, Callable[[str], Any]], text: str) -> Any:
    if callable(kind):
        return kind(text)
    table = {"str": str, "int": int, "float": float, "float32": np.float32, "float64": np.float64,
             "set": set, "list": list}
    key = kind.lower()
    if key == "dict":
        if "=" not in text:
            raise ValueError("dict conversion needs 'k=v' items separated by ';'")
        return {item.strip().split("=")[0]: "=".join(item.strip().split("=")[1:]) for item in text.strip().split(";")}
    if key not in table:
        raise ValueError(f"type function: `{kind}` is not supported")
    return table[key](text)


def str2list(text: str, sep: str = ",", trans_type: Union[type, str] = str) -> List[Any]:
    """'a, b,,c' -> ['a', 'b', 'c'] (blank items dropped, items stripped, then converted)."""
    return [_convert(trans_type, piece.strip()) for piece in text.split(sep) if piece.strip()]


def str2dict(text: str, trans_type: Union[type, str] = str) -> Dict[str, Any]:
    """'a=1;b=2' -> {'a': '1', 'b': '2'}."""
    out: Dict[str, Any] = {}
    for item in text.strip().split(";"):
        k, v = item.strip().split("=")
        out[k.strip()] = _convert(trans_type, v.strip())
    return out


def str2bool(text: str) -> bool:
    return text.lower() == "true"
