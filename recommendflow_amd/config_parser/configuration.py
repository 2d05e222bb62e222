"""YAML config -> Configuration (reference: config_parser/configuration.py:16-270).

Grammar kept verbatim (conf/CONF_README.md):
* every string `$key` is replaced by the first value found under `key` anywhere in the YAML tree
  (depth-first, first match, configuration.py:104-122); a string that is exactly `$key` takes the
  value itself (any type), a `$key` embedded in a longer string is split at punctuation other than
  `_` and `$` and must resolve to a scalar (configuration.py:124-162);
* substitution walks the tree in YAML order and rewrites it in place, so later keys see earlier
  keys already substituted (configuration.py:170-207);
* `Features.features` / `Experiments.experiments` are whitespace-separated CSV rows (:164-168).

Deviation D-slotmap: the reference never passes a slot map (configuration.py:30). The build reads
``slot_map_path`` from the argument, else from a `slot_map` key in the YAML, else from the side-car
``<config stem>.feature.map`` next to the YAML.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional

import pandas as pd
import yaml

from ..utils.str_parser import str2dict, str2list
from .config_proto import FeatureDeal
from .config_utils import is_punctuation, side_car_slot_map
from .features import Features

_SEP = "\x00"


class Configuration:
    """Levels: Features, Networks, Datasets, Experiments, ... (free-form except Features)."""

    def __init__(self, config_path: str, slot_map_path: Optional[str] = None, ellipsis: str = "inclusive"):
        self.config_path = config_path
        with open(config_path, encoding="utf-8") as f:
            self.conf = yaml.safe_load(f.read())
        self._split_rows()
        self._substitute_tree()
        slot_map = slot_map_path or self._find("slot_map") or side_car_slot_map(config_path)
        self.features = Features(self.conf, self.get_conf_value("vocabs"), self.get_conf_value("seeds"),
                                 slot_map_path=slot_map or None, ellipsis=ellipsis)
        self.networks = self.conf.get("Networks", {}) or {}
        self.exp_conf = self.conf.get("Experiments")
        if not self.exp_conf or not self.exp_conf.get("experiments"):
            self.experiment_field: List[str] = []
            self.experiments = pd.DataFrame()
        else:
            fields = self.exp_conf["experiment_fields"]
            self.experiment_field = str2list(fields) if isinstance(fields, str) else list(fields)
            if self.experiment_field[0] != "exp_id":
                raise AssertionError("The first field must be exp_id")
            rows = [self._parse_exp(r) for r in self.exp_conf["experiments"]]
            self.experiments = pd.DataFrame(rows, columns=self.experiment_field).set_index("exp_id")
        self.need_parse_second = self.features.contain_deal(FeatureDeal.Image) or self.features.contain_deal(FeatureDeal.Embedding)

    # -- public -------------------------------------------------------------------------------
    @property
    def train_features(self):
        return self.features.train_features

    @property
    def train_feature_names(self):
        return self.features.train_feature_names

    def get_conf_value(self, key: str, dtype: type = None):
        v = self._find(key)
        if v is None:
            raise KeyError(f"Could not find key='{key}' in configuration.")
        return dtype(v) if dtype else v

    def active_experiment(self, exp_id):
        """Apply an experiment row's `±feature` toggles (configuration.py:76-102); name before field."""
        if "features" in self.experiments.columns:
            toggles = self.experiments.loc[exp_id]["features"]
            if not isinstance(toggles, list):
                raise AssertionError("Experiments field features must be a feature name list.")
            for t in toggles:
                if t[0] not in "+-":
                    raise ValueError("Feature first latter must be '+/-' represent feature valid/invalid.")
                on, key = t[0] == "+", t[1:]
                by_name = any(f.name == key for f in self.features.features)
                if on:
                    self.features.set_feature_valid(name=key) if by_name else self.features.set_feature_valid(field=key)
                else:
                    self.features.set_feature_invalid(name=key) if by_name else self.features.set_feature_invalid(field=key)
        self.need_parse_second = self.features.contain_deal(FeatureDeal.Image) or self.features.contain_deal(FeatureDeal.Embedding)
        return self.experiments.loc[exp_id].to_dict()

    def print_features(self, scale: str = "train", blank_size: int = 2):
        feats = self.features.features if scale == "all" else self.train_features
        rows = [[f"name={f.name}", f"field={f.field_name}", f"tower={f.tower.value}", f"deal={f.deal.value}",
                 f"type={f.type}", f"working={f.working}"] for f in feats]
        widths = [max((len(r[c]) for r in rows), default=0) for c in range(6)]
        for i, r in enumerate(rows):
            cells = [r[c] + " " * (widths[c] - len(r[c]) + blank_size) for c in range(5)] + [r[5]]
            print(f"Feature {i}:\t[{''.join(cells)}]")

    # -- internals ----------------------------------------------------------------------------
    def _find(self, key: str):
        def walk(d: Dict[str, Any]):
            if key in d:
                return d.get(key)
            for v in d.values():
                if isinstance(v, dict):
                    r = walk(v)
                    if r is not None:
                        return r
            return None

        return walk(self.conf)

    def _split_rows(self):
        self.conf["Features"]["features"] = [line.split(",") for line in str(self.conf["Features"]["features"]).split()]
        exp = self.conf.get("Experiments")
        if isinstance(exp, dict):
            rows = exp.get("experiments")
            exp["experiments"] = [line.split(",") for line in str(rows).split()] if rows else []

    def _set_value(self, v: Any):
        if not isinstance(v, str):
            return v
        plain = not any(is_punctuation(c, "_$") for c in v)
        if plain and v.startswith("$"):
            return self.get_conf_value(v[1:])
        if "$" in v:
            return self._set_str(v)
        return v

    def _set_str(self, v: Any):
        if not isinstance(v, str):
            return v
        pieces: List[str] = []
        buf = ""
        for c in v:
            if c == "$" or is_punctuation(c, "_$"):
                pieces.append(buf)
                buf = c
            else:
                buf += c
        pieces.append(buf)
        out = []
        for p in pieces:
            val = self.get_conf_value(p[1:]) if p.startswith("$") else p
            if not isinstance(val, (str, int, float, bool)):
                raise Exception(f"'$' symbol in sub string only support [str, int, float, bool], got {type(val).__name__}. "
                                f"map_value: {val}.")
            out.append(str(val))
        return "".join(out)

    def _substitute_tree(self):
        def sub_list(items):
            res = []
            for i in items:
                if isinstance(i, list):
                    res.append(sub_list(i))
                elif isinstance(i, dict):
                    res.append(sub_dict(i))
                else:
                    res.append(self._set_value(i))
            return res

        def sub_dict(d):
            for k, v in d.items():
                if isinstance(v, dict):
                    sub_dict(v)
                elif isinstance(v, list):
                    res = []
                    for i in v:
                        s = self._set_value(i)
                        if isinstance(s, (int, str, float)):
                            res.append(s)
                        elif isinstance(s, list):
                            res.append(sub_list(s))
                        else:
                            raise ValueError(f"'$' symbol in list must be [str, int, float], got {type(s).__name__}, sub_i: {s}")
                    d[k] = res
                else:
                    d[k] = self._set_value(v)
            return d

        sub_dict(self.conf)

    def _parse_exp(self, row: List[Any]):
        try:
            exp_id = int(row[0])
        except Exception as e:  # noqa: BLE001
            raise Exception(f"Experiment first col must be integer type exp_id, got {type(row[0]).__name__}, detail: {e}")
        out: List[Any] = [exp_id]
        for e in row[1:]:
            if not isinstance(e, str):
                out.append(e)
            elif e.startswith("{") and e.endswith("}"):
                out.append(str2dict(e[1:-1]))
            elif (e.startswith("[") and e.endswith("]")) or (e.startswith("(") and e.endswith(")")):
                out.append(str2list(e[1:-1], sep=";"))
            else:
                out.append(self._set_str(e))
        return out
