"""Typed feature list parsed from the `Features:` block (reference: config_parser/features.py).

A feature row is `group,type,tower,deal,vocab,embedding_dim,pooling,working` (feature_fields);
`group` expands through `feature_group` to member names or slot ids (features.py:208-228), slot ids
resolve through the slot map (:228). The parse rules follow Features.__parse_feature
(features.py:208-275); deviations:

* D-ellipsis: `[a, b, ..., c]` keeps `a` (the reference slices it away, features.py:224). Pass
  ``ellipsis="reference"`` to reproduce the reference's expansion exactly.
* D-cls: pooling `cls` == `first` (config_proto.FeaturePooling).
* D-slotmap: Spark type names in the slot map (config_utils.load_slot_map).
* Feature.type is the type NAME ('int' | 'float' | 'str') — the reference stores a TF dtype there and
  then compares it with the name in LookupEmbedding (preprocess_layers.py:148), which can never match
  (part of D-lookup).
"""
from __future__ import annotations

import os
from typing import Any, Dict, List, Optional, Union

import pandas as pd

from ..utils.str_parser import str2list
from .config_proto import (DEFAULT_MAP, SUPPORT_TYPE, TYPE_MAP, FeatureDeal, FeaturePooling, FeatureTower)
from .config_utils import load_slot_map, load_vocab

_NO_DIM_DEALS = (FeatureDeal.Numeric, FeatureDeal.Null, FeatureDeal.TokenId, FeatureDeal.Image,
                 FeatureDeal.Embedding, FeatureDeal.BertEncode)
_CONVERT = {"int": int, "float": float, "str": str}


class Feature:
    """One input feature (reference: features.py:17-89). Compares and hashes by name."""

    def __init__(self, name: str, field_name: str, ftype: str, tower: FeatureTower, deal: FeatureDeal,
                 vocab_size: int = -1, embedding_dim: int = -1, pooling: FeaturePooling = FeaturePooling.Null,
                 working: bool = True, vocabs: Union[List[Any], str, None] = None,
                 seeds: Union[List[int], int, None] = None, multivalued: Optional[bool] = None):
        t = ftype.lower()
        if t not in SUPPORT_TYPE:
            raise AssertionError(f"Feature type field only support: {SUPPORT_TYPE}, got {ftype}, field: {field_name}")
        self.name = name
        self.field_name = field_name
        self.type = t
        self.np_dtype = TYPE_MAP[t]
        self.tower = tower
        self.deal = deal
        self.vocab_size = vocab_size
        self.embedding_dim = embedding_dim
        self.pooling = pooling
        self.default = DEFAULT_MAP[t]
        self.working = working
        self.vocabs = [_CONVERT[t](v) for v in vocabs] if isinstance(vocabs, list) else vocabs
        self.hash_seeds = seeds
        # None = unknown (YAML-named feature); True/False from an ArrayType / scalar slot-map type
        self.multivalued = multivalued

    def is_auto_vocabs(self):
        return isinstance(self.vocabs, str) and self.vocabs.upper() == "__AUTO__"

    def is_token_id(self):
        return self.deal == FeatureDeal.TokenId

    def is_lookup(self):
        return self.deal == FeatureDeal.Lookup

    def is_hashing(self):
        return self.deal == FeatureDeal.Hashing

    def is_discrete(self):
        return self.deal == FeatureDeal.Discrete

    def is_image(self):
        return self.deal == FeatureDeal.Image

    def is_embedding(self):
        return self.deal == FeatureDeal.Embedding

    def is_numeric(self):
        return self.deal == FeatureDeal.Numeric

    def is_bert_encode(self):
        return self.deal == FeatureDeal.BertEncode

    def __hash__(self):
        return hash(self.name)

    def __eq__(self, other):
        return self.name == getattr(other, "name", other)

    def __lt__(self, other):
        return self.name < getattr(other, "name", other)

    def __gt__(self, other):
        return self.name > getattr(other, "name", other)

    def __repr__(self):
        return (f"Feature(name={self.name!r}, field={self.field_name!r}, type={self.type}, tower={self.tower.value}, "
                f"deal={self.deal.value}, vocab_size={self.vocab_size}, dim={self.embedding_dim}, "
                f"pooling={self.pooling.value}, working={self.working})")

    def to_dict(self) -> Dict[str, Any]:
        return {"name": self.name, "field_name": self.field_name, "type": self.type, "tower": self.tower.value,
                "deal": self.deal.value, "vocab_size": self.vocab_size, "embedding_dim": self.embedding_dim,
                "pooling": self.pooling.value, "working": self.working, "vocabs": self.vocabs,
                "hash_seeds": self.hash_seeds, "default": self.default}


def _match(feature: Feature, flag=None, field=None, tower=None, deal=None) -> bool:
    """All '|'-separated alternatives of each given criterion must hold (reference filter_feature :388-400)."""
    if flag and any(f not in feature.name for f in flag.split("|")):
        return False
    if tower and any(feature.tower != FeatureTower(t) for t in tower.split("|")):
        return False
    if deal and any(feature.deal != FeatureDeal(d) for d in deal.split("|")):
        return False
    if field and any(feature.field_name != f for f in field.split("|")):
        return False
    return True


def _exclude(feature: Feature, flag=None, field=None, tower=None, deal=None) -> bool:
    """False if any given alternative matches (reference except_feature :403-415)."""
    if flag and any(f in feature.name for f in flag.split("|")):
        return False
    if tower and any(feature.tower == FeatureTower(t) for t in tower.split("|")):
        return False
    if deal and any(feature.deal == FeatureDeal(d) for d in deal.split("|")):
        return False
    if field and any(feature.field_name == f for f in field.split("|")):
        return False
    return True


filter_feature = _match
except_feature = _exclude


def expand_ellipsis(names: List[Any], mode: str = "inclusive") -> List[Any]:
    """`[1, 4, ..., 7]` -> `[1, 4, 5, 6, 7]`; mode "reference" reproduces features.py:218-224 (drops `1`)."""
    names = list(names)
    while "..." in names:
        i = names.index("...")
        lo, hi = names[i - 1], names[i + 1]
        if not (isinstance(lo, int) and isinstance(hi, int)):
            raise AssertionError(f"Except int, got start={lo}, end={hi}.")
        if lo >= hi:
            raise AssertionError(f"Got start={lo}, end={hi}, start must smaller than end.")
        head = names[: max(0, i - 2)] if mode == "reference" else names[: i - 1]
        names = head + list(range(lo, hi + 1)) + names[i + 2:]
    return names


class Features:
    """Ordered feature list + query helpers (reference: features.py:92-385)."""

    def __init__(self, conf: Dict[str, Any], vocabs_map: Optional[Dict[str, Any]] = None,
                 seeds: Union[int, List[int], None] = None, slot_map_path: Optional[str] = None,
                 ellipsis: str = "inclusive"):
        self.conf = conf
        self.slot_map = load_slot_map(slot_map_path) if slot_map_path else {}
        self.ellipsis = ellipsis
        fields = conf["Features"]["feature_fields"]
        self.field_names = fields if isinstance(fields, list) else str2list(fields)
        self.vocabs_map = vocabs_map or {}
        self.seeds = seeds
        groups = conf["Features"].get("feature_group") or {}
        self.feature_group = {}
        for k, v in groups.items():
            if isinstance(v, str):
                self.feature_group[k.lower()] = str2list(v)
            elif isinstance(v, list):
                self.feature_group[k.lower()] = v
            else:
                raise Exception(f"Feature group except str or list, but got {type(v).__name__}.")
        self.features: List[Feature] = []
        owner: Dict[str, str] = {}
        for row in conf["Features"]["features"]:
            for f in self._parse_row(row):
                if f.name in owner:
                    raise Exception(f"Feature: [{self.field_names[0]}='{f.field_name}', name='{f.name}'] was conflicted with "
                                    f"Feature: [{self.field_names[0]}='{owner[f.name]}', name='{f.name}']")
                owner[f.name] = f.field_name
                self.features.append(f)
        self._refresh_deal_attrs()

    # -- parsing ------------------------------------------------------------------------------
    def _vocab(self, key: str, read: bool = True):
        v = self.vocabs_map[key]
        if isinstance(v, list):
            return v
        if isinstance(v, str):
            if not read:
                return v
            df = pd.read_csv(v, sep="\t", dtype=str, names=["vocab_id", "vocab_name"]).fillna("-1")
            vals = df[df.columns[0]].astype(str).unique().tolist()
            self.vocabs_map[key] = vals
            return vals
        raise Exception(f"Vocab={key}, value={v}, type={type(v)}, expect list or string.")

    def _parse_row(self, row: List[Any]) -> List[Feature]:
        d = dict(zip(self.field_names, row))
        if len(d) != len(self.field_names):
            raise AssertionError(f"Conf_str = {row} is invalid, please check.")
        group = str(d[self.field_names[0]]).lower()
        names = self.feature_group.get(group, [group])
        if any(isinstance(n, int) and not isinstance(n, bool) for n in names) and not self.slot_map:
            raise AssertionError("If you want to set feature slot id to locate feature, you must prepare slot map file.")
        names = expand_ellipsis(names, self.ellipsis)
        ftype = str(d["type"]).lower()
        for n in names:
            if isinstance(n, int) and n not in self.slot_map:
                raise Exception(f"Feature: [group={group}, slot_id={n}] was not in slot_map_file, please check!")
        typed = []
        for n in names:
            if isinstance(n, int):
                nm, t, multi = self.slot_map[n]
                typed.append((nm, t, multi))
            else:
                typed.append((n, ftype, None))
        tower = FeatureTower(str(d["tower"]).lower())
        deal = FeatureDeal(str(d["deal"]).lower())
        pooling = FeaturePooling(str(d["pooling"]).lower())
        working = str(d["working"]).lower() == "true"
        seeds = self.seeds if deal == FeatureDeal.Hashing else None
        vocab = d["vocab"].lower() if isinstance(d["vocab"], str) else d["vocab"]
        dim = -1 if deal in _NO_DIM_DEALS else int(d["embedding_dim"])

        vocabs: Any = None
        vocab_size = -1
        if deal in (FeatureDeal.Lookup, FeatureDeal.Discrete) and working:
            if not isinstance(vocab, str):
                vocabs, vocab_size = vocab, len(vocab)
            elif vocab.startswith("$"):
                vocabs = self._vocab(vocab[1:], read=True)
                vocab_size = len(vocabs)
            else:
                try:
                    vocab_size = int(vocab)
                    vocabs = "__AUTO__"
                    if vocab_size <= 0:
                        raise AssertionError("Vocab size must be set larger than 0, it means automatically adapt vocabs.")
                except ValueError as e:
                    if vocab == "null":
                        raise ValueError("Vocab or vocab size must be given in vocab field when feature deal method "
                                         "set in ['string_lookup', 'integer_lookup', 'discrete']")
                    if vocab in self.vocabs_map:
                        raise Exception(f"Feature field: {group} get vocab symbol: '{vocab}', you may want to set as '${vocab}'?")
                    raise Exception(f"Get unknown vocab symbol: '{vocab}', details: {e}.")
        elif deal == FeatureDeal.BertEncode:
            vocabs = self._vocab(vocab[1:], read=False) if vocab.startswith("$") else None
            if vocabs is None:
                raise Exception("Bert encode vocab must given.")
            if not os.path.isfile(vocabs):
                raise FileNotFoundError(f"bert dict vocab path: {vocabs} dose not exist.")
            vocab_size = len(load_vocab(vocabs))
        elif deal == FeatureDeal.Hashing:
            vocab_size = int(vocab)
        return [Feature(nm, group, t, tower, deal, vocab_size, dim, pooling, working, vocabs, seeds, multi)
                for nm, t, multi in typed]

    def _refresh_deal_attrs(self):
        for deal in FeatureDeal:
            if deal != FeatureDeal.Null:
                setattr(self, f"{deal.value}_features", self.get_deal_features(deal.value))
                setattr(self, f"{deal.value}_feature_names", self.get_deal_features(deal.value, True))

    # -- queries ------------------------------------------------------------------------------
    @property
    def train_features(self) -> List[Feature]:
        return [f for f in self.features if f.working]

    @property
    def train_feature_names(self) -> List[str]:
        return [f.name for f in self.features if f.working]

    def get_tower_features(self, tower: str, name_only: bool = False):
        t = FeatureTower(tower)
        return [f.name if name_only else f for f in self.train_features if f.tower == t]

    def get_deal_features(self, deal: str, name_only: bool = False):
        dl = FeatureDeal(deal)
        return [f.name if name_only else f for f in self.train_features if f.deal == dl]

    user_features = property(lambda self: self.get_tower_features("user"))
    user_feature_names = property(lambda self: self.get_tower_features("user", True))
    ad_features = property(lambda self: self.get_tower_features("ad"))
    ad_feature_names = property(lambda self: self.get_tower_features("ad", True))
    context_features = property(lambda self: self.get_tower_features("context"))
    context_feature_names = property(lambda self: self.get_tower_features("context", True))
    labels = property(lambda self: self.get_tower_features("label"))
    label_names = property(lambda self: self.get_tower_features("label", True))

    def _fields_map(self, keep, name_rlike=None, tower=None, deal=None, name_only=False, train_only=True):
        res: Dict[str, list] = {}
        for f in self.train_features if train_only else self.features:
            if keep(f, flag=name_rlike, tower=tower, deal=deal):
                res.setdefault(f.field_name, []).append(f.name if name_only else f)
        return res

    def get_fields_map(self, name_rlike=None, tower=None, deal=None, name_only=False, train_only=True):
        return self._fields_map(_match, name_rlike, tower, deal, name_only, train_only)

    def get_fields_map_except(self, name_rlike=None, tower=None, deal=None, name_only=False, train_only=True):
        return self._fields_map(_exclude, name_rlike, tower, deal, name_only, train_only)

    def get_fields(self, name_rlike=None, tower=None, deal=None, train_only=True):
        return list(self.get_fields_map(name_rlike, tower, deal, True, train_only))

    def get_fields_except(self, name_rlike=None, tower=None, deal=None, train_only=True):
        return list(self.get_fields_map_except(name_rlike, tower, deal, True, train_only))

    def index_of_fields(self, fields_list, name_rlike=None, tower=None, deal=None, train_only=True):
        allf = self.get_fields(name_rlike, tower, deal, train_only)
        return [allf.index(i) for i in fields_list]

    def get_fields_feature_tuple(self, name_rlike=None, tower=None, deal=None, name_only=False, train_only=True):
        return list(self.get_fields_map(name_rlike, tower, deal, name_only, train_only).values())

    def get_feature(self, name: str) -> Feature:
        for f in self.train_features:
            if f.name == name:
                return f
        raise Exception(f"Feature name = {name} dose not exist.")

    def feature_filter(self, name_rlike=None, field=None, tower=None, deal=None, train_only=True):
        return [f for f in (self.train_features if train_only else self.features) if _match(f, name_rlike, field, tower, deal)]

    def feature_except(self, name_rlike=None, field=None, tower=None, deal=None, train_only=True):
        return [f for f in (self.train_features if train_only else self.features) if _exclude(f, name_rlike, field, tower, deal)]

    get_features = feature_filter

    def index_of_features(self, names, name_rlike=None, field=None, tower=None, deal=None, train_only=True):
        allf = [f.name for f in self.feature_filter(name_rlike, field, tower, deal, train_only)]
        return [allf.index(n) for n in names]

    def get_features_by_name(self, names=None, prefix: str = "", suffix: str = ""):
        if names:
            return [f for f in self.train_features if f.name in names]
        if prefix:
            return [f for f in self.train_features if f.name.startswith(prefix)]
        if suffix:
            return [f for f in self.train_features if f.name.endswith(suffix)]
        raise ValueError("Names, prefix or suffix must given only one.")

    def _set_status(self, name: str = "", field: str = "", status: bool = True):
        if not (name or field):
            raise AssertionError("Name or field must given at least one of them")
        for f in self.features:
            if (name and f.name == name) or (not name and field and f.field_name == field):
                f.working = status
        self._refresh_deal_attrs()

    def set_feature_valid(self, name: str = "", field: str = ""):
        self._set_status(name, field, True)

    def set_feature_invalid(self, name: str = "", field: str = ""):
        self._set_status(name, field, False)

    def contain(self, name: str) -> bool:
        return any(f.name == name for f in self.train_features)

    def contain_field(self, field: str) -> bool:
        return any(f.field_name == field for f in self.train_features)

    def contain_deal(self, deal: FeatureDeal) -> bool:
        return any(f.deal == deal for f in self.train_features)

    def get_image_features(self):
        return self.get_deal_features("image")

    def get_embedding_features(self):
        return self.get_deal_features("embedding")

    def __iter__(self):
        return iter(self.features)

    def __len__(self):
        return len(self.features)
