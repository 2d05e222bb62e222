"""Runs only bench.py's feature-pipe leg (bench_pipe) on cuda:0 and prints its JSON."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from recommendflow_amd.backend.encoder.sparse_encoder import FusedSparseEncoder, SlotSpec  # noqa: E402
from recommendflow_amd.config_parser.configuration import Configuration  # noqa: E402

args = bench.parse()
conf = Configuration(os.path.join(bench.ROOT, "tests", "golden", "conf", "base_recall_sdpa.yaml"))
feats = conf.features.hashing_features
n_bins = args.table_rows // (2 * len(feats))
specs = [SlotSpec(f.name, n_bins, tuple(f.hash_seeds), f.pooling.value) for f in feats]
enc = FusedSparseEncoder(specs, args.dim, table_dtype=torch.float32, seed=2023)
print(json.dumps(bench.bench_pipe(args, enc, specs, [bool(f.multivalued) for f in feats]), indent=1))
