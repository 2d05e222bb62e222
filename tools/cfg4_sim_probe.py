"""cfg4 rank 0 of P on one GPU (diagnostics; rocprofv3 --kernel-trace target): bench.py's bench_sharded_sim leg
alone (route -> id exchange -> owner gather -> row exchange -> pool, LoopbackComm) and its JSON.
python tools/cfg4_sim_probe.py [--P 8] [--shard-batch 8192] [--shard-rows 125000000] [--steps 25]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from recommendflow_amd.backend.encoder.sparse_encoder import SlotSpec  # noqa: E402
from recommendflow_amd.config_parser.configuration import Configuration  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=8)
    ap.add_argument("--shard-batch", type=int, default=8192)
    ap.add_argument("--shard-rows", type=int, default=125_000_000)
    ap.add_argument("--shard-dim", type=int, default=128)
    ap.add_argument("--steps", type=int, default=25)
    a = ap.parse_args()
    conf = Configuration(os.path.join(ROOT, "tests", "golden", "conf", "base_recall_sdpa.yaml"))
    feats = conf.features.hashing_features
    specs = [SlotSpec(f.name, 1, tuple(f.hash_seeds), f.pooling.value) for f in feats]
    multi = [bool(f.multivalued) for f in feats]
    res = bench.bench_sharded_sim(a, specs, multi, a.P)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
