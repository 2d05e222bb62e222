"""cfg4 route stage at P ranks on one GPU (diagnostics; rocprofv3 --kernel-trace target): ShardedFusedEncoder as
rank 0 of P with the LoopbackComm, cfg2 slots, shard_rows x dim fp32 shard, B examples; times route_exchange and
prints the per-step ms. python tools/route_probe.py [--P 8] [--batch 8192] [--shard-rows 125000000] [--reps 20]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch

from recommendflow_amd.backend.encoder.sharded_encoder import LoopbackComm, ShardedFusedEncoder
from recommendflow_amd.backend.encoder.sparse_encoder import SlotSpec
from recommendflow_amd.config_parser.configuration import Configuration
from recommendflow_amd.runtime.batch import synthetic_batch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=8)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--shard-rows", type=int, default=125_000_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    conf = Configuration(os.path.join(ROOT, "tests", "golden", "conf", "base_recall_sdpa.yaml"))
    feats = conf.features.hashing_features
    n_bins = a.shard_rows * a.P // (2 * len(feats))
    sp = [SlotSpec(f.name, n_bins, tuple(f.hash_seeds), f.pooling.value) for f in feats]
    multi = [bool(f.multivalued) for f in feats]
    enc = ShardedFusedEncoder(sp, a.dim, 0, a.P, comm=LoopbackComm(a.P), seed=2024)
    batches = [synthetic_batch(a.batch, multi, seed=4321 + i).to("cuda") for i in range(2)]
    for i in range(3):
        enc.route_exchange(batches[i % 2], local_fast=enc.local_fast)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.reps):
        r, _ = enc.route_exchange(batches[i % 2], local_fast=enc.local_fast)
    torch.cuda.synchronize()
    print(f"route P={a.P}: {(time.perf_counter() - t0) / a.reps * 1e3:.4f} ms/step, requests after dedup {r.n_requests}, "
          f"logical rows {r.n_logical}")


if __name__ == "__main__":
    main()
