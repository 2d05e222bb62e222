"""Microbench of rf_route_rows (dedup + owner routing) on the cfg4 request stream vs synthetic streams (diagnostics)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommendflow_amd.backend.encoder.sharded_encoder import GpuShardOps, build_slot_desc  # noqa: E402
from recommendflow_amd.backend.encoder.sparse_encoder import SlotSpec  # noqa: E402
from recommendflow_amd.config_parser.configuration import Configuration  # noqa: E402
from recommendflow_amd.runtime.batch import synthetic_batch  # noqa: E402


def timeit(fn, n=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n


def main():
    ops = GpuShardOps()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    conf = Configuration(os.path.join(root, "tests", "golden", "conf", "base_recall_sdpa.yaml"))
    feats = conf.features.hashing_features
    n_bins = 125_000_000 // (2 * len(feats))
    sp = [SlotSpec(f.name, n_bins, tuple(f.hash_seeds), f.pooling.value) for f in feats]
    desc, _ = build_slot_desc(sp, 128)
    d = ops.upload_desc(desc)
    b = synthetic_batch(8192, [bool(f.multivalued) for f in feats], seed=5).to("cuda")
    rows = ops.hash_rows(d, len(sp), b)
    res = {}
    streams = {
        "cfg4_requests": rows,
        "cfg4_sorted": torch.sort(rows).values,
        "cfg4_shuffled": rows[torch.randperm(rows.numel(), device="cuda")],
        "uniform_unique": torch.randperm(rows.numel(), device="cuda").to(torch.int64) * 131,
    }
    for name, r in streams.items():
        for P in (1, 8):
            R = 125_000_000 * P if name.startswith("cfg4") else int(r.max()) + 1
            ms = timeit(lambda: ops.route(r, P, R))
            c, _, _ = ops.route(r, P, R)
            res[f"{name}_P{P}"] = {"ms": round(ms, 4), "n": r.numel(), "uniq": int(c.sum())}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
