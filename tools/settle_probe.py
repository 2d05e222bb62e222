"""Why the headline kernel's first launches are slower: per-launch HIP-event durations of the
cfg2 fused encoder for the first N launches of a process, then again after the GPU idled (sleep), then after the
GPU ran an unrelated dense workload (fp32 GEMMs for ~0.3 s, no table traffic), then after a pass over the table
rows' pages by another kernel (a full-table copy). Clock ramp shows as a slope after idle that a busy phase removes;
cache / TLB warm-up as a slope that only touching the table removes. Diagnostics only.

usage: python tools/settle_probe.py [--n 100]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100)
    a = ap.parse_args()
    from recommendflow_amd.backend.encoder.sparse_encoder import FusedSparseEncoder, SlotSpec
    from recommendflow_amd.config_parser.configuration import Configuration
    from recommendflow_amd.runtime.batch import synthetic_batch

    conf = Configuration(os.path.join(ROOT, "tests", "golden", "conf", "base_recall_sdpa.yaml"))
    feats = conf.features.hashing_features
    S = len(feats)
    n_bins = 10_000_000 // (2 * S)
    specs = [SlotSpec(f.name, n_bins, tuple(f.hash_seeds), f.pooling.value) for f in feats]
    enc = FusedSparseEncoder(specs, 64, table_dtype=torch.float32, seed=2023)
    multi = [bool(f.multivalued) for f in feats]
    dev = [synthetic_batch(4096, multi, seed=1234 + i).to("cuda") for i in range(4)]
    out = torch.empty((4096, enc.out_width), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()

    def series(tag):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.n)]
        for i in range(a.n):
            ev[i][0].record()
            enc(dev[i % 4], out=out)
            ev[i][1].record()
        torch.cuda.synchronize()
        us = [s.elapsed_time(e) * 1e3 for s, e in ev]
        win = lambda lo, hi: round(sum(us[lo:hi]) / len(us[lo:hi]), 1)
        rec = {"phase": tag, "first5": [round(x, 1) for x in us[:5]], "l5_24": win(5, 25), "l25_49": win(25, 50),
               "l50_99": win(50, min(100, a.n))}
        print(json.dumps(rec), flush=True)
        return us

    series("cold (process start, after table init)")
    time.sleep(2.0)
    series("after 2 s idle")
    x = torch.randn(4096, 8192, device="cuda")
    w = torch.randn(8192, 4096, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        torch.mm(x, w)
    torch.cuda.synchronize()
    series("right after 0.3 s of fp32 GEMMs (no table traffic)")
    time.sleep(2.0)
    t2 = enc.table.clone()
    torch.cuda.synchronize()
    del t2
    series("after 2 s idle + one table copy")
    time.sleep(2.0)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        torch.mm(x, w)
    enc(dev[0], out=out)
    torch.cuda.synchronize()
    series("after 2 s idle + 0.3 s GEMMs + 1 launch")


if __name__ == "__main__":
    main()
