"""Micro-benchmarks for the sparse path (diagnostics, not the headline bench).

Times with HIP events on the launch stream: the fused kernel on cfg2 (Zipf and uniform ids), the
hash-only kernel over the same tokens, a pure row gather of the same rows, and a device copy.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np
import torch

from recommendflow_amd.backend.encoder.sparse_encoder import FusedSparseEncoder, SlotSpec
from recommendflow_amd.config_parser.configuration import Configuration
from recommendflow_amd.runtime import lib as L
from recommendflow_amd.runtime.batch import synthetic_batch


def timeit(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    s = [torch.cuda.Event(enable_timing=True) for _ in range(reps)]
    e = [torch.cuda.Event(enable_timing=True) for _ in range(reps)]
    for i in range(reps):
        s[i].record()
        fn()
        e[i].record()
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in zip(s, e))
    return t[len(t) // 2]


def main():
    res = {}
    conf = Configuration(os.path.join(ROOT, "tests", "golden", "conf", "base_recall_sdpa.yaml"))
    feats = conf.features.hashing_features
    S = len(feats)
    nb = 10_000_000 // (2 * S)
    specs = [SlotSpec(f.name, nb, tuple(f.hash_seeds), "sum") for f in feats]
    enc = FusedSparseEncoder(specs, 64, seed=1)
    multi = [bool(f.multivalued) for f in feats]
    for name, kw in [("zipf", {}), ("uniform", {"uniform": True})]:
        hb = synthetic_batch(4096, multi, seed=1234, **kw)
        db = hb.to("cuda")
        out = torch.empty((4096, enc.out_width), device="cuda")
        by = enc.algorithmic_bytes(hb)
        ms = timeit(lambda: enc(db, out=out))
        res[f"fused_{name}"] = {"ms": ms, "GBs": by / ms / 1e6}
        if name == "zipf":
            for tag, bits in [("nohash", 1 << 12), ("nopool", 1 << 13), ("nopad", 1 << 14), ("nohash_nopad", (1 << 12) | (1 << 14))]:
                enc.extra_flags = bits
                res[f"fused_zipf_abl_{tag}"] = {"ms": timeit(lambda: enc(db, out=out)), "GBs": 0}
        enc.extra_flags = 0
    # scalar-only batch (every slot L = 1)
    hb1 = synthetic_batch(4096, [False] * S, seed=7)
    db1 = hb1.to("cuda")
    out = torch.empty((4096, enc.out_width), device="cuda")
    ms = timeit(lambda: enc(db1, out=out))
    res["fused_scalar_only"] = {"ms": ms, "GBs": enc.algorithmic_bytes(hb1) / ms / 1e6}
    # hash-only over the cfg2 tokens
    hb = synthetic_batch(4096, multi, seed=1234)
    db = hb.to("cuda")
    bins = torch.empty(hb.n_tokens, dtype=torch.int64, device="cuda")
    ms = timeit(lambda: L.call("rf_siphash_bucket", L.ptr(db.tok_bytes), L.ptr(db.tok_off), hb.n_tokens, 2022, 2022,
                               21834, 1, L.ptr(bins), L.stream_ptr()))
    res["hash_only_1key"] = {"ms": ms, "Mtok_s": hb.n_tokens / ms / 1e3}
    # emit-idx path gives the real rows; pure gather of all 2*Ntok rows into a dense buffer
    _, idx = enc(db, emit_idx=True)
    seg = torch.from_numpy(np.repeat(enc.host_desc["row_base"], np.diff(hb.bag_off).reshape(4096, S).sum(0) * 0 + 1, axis=0)).cuda()
    lens = torch.from_numpy(np.diff(hb.bag_off).astype(np.int64)).cuda()
    slot_of_tok = torch.repeat_interleave(torch.arange(4096 * S, device="cuda") % S, lens)
    rb = torch.from_numpy(enc.host_desc["row_base"].astype(np.int64)).cuda()
    rows = (idx + rb[slot_of_tok]).reshape(-1).contiguous()
    g = torch.empty((rows.numel(), 64), device="cuda")
    ms = timeit(lambda: L.call("rf_gather_rows", L.ptr(rows), rows.numel(), L.ptr(enc.table), 0, enc.table.shape[0], 64,
                               L.ptr(g), L.stream_ptr()))
    res["gather_rows"] = {"ms": ms, "GBs": 2 * rows.numel() * 256 / ms / 1e6, "rows": rows.numel()}
    srt = torch.sort(rows).values
    ms = timeit(lambda: L.call("rf_gather_rows", L.ptr(srt), srt.numel(), L.ptr(enc.table), 0, enc.table.shape[0], 64,
                               L.ptr(g), L.stream_ptr()))
    res["gather_rows_sorted"] = {"ms": ms, "GBs": 2 * srt.numel() * 256 / ms / 1e6}
    x = torch.empty(2 * 1024 ** 3 // 4, device="cuda")
    y = torch.empty_like(x)
    ms = timeit(lambda: y.copy_(x))
    res["copy_2GiB"] = {"ms": ms, "GBs": 2 * x.numel() * 4 / ms / 1e6}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
