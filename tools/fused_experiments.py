"""Layout experiments on the cfg2 fused kernel (diagnostics): output layout [B][S*2D] (the API's) vs
slot-major [S][B][2D] (each 64-example item writes 32 KB contiguously), and the ablation bits."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from recommendflow_amd.backend.encoder.sparse_encoder import FusedSparseEncoder, SlotSpec  # noqa: E402
from recommendflow_amd.config_parser.configuration import Configuration  # noqa: E402
from recommendflow_amd.runtime import lib as L  # noqa: E402
from recommendflow_amd.runtime.batch import synthetic_batch  # noqa: E402
from tools.kbench import timeit  # noqa: E402


def main():
    conf = Configuration(os.path.join(ROOT, "tests", "golden", "conf", "base_recall_sdpa.yaml"))
    feats = conf.features.hashing_features
    S, B, D = len(feats), 4096, 64
    specs = [SlotSpec(f.name, 10_000_000 // (2 * S), tuple(f.hash_seeds), "sum") for f in feats]
    enc = FusedSparseEncoder(specs, D, seed=1)
    hb = synthetic_batch(B, [bool(f.multivalued) for f in feats], seed=1234)
    db = hb.to("cuda")
    by = enc.algorithmic_bytes(hb)
    res = {}
    out = torch.empty((B, enc.out_width), device="cuda")

    def run(desc, o, stride, flags=0):
        L.call("rf_diag_fused_hash_embed_fwd", L.ptr(desc), S, L.ptr(db.tok_bytes), L.ptr(db.tok_off), L.ptr(db.bag_off),
               L.ptr(db.lmax), B, L.ptr(enc.table), 0, enc.table.shape[0], D, L.ptr(o), 0, stride, flags, None,
               L.stream_ptr())

    res["api_layout"] = timeit(lambda: run(enc.desc, out, enc.out_width))
    h = enc.host_desc.copy()
    h["out_off"] = np.arange(S) * B * 2 * D
    dsm = torch.from_numpy(h.view(np.uint8).copy()).cuda()
    res["slot_major_layout"] = timeit(lambda: run(dsm, out, 2 * D))
    for tag, bits in [("nohash", 1 << 12), ("nopool", 1 << 13), ("nopad", 1 << 14)]:
        res[f"abl_{tag}"] = timeit(lambda: run(enc.desc, out, enc.out_width, bits))
    res = {k: {"ms": round(v, 4), "GBs": round(by / v / 1e6, 1)} for k, v in res.items()}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
