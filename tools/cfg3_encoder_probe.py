"""cfg3 sparse-encoder ablations (diagnostics): one tower = 100 single-valued slots x 1M bins x 2 tables,
D = 64 bf16, B = 4096, through rf_fused_hash_embed_fwd with the kernel's ablation flags
(1<<12: rows from a cheap formula instead of SipHash; 1<<13: hash only, no gather/pool)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch

from recommendflow_amd.backend.encoder.sparse_encoder import FusedSparseEncoder, SlotSpec
from recommendflow_amd.runtime.batch import synthetic_batch


def main():
    B, Ls = 4096, 100
    specs = [SlotSpec(f"u{i:03d}", 1_000_000, (2022, 2023)) for i in range(Ls)]
    enc = FusedSparseEncoder(specs, 64, table_dtype=torch.bfloat16, seed=3)
    hb = synthetic_batch(B, [False] * Ls, seed=77, slot_ids=range(Ls)).to("cuda")
    out = torch.empty((B, enc.out_width), dtype=torch.bfloat16, device="cuda")
    res = {}
    for name, fl, st in (("single_token_kernel", 0, True), ("general_kernel_lean", 0, False),
                         ("general_phase2", 1 << 15, False), ("no_hash", 1 << 12, False), ("hash_only", 1 << 13, False)):
        enc.extra_flags = fl
        enc.single_token = st

        def run():
            enc(hb, out=out)

        for _ in range(20):
            run()
        s = [torch.cuda.Event(enable_timing=True) for _ in range(30)]
        e = [torch.cuda.Event(enable_timing=True) for _ in range(30)]
        for i in range(30):
            s[i].record()
            run()
            e[i].record()
        torch.cuda.synchronize()
        res[name] = round(sorted(a.elapsed_time(b) for a, b in zip(s, e))[15], 4)
    # cfg2 (the headline kernel): 229 slots, 198 of them single-valued
    from recommendflow_amd.config_parser.configuration import Configuration

    conf = Configuration(os.path.join(ROOT, "tests", "golden", "conf", "base_recall_sdpa.yaml"))
    feats = conf.features.hashing_features
    nb = 10_000_000 // (2 * len(feats))
    enc2 = FusedSparseEncoder([SlotSpec(f.name, nb, tuple(f.hash_seeds), f.pooling.value) for f in feats], 64, seed=2023)
    hb2 = synthetic_batch(4096, [bool(f.multivalued) for f in feats], seed=1234).to("cuda")
    out2 = torch.empty((4096, enc2.out_width), device="cuda")
    for name, fl in (("cfg2_full", 0), ("cfg2_general_phase2", 1 << 15), ("cfg2_xcd_order", 1 << 11),
                     ("cfg2_full_again", 0)):
        enc2.extra_flags = fl
        for _ in range(60):
            enc2(hb2, out=out2)
        s = [torch.cuda.Event(enable_timing=True) for _ in range(50)]
        e = [torch.cuda.Event(enable_timing=True) for _ in range(50)]
        for i in range(50):
            s[i].record()
            enc2(hb2, out=out2)
            e[i].record()
        torch.cuda.synchronize()
        res[name] = round(sorted(a.elapsed_time(b) for a, b in zip(s, e))[25], 4)
    by = 2 * B * Ls * 128 + B * Ls * 256 + int(hb.tok_bytes.numel()) + 4 * hb.n_tokens
    res["single_token_GBs"] = round(by / res["single_token_kernel"] / 1e6, 1)
    res["general_lean_GBs"] = round(by / res["general_kernel_lean"] / 1e6, 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
