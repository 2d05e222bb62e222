"""ESIM gather-form attention micro-benchmark (diagnostics): rf_esim_gather_fwd at cfg3's configured shape
(100 + 100 single-valued slots, 1 M bins per hash, 2 x 200 M x 64 bf16 fused tables = 51.2 GB, B = 4096, L = 100,
d = 128). The ids come from rf_single_token_ids_fwd over synthetic Zipf(1.1) (or --uniform) batches; two batches
alternate, HIP-event timed on the launch stream. Also the rocprofv3 --pmc target for this kernel.
    python tools/esim_gather_probe.py [--reps 50] [--uniform] [--batch 4096] [--bins 1000000]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch

from recommendflow_amd.backend.encoder.sparse_encoder import SlotSpec
from recommendflow_amd.models.ranking.esim import Esim
from recommendflow_amd.runtime.batch import synthetic_batch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--L", type=int, default=100)
    ap.add_argument("--bins", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--uniform", action="store_true")
    ap.add_argument("--stamp", action="store_true", help="one stamped launch: per-phase shader-clock cycles")
    a = ap.parse_args()
    B, Ls = a.batch, a.L
    user = [SlotSpec(f"u{i:03d}", a.bins, (2022, 2023)) for i in range(Ls)]
    ad = [SlotSpec(f"a{i:03d}", a.bins, (2022, 2023)) for i in range(Ls)]
    model = Esim(user, ad, n_dense=16, dim=64, table_dtype=torch.bfloat16, seed=3)
    hu = [synthetic_batch(B, [False] * Ls, seed=77 + i, slot_ids=range(Ls), uniform=a.uniform).to("cuda") for i in range(2)]
    ha = [synthetic_batch(B, [False] * Ls, seed=99 + i, slot_ids=range(Ls, 2 * Ls), uniform=a.uniform).to("cuda")
          for i in range(2)]
    ids = [model.token_ids(hu[p], ha[p]) for p in (0, 1)]
    pooled = torch.empty((B, model.pooled_width), device="cuda")
    for i in range(10):
        model.attention_gather(*ids[i & 1], pooled)
    torch.cuda.synchronize()
    s = [torch.cuda.Event(enable_timing=True) for _ in range(a.reps)]
    e = [torch.cuda.Event(enable_timing=True) for _ in range(a.reps)]
    for i in range(a.reps):
        s[i].record()
        model.attention_gather(*ids[i & 1], pooled)
        e[i].record()
    torch.cuda.synchronize()
    if a.stamp:
        stamp_report(model, ids[0], pooled, B)
    t = sorted(x.elapsed_time(y) for x, y in zip(s, e))
    ms = t[len(t) // 2]
    flops = 2 * Ls * Ls * model.d * 3 * B
    by = 2 * B * Ls * model.d * 2 + B * 6 * model.d * 4
    print(json.dumps({"kernel": "esim2_kernel<GATHER>", "ms_median": round(ms, 4), "ms_min": round(t[0], 4),
                      "TFLOPs": round(flops / ms / 1e9, 1), "GBs": round(by / ms / 1e6, 1), "batch": B, "L": Ls,
                      "d": model.d, "bins": a.bins, "ids": "uniform" if a.uniform else "zipf1.1",
                      "checksum": float(pooled[:, model.d_emb:].double().sum())}))


def stamp_report(model, ids, pooled, B):
    """rf_diag_esim_gather_stamped once: mean shader cycles per phase and wave-example, split by the wave's stripe
    count (2 or 1 of the 7 stripes at L = 100), in the loop's order of points."""
    import numpy as np

    from recommendflow_amd.runtime import lib as L

    cus = torch.cuda.get_device_properties(0).multi_processor_count
    split = False  # the d-split 3-workgroup kernel (v8) was measured slower and removed (profiles/r04)
    grid = min(B, (3 if split else 2) * cus)
    EX, P = -(-B // grid) + 1, 10
    st = torch.zeros(grid * 4 * EX * P, dtype=torch.int32, device="cuda")
    eq, ea = model.enc_q, model.enc_a
    L.call("rf_diag_esim_gather_stamped", L.ptr(ids[0]), L.ptr(ids[1]), L.ptr(eq.table), eq.table.shape[0], L.ptr(ea.table),
           ea.table.shape[0], L.DT_BF16, B, model.L, model.d, L.ptr(pooled), pooled.stride(0), model.d_emb, L.ptr(st), EX,
           L.stream_ptr(None))
    torch.cuda.synchronize()
    t = st.cpu().numpy().view(np.uint32).astype(np.int64).reshape(grid, 4, EX, P)
    order = [0, 1, 7, 8, 9, 2, 3, 4, 5, 6]
    names = ["issue next loads", "scores (E^T)", "softmax", "P@V+stats side 0", "P@V+stats side 1", "compute barrier",
             "stage next images", "reduce pooled", "second barrier"]
    if split:  # esim_split_kernel's points (rf_attn.hip)
        order = [0, 1, 2, 3, 4, 5, 6, 7]
        names = ["P1 scores over hash-0 half (+ loads issued)", "barrier, stage hash-1 half, barrier",
                 "P2 scores over hash-1 half + softmax", "P2 P@V + stats cols 64..127", "barrier, stage hash-0, barrier",
                 "P3 P@V + stats cols 0..63", "barrier, stage next, reduce, barrier"]
    rows = {1: [], 2: []}
    for g in range(grid):
        n_g = len(range(g, B, grid))
        for w in range(4):
            for k in range(n_g):
                sp0 = (w + k) & 3
                v = t[g, w, k]
                d = [(v[order[i + 1]] - v[order[i]]) % (1 << 32) for i in range(len(order) - 1)]
                nxt = t[g, w, k + 1, order[0]] if k + 1 < n_g else None
                tot = (nxt - v[0]) % (1 << 32) if nxt is not None else None
                rows[2 if sp0 + 4 < 7 else 1].append(d + [tot if tot is not None else -1])
    out = {}
    for ns, r in rows.items():
        r = np.asarray(r, np.float64)
        m = {names[i]: round(float(np.median(r[:, i])), 0) for i in range(len(names))}
        tot = r[:, -1][r[:, -1] >= 0]
        m["example total (loop top to loop top)"] = round(float(np.median(tot)), 0) if len(tot) else None
        out[f"{ns}-stripe waves (median shader cycles)"] = m
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
