"""Grouped vs separate rf_gemm_f32 launches on the DSSM towers' layers at cfg2 (diagnostics): the inputs are
column blocks of one [4096, 29184] encoder output, as in the model. HIP-event times per variant."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from recommendflow_amd.runtime import gemm as G


def t(fn, reps=20):
    for _ in range(3):
        fn()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    for _ in range(reps):
        fn()
    e[1].record()
    torch.cuda.synchronize()
    return e[0].elapsed_time(e[1]) / reps


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(4096, 8704 + 20480, device="cuda", generator=g) * 0.05
    xu, xa = x[:, :8704], x[:, 8704:]
    xu_c, xa_c = xu.contiguous(), xa.contiguous()
    Wu = torch.randn(1024, 8704, device="cuda", generator=g) * 0.01
    Wa = torch.randn(1024, 20480, device="cuda", generator=g) * 0.01
    h1 = torch.randn(4096, 1024, device="cuda", generator=g)
    h1b = torch.randn(4096, 1024, device="cuda", generator=g)
    W2 = torch.randn(512, 1024, device="cuda", generator=g)
    W2b = torch.randn(512, 1024, device="cuda", generator=g)
    h2 = torch.randn(4096, 512, device="cuda", generator=g)
    h2b = torch.randn(4096, 512, device="cuda", generator=g)
    W3 = torch.randn(256, 512, device="cuda", generator=g)
    W3b = torch.randn(256, 512, device="cuda", generator=g)
    for _ in range(30):  # clocks up
        G.gemm_f32(xa, Wa, trans_b=True)
    r = {}
    r["L1_separate_views"] = t(lambda: (G.gemm_f32(xu, Wu, trans_b=True), G.gemm_f32(xa, Wa, trans_b=True)))
    r["L1_separate_contig"] = t(lambda: (G.gemm_f32(xu_c, Wu, trans_b=True), G.gemm_f32(xa_c, Wa, trans_b=True)))
    r["L1_user_view"] = t(lambda: G.gemm_f32(xu, Wu, trans_b=True))
    r["L1_ad_view"] = t(lambda: G.gemm_f32(xa, Wa, trans_b=True))
    r["L1_grouped_views"] = t(lambda: G.gemm_f32_grouped([(xu, Wu, None, "none", None), (xa, Wa, None, "none", None)], trans_b=True))
    r["L2_separate"] = t(lambda: (G.gemm_f32(h1, W2, trans_b=True), G.gemm_f32(h1b, W2b, trans_b=True)))
    r["L2_grouped"] = t(lambda: G.gemm_f32_grouped([(h1, W2, None, "none", None), (h1b, W2b, None, "none", None)], trans_b=True))
    r["L3_separate"] = t(lambda: (G.gemm_f32(h2, W3, trans_b=True), G.gemm_f32(h2b, W3b, trans_b=True)))
    r["L3_grouped"] = t(lambda: G.gemm_f32_grouped([(h2, W3, None, "none", None), (h2b, W3b, None, "none", None)], trans_b=True))
    fl = {"L1": 2 * 4096 * 1024 * (8704 + 20480), "L2": 2 * 2 * 4096 * 512 * 1024, "L3": 2 * 2 * 4096 * 256 * 512}
    for k, v in r.items():
        f = fl[k[:2]] if not k.startswith("L1_user") and not k.startswith("L1_ad") else \
            2 * 4096 * 1024 * (8704 if "user" in k else 20480)
        print(json.dumps({"case": k, "ms": round(v, 4), "frac_157TF": round(f / v / 1e9 / 157.3, 4)}))


if __name__ == "__main__":
    main()
