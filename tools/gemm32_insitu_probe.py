"""Why the towers' input-layer GEMMs run slower inside the DSSM forward than alone (diagnostics): the same
rf_gemm_f32 launch timed (a) back to back, (b) right after its A operand was rewritten (as the encoder writes it),
(c) after an HBM-bound kernel of the encoder's size that writes other memory, (d) with its own launches separated
by idle gaps. HIP events around the GEMM only."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from recommendflow_amd.runtime import gemm as G


def timed(pre, fn, reps=20):
    ms = []
    for i in range(reps + 3):
        pre()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        if i >= 3:
            ms.append(e0.elapsed_time(e1))
    return round(sum(ms) / len(ms), 4), round(min(ms), 4)


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    xa = torch.randn(4096, 20480, device="cuda", generator=g) * 0.05
    xa2 = torch.randn(4096, 20480, device="cuda", generator=g) * 0.05
    Wa = torch.randn(1024, 20480, device="cuda", generator=g) * 0.01
    big = torch.empty(4096 * 29184, device="cuda")
    for _ in range(30):
        G.gemm_f32(xa, Wa, trans_b=True)
    fl = 2 * 4096 * 1024 * 20480
    res = {}
    res["a_back_to_back"] = timed(lambda: None, lambda: G.gemm_f32(xa, Wa, trans_b=True))
    res["b_after_A_rewrite"] = timed(lambda: xa.copy_(xa2), lambda: G.gemm_f32(xa, Wa, trans_b=True))
    res["c_after_other_write"] = timed(lambda: big.fill_(1.0), lambda: G.gemm_f32(xa, Wa, trans_b=True))
    res["d_after_1ms_idle"] = timed(lambda: (torch.cuda.synchronize(), time.sleep(0.001)), lambda: G.gemm_f32(xa, Wa, trans_b=True))
    res["e_after_50ms_idle"] = timed(lambda: (torch.cuda.synchronize(), time.sleep(0.05)), lambda: G.gemm_f32(xa, Wa, trans_b=True), reps=10)
    for k, (avg, mn) in res.items():
        print(json.dumps({"case": k, "ms_avg": avg, "ms_min": mn, "frac_avg": round(fl / avg / 1e9 / 157.3, 4)}))


if __name__ == "__main__":
    main()
