"""cfg5 recall search in isolation (diagnostics): FaissSearcher Flat IP, 1024 l2-normalised queries x 1M items x 256
(the cascade's recall shapes), top-200. Times search_index (HIP events, after a warm-up; the block loop and the
screened form), the bf16 form of its score
GEMM for one 32768-item block, and counts, for a bf16 screen, how many items score within 2 delta of each query's
200th screened score (delta = the bf16 rounding bound of a unit-vector dot product).
    python tools/flat_probe.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from recommendflow_amd.backend.third_party_components.faiss_searcher import BLOCK, FaissSearcher  # noqa: E402
from recommendflow_amd.runtime import lib as L  # noqa: E402

N, E, B, K = 1_000_000, 256, 1024, 200
g = torch.Generator(device="cuda").manual_seed(3)
items = torch.randn((N, E), device="cuda", generator=g)
items = items / items.norm(dim=1, keepdim=True)
q = torch.randn((B, E), device="cuda", generator=g)
q = q / q.norm(dim=1, keepdim=True)
s = FaissSearcher(items=items[:8].cpu().numpy(), index_param="Flat", measurement="ip")
s.index = items.contiguous()


def ev(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        fn()
        torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


s.screen = False
res = {"search_index_block_loop_ms": round(ev(lambda: s.search_index(q, K)), 3)}
s.screen, s.screen_bf16 = True, False
res["search_index_screened_fp32_ms"] = round(ev(lambda: s.search_index(q, K)), 3)
s.screen_bf16 = True
res["search_index_screened_ms"] = round(ev(lambda: s.search_index(q, K)), 3)
a_v, a_i = s.search_index(q, K)
s.screen = False
b_v, b_i = s.search_index(q, K)
s.screen = True
res["screened_equals_block_loop"] = bool(torch.equal(a_i, b_i) and torch.equal(a_v, b_v))
# the screen's stages alone: the candidate pass over one block and over the rest, real thresholds and +inf
v0, _ = s.search_index(q[:, :], K)
thr = v0[:, K - 1].contiguous()
inf = torch.full_like(thr, float("inf"))
cap = 32768
cnt = torch.zeros(B, dtype=torch.int32, device="cuda")
cv = torch.empty((B, cap), device="cuda")
ci = torch.empty((B, cap), dtype=torch.int32, device="cuda")


def cand(t, n0, n):
    cnt.zero_()
    L.call("rf_ip_candidates_f32", L.ptr(q), E, B, L.ptr(items[n0:]), n, E, L.ptr(t), cap, L.ptr(cnt), L.ptr(cv), L.ptr(ci),
           n0, L.stream_ptr())


res["cand_one_block_inf_ms"] = round(ev(lambda: cand(inf, BLOCK, BLOCK)), 4)
res["cand_one_block_thr_ms"] = round(ev(lambda: cand(thr, BLOCK, BLOCK)), 4)
res["cand_rest_thr_ms"] = round(ev(lambda: cand(thr, BLOCK, N - BLOCK)), 4)
res["cand_rest_inf_ms"] = round(ev(lambda: cand(inf, BLOCK, N - BLOCK)), 4)
blk = items[:BLOCK].contiguous()
sc = torch.empty((B, BLOCK), device="cuda")
res["fp32_block_gemm_ms"] = round(ev(lambda: L.call("rf_linear_fwd", L.ptr(q), L.DT_F32, B, E, E, L.ptr(blk), BLOCK, None, 0,
                                                    L.ptr(sc), BLOCK, L.stream_ptr())), 4)
qb, bb = q.to(torch.bfloat16), blk.to(torch.bfloat16)
res["bf16_block_gemm_ms"] = round(ev(lambda: L.call("rf_linear_fwd", L.ptr(qb), L.DT_BF16, B, E, E, L.ptr(bb), BLOCK, None,
                                                    0, L.ptr(sc), BLOCK, L.stream_ptr())), 4)
from recommendflow_amd.runtime import gemm as G  # noqa: E402

res["gemm_f32_block_ms"] = round(ev(lambda: G.gemm_f32(q, blk, trans_b=True, out=sc)), 4)
# screen: the exact scores and the bf16 screened scores of every item, one 64-query slice at a time
delta = 2.0 ** -7 + E * 2.0 ** -23
ib = items.to(torch.bfloat16)
cnt = []
for r0 in range(0, 256, 64):
    qs = q[r0:r0 + 64]
    ss = (qs.to(torch.bfloat16).float() @ ib.float().t())
    t = torch.topk(ss, K, dim=1).values[:, -1:]
    cnt.append((ss >= t - 2 * delta).sum(dim=1))
cnt = torch.cat(cnt).float()
res["screen_candidates"] = {"mean": round(cnt.mean().item(), 1), "max": int(cnt.max().item()), "delta": delta}
print(json.dumps(res))
