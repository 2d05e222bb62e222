"""cfg5 Flat search (1024 unit queries x 1M items x 256, top-200): search_index time against the number of exactly
scored lead blocks before the bf16 screen (faiss_searcher.SCREEN_EXACT_BLOCKS), HIP events after a warm-up, and
whether the result equals the block loop bit for bit (diagnostics).
    python tools/flat_lead_sweep.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from recommendflow_amd.backend.third_party_components import faiss_searcher as F  # noqa: E402

N, E, B, K = 1_000_000, 256, 1024, 200
g = torch.Generator(device="cuda").manual_seed(3)
items = torch.randn((N, E), device="cuda", generator=g)
items = items / items.norm(dim=1, keepdim=True)
q = torch.randn((B, E), device="cuda", generator=g)
q = q / q.norm(dim=1, keepdim=True)
s = F.FaissSearcher(items=items[:8].cpu().numpy(), index_param="Flat", measurement="ip")
s.index = items.contiguous()
s.screen = False
want_v, want_i = s.search_index(q, K)
s.screen = True


def ev(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


res = {}
for lead in (1, 2, 3, 4, 6):
    F.SCREEN_EXACT_BLOCKS = lead
    v, i = s.search_index(q, K)
    res[lead] = {"ms": round(ev(lambda: s.search_index(q, K)), 3), "bit_equal": bool(torch.equal(v, want_v) and torch.equal(i, want_i))}
    print(json.dumps({"lead_blocks": lead, **res[lead]}), flush=True)
