"""rocprof target (diagnostics): the screened Flat search at the cfg5 shapes (1024 unit queries x 1M unit items x 256,
top-200), 20 calls after a warm-up, so `rocprofv3 --kernel-trace --stats` splits it per kernel.
    python tools/flat_search_trace.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from recommendflow_amd.backend.third_party_components.faiss_searcher import FaissSearcher  # noqa: E402

N, E, B, K = 1_000_000, 256, 1024, 200
g = torch.Generator(device="cuda").manual_seed(3)
items = torch.randn((N, E), device="cuda", generator=g)
items = items / items.norm(dim=1, keepdim=True)
q = torch.randn((B, E), device="cuda", generator=g)
q = q / q.norm(dim=1, keepdim=True)
s = FaissSearcher(items=items[:8].cpu().numpy(), index_param="Flat", measurement="ip")
s.index = items.contiguous()
for _ in range(25):
    s.search_index(q, K)
torch.cuda.synchronize()
print("ok")
