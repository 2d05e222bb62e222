"""cfg3 id pass in isolation (diagnostics): Esim.token_ids (rf_single_token_ids_multi_fwd, both towers, 2 x 100
single-valued slots x 4096) captured 20 times into one hipGraph, HIP events around 10 replays after a 0.3 s warm-up:
the kernel's time per call without a graph launch per call. Small tables (the pass reads no table rows).
    python tools/ids_probe.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from recommendflow_amd.backend.encoder.sparse_encoder import SlotSpec  # noqa: E402
from recommendflow_amd.models.ranking.esim import Esim  # noqa: E402
from recommendflow_amd.runtime.batch import synthetic_batch  # noqa: E402
from recommendflow_amd.runtime.graphs import CapturedGraph  # noqa: E402

B, Ls = 4096, 100
model = Esim([SlotSpec(f"u{i:03d}", 1_000_000, (2022, 2023)) for i in range(Ls)],
             [SlotSpec(f"a{i:03d}", 1_000_000, (2022, 2023)) for i in range(Ls)], n_dense=16, dim=64,
             table_dtype=torch.bfloat16, seed=3)
hu = synthetic_batch(B, [False] * Ls, seed=77, slot_ids=range(Ls)).to("cuda")
ha = synthetic_batch(B, [False] * Ls, seed=99, slot_ids=range(Ls, 2 * Ls)).to("cuda")
g = CapturedGraph(lambda: [model.token_ids(hu, ha) for _ in range(20)])
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.3:
    g.replay()
    torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(10):
    g.replay()
b.record()
torch.cuda.synchronize()
us = a.elapsed_time(b) / 200 * 1e3
tok = sum(h.n_tokens for h in (hu, ha))
print(json.dumps({"token_ids_us": round(us, 2), "tokens": tok, "Mtok_per_s": round(tok / us, 1)}))
