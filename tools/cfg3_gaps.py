"""rocprof target (diagnostics): the cfg3 ESIM forward as the bench runs it (one hipGraph per forward, two
resident batches alternating), replayed 40 times; `rocprofv3 --kernel-trace` of this run gives every kernel's
start/end, so tools/trace_gaps.py can split a forward into kernel time and the idle gaps between kernels.
    python tools/cfg3_gaps.py [--eager] [--serial-mlp] [--gather] [--uniform] [--unfused]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch

from recommendflow_amd.backend.encoder.sparse_encoder import SlotSpec
from recommendflow_amd.models.ranking.esim import Esim
from recommendflow_amd.runtime.batch import synthetic_batch
from recommendflow_amd.runtime.graphs import CapturedGraph

B, Ls = 4096, 100
user = [SlotSpec(f"u{i:03d}", 1_000_000, (2022, 2023)) for i in range(Ls)]
ad = [SlotSpec(f"a{i:03d}", 1_000_000, (2022, 2023)) for i in range(Ls)]
model = Esim(user, ad, n_dense=16, dim=64, table_dtype=torch.bfloat16, seed=3)
uni = "--uniform" in sys.argv  # uniform ids (no Zipf-hot rows) instead of Zipf(1.1)
hu = [synthetic_batch(B, [False] * Ls, seed=77 + i, slot_ids=range(Ls), uniform=uni).to("cuda") for i in range(2)]
ha = [synthetic_batch(B, [False] * Ls, seed=99 + i, slot_ids=range(Ls, 2 * Ls), uniform=uni).to("cuda") for i in range(2)]
dense = torch.randn(B, 16, device="cuda")
model.concurrent_input_mlp = "--serial-mlp" not in sys.argv
model.gather = "--gather" in sys.argv
model.fused_scorer = "--unfused" not in sys.argv  # A/B: pooled fp32 -> LayerNorm pass -> GEMMs -> head
if "--eager" in sys.argv:
    run = [lambda p=p: model(hu[p], ha[p], dense) for p in (0, 1)]
else:
    g = [CapturedGraph(lambda p=p: model(hu[p], ha[p], dense)) for p in (0, 1)]
    run = [gg.replay for gg in g]
for i in range(20):
    run[i & 1]()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for i in range(40):
    run[i & 1]()
e.record()
torch.cuda.synchronize()
print(f"forward {s.elapsed_time(e) / 40:.4f} ms")
