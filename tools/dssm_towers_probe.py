"""rocprof target (diagnostics): the cfg2 DSSM fp32 towers exactly as bench_dssm's `fp32_towers` stage runs them
(user [B, 8832] and ad [B, 20480] fp32 inputs -> Dense 1024 / 512 / 256 selu + BatchNorm folded -> l2norm -> dot),
replayed as one hipGraph 30 times; prints the graph-timed ms per forward."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from recommendflow_amd.backend.encoder.sparse_encoder import FusedSparseEncoder, SlotSpec  # noqa: E402
from recommendflow_amd.config_parser.configuration import Configuration  # noqa: E402
from recommendflow_amd.models.matching.dssm import Dssm  # noqa: E402
from recommendflow_amd.runtime.graphs import CapturedGraph  # noqa: E402

B = 4096
conf = Configuration(os.path.join(ROOT, "tests", "golden", "conf", "base_recall_sdpa.yaml"))
feats = conf.features.hashing_features
users = [f for f in feats if f.tower.value == "user"]
ads = [f for f in feats if f.tower.value == "ad"]
eu = FusedSparseEncoder([SlotSpec(f.name, 1000, tuple(f.hash_seeds), f.pooling.value) for f in users], 64)
ea = FusedSparseEncoder([SlotSpec(f.name, 1000, tuple(f.hash_seeds), f.pooling.value) for f in ads], 64)
model = Dssm(eu, ea, seed=5)
xu = torch.randn((B, eu.out_width), device="cuda") * 0.05
xa = torch.randn((B, ea.out_width), device="cuda") * 0.05


def towers():
    u = torch.nn.functional.normalize(model.user_dense(xu), dim=-1, eps=1e-6)
    v = torch.nn.functional.normalize(model.ad_dense(xa), dim=-1, eps=1e-6)
    (u * v).sum(-1)


towers()
g = CapturedGraph(towers)
for _ in range(5):
    g.replay()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(30):
    g.replay()
e.record()
e.synchronize()
ms = s.elapsed_time(e) / 30
fl = model.flops_per_example() * B
print(f"towers {ms:.4f} ms  {fl / ms / 1e9:.1f} TF/s  frac {fl / ms / 1e9 / 157.3:.4f}")
