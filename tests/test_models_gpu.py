"""Model-level parity (GPU vs the CPU oracle composed stage by stage), small shapes.

ESIM (cfg3 structure): sparse slots -> bf16 tables -> q, a token sequences (bit-exact vs the oracle)
-> ESIM pooling + MLPs (float64 oracle). Bar: |dp| <= 1e-2 on the softmax outputs,
>= 99.9% arg-max agreement (here: all rows, on a batch of 256).
DSSM (cfg2 structure): fp32 towers on the exact-fp32 MFMA path, rtol 1e-4 on the cosine score.
"""
import numpy as np
import pytest
import torch

from recommendflow_amd.backend.encoder.sparse_encoder import FusedSparseEncoder, SlotSpec
from recommendflow_amd.models.matching.dssm import Dssm
from recommendflow_amd.models.ranking.esim import Esim
from recommendflow_amd.runtime.batch import synthetic_batch

pytestmark = pytest.mark.gpu


def enc_ref(O, enc, hb):
    t = enc.table.cpu()
    tab = t.view(torch.int16).numpy().view(np.uint16) if t.dtype == torch.bfloat16 else t.numpy()
    odt = O.DT_BF16 if enc.out_dtype == torch.bfloat16 else O.DT_F32
    out, _ = O.fused_hash_embed(enc.host_desc, hb.tok_bytes, hb.tok_off, hb.bag_off, hb.lmax, hb.batch, tab, enc.dim,
                                enc.out_width, out_dtype=odt)
    return O.bf16_to_f32(out) if odt == O.DT_BF16 else out


def mlp_params(m):
    return [{"W": dn.weight.float().cpu().numpy().T, "b": dn.bias.cpu().numpy(), "gamma": nm.gamma.cpu().numpy(),
             "beta": nm.beta.cpu().numpy(), "mean": None if nm.mean is None else nm.mean.cpu().numpy(),
             "var": None if nm.var is None else nm.var.cpu().numpy()} for nm, dn in zip(m.norms, m.denses)]


def test_esim_model_vs_oracle(O, cuda):
    Lq, B, D = 24, 256, 64
    user = [SlotSpec(f"u{i}", 5000 + i, (2022, 2023)) for i in range(Lq)]
    ad = [SlotSpec(f"a{i}", 7000 + i, (2022, 2023)) for i in range(Lq)]
    model = Esim(user, ad, n_dense=16, dim=D, seed=5)
    hu = synthetic_batch(B, [False] * Lq, seed=1)
    ha = synthetic_batch(B, [i % 5 == 0 for i in range(Lq)], seed=2)
    dense = torch.randn(B, 16, generator=torch.Generator().manual_seed(3))
    p = model(hu.to("cuda"), ha.to("cuda"), dense.cuda()).cpu().numpy()
    q = enc_ref(O, model.enc_q, hu).reshape(B, Lq, 2 * D)
    a = enc_ref(O, model.enc_a, ha).reshape(B, Lq, 2 * D)
    d_emb = O.mlp(dense.numpy(), mlp_params(model.input_mlp), "gelu", "ln")
    pooled = np.concatenate([d_emb, O.esim_pool(q, a)], axis=1)
    x = O.mlp(pooled, mlp_params(model.output_mlp), "gelu", "ln")
    W = model.dense_output.weight.float().cpu().numpy()
    want = O.activation(x @ W.T.astype(np.float64) + model.dense_output.bias.cpu().numpy(), "softmax")
    assert np.abs(p - want).max() <= 1e-2
    assert (p.argmax(1) == want.argmax(1)).mean() >= 0.999
    np.testing.assert_allclose(p.sum(1), 1.0, atol=1e-5)


def test_dssm_model_vs_oracle(O, cuda):
    B, D = 128, 16
    us = [SlotSpec(f"u{i}", 3000, (2022, 2023)) for i in range(6)]
    as_ = [SlotSpec(f"a{i}", 3000, (2022, 2023)) for i in range(9)]
    eu, ea = FusedSparseEncoder(us, D, seed=1), FusedSparseEncoder(as_, D, seed=2)
    m = Dssm(eu, ea, units=(128, 64, 32), seed=4)
    hu = synthetic_batch(B, [i % 2 == 0 for i in range(6)], seed=7)
    ha = synthetic_batch(B, [False] * 9, seed=8)
    score = m(hu.to("cuda"), ha.to("cuda")).cpu().numpy()
    u = O.l2_normalize(O.mlp(enc_ref(O, eu, hu), mlp_params(m.user_dense), "selu", "bn"))
    v = O.l2_normalize(O.mlp(enc_ref(O, ea, ha), mlp_params(m.ad_dense), "selu", "bn"))
    np.testing.assert_allclose(score, (u * v).sum(1), rtol=1e-4, atol=1e-5)
