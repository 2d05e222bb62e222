"""Shared test helpers: the oracle's view of a fused encoder's output and of an MLP's parameters."""
import numpy as np
import torch


def enc_ref(O, enc, hb):
    """oracle.fused_hash_embed over the encoder's own table (bf16 tables read as raw bits) -> float32."""
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
