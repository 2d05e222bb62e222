"""Training losses: the float64 oracle against a direct transcription of the reference formulas
(CPU), and the HIP kernels (rf_cosent_loss, rf_inbatch_ce_loss) against the oracle (GPU)."""
import numpy as np
import pytest
from scipy.special import logsumexp

from oracle import oracle as O


def ref_cosent(y, s, scale=20):
    # match_losses.py:42-56 verbatim in numpy float64: mask with -1e12, prepend 0, logsumexp
    yt = (y[:, None] < y[None, :]).astype(np.float64)
    yp = s * scale
    yp = yp[:, None] - yp[None, :]
    yp = (yp - (1 - yt) * 1e12).reshape(-1)
    return logsumexp(np.concatenate([[0.0], yp]))


def ref_inbatch(y, q, d, scale=20):
    # match_losses.py:150-165 verbatim
    yp = q @ d.T
    num = np.diag(np.exp(scale * yp))
    den = np.exp(scale * yp).sum(-1)
    return np.mean(-np.log(num / den) * y)


@pytest.mark.parametrize("B", [1, 5, 64])
def test_oracle_cosent_matches_reference_formula_and_gradient(B):
    rng = np.random.default_rng(B)
    y = rng.integers(0, 3, B).astype(np.float64)
    s = rng.uniform(-1, 1, B)
    loss, ds = O.cosent_loss(y, s)
    assert np.isclose(loss, ref_cosent(y, s), rtol=1e-12, atol=1e-12)
    eps = 1e-6
    num = np.array([(ref_cosent(y, s + eps * np.eye(B)[i]) - ref_cosent(y, s - eps * np.eye(B)[i])) / (2 * eps)
                    for i in range(B)])
    np.testing.assert_allclose(ds, num, rtol=1e-5, atol=1e-7)


def test_oracle_inbatch_ce_matches_reference_formula_and_gradient():
    rng = np.random.default_rng(0)
    B, E = 6, 5
    q = rng.normal(size=(B, E)) * 0.3
    d = rng.normal(size=(B, E)) * 0.3
    y = rng.integers(0, 2, B).astype(np.float64)
    loss, dP = O.inbatch_ce_loss(y, q @ d.T)
    assert np.isclose(loss, ref_inbatch(y, q, d), rtol=1e-10)
    # chain rule through P = q d^T, compared with finite differences on q
    dq = dP @ d
    eps = 1e-6
    for i in range(B):
        for e in range(E):
            qp, qm = q.copy(), q.copy()
            qp[i, e] += eps
            qm[i, e] -= eps
            fd = (ref_inbatch(y, qp, d) - ref_inbatch(y, qm, d)) / (2 * eps)
            assert np.isclose(dq[i, e], fd, rtol=1e-4, atol=1e-8)


@pytest.mark.gpu
@pytest.mark.parametrize("B", [1, 7, 300, 4096])
def test_cosent_kernel(cuda, B):
    import torch

    from recommendflow_amd.backend.losses.match_losses import _Cosent

    rng = np.random.default_rng(B)
    y = rng.integers(0, 2 if B > 7 else 4, B).astype(np.float32)
    s = rng.uniform(-1, 1, B).astype(np.float32)
    st = torch.tensor(s, device="cuda", requires_grad=True)
    loss = _Cosent.apply(st, torch.tensor(y, device="cuda"), 20.0)
    loss.backward()
    want, wds = O.cosent_loss(y, s)
    assert abs(float(loss.detach()) - want) <= 1e-5 * max(1.0, abs(want))
    np.testing.assert_allclose(st.grad.cpu().numpy(), wds, rtol=1e-4, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("B,K", [(1, 64), (33, 64), (2048, 64), (4096, 256)])
def test_inbatch_ce_kernel(cuda, B, K):
    import torch

    from recommendflow_amd.backend.losses.match_losses import batch_neg_sample_scaled_multi_class_ce_loss

    rng = np.random.default_rng(B)
    q = torch.nn.functional.normalize(torch.tensor(rng.normal(size=(B, K)), dtype=torch.float32), dim=-1).cuda()
    d = torch.nn.functional.normalize(torch.tensor(rng.normal(size=(B, K)), dtype=torch.float32), dim=-1).cuda()
    q.requires_grad_(True)
    d.requires_grad_(True)
    y = torch.tensor(rng.integers(0, 2, B), dtype=torch.float32, device="cuda")
    loss = batch_neg_sample_scaled_multi_class_ce_loss(y, q, d)
    loss.backward()
    P = (q.detach().double() @ d.detach().double().t()).cpu().numpy()
    want, dP = O.inbatch_ce_loss(y.cpu().numpy(), P)
    assert abs(float(loss.detach()) - want) <= 1e-5 * max(1.0, abs(want))
    np.testing.assert_allclose(q.grad.cpu().numpy(), dP @ d.detach().cpu().numpy(), rtol=1e-4, atol=1e-6)
    # the logits' backward products run on librf (rf_linear_fwd) where the rows allow it: dd = dP^T q
    np.testing.assert_allclose(d.grad.cpu().numpy(), dP.T @ q.detach().cpu().numpy(), rtol=1e-4, atol=1e-6)
