"""CPU: the float64 ESIM training oracle (oracle.esim_train_loss, esim_pool_bwd, ln_mlp_train_bwd) against central
finite differences of its own forward. This pins the analytic backward the GPU training path is checked against
(tests/test_esim_train_gpu.py): for every parameter group a random direction v, (f(t + h v) - f(t - h v)) / 2h vs
<grad, v>, rtol 1e-6 in float64. The forward follows esim.py:45-53,69-89, attention_layers.py:33-74, mlp.py:4-15;
parity of the forward itself with the reference is unpinned (TensorFlow is not importable)."""
import numpy as np
import pytest

from oracle import oracle as O


def _model(rng, B=6, L=5, d=8, n_dense=4, inu=(8, 12), outu=(16, 8)):
    def layers(k, units):
        out = []
        for u in units:
            out.append({"W": rng.normal(0, 0.4, (u, k)), "b": rng.normal(0, 0.1, u), "gamma": 1 + rng.normal(0, 0.1, k),
                        "beta": rng.normal(0, 0.1, k)})
            k = u
        return out

    q = rng.normal(0, 1.0, (B, L, d))
    a = rng.normal(0, 1.0, (B, L, d))
    dense = rng.normal(0, 1.0, (B, n_dense))
    lin = layers(n_dense, inu)
    lout = layers(inu[-1] + 6 * d, outu)
    Wo = rng.normal(0, 0.4, (2, outu[-1]))
    bo = rng.normal(0, 0.1, 2)
    y = rng.integers(0, 2, B)
    return q, a, dense, y, lin, lout, Wo, bo


def _fd(f, x, v, h=1e-6):
    return (f(x + h * v) - f(x - h * v)) / (2 * h)


@pytest.mark.parametrize("rate", [0.0, 0.3])
def test_esim_train_grads_match_finite_differences(rate):
    rng = np.random.default_rng(7)
    q, a, dense, y, lin, lout, Wo, bo = _model(rng)
    seeds = ([11, 12], 13, [14, 15])
    loss, _, g = O.esim_train_loss(q, a, dense, y, lin, lout, Wo, bo, rate=rate, seeds=seeds, grads=True)

    def L(q_=q, a_=a, lin_=lin, lout_=lout, Wo_=Wo, bo_=bo):
        return O.esim_train_loss(q_, a_, dense, y, lin_, lout_, Wo_, bo_, rate=rate, seeds=seeds)[0]

    checks = []
    v = rng.normal(size=q.shape)
    checks.append(("q", _fd(lambda t: L(q_=t), q, v), (g["q"] * v).sum()))
    v = rng.normal(size=a.shape)
    checks.append(("a", _fd(lambda t: L(a_=t), a, v), (g["a"] * v).sum()))
    v = rng.normal(size=Wo.shape)
    checks.append(("W_out", _fd(lambda t: L(Wo_=t), Wo, v), (g["W_out"] * v).sum()))
    v = rng.normal(size=bo.shape)
    checks.append(("b_out", _fd(lambda t: L(bo_=t), bo, v), (g["b_out"] * v).sum()))
    for name, layers, key in (("input", lin, "lin_"), ("output", lout, "lout_")):
        for li, p in enumerate(layers):
            for k in ("W", "b", "gamma", "beta"):
                v = rng.normal(size=p[k].shape)

                def f(t, li=li, k=k, layers=layers, key=key):
                    ls = [dict(x) for x in layers]
                    ls[li][k] = t
                    return L(**{key: ls})

                checks.append((f"{name}[{li}].{k}", _fd(f, p[k], v), (g[name][li][k] * v).sum()))
    for name, fd, an in checks:
        assert abs(fd - an) <= 1e-6 * max(1.0, abs(fd)) + 1e-9, (name, fd, an)
    assert np.isfinite(loss)
