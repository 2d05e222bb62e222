"""CPU: the float64 DSSM tower-training oracle (oracle.tower_train_fwd / tower_train_bwd, the checker of
tests/test_tower_train_gpu.py) against central finite differences of its own forward, so the restated backward
(BatchNormalization with batch statistics, SELU, dropout, Dense) is pinned by calculus rather than by itself."""
import numpy as np
import pytest


def _layers(rng, widths):
    out = []
    for k, n in zip(widths[:-1], widths[1:]):
        out.append({"W": rng.normal(0, 0.4, (n, k)), "b": rng.normal(0, 0.1, n), "gamma": rng.uniform(0.5, 1.5, k),
                    "beta": rng.normal(0, 0.1, k)})
    return out


@pytest.mark.parametrize("rate", [0.0, 0.3])
def test_tower_backward_matches_finite_differences(O, rate):
    rng = np.random.default_rng(3)
    M, widths, seeds = 12, [5, 4, 3], [11, 12]
    x = rng.normal(0.2, 1.0, (M, widths[0]))
    layers = _layers(rng, widths)
    dout = rng.normal(0, 1, (M, widths[-1]))

    def f(xv, lv):
        out, _ = O.tower_train_fwd(xv, lv, rate, seeds)
        return float((out * dout).sum())

    out, cache = O.tower_train_fwd(x, layers, rate, seeds)
    dx, grads = O.tower_train_bwd(dout, layers, cache, rate)
    h = 1e-6
    num = np.zeros_like(x)
    for i in range(M):
        for j in range(widths[0]):
            xp, xm = x.copy(), x.copy()
            xp[i, j] += h
            xm[i, j] -= h
            num[i, j] = (f(xp, layers) - f(xm, layers)) / (2 * h)
    np.testing.assert_allclose(dx, num, rtol=1e-5, atol=1e-7)
    for li in range(len(layers)):
        for name in ("W", "b", "gamma", "beta"):
            p = layers[li][name]
            g = np.zeros_like(p)
            for idx in np.ndindex(p.shape):
                lp = [dict(d) for d in layers]
                lm = [dict(d) for d in layers]
                lp[li][name] = p.copy()
                lm[li][name] = p.copy()
                lp[li][name][idx] += h
                lm[li][name][idx] -= h
                g[idx] = (f(x, lp) - f(x, lm)) / (2 * h)
            np.testing.assert_allclose(grads[li][name], g, rtol=1e-5, atol=1e-7, err_msg=f"layer {li} {name}")


def test_dropout_keep_rate(O):
    k = O.dropout_keep(2024, 300, 257, 0.3)
    assert abs(k.mean() - 0.7) < 0.01
    assert not np.array_equal(k, O.dropout_keep(2025, 300, 257, 0.3))
