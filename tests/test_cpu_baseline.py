"""The float32 CPU baseline of cfg3's dense stages (oracle.esim_scorer_f32, timed by bench.py) computes
the same function as the float64 restatement composed stage by stage (esim_pool, mlp, Dense(2, softmax))."""
import numpy as np

from oracle import oracle as O


def _layers(rng, dims):
    return [{"W": rng.normal(0, (2.0 / (k + n)) ** 0.5, (k, n)), "b": rng.normal(0, 0.1, n),
             "gamma": rng.uniform(0.5, 1.5, k), "beta": rng.normal(0, 0.1, k)} for k, n in zip(dims[:-1], dims[1:])]


def test_esim_scorer_f32_matches_f64():
    rng = np.random.default_rng(0)
    B, L, d = 12, 20, 32
    q = rng.uniform(-0.1, 0.1, (B, L, d)).astype(np.float32)
    a = rng.uniform(-0.1, 0.1, (B, L, d)).astype(np.float32)
    dense = rng.normal(size=(B, 16)).astype(np.float32)
    pin, pout = _layers(rng, [16, 32, 48]), _layers(rng, [48 + 6 * d, 64, 32])
    Wo, bo = rng.normal(0, 0.2, (32, 2)), rng.normal(0, 0.1, 2)
    got = O.esim_scorer_f32(q, a, dense, pin, pout, Wo, bo)
    pooled = np.concatenate([O.mlp(dense, pin, "gelu", "ln"), O.esim_pool(q, a)], axis=1)
    want = O.activation(O.mlp(pooled, pout, "gelu", "ln") @ Wo + bo, "softmax")
    assert got.dtype == np.float32
    np.testing.assert_allclose(got, want, rtol=0, atol=2e-5)


def test_bench_timed_runs_protocol():
    import importlib.util
    import os

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(os.path.dirname(__file__), "..", "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    calls = []
    r = bench.timed_runs(lambda: calls.append(1), examples=100, budget_s=0.0, warmup=5, min_runs=7)
    assert len(calls) == 12 and r["runs"] == 7
    assert r["p90"] >= r["median"] > 0
    model, n = bench.host_cpu()
    assert isinstance(model, str) and n >= 1
