"""Committed golden fixtures (tests/golden/, made by make_golden.py from the oracle):
the oracle and the generator must keep reproducing them exactly."""
import os

import numpy as np
import pytest

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(G, name))  # allow_pickle=False (default)


def test_density_kats(po):
    g = load("density_kats.npz")
    for name, d in [("tanh1", po.Density("tanh", 1.0)), ("exp01", po.Density("exp", 0.1)), ("cube", po.Density("cube"))]:
        psi, dpsi = d.score_and_der(g["grid"][None, :])
        assert np.array_equal(psi[0], g[f"{name}_psi"]) and np.array_equal(dpsi[0], g[f"{name}_dpsi"])
        assert np.array_equal(d.log_lik(g["grid"]), g[f"{name}_ll"])


def test_generator_digest(dg):
    g = load("c1_data_digest.npz")
    x, s, a = dg.generate_data(8, 10000, 42)
    assert np.array_equal(a, g["a"])
    assert np.array_equal(x[:, :64], g["x_first"]) and np.array_equal(x[:, -64:], g["x_last"])
    assert np.array_equal(s.sum(axis=1), g["s_rowsum"])


def test_pass_stats(po, c1_data):
    g = load("c1_pass_stats.npz")
    x, _, _ = c1_data
    st = po.pass_stats(g["w"], g["mu"], x, po.Density("tanh", 1.0), True)
    for k in st:
        assert np.allclose(st[k], g[k], rtol=1e-13, atol=0), k


@pytest.mark.parametrize("tag,kw", [("ortho_ext", dict(ortho=True, extended=True)),
                                    ("nonortho", dict(ortho=False, extended=False))])
def test_trajectories(po, c1_data, tag, kw):
    g = load("c1_trajectories.npz")
    x, _, a = c1_data
    r = po.fit_with_config(x, po.PicardConfig(w_init=np.eye(8), **kw))
    assert r.n_iterations == int(g[f"{tag}_n_iter"])
    assert np.allclose(r.info.trace_loss, g[f"{tag}_loss"], rtol=1e-12, atol=0)
    assert np.allclose(r.unmixing, g[f"{tag}_unmixing"], rtol=0, atol=1e-10)
