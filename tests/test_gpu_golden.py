"""GPU path against the committed golden fixtures (tests/golden/)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(G, name))


def test_pass_stats_vs_golden(pa, c1_data):
    g = load("c1_pass_stats.npz")
    x, _, _ = c1_data
    ctx = pa.DeviceContext(0)
    ctx.load(x)
    st = ctx.eval(g["w"], g["mu"], pa.DensityType.tanh(), True)
    for k in ("G", "H", "dpsi", "ll", "y2"):
        err = np.max(np.abs(st[k] - g[k])) / np.max(np.abs(g[k]))
        assert err <= 1e-12, (k, err)


def test_generated_data_vs_golden(pa):
    g = load("c1_data_digest.npz")
    ctx = pa.DeviceContext(0)
    a = ctx.generate(8, 10000, 42)
    x = ctx.download()
    assert np.array_equal(a, g["a"])
    assert np.max(np.abs(x[:, :64] - g["x_first"])) <= 1e-12 * np.max(np.abs(g["x_first"]))
    assert np.max(np.abs(x.sum(axis=1) - g["x_rowsum"])) <= 1e-9


@pytest.mark.parametrize("tag,kw", [("ortho_ext", dict(ortho=True, extended=True)),
                                    ("ortho", dict(ortho=True, extended=False)),
                                    ("nonortho_ext", dict(ortho=False, extended=True)),
                                    ("nonortho", dict(ortho=False, extended=False))])
def test_stepping_trajectory_vs_golden(pa, c1_data, tag, kw):
    """pc_solver_step one iteration at a time: per-iteration loss and gradient norm
    follow the golden trajectory (first iterations to 1e-9 relative; rounding may move
    a near-tie line-search decision late in the run, so the tail is checked by outcome)."""
    g = load("c1_trajectories.npz")
    x, _, a = c1_data
    ctx = pa.DeviceContext(0)
    ctx.load(x)
    s = pa.Solver(ctx, pa.PicardConfig(w_init=np.eye(8), **kw))
    losses, gnorms = [], []
    done = False
    while not done:
        done = s.step()
        loss, gn, _ = s.last()
        losses.append(loss)
        gnorms.append(gn)
    r = s.finish()
    k = min(5, len(g[f"{tag}_loss"]))
    assert np.allclose(losses[:k], g[f"{tag}_loss"][:k], rtol=1e-9, atol=0)
    assert np.allclose(gnorms[:k], g[f"{tag}_gnorm"][:k], rtol=1e-6, atol=0)
    assert r.converged and abs(r.n_iterations - int(g[f"{tag}_n_iter"])) <= 2
    assert abs(pa.utils.amari_distance(r.full_unmixing(), a) - float(g[f"{tag}_amari"])) <= 1e-6


def test_c2_fit_vs_golden(pa):
    """BASELINE config 2 whole on the device (64 × 1e6 bench mixture, seed 42, Picard-O
    extended tanh, w_init = I: the int8 digit Y stage, screens, paired screens and curvature
    rejections all active) against the oracle's fit of the same data (tests/golden/c2_fit.npz,
    make_golden.py c2): the per-iteration losses follow the oracle's, both converge in the same
    number of iterations (±2), and the Amari distances to the generated mixing agree to 1e-6
    (north_star's fp64 tolerance)."""
    g = load("c2_fit.npz")
    ctx = pa.DeviceContext(0)
    a = ctx.generate(64, 1_000_000, 42)
    assert np.array_equal(a, g["a"])
    s = pa.Solver(ctx, pa.PicardConfig(w_init=np.eye(64), want_sources=False))
    losses = []
    done = False
    while not done:
        done = s.step()
        losses.append(s.last()[0])
    r = s.finish()
    assert ctx.int8_passes > 0
    assert np.max(np.abs(r.mean - g["mean"])) <= 1e-12 * np.max(np.abs(g["mean"])) + 1e-15
    k = min(5, len(g["loss"]))
    assert np.allclose(losses[:k], g["loss"][:k], rtol=1e-9, atol=0)
    assert r.converged and abs(r.n_iterations - int(g["n_iter"])) <= 2
    amari = pa.utils.amari_distance(r.full_unmixing(), a)
    assert abs(amari - float(g["amari"])) <= 1e-6, (amari, float(g["amari"]))
