"""The 32x32x32 form of the line-search screen (k_screen_oz32, PICARD_SCREEN32=1).

Its estimate groups each row's samples differently from k_screen_oz2 (4 groups of 4 samples per
lane of a 32-sample step instead of the 4 samples of a 16-sample block), with the same
per-element fp32 arithmetic, so the same rigorous bound must cover it: |Σℓ_exact − Σℓ_screen| ≤
bound for every row, over W of very different scales, ragged T (a last step with one block),
a loud and a silent sample; the two screens' estimates lie within the sum of their bounds, and
their bounds agree (only the κ1·Σ|ỹ| term depends on the kernel).
A screened fit on it takes exactly the exact fit's decisions (bit-identical unmixing).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _mix(rng, n, t):
    s = rng.laplace(size=(n, t))
    a = rng.uniform(-0.5, 0.5, size=(n, n)) + np.eye(n)
    return a @ s


@pytest.mark.parametrize("n", [72, 100, 128])
@pytest.mark.parametrize("alpha", [1.0, 0.5])
@pytest.mark.parametrize("t", [30011, 4099])
def test_screen32_bound_covers_exact(pa, n, alpha, t, monkeypatch):
    monkeypatch.setenv("PICARD_SCREEN_DMAX", "3")  # the 32x32x32 form is a D ≤ 3 screen
    rng = np.random.default_rng(n + t)
    x = _mix(rng, n, t)
    x[:, 7] *= 1e3  # one loud sample
    x[:, 11] = 0.0  # one silent sample
    mu = x.mean(axis=1)
    xc = x - mu[:, None]
    k = np.linalg.cholesky(np.linalg.inv(xc @ xc.T / x.shape[1])).T
    d = pa.DensityType.tanh(alpha)
    monkeypatch.delenv("PICARD_SCREEN32", raising=False)
    c2 = pa.DeviceContext(0)
    c2.load(x)
    monkeypatch.setenv("PICARD_SCREEN32", "1")
    c32 = pa.DeviceContext(0)
    c32.load(x)
    for scale in (1e-4, 0.3, 1.0, 10.0, 300.0):
        w = scale * (np.linalg.qr(rng.normal(size=(n, n)))[0] @ k)
        ll32, b32 = c32.eval_loss_screen(w, mu, d)
        ll2, b2 = c2.eval_loss_screen(w, mu, d)
        lo, _, _ = c32.eval_split(w, mu, d, False, need_y2=False)
        exact = lo["ll"]
        assert np.all(np.abs(exact - ll32) <= b32), (scale, np.max(np.abs(exact - ll32) / b32))
        assert np.all(np.abs(ll32 - ll2) <= b32 + b2)
        assert np.allclose(b32, b2, rtol=1e-3, atol=0.0)  # the same bound (its Σ|ỹ| term per kernel)
    assert c32.screen_stats()[1] == 5


@pytest.mark.parametrize("seed", [1, 2])
def test_screen32_fit_bit_identical(pa, seed, monkeypatch):
    """Picard-O at N = 96 on the int8 stage: the fit screened on k_screen_oz32 takes the same
    decisions as the exact mode (every try evaluated in full)."""
    monkeypatch.setenv("PICARD_SCREEN_DMAX", "3")
    rng = np.random.default_rng(seed)
    x = _mix(rng, 96, 40011)
    cfg = dict(max_iter=60, random_state=seed)

    def fit(mode):
        ctx = pa.DeviceContext(0)
        ctx.load(x)
        ctx.set_y_stage(mode)
        sv = pa.Solver(ctx, pa.PicardConfig(**cfg))
        while not sv.step():
            pass
        r = sv.finish()
        sv.close()
        return r, ctx.screen_stats()[1]

    monkeypatch.setenv("PICARD_SCREEN32", "1")
    r32, ns = fit("auto")
    re_, ne = fit("int8-exact")
    assert ns > 0 and ne == 0
    assert r32.n_iterations == re_.n_iterations and r32.converged == re_.converged
    assert np.array_equal(r32.unmixing, re_.unmixing)
