"""The line-search screen's statistical tail bound and the D ≤ 2 screen (DeviceCtx::screen_rank_bound).

The exact stage's y differs from a D ≤ dmax screen's by Σ_{dmax < a+b ≤ 6} W_a·X_b (the digit
levels of W and X). Besides the worst case (every digit at its largest) the bound now takes, per
row, Σ 2^(f_i−12−8(a+b))·√(S4·λ_b·‖w_a,i‖²) — Cauchy–Schwarz over the samples with weights 2^e_t
and the largest eigenvalue of the digit Gram D_b = Σ_t d_b,t·d_b,tᵀ — whichever is smaller. Here:
the device's digit Grams (k_digit_gram) give exactly numpy's Gershgorin bounds of the image's
digits, the D ≤ 2 screen's bound covers the exact pass, and fits screened from D ≤ 2 or D ≤ 3 stay
bit-identical to the unscreened int8 fit."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _digits7(v):
    """ozaki.inc oz_digits: 7 round-to-nearest radix-256 digits, ±128/±129 folded upward"""
    dg = []
    for _ in range(7):
        r = np.rint(v)
        dg.append(r.astype(np.int64))
        v = (v - r) * 256.0
    for b in range(6, 0, -1):
        hi, lo = dg[b] > 127, dg[b] < -128
        dg[b] = np.where(hi, dg[b] - 256, np.where(lo, dg[b] + 256, dg[b]))
        dg[b - 1] = dg[b - 1] + hi.astype(np.int64) - lo.astype(np.int64)
    return dg


def _laplace_mix(rng, n, t):
    s = rng.laplace(size=(n, t))
    a = rng.uniform(-0.5, 0.5, size=(n, n)) + np.eye(n)
    return a @ s


@pytest.mark.parametrize("n,t", [(128, 40011), (100, 20000), (64, 30001), (48, 16 * 2047 * 4 + 37)])
def test_digit_gram_matches_numpy(pa, n, t):
    """k_digit_gram's Gershgorin bounds equal numpy's on the same digits (exact integers), for
    both image layouts (nf ≤ 64: one k-step) and a workgroup range that fills DG_MAX_CHUNKS."""
    rng = np.random.default_rng(n + t)
    x = _laplace_mix(rng, n, t)
    x[:, 5] = 0.0  # a silent sample: zero digits, scale 1
    mu = x.mean(axis=1)
    ctx = pa.DeviceContext(0)
    ctx.load(x)
    w = np.linalg.qr(rng.normal(size=(n, n)))[0]
    ctx.eval_loss_screen(w, mu, pa.DensityType.tanh())  # centres the resident X, builds the image
    lam, s4 = ctx.screen_digit_gram()
    ctx.close()
    xc = x - mu[:, None]
    e = np.frexp(np.abs(xc).max(axis=0))[1]
    dg = _digits7(xc * np.ldexp(1.0, 6 - e)[None, :])
    for b in range(7):
        d = dg[b].astype(np.float64)
        gersh = np.abs(d @ d.T).sum(axis=1).max()
        assert lam[b] == pytest.approx(gersh, rel=1e-11), (b, lam[b], gersh)
        assert lam[b] >= gersh
    s4_np = np.sum(np.ldexp(1.0, 2 * e))
    pad = s4 - s4_np  # padding samples carry 4^0 = 1 each
    assert 0.0 <= pad <= 1e-7 * s4 + 16 * 2048, (s4, s4_np)


@pytest.mark.parametrize("n", [128, 96])
def test_d2_screen_bound_covers_exact(pa, n, monkeypatch):
    """The D ≤ 2 fp32 screen (statistical tail) against the exact loss-only pass on the bench
    mixture: covered, and the bound small enough to decide the C3 searches' rejections
    (≈ 1e-2 per sample at the fit's scale, W = Q·P: DESIGN.md §3)."""
    monkeypatch.setenv("PICARD_SCREEN_DMAX", "2")
    rng = np.random.default_rng(3 * n)
    t = 200003
    ctx = pa.DeviceContext(0)
    ctx.generate(n, t, 42)
    mu = ctx.rowsum() / t
    d = pa.DensityType.tanh()
    # whitening of the generated mixture (the solver's P), so W·P has the fit's scales
    g = ctx.gram(mu) / t
    ev, evec = np.linalg.eigh(g)
    p = (evec / np.sqrt(ev)).T
    worst = 0.0
    for scale in (0.5, 1.0, 2.0):
        w = scale * (np.linalg.qr(rng.normal(size=(n, n)))[0] @ p)
        ll, bnd = ctx.eval_loss_screen(w, mu, d)
        lo, _, _ = ctx.eval_split(w, mu, d, False, need_y2=False)
        exact = lo["ll"]
        assert np.all(np.abs(exact - ll) <= bnd), (scale, np.max(np.abs(exact - ll) / bnd))
        worst = max(worst, bnd.sum() / t)
    ctx.close()
    print(f"n={n}: D<=2 bound {worst:.3e} per sample (sum over rows)")
    assert worst <= 3e-2


@pytest.mark.parametrize("dmax", ["2", "3"])
@pytest.mark.parametrize("n,seed", [(128, 42), (64, 42)])
def test_screen_chain_fit_bit_identical(pa, n, seed, dmax, capfd, monkeypatch):
    """Picard-O on the bench mixture screened from D ≤ dmax (with the finer levels after it) and
    unscreened (int8-exact): identical iterations, bit-identical unmixing."""
    monkeypatch.setenv("PICARD_TRACE", "1")
    monkeypatch.setenv("PICARD_SCREEN_DMAX", dmax)
    res = {}
    for mode in ("auto", "int8-exact"):
        ctx = pa.DeviceContext(0)
        ctx.generate(n, 200003, seed)
        ctx.set_y_stage(mode)
        sv = pa.Solver(ctx, pa.PicardConfig(random_state=42, max_iter=60))
        while not sv.step():
            pass
        res[mode] = (sv.finish(), ctx.screen_stats()[1])
        sv.close()
        ctx.close()
    err = capfd.readouterr().err
    (r, ns), (r0, ns0) = res["auto"], res["int8-exact"]
    assert ns > 0 and ns0 == 0
    assert r.n_iterations == r0.n_iterations and r.converged == r0.converged
    assert np.array_equal(r.unmixing, r0.unmixing)
    rej = sum(1 for line in err.splitlines() if line.startswith("[picard-screen]") and line.endswith("reject")
              or "reject (pair" in line)
    fine = sum(1 for line in err.splitlines() if line.startswith("[picard-screen] fine"))
    print(f"dmax {dmax}: screen passes {ns}, rejections {rej}, finer screens {fine}")
    assert rej > 0
