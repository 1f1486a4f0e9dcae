"""The C++ host driver (core::run, L-BFGS, line search, whitening, warm starts)
run through pc_fit_with_evaluator with the per-pass statistics supplied by
callbacks. The callbacks compute the same sums the HIP pass produces, so this
checks the host logic against the oracle on a CPU-only machine. The product
path never uses these callbacks (they are a test hook of the C ABI)."""
import numpy as np
import pytest

from conftest import density_of


def host_fit(pa, po, x, cfg):
    def ev(w, mu, d, need_h):
        return po.pass_stats(w, mu, x, density_of(po, d), need_h)

    def gram(mu):
        xc = x - mu[:, None] if mu is not None else x
        return xc @ xc.T

    def sources(w, mu):
        return w @ (x - mu[:, None] if mu is not None else x)

    def m4(w, mu):
        y = sources(w, mu)
        n = y.shape[0]
        z = np.stack([y[i] * y[j] for i in range(n) for j in range(i, n)])
        return z @ z.T

    return pa.fit_with_host_evaluator(x.shape[0], x.shape[1], cfg, rowsum=lambda: x.sum(axis=1), gram=gram,
                                      eval=ev, sources=sources, moments4=m4)


@pytest.mark.parametrize("ortho,extended", [(True, True), (True, False), (False, True), (False, False)])
def test_core_run_matches_oracle(pa, po, c1_data, ortho, extended):
    x, s, a = c1_data
    r = host_fit(pa, po, x, pa.PicardConfig(w_init=np.eye(8), ortho=ortho, extended=extended))
    ro = po.fit_with_config(x, po.PicardConfig(w_init=np.eye(8), ortho=ortho, extended=extended))
    assert r.converged and ro.converged
    assert abs(r.n_iterations - ro.n_iterations) <= 2
    if ortho:  # identical trajectories: same pass count, W to rounding
        assert r.n_iterations == ro.n_iterations and r.n_evaluations == ro.info.n_evals
        assert np.max(np.abs(r.unmixing - ro.unmixing)) < 1e-10
    assert abs(pa.utils.amari_distance(r.full_unmixing(), a) - po.amari_distance(ro.full_unmixing(), a)) < 1e-6
    assert np.max(np.abs(r.whitening - ro.whitening)) < 1e-8


@pytest.mark.parametrize("kw", [dict(n_components=5), dict(whiten=False), dict(centering=False),
                                dict(whiten=False, extended=True, ortho=False), dict(fastica_it=5),
                                dict(jade_it=2), dict(m=2, ls_tries=3), dict(lambda_min=0.5), dict(tol=1e-4)])
def test_config_variants(pa, po, c1_data, kw):
    x, s, a = c1_data
    nc = kw.get("n_components", 8)
    r = host_fit(pa, po, x, pa.PicardConfig(w_init=np.eye(nc), max_iter=300, **kw))
    ro = po.fit_with_config(x, po.PicardConfig(w_init=np.eye(nc), max_iter=300, **kw))
    assert r.converged == ro.converged
    fw, fwo = r.full_unmixing(), ro.full_unmixing()
    assert np.max(np.abs(fw - fwo)) <= 1e-6 * np.max(np.abs(fwo))
    assert (r.whitening is None) == (ro.whitening is None)
    assert (r.mean is None) == (ro.mean is None)


@pytest.mark.parametrize("dens", [("exp", 1.0), ("cube", 1.0), ("tanh", 0.5)])
def test_densities(pa, po, c1_data, dens):
    x, s, a = c1_data
    pd = pa.DensityType(["tanh", "exp", "cube"].index(dens[0]), dens[1])
    r = host_fit(pa, po, x, pa.PicardConfig(w_init=np.eye(8), density=pd, max_iter=200))
    ro = po.fit_with_config(x, po.PicardConfig(w_init=np.eye(8), density=po.Density(*dens), max_iter=200))
    assert r.n_iterations == ro.n_iterations and r.converged == ro.converged
    assert np.max(np.abs(r.unmixing - ro.unmixing)) < 1e-8


def test_max_iter_and_counts(pa, po, c1_data):
    x, s, a = c1_data
    r = host_fit(pa, po, x, pa.PicardConfig(w_init=np.eye(8), max_iter=3))
    ro = po.fit_with_config(x, po.PicardConfig(w_init=np.eye(8), max_iter=3))
    assert r.n_iterations == ro.n_iterations == 3  # core.rs:396 (last iter + 1)
    assert not r.converged
    assert np.max(np.abs(r.unmixing - ro.unmixing)) < 1e-10


def test_verbose_lines(pa, po, c1_data, capfd):
    x, s, a = c1_data
    host_fit(pa, po, x, pa.PicardConfig(w_init=np.eye(8), max_iter=2, verbose=True))
    out = capfd.readouterr().out.splitlines()
    assert out[0] == "Running Picard..."
    assert out[1].startswith("iteration 1, gradient norm = ") and ", loss = " in out[1]
    ro = po.fit_with_config(x, po.PicardConfig(w_init=np.eye(8), max_iter=2))
    assert out[1] == (f"iteration 1, gradient norm = {po.rust_e4(ro.info.trace_gnorm[0])}, "
                      f"loss = {po.rust_e4(ro.info.trace_loss[0])}")


def test_errors(pa, po, c1_data):
    x, s, a = c1_data
    with pytest.raises(pa.InvalidDimensions, match=r"w_init shape \[3, 3\] doesn't match expected \(8, 8\)"):
        host_fit(pa, po, x, pa.PicardConfig(w_init=np.eye(3)))
    with pytest.raises(pa.InvalidConfig):
        host_fit(pa, po, x, pa.PicardConfig(m=0))
    with pytest.raises(pa.SingularMatrix):
        host_fit(pa, po, np.ones((3, 50)), pa.PicardConfig())


def test_seeded_random_init_is_deterministic(pa, po, c1_data):
    x, s, a = c1_data
    r1 = host_fit(pa, po, x, pa.PicardConfig(random_state=7))
    r2 = host_fit(pa, po, x, pa.PicardConfig(random_state=7))
    assert np.array_equal(r1.unmixing, r2.unmixing)
    assert r1.converged and po.amari_distance(r1.full_unmixing(), a) < 0.01


@pytest.mark.parametrize("n,t,extended", [(16, 20000, True), (12, 15000, False)])
def test_screened_line_search_decisions_unchanged(pa, po, dg, n, t, extended):
    """The orthogonal line-search screen (Evaluator::eval_loss_screen) changes no decision:
    with a screen that returns the exact Σℓ moved anywhere inside its stated bound, the fit
    is bit-identical to the unscreened one (same iterations, same unmixing bits), the screen
    rejects tries (fewer exact passes) and no try is rejected that the exact pass accepts."""
    x, _ = dg.generate_data(n, t, 42)[:2]
    rng = np.random.default_rng(0)
    calls = {"screen": 0, "eval": 0}

    def ev(w, mu, d, need_h):
        calls["eval"] += 1
        return po.pass_stats(w, mu, x, density_of(po, d), need_h)

    def screen(w, mu, d):
        calls["screen"] += 1
        ll = po.pass_stats(w, mu, x, density_of(po, d), False)["ll"]
        bnd = 1e-9 * np.abs(ll) + 1e-12
        return ll + rng.uniform(-0.9, 0.9, size=ll.shape) * bnd, bnd

    def fit(with_screen):
        calls.update(screen=0, eval=0)
        kw = dict(eval_loss_screen=screen) if with_screen else {}
        r = pa.fit_with_host_evaluator(
            x.shape[0], x.shape[1], pa.PicardConfig(random_state=42, extended=extended, max_iter=60),
            rowsum=lambda: x.sum(axis=1), gram=lambda mu: (x - mu[:, None]) @ (x - mu[:, None]).T,
            eval=ev, sources=lambda w, mu: w @ (x - mu[:, None]), **kw)
        return r, dict(calls)

    r0, c0 = fit(False)
    r1, c1 = fit(True)
    assert c0["screen"] == 0 and c1["screen"] > 0
    assert r1.n_iterations == r0.n_iterations and r1.converged == r0.converged
    assert np.array_equal(r1.unmixing, r0.unmixing)
    assert c1["eval"] < c0["eval"]  # rejected tries ran no exact pass


def test_curvature_rejection_decisions_unchanged(pa, po, dg, capfd, monkeypatch):
    """Orthogonal tries rejected by the curvature bound (Solver::set_curvature) run no pass and
    change no decision: the bench mixture at N=16 has searches along non-descent directions
    whose small-α tries the bound rejects; the fit is bit-identical to the every-try-exact one."""
    monkeypatch.setenv("PICARD_TRACE", "1")
    x, _ = dg.generate_data(16, 20000, 42)[:2]

    def ev(w, mu, d, need_h):
        return po.pass_stats(w, mu, x, density_of(po, d), need_h)

    def screen(w, mu, d):
        ll = po.pass_stats(w, mu, x, density_of(po, d), False)["ll"]
        return ll, 1e-9 * np.abs(ll) + 1e-12

    def fit(with_screen):
        kw = dict(eval_loss_screen=screen) if with_screen else {}
        return pa.fit_with_host_evaluator(
            x.shape[0], x.shape[1], pa.PicardConfig(random_state=42, max_iter=60),
            rowsum=lambda: x.sum(axis=1), gram=lambda mu: (x - mu[:, None]) @ (x - mu[:, None]).T,
            eval=ev, sources=lambda w, mu: w @ (x - mu[:, None]), **kw)

    r0 = fit(False)
    n0 = capfd.readouterr().err.count("[picard-curv]")
    r1 = fit(True)
    n1 = capfd.readouterr().err.count("[picard-curv]")
    assert n0 == 0 and n1 > 0  # only once the evaluator screens
    assert r1.n_iterations == r0.n_iterations and r1.converged == r0.converged
    assert np.array_equal(r1.unmixing, r0.unmixing)


@pytest.mark.parametrize("a,mixed,aniso", [(1.0, True, False), (1.0, False, False), (0.5, True, False),
                                           (2.0, False, False), (1.0, True, True), (2.0, True, True)])
def test_curvature_bound_holds(a, mixed, aniso):
    """The bound behind the curvature rejection (Solver::set_curvature / curvature_lower_bound):
    on whitened data, along W(α) = expm(αD)·W with D skew-symmetric, the tanh loss
    L(α) = Σ_i s_i mean_t ℓ(y_it) satisfies L(α) − L(0) ≥ α·s + ∫_0^α (α − β)·m(β) dβ with
    m(β) = max(q − β·K3, −M), A_k = tr(D^k·Cy·D^kᵀ), Cy = mean_t y_t y_tᵀ, A1⁻ = the rows of A1
    with s_i < 0, q = v0 − a·A1⁻, M = a·(A1⁻ + √(A0·A2)), K3 = a·(√(A1·A2) + √(A0·A3)),
    v0 = ⟨g_s, D²⟩ (g_s = s_i·(ψ·Yᵀ)_ij/T), s = ⟨g_s, D⟩ (no margins here: the solver takes
    1.01·Cy). The bound is at least the round-2 pair max(α·s − α²·a·(A1 + √(A0·A2))/2,
    α·s + α²·q/2 − α³·K3/6). A1⁻ = min(A1, λ·Σ_{s_i<0}(D·Dᵀ)_ii), λ = the Gershgorin bound on
    λmax(Cy): it bounds the negative rows at every α, so the bound holds for an anisotropic Cy
    too (aniso: rows scaled up to 4x after whitening)."""
    from scipy.linalg import expm
    rng = np.random.default_rng(5)
    n, t = 8, 4000
    x = rng.laplace(size=(n, t))
    x -= x.mean(axis=1, keepdims=True)
    ev, u = np.linalg.eigh(x @ x.T / t)
    x = (u / np.sqrt(ev)).T @ x  # whitened: covariance I
    if aniso:  # far from isotropic, with a rotation so Cy is not diagonal
        q0 = np.linalg.qr(rng.normal(size=(n, n)))[0]
        x = q0 @ (np.geomspace(0.25, 4.0, n)[:, None] * x)
    w = np.linalg.qr(rng.normal(size=(n, n)))[0]
    s = np.sign(rng.normal(size=n)) if mixed else np.ones(n)
    if aniso:
        s[: n // 2] = -1.0  # several negative rows

    def ell(y):  # density.rs Tanh log_lik: |y| + log1p(exp(-2a|y|))/a
        return np.abs(y) + np.log1p(np.exp(-2 * a * np.abs(y))) / a

    def loss(wm):
        return float(np.sum(s * ell(wm @ x).mean(axis=1)))

    y = w @ x
    gs = s[:, None] * (np.tanh(a * y) @ y.T) / t
    cy = y @ y.T / t
    tr = lambda m: float(np.trace(m @ cy @ m.T))  # noqa: E731
    for _ in range(20):
        d = rng.normal(size=(n, n)) * rng.uniform(0.01, 1.0)
        d = (d - d.T) / 2
        slope = float(np.sum(gs * d))
        d2 = d @ d
        a0, a1, a2, a3 = float(np.trace(cy)), tr(d), tr(d2), tr(d2 @ d)
        lam = float(np.max(np.sum(np.abs(cy), axis=1)))
        a1n = min(a1, lam * float(np.sum((d * d)[s < 0])))
        m_old = a * (a1 + np.sqrt(a0 * a2))
        m = a * (a1n + np.sqrt(a0 * a2))
        q = float(np.sum(gs * d2)) - a * a1n
        k3 = a * (np.sqrt(a1 * a2) + np.sqrt(a0 * a3))
        for alpha in 2.0 ** -np.arange(0, 10):
            lhs = loss(expm(alpha * d) @ w) - loss(w)
            b = min(max((q + m) / k3, 0.0), alpha)
            bound = (alpha * slope + q * b * (alpha - b / 2) - k3 * b * b * (alpha / 2 - b / 3)
                     - m * (alpha - b) ** 2 / 2)
            b2 = alpha * slope - alpha * alpha * m_old / 2
            b3 = alpha * slope + alpha * alpha * q / 2 - alpha ** 3 * k3 / 6
            assert bound >= max(b2, b3) - 1e-15 * (1 + abs(bound)), (alpha, bound, b2, b3)
            assert lhs >= bound - 1e-12, (alpha, lhs, bound)


@pytest.mark.parametrize("n,t,seed", [(16, 20000, 42), (24, 20000, 42)])
def test_model_schedule_decisions_unchanged(pa, po, dg, n, t, seed, capfd, monkeypatch):
    """The quadratic-model schedule (Solver::step's first-try cells, line_search's later-try
    full passes, "[picard-model]") changes no decision: with a screen the fit runs some later
    tries as full passes straight away, and stays bit-identical to the every-try-exact fit."""
    monkeypatch.setenv("PICARD_TRACE", "1")
    x, _ = dg.generate_data(n, t, seed)[:2]

    def ev(w, mu, d, need_h):
        return po.pass_stats(w, mu, x, density_of(po, d), need_h)

    def screen(w, mu, d):
        ll = po.pass_stats(w, mu, x, density_of(po, d), False)["ll"]
        return ll, 1e-9 * np.abs(ll) + 1e-12

    def fit(with_screen):
        kw = dict(eval_loss_screen=screen) if with_screen else {}
        return pa.fit_with_host_evaluator(
            x.shape[0], x.shape[1], pa.PicardConfig(random_state=42, max_iter=60),
            rowsum=lambda: x.sum(axis=1), gram=lambda mu: (x - mu[:, None]) @ (x - mu[:, None]).T,
            eval=ev, sources=lambda w, mu: w @ (x - mu[:, None]), **kw)

    r0 = fit(False)
    capfd.readouterr()
    r1 = fit(True)
    err = capfd.readouterr().err
    assert "[picard-model]" in err and "[picard-pred]" in err
    assert r1.n_iterations == r0.n_iterations and r1.converged == r0.converged
    assert np.array_equal(r1.unmixing, r0.unmixing)


@pytest.mark.parametrize("group", [1, 3])
def test_staged_multi_try_decisions_unchanged(pa, po, dg, group, monkeypatch):
    """Non-orthogonal searches with the tries split over two multi-try passes (the first covers
    `group` tries, PICARD_MULTI_GROUP) decide exactly as with all tries in one pass: each try's
    sums do not depend on the pass that carries it. Counts the passes to show the split ran."""
    x, _ = dg.generate_data(12, 8000, 42)[:2]
    calls = []

    def ev(w, mu, d, need_h):
        return po.pass_stats(w, mu, x, density_of(po, d), need_h)

    def multi(w, z, alphas, mu, d):
        calls.append(len(alphas))
        ll, y2 = [], []
        for a in alphas:
            st = po.pass_stats(w + a * z, mu, x, density_of(po, d), False)
            ll.append(st["ll"])
            y2.append(st["y2"])
        return np.array(ll), np.array(y2)

    def fit():
        calls.clear()
        r = pa.fit_with_host_evaluator(
            x.shape[0], x.shape[1], pa.PicardConfig(ortho=False, extended=False, random_state=7, max_iter=80),
            rowsum=lambda: x.sum(axis=1), gram=lambda mu: (x - mu[:, None]) @ (x - mu[:, None]).T,
            eval=ev, sources=lambda w, mu: w @ (x - mu[:, None]), eval_loss_multi=multi)
        return r, list(calls)

    monkeypatch.delenv("PICARD_MULTI_GROUP", raising=False)
    r0, c0 = fit()
    monkeypatch.setenv("PICARD_MULTI_GROUP", str(group))
    r1, c1 = fit()
    assert c0 and max(c0) > group  # one pass per search carried more than `group` tries
    assert max(c1[i] for i in range(len(c1))) >= 1 and all(n <= max(c0) for n in c1)
    assert any(n == group for n in c1)  # first passes capped at `group` tries
    assert r1.n_iterations == r0.n_iterations and r1.converged == r0.converged
    assert np.array_equal(r1.unmixing, r0.unmixing)


@pytest.mark.parametrize("a,aniso", [(1.0, False), (0.5, False), (2.0, False), (1.0, True)])
def test_convexity_bound_holds(a, aniso):
    """The bound behind the non-orthogonal convexity rejection (Solver::convexity_trim): along
    W(α) = (I + αD)·W the tanh loss L(α) = −log|det W(α)| + Σ_i mean_t ℓ(y_it(α)) satisfies
    L(α) − L(0) ≥ α·Σ_ij D_ij·G_ij/T − Σ_k ½·log((1 + α·D_kk)² + α²·Σ_{j≠k} D_kj²) with
    G = ψ(Y)·Yᵀ (convexity of ℓ along the affine y(α), Hadamard's inequality for the determinant),
    for general D (descent and non-descent, small and large) and W."""
    rng = np.random.default_rng(11)
    n, t = 8, 4000
    x = rng.laplace(size=(n, t))
    x -= x.mean(axis=1, keepdims=True)
    ev, u = np.linalg.eigh(x @ x.T / t)
    x = (u / np.sqrt(ev)).T @ x
    if aniso:
        x = np.geomspace(0.25, 4.0, n)[:, None] * x

    def ell(y):  # density.rs Tanh log_lik
        return np.abs(y) + np.log1p(np.exp(-2 * a * np.abs(y))) / a

    def loss(wm):
        return -np.linalg.slogdet(wm)[1] + float(np.sum(ell(wm @ x).mean(axis=1)))

    hits = 0
    for _ in range(30):
        w = rng.normal(size=(n, n)) + 2 * np.eye(n)
        y = w @ x
        g = np.tanh(a * y) @ y.T / t
        d = rng.normal(size=(n, n)) * rng.uniform(0.01, 2.0)
        fp = float(np.sum(d * g))
        off = np.sum(d * d, axis=1) - np.diag(d) ** 2
        for alpha in 2.0 ** -np.arange(0, 10):
            h = 0.5 * np.sum(np.log((1 + alpha * np.diag(d)) ** 2 + alpha * alpha * off))
            bound = alpha * fp - h
            lhs = loss((np.eye(n) + alpha * d) @ w) - loss(w)
            assert lhs >= bound - 1e-12 * (1 + abs(lhs)), (alpha, lhs, bound)
            hits += bound > 0
    assert hits > 0  # the bound does reject tries in this sample


def test_convexity_rejection_decisions_unchanged(pa, po, dg, capfd, monkeypatch):
    """Non-orthogonal tries rejected by the convexity bound (Solver::convexity_trim) run no pass
    and change no decision: on the bench mixture some L-BFGS directions do not descend, their
    trailing tries (all of them, for some searches) are dropped, and the fit is bit-identical to
    the one with every try evaluated (PICARD_CVX=0)."""
    monkeypatch.setenv("PICARD_TRACE", "1")
    x, _ = dg.generate_data(12, 8000, 42)[:2]
    calls = []

    def ev(w, mu, d, need_h):
        return po.pass_stats(w, mu, x, density_of(po, d), need_h)

    def multi(w, z, alphas, mu, d):
        calls.append(len(alphas))
        ll, y2 = [], []
        for al in alphas:
            st = po.pass_stats(w + al * z, mu, x, density_of(po, d), False)
            ll.append(st["ll"])
            y2.append(st["y2"])
        return np.array(ll), np.array(y2)

    def fit(cvx):
        monkeypatch.setenv("PICARD_CVX", "1" if cvx else "0")
        calls.clear()
        r = pa.fit_with_host_evaluator(
            x.shape[0], x.shape[1], pa.PicardConfig(ortho=False, extended=False, random_state=7, max_iter=80),
            rowsum=lambda: x.sum(axis=1), gram=lambda mu: (x - mu[:, None]) @ (x - mu[:, None]).T,
            eval=ev, sources=lambda w, mu: w @ (x - mu[:, None]), eval_loss_multi=multi)
        return r, sum(calls), capfd.readouterr().err

    r0, t0, e0 = fit(False)
    r1, t1, e1 = fit(True)
    assert "[picard-cvx]" not in e0 and "[picard-cvx]" in e1
    assert t1 < t0  # fewer tries evaluated
    assert r1.n_iterations == r0.n_iterations and r1.converged == r0.converged
    assert np.array_equal(r1.unmixing, r0.unmixing)
