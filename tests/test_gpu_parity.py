"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Tolerances (fp64 throughout; differences are summation order only):
  * fused-pass statistics (G_raw, H_raw, Σψ′, Σℓ, Σy²): max-abs error ≤ 1e-12 × max|oracle|
  * rowsum / Gram / sources / fourth moments: the same 1e-12 relative bound
  * end-to-end fits on BASELINE config 1 (8 × 10k): both converge, Amari distance
    within 1e-6 of the oracle's (north_star), unmixing within 1e-6, iteration
    count within ±2 (rounding can move a line-search accept near tol).
"""
import numpy as np
import pytest

from conftest import density_of, rel_err

pytestmark = pytest.mark.gpu

TOL = 1e-12


@pytest.fixture(scope="module")
def rng():
    return np.random.default_rng(1234)


def laplace_mix(rng, nf, t):
    s = rng.laplace(size=(nf, t))
    a = rng.uniform(-0.5, 0.5, size=(nf, nf)) + np.eye(nf)
    return a @ s + rng.normal(size=(nf, 1))


def ctx_with(pa, x):
    ctx = pa.DeviceContext(0)
    ctx.load(x)
    return ctx


DENSITIES = [("tanh", 1.0), ("tanh", 0.7), ("exp", 1.0), ("exp", 0.1), ("cube", 1.0)]


@pytest.mark.parametrize("n", [8, 16, 30, 64, 100, 128, 160, 256])
@pytest.mark.parametrize("dens", DENSITIES)
@pytest.mark.parametrize("need_h", [False, True])
def test_eval_stats_vs_oracle(pa, po, rng, n, dens, need_h):
    t = 5003  # ragged: not a multiple of any block size
    x = laplace_mix(rng, n, t)
    ctx = ctx_with(pa, x)
    w = rng.normal(size=(n, n)) / np.sqrt(n)
    mu = x.mean(axis=1)
    d = pa.DensityType(["tanh", "exp", "cube"].index(dens[0]), dens[1])
    got = ctx.eval(w, mu, d, need_h)
    want = po.pass_stats(w, mu, x, density_of(po, d), need_h)
    for k in want:
        assert rel_err(got[k], want[k]) <= TOL, (k, rel_err(got[k], want[k]))


@pytest.mark.parametrize("nc,nf", [(5, 12), (3, 8), (16, 40), (64, 200), (20, 128)])
def test_eval_rectangular(pa, po, rng, nc, nf):
    t = 3001
    x = laplace_mix(rng, nf, t)
    ctx = ctx_with(pa, x)
    w = rng.normal(size=(nc, nf)) / np.sqrt(nf)
    mu = x.mean(axis=1)
    got = ctx.eval(w, mu, pa.DensityType.tanh(), True)
    want = po.pass_stats(w, mu, x, po.Density("tanh", 1.0), True)
    for k in want:
        assert rel_err(got[k], want[k]) <= TOL, k


def test_eval_no_mean_and_tiny_t(pa, po, rng):
    for t in [1, 2, 15, 17, 129]:
        x = laplace_mix(rng, 8, t)
        ctx = ctx_with(pa, x)
        w = rng.normal(size=(8, 8))
        got = ctx.eval(w, None, pa.DensityType.tanh(), False)
        want = po.pass_stats(w, None, x, po.Density("tanh", 1.0), False)
        for k in want:
            assert rel_err(got[k], want[k]) <= TOL, (t, k)


@pytest.mark.parametrize("n", [8, 64, 128])
@pytest.mark.parametrize("dens", DENSITIES)
def test_skip_y2_changes_nothing_else(pa, rng, n, dens):
    """PC_EVAL_SKIP_Y2 (the orthogonal solver's mode): Σy² reads 0, every other
    statistic is bit-identical to the pass that accumulates Σy²."""
    x = laplace_mix(rng, n, 3001)
    ctx = ctx_with(pa, x)
    w = rng.normal(size=(n, n)) / np.sqrt(n)
    mu = x.mean(axis=1)
    d = pa.DensityType(["tanh", "exp", "cube"].index(dens[0]), dens[1])
    a = ctx.eval(w, mu, d, False, need_y2=True)
    b = ctx.eval(w, mu, d, False, need_y2=False)
    for k in ("G", "dpsi", "ll"):
        assert np.array_equal(a[k], b[k]), k
    if dens[0] != "cube":  # cube keeps Σy² (its Σψ′ = 3·Σy²)
        assert not b["y2"].any()


@pytest.mark.parametrize("n", [8, 30, 64, 128, 200])
@pytest.mark.parametrize("dens", [("tanh", 1.0), ("exp", 0.5), ("cube", 1.0)])
@pytest.mark.parametrize("need_h,need_y2", [(False, True), (True, True), (False, False)])
def test_split_eval_bit_identical(pa, rng, n, dens, need_h, need_y2):
    """Loss-only try + completion from the kept Y == one fused pass, bit for bit (fp64 Y
    stage in both; the int8-slice stage is checked against these in test_gpu_int8.py)."""
    x = laplace_mix(rng, n, 4099)
    ctx = ctx_with(pa, x)
    ctx.set_y_stage("f64")
    w = rng.normal(size=(n, n)) / np.sqrt(n)
    mu = x.mean(axis=1)
    d = pa.DensityType(["tanh", "exp", "cube"].index(dens[0]), dens[1])
    full = ctx.eval(w, mu, d, need_h, need_y2=need_y2)
    loss_only, kept, done = ctx.eval_split(w, mu, d, need_h, need_y2=need_y2)
    assert np.array_equal(loss_only["ll"], full["ll"]) and np.array_equal(loss_only["y2"], full["y2"])
    if kept:
        assert np.isnan(loss_only["G"]).all()
    for k in full:
        assert np.array_equal(done[k], full[k]), k


@pytest.mark.parametrize("nc,nf", [(8, 8), (30, 30), (64, 64), (100, 100), (256, 256), (20, 70)])
@pytest.mark.parametrize("dens", [("tanh", 1.0), ("tanh", 0.6), ("exp", 0.5), ("cube", 1.0)])
def test_multi_try_loss_pass(pa, rng, nc, nf, dens):
    """Non-ortho line search in one pass: Σℓ, Σy² of (w + α_j z)(X − μ) for every try α_j
    equal a separate pass at each try to 1e-12 relative (Y_j is formed as Y + α_j Z,
    so they differ by rounding only). 13 tries exercise the 12-per-pass chunking."""
    x = laplace_mix(rng, nf, 3001)
    ctx = ctx_with(pa, x)
    w = rng.normal(size=(nc, nf)) / np.sqrt(nf)
    z = rng.normal(size=(nc, nf)) / np.sqrt(nf)
    mu = x.mean(axis=1)
    d = pa.DensityType(["tanh", "exp", "cube"].index(dens[0]), dens[1])
    alphas = 0.5 ** np.arange(1, 14)
    ll, y2 = ctx.eval_loss_multi(w, z, alphas, mu, d)
    for j, a in enumerate(alphas):
        ref = ctx.eval(w + a * z, mu, d)
        assert rel_err(ll[j], ref["ll"]) <= TOL, j
        assert rel_err(y2[j], ref["y2"]) <= TOL, j


def test_multi_try_schedule_matches_per_try(pa, rng, monkeypatch):
    """A non-ortho fit with the one-pass line search takes the same iterations as one
    with a pass per try (PICARD_NO_MULTI=1) and lands on the same unmixing."""
    x = laplace_mix(rng, 40, 20000)
    cfg = dict(ortho=False, extended=True, max_iter=200, random_state=3)
    r1 = pa.Picard.fit_with_config(x, pa.PicardConfig(**cfg))
    monkeypatch.setenv("PICARD_NO_MULTI", "1")
    r2 = pa.Picard.fit_with_config(x, pa.PicardConfig(**cfg))
    assert r1.converged and r2.converged
    assert abs(r1.n_iterations - r2.n_iterations) <= 2
    assert np.max(np.abs(r1.unmixing - r2.unmixing)) <= 1e-6


@pytest.mark.parametrize("knob", ["PICARD_KEEP_Y", "PICARD_SPLIT_FIRST"])
def test_ortho_schedule_knobs_bit_identical(pa, rng, monkeypatch, knob):
    """The orthogonal line-search schedules (host_solver.hpp: Y kept in HBM for the
    completion; try 1 loss-only) change which passes run, never the sums: the fit is
    bit-identical to the default schedule (64 < N ≤ 128: the split kernels)."""
    x = laplace_mix(rng, 96, 20000)
    cfg = dict(max_iter=40, random_state=5)

    def fit():
        ctx = ctx_with(pa, x)
        ctx.set_y_stage("f64")  # one Y-stage arithmetic for every pass kind
        sv = pa.Solver(ctx, pa.PicardConfig(**cfg))
        while not sv.step():
            pass
        r = sv.finish()
        sv.close()
        return r

    r1 = fit()
    monkeypatch.setenv(knob, "1")
    r2 = fit()
    assert r1.n_iterations == r2.n_iterations and r1.converged == r2.converged
    assert np.array_equal(r1.unmixing, r2.unmixing)


def test_eval_deterministic(pa, rng):
    x = laplace_mix(rng, 64, 20000)
    ctx = ctx_with(pa, x)
    w = rng.normal(size=(64, 64))
    a = ctx.eval(w, None, pa.DensityType.tanh(), False)
    b = ctx.eval(w, None, pa.DensityType.tanh(), False)
    for k in a:
        assert np.array_equal(a[k], b[k])


def test_rowsum_gram_sources(pa, rng):
    for nf in [8, 64, 150]:
        x = laplace_mix(rng, nf, 4097)
        ctx = ctx_with(pa, x)
        assert rel_err(ctx.rowsum(), x.sum(axis=1)) <= TOL
        mu = x.mean(axis=1)
        xc = x - mu[:, None]
        assert rel_err(ctx.gram(mu), xc @ xc.T) <= TOL
        assert rel_err(ctx.gram(None), x @ x.T) <= TOL
        w = rng.normal(size=(nf // 2, nf))
        assert rel_err(ctx.sources(w, mu), w @ xc) <= TOL


@pytest.mark.parametrize("n", [8, 64, 128])
def test_resident_centring_is_exact(pa, rng, n):
    """The first pass with a mean μ centres the resident X in place (DeviceCtx::resident_mu):
    its statistics are bit-identical to a pass over data centred on the host (the same IEEE
    subtraction), rowsum() still returns the caller's sums, and download() restores X."""
    x = laplace_mix(rng, n, 4099)
    mu = x.mean(axis=1)
    w = rng.normal(size=(n, n)) / np.sqrt(n)
    d = pa.DensityType.tanh()
    ctx = ctx_with(pa, x)
    sums = ctx.rowsum()
    got = ctx.eval(w, mu, d, False, need_y2=True)
    ref_ctx = ctx_with(pa, x - mu[:, None])
    want = ref_ctx.eval(w, None, d, False, need_y2=True)
    for k in want:
        assert np.array_equal(got[k], want[k]), k
    assert np.array_equal(ctx.rowsum(), sums)
    again = ctx.eval(w, mu, d, False, need_y2=True)  # same μ: no second shift
    for k in want:
        assert np.array_equal(again[k], want[k]), k
    assert rel_err(ctx.download(), x) <= 1e-15


def test_moments4(pa, rng):
    n = 6
    x = laplace_mix(rng, n, 3000)
    ctx = ctx_with(pa, x)
    w = rng.normal(size=(n, n))
    y = w @ x
    pairs = [(i, j) for i in range(n) for j in range(i, n)]
    z = np.stack([y[i] * y[j] for i, j in pairs])
    assert rel_err(ctx.moments4(w), z @ z.T) <= TOL


def test_generate_matches_reference_generator(pa, dg):
    ctx = pa.DeviceContext(0)
    a = ctx.generate(8, 10000, 42)
    x = ctx.download()
    xr, s, ar = dg.generate_data(8, 10000, 42)
    assert np.array_equal(a, ar)  # mixing matrix: bit-exact (benchmarks.rs:26-32)
    assert rel_err(x, xr) <= TOL  # X = A·S: GEMM summation order only


def _fit_both(pa, po, x, **kw):
    n = x.shape[0]
    cfg = pa.PicardConfig(w_init=np.eye(n), **kw)
    r = pa.Picard.fit_with_config(x, cfg)
    ro = po.fit_with_config(x, po.PicardConfig(w_init=np.eye(n), **kw))
    return r, ro


@pytest.mark.parametrize("ortho,extended", [(True, True), (True, False), (False, True), (False, False)])
def test_fit_c1_vs_oracle(pa, po, c1_data, ortho, extended):
    x, s, a = c1_data
    r, ro = _fit_both(pa, po, x, ortho=ortho, extended=extended)
    assert r.converged and ro.converged
    assert r.gradient_norm < 1e-7
    assert abs(r.n_iterations - ro.n_iterations) <= 2
    am, amo = pa.utils.amari_distance(r.full_unmixing(), a), po.amari_distance(ro.full_unmixing(), a)
    assert abs(am - amo) <= 1e-6
    assert np.max(np.abs(r.unmixing - ro.unmixing)) <= 1e-6
    assert np.max(np.abs(r.whitening - ro.whitening)) <= 1e-8 * np.max(np.abs(ro.whitening))
    assert np.max(np.abs(r.sources - ro.sources)) <= 1e-5
    if extended:
        assert np.array_equal(r.signs, ro.signs)


@pytest.mark.parametrize("kw", [dict(density=("exp", 1.0)), dict(density=("cube", 1.0), ortho=True, extended=True),
                                dict(n_components=5), dict(whiten=False), dict(centering=False),
                                dict(fastica_it=10), dict(jade_it=3), dict(m=3, ls_tries=4)])
def test_fit_variants_vs_oracle(pa, po, c1_data, kw):
    x, s, a = c1_data
    kw = dict(kw)
    pk, ok = dict(kw), dict(kw)
    if "density" in kw:
        k, al = kw["density"]
        pk["density"] = getattr(pa.DensityType, k)(al) if k != "cube" else pa.DensityType.cube()
        ok["density"] = po.Density(k, al)
    nc = kw.get("n_components", 8)
    r = pa.Picard.fit_with_config(x, pa.PicardConfig(w_init=np.eye(nc), max_iter=200, **pk))
    ro = po.fit_with_config(x, po.PicardConfig(w_init=np.eye(nc), max_iter=200, **ok))
    assert r.converged == ro.converged
    assert abs(r.n_iterations - ro.n_iterations) <= max(2, ro.n_iterations // 10)
    fw, fwo = r.full_unmixing(), ro.full_unmixing()
    if nc == 8:
        assert abs(pa.utils.amari_distance(fw, a) - po.amari_distance(fwo, a)) <= 1e-6
    assert np.max(np.abs(fw - fwo)) <= 1e-5 * np.max(np.abs(fwo))


@pytest.mark.parametrize("jade_it", [1, 3])
def test_jade_device_sweeps_match_host(pa, c1_data, monkeypatch, capfd, jade_it):
    """The Jacobi sweeps as one cooperative device launch (the default,
    DeviceCtx::jade_sweeps) against the host sweeps (PICARD_HOST_JADE=1) on the same
    cumulant matrices: the angles differ only by summation order, so after a few sweeps
    they agree to ~1e-12. PICARD_TRACE names the sweeps that actually ran."""
    x, s, a = c1_data
    cfg = dict(jade_it=jade_it, max_iter=1, w_init=np.eye(8))
    monkeypatch.setenv("PICARD_TRACE", "1")
    monkeypatch.setenv("PICARD_HOST_JADE", "1")
    host = pa.Picard.fit_with_config(x, pa.PicardConfig(**cfg)).full_unmixing()
    assert "host sweeps" in capfd.readouterr().err
    monkeypatch.delenv("PICARD_HOST_JADE")
    dev = pa.Picard.fit_with_config(x, pa.PicardConfig(**cfg)).full_unmixing()
    assert "device sweeps" in capfd.readouterr().err
    assert np.max(np.abs(dev - host)) <= 1e-9 * np.max(np.abs(host))


def test_jade_long_run_properties(pa, c1_data):
    """jade.rs:22-72 as written never reaches its 1e-6 angle tolerance on this data:
    every sweep rotates by ~0.75 rad and a 1e-15 relative perturbation of the input
    changes the 20-sweep output by O(1) (chaotic). Only the
    reference's own property is checkable: the warm start is orthogonal
    (jade.rs:245-255) and Picard then converges."""
    x, s, a = c1_data
    r = pa.Picard.fit_with_config(x, pa.PicardConfig(jade_it=20, random_state=1))
    assert r.converged
    w = r.unmixing
    assert np.max(np.abs(w @ w.T - np.eye(8))) < 1e-6


def test_c4_shape_nonortho_vs_oracle(pa, po, dg):
    """BASELINE config 4's shape (N = 256, non-ortho, m = 7) at a T the oracle runs in
    seconds: the tiled MFMA path end to end, first iterations against the oracle."""
    x, s, a = dg.generate_data(256, 20000, 42)
    kw = dict(ortho=False, extended=False, m=7, max_iter=6)
    ctx = pa.DeviceContext(0)
    ctx.load(x)
    sv = pa.Solver(ctx, pa.PicardConfig(w_init=np.eye(256), **kw))
    losses = []
    done = False
    while not done:
        done = sv.step()
        losses.append(sv.last()[0])
    r = sv.finish()
    ro = po.fit_with_config(x, po.PicardConfig(w_init=np.eye(256), **kw))
    assert r.n_iterations == ro.n_iterations == 6
    assert np.allclose(losses, ro.info.trace_loss, rtol=1e-10, atol=0)
    assert np.max(np.abs(r.unmixing - ro.unmixing)) <= 1e-8


def test_transform_and_mixing(pa, po, c1_data):
    x, s, a = c1_data
    r, ro = _fit_both(pa, po, x)
    y = pa.Picard.transform(x, r)
    assert rel_err(y, po.transform(x, ro)) <= 1e-6
    assert rel_err(y, r.sources) <= 1e-10
    assert rel_err(r.mixing(), ro.mixing()) <= 1e-6


def test_errors(pa):
    with pytest.raises(pa.InvalidDimensions, match="Input matrix cannot be empty"):
        pa.Picard.fit(np.zeros((0, 10)))
    with pytest.raises(pa.InvalidConfig, match="max_iter"):
        pa.Picard.fit_with_config(np.ones((2, 10)), pa.PicardConfig(max_iter=0))
    x = np.random.default_rng(0).laplace(size=(3, 100))
    with pytest.raises(pa.InvalidDimensions, match=r"w_init shape \[2, 2\] doesn't match expected \(3, 3\)"):
        pa.Picard.fit_with_config(x, pa.PicardConfig(w_init=np.eye(2)))
    with pytest.raises(pa.SingularMatrix):
        pa.Picard.fit(np.ones((3, 100)))  # rank-1 after centering → whiten min-sv check


def test_reference_solver_tests(pa, rng):
    """solver.rs:288-398 restated (shapes / bounds; the reference pins no values)."""
    def gen(n, t, seed):
        r = np.random.default_rng(seed)
        s = np.sign(r.uniform(-1, 1, size=(n, t))) * -np.log(r.uniform(size=(n, t)))
        a = r.normal(size=(n, n))
        return a @ s
    x = gen(3, 1000, 42)
    res = pa.Picard.fit(x)
    assert res.sources.shape == (3, 1000) and res.unmixing.shape == (3, 3)
    res = pa.Picard.fit_with_config(x, pa.PicardConfig.builder().max_iter(100).random_state(42).build())
    assert res.n_iterations <= 100
    res = pa.Picard.fit_with_config(x, pa.PicardConfig.builder().jade_it(50).random_state(42).build())
    assert res.sources.shape[0] == 3 and (res.converged or res.n_iterations > 0)
    x4 = gen(4, 2000, 123)
    rj = pa.Picard.fit_with_config(x4, pa.PicardConfig.builder().jade_it(30).random_state(42).build())
    assert rj.converged or rj.gradient_norm < 1.0
    x5 = gen(5, 1000, 42)
    rn = pa.Picard.fit_with_config(x5, pa.PicardConfig.builder().n_components(3).random_state(42).build())
    assert rn.sources.shape[0] == 3 and rn.unmixing.shape[0] == 3
    rt = pa.Picard.fit_with_config(x, pa.PicardConfig.builder().random_state(42).build())
    assert pa.Picard.transform(x, rt).shape == rt.sources.shape
    rw = pa.Picard.fit_with_config(x, pa.PicardConfig.builder().whiten(False).random_state(42).build())
    assert rw.whitening is None


def test_large_t_shard_additivity(pa, rng):
    """Size-independent property at C2 scale (64 × 1e6): stats are sums over t,
    so the two halves' stats add up to the whole (checksum of checksums)."""
    n, t = 64, 1_000_000
    ctx = pa.DeviceContext(0)
    a = ctx.generate(n, t, 7)
    x = ctx.download()
    w = np.linalg.qr(rng.normal(size=(n, n)))[0]
    mu = ctx.rowsum() / t
    full = ctx.eval(w, mu, pa.DensityType.tanh(), False)
    half = t // 2
    parts = []
    for lo, hi in [(0, half), (half, t)]:
        c = pa.DeviceContext(0)
        c.load(np.ascontiguousarray(x[:, lo:hi]))
        parts.append(c.eval(w, mu, pa.DensityType.tanh(), False))
    for k in full:
        assert rel_err(parts[0][k] + parts[1][k], full[k]) <= 1e-11, k
    # ortho Picard gradient at the true unmixing is small; at a random W it is not
    assert np.isfinite(full["G"]).all() and np.isfinite(full["ll"]).all()


@pytest.mark.parametrize("n,t", [(64, 100_000), (128, 100_000)])
def test_fit_c2_c3_shapes_vs_oracle(pa, po, dg, n, t):
    """BASELINE configs 2 and 3 (Picard-O extended tanh at N = 64 / 128) at a T the
    oracle fits in seconds: the register-resident fused / loss-only / split schedule
    end to end against core::run. Both converge; Amari distance within 1e-6
    (north_star); unmixing within 1e-6 relative; signs identical."""
    x, s, a = dg.generate_data(n, t, 42)
    r, ro = _fit_both(pa, po, x, max_iter=200)
    assert r.converged and ro.converged
    assert r.gradient_norm < 1e-7
    am, amo = pa.utils.amari_distance(r.full_unmixing(), a), po.amari_distance(ro.full_unmixing(), a)
    assert abs(am - amo) <= 1e-6
    assert np.max(np.abs(r.full_unmixing() - ro.full_unmixing())) <= 1e-6 * np.max(np.abs(ro.full_unmixing()))
    assert np.array_equal(r.signs, ro.signs)
