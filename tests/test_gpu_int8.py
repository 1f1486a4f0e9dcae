"""GPU parity of the int8-slice Y stage (ozaki.inc) against the CPU oracle.

The loss-only line-search pass and the fused pass at 64 < nc ≤ 128, n_features ≤ 128
(NB = 8: k_eval_loss_oz, k_eval_fused_ws) and at 32 < nc ≤ 64, n_features ≤ 64 (NB = 4:
k_eval_loss_oz<…, 4>, k_eval_fused<4, …, OZ>), no H, form Y = W·(X − μ)
from exact int8 digits (7 radix-256 digits per value of X and of W, exact int32 diagonal sums, fp64
combine). Tolerances: the statistics against the fp64 oracle at the file-wide 1e-12
relative bound of test_gpu_parity.py; against the context's own fp64 Y stage
(pc_ctx_set_y_stage F64) at 1e-13 relative (both are fp64-accurate, the difference is
rounding). Every test asserts that the int8 kernel actually ran (pc_ctx_int8_passes).
"""
import numpy as np
import pytest

from conftest import density_of, rel_err

pytestmark = pytest.mark.gpu

TOL = 1e-12
TOL_MODES = 1e-13
DENSITIES = [("tanh", 1.0), ("tanh", 0.7), ("exp", 1.0), ("exp", 0.1), ("cube", 1.0)]


@pytest.fixture(scope="module")
def rng():
    return np.random.default_rng(4321)


def laplace_mix(rng, nf, t):
    s = rng.laplace(size=(nf, t))
    a = rng.uniform(-0.5, 0.5, size=(nf, nf)) + np.eye(nf)
    return a @ s + rng.normal(size=(nf, 1))


def dens_of(pa, dens):
    return pa.DensityType(["tanh", "exp", "cube"].index(dens[0]), dens[1])


def loss_only(ctx, w, mu, d, need_y2=True):
    lo, kept, done = ctx.eval_split(w, mu, d, False, need_y2=need_y2)
    return lo, kept, done


@pytest.mark.parametrize("n", [40, 64, 65, 100, 128])
@pytest.mark.parametrize("dens", DENSITIES)
def test_int8_loss_vs_oracle(pa, po, rng, n, dens):
    t = 5003  # ragged: the last 16-sample block is partly padding
    x = laplace_mix(rng, n, t)
    ctx = pa.DeviceContext(0)
    ctx.load(x)
    w = rng.normal(size=(n, n)) / np.sqrt(n)
    mu = x.mean(axis=1)
    d = dens_of(pa, dens)
    before = ctx.int8_passes
    lo, _, _ = loss_only(ctx, w, mu, d)
    assert ctx.int8_passes >= before + 1
    want = po.pass_stats(w, mu, x, density_of(po, d), False)
    for k in ("ll", "y2"):
        assert rel_err(lo[k], want[k]) <= TOL, (k, rel_err(lo[k], want[k]))


@pytest.mark.parametrize("nc,nf", [(128, 128), (80, 128), (72, 100), (65, 65), (64, 64), (40, 64), (48, 60)])
def test_int8_vs_f64_stage(pa, rng, nc, nf):
    """Same context, same W: the int8 stage against the fp64 MFMA stage."""
    x = laplace_mix(rng, nf, 20011)
    ctx = pa.DeviceContext(0)
    ctx.load(x)
    w = rng.normal(size=(nc, nf)) / np.sqrt(nf)
    mu = x.mean(axis=1)
    d = pa.DensityType.tanh()
    a, _, _ = loss_only(ctx, w, mu, d)
    n8 = ctx.int8_passes
    ctx.set_y_stage("f64")
    b, _, _ = loss_only(ctx, w, mu, d)
    assert ctx.int8_passes == n8 and n8 >= 1
    for k in ("ll", "y2"):
        assert rel_err(a[k], b[k]) <= TOL_MODES, (k, rel_err(a[k], b[k]))


@pytest.mark.parametrize("g_stage", ["f64", "auto"])
def test_int8_kept_y_completion_vs_oracle(pa, po, rng, g_stage):
    """The loss-only pass keeps its (int8-stage) Y in HBM and the completion forms G,
    Σψ′ from it: G = ψ(Y)·Yᵀ checks Y itself element-wise against the oracle. (With G on int8
    digits — g_stage "auto" — the completion recomputes the fused pass instead, so the accepted
    try's G has the fused pass's bits; the same check then covers that path.)"""
    n, t = 128, 8191
    x = laplace_mix(rng, n, t)
    ctx = pa.DeviceContext(0)
    ctx.set_g_stage(g_stage)
    ctx.load(x)
    w = rng.normal(size=(n, n)) / np.sqrt(n)
    mu = x.mean(axis=1)
    d = pa.DensityType.tanh()
    lo, kept, done = loss_only(ctx, w, mu, d)
    assert ctx.int8_passes >= 1
    want = po.pass_stats(w, mu, x, density_of(po, d), False)
    for k in ("G", "dpsi", "ll"):
        assert rel_err(done[k], want[k]) <= TOL, (k, kept, rel_err(done[k], want[k]))


def test_int8_wide_dynamic_range(pa, po, rng):
    """Per-sample exponents: samples spanning 2^±40, exact-zero samples (a zero
    column gives zero slices and y = 0, like the padding) and one huge outlier."""
    n, t = 128, 4000
    x = laplace_mix(rng, n, t)
    x *= np.exp2(rng.integers(-40, 40, size=t))[None, :]
    x[:, 17] = 0.0
    x[:, 1000:1016] = 0.0
    x[5, 2000] = 1e12
    ctx = pa.DeviceContext(0)
    ctx.load(x)
    w = rng.normal(size=(n, n)) / np.sqrt(n)
    w[3] *= 1e-30  # a row far below the others: its own exponent
    w[7] = 0.0
    d = pa.DensityType.cube()  # no saturation: every sample's y enters Σy⁴, Σy²
    lo, _, _ = loss_only(ctx, w, None, d)
    assert ctx.int8_passes >= 1
    want = po.pass_stats(w, None, x, density_of(po, d), False)
    for k in ("ll", "y2"):
        # per row: rows differ by many orders of magnitude
        for i in range(n):
            if want[k][i] != 0:
                assert abs(lo[k][i] - want[k][i]) <= TOL * abs(want[k][i]), (k, i)
            else:
                assert lo[k][i] == 0, (k, i)


def test_int8_reslices_after_mean_change(pa, po, rng):
    """The slice image follows the resident X: a pass with another μ (X un-shifted and
    re-centred in place) and a pass with μ = None both match the oracle."""
    n, t = 100, 6000
    x = laplace_mix(rng, n, t)
    ctx = pa.DeviceContext(0)
    ctx.load(x)
    w = rng.normal(size=(n, n)) / np.sqrt(n)
    d = pa.DensityType.tanh()
    for mu in (x.mean(axis=1), np.zeros(n) + 0.25, None, x.mean(axis=1)):
        lo, _, _ = loss_only(ctx, w, mu, d)
        want = po.pass_stats(w, mu, x, density_of(po, d), False)
        assert rel_err(lo["ll"], want["ll"]) <= TOL
    assert ctx.int8_passes >= 4


def test_int8_fit_matches_f64_fit(pa, rng):
    """A Picard-O fit at N = 96 (loss-only tries on the int8 stage) converges like the
    oracle-checked fp64 path: same iteration count ±2, unmixing within 1e-6."""
    x = laplace_mix(rng, 96, 20000)
    cfg = dict(max_iter=200, random_state=5)
    res = {}
    for mode in ("auto", "f64"):
        ctx = pa.DeviceContext(0)
        ctx.load(x)
        ctx.set_y_stage(mode)
        sv = pa.Solver(ctx, pa.PicardConfig(**cfg))
        while not sv.step():
            pass
        res[mode] = (sv.finish(), ctx.int8_passes)
        sv.close()
    (r, n8), (r64, n64) = res["auto"], res["f64"]
    assert n8 >= 1 and n64 == 0
    assert r.converged and r64.converged
    assert abs(r.n_iterations - r64.n_iterations) <= 2
    assert np.max(np.abs(r.unmixing - r64.unmixing)) <= 1e-6


@pytest.mark.parametrize("n", [40, 64, 100, 128])
@pytest.mark.parametrize("dens", [("tanh", 1.0), ("exp", 0.5), ("cube", 1.0)])
@pytest.mark.parametrize("need_y2", [False, True])
def test_int8_split_eval_bit_identical(pa, rng, n, dens, need_y2):
    """Loss-only try + completion == one fused pass, bit for bit, on the int8 stage
    (both kernels run oz_ystage + oz_combine and the same row-term order)."""
    x = laplace_mix(rng, n, 4099)
    ctx = pa.DeviceContext(0)
    ctx.load(x)
    w = rng.normal(size=(n, n)) / np.sqrt(n)
    mu = x.mean(axis=1)
    d = dens_of(pa, dens)
    full = ctx.eval(w, mu, d, False, need_y2=need_y2)
    assert ctx.int8_passes == 1
    lo, kept, done = ctx.eval_split(w, mu, d, False, need_y2=need_y2)
    assert ctx.int8_passes >= 2
    assert np.array_equal(lo["ll"], full["ll"]) and np.array_equal(lo["y2"], full["y2"])
    for k in full:
        assert np.array_equal(done[k], full[k]), k


@pytest.mark.parametrize("n", [40, 64, 65, 100, 128])
@pytest.mark.parametrize("dens", DENSITIES)
def test_int8_fused_vs_oracle_and_f64(pa, po, rng, n, dens):
    """The fused pass on the int8 stage (G, Σψ′, Σℓ, Σy²) against the oracle (1e-12) and
    against the fp64 Y stage of the same context (1e-13). G on fp64 MFMA here, so the check
    isolates the Y stage (G on int8 digits: test_gpu_g8.py)."""
    x = laplace_mix(rng, n, 5003)
    ctx = pa.DeviceContext(0)
    ctx.set_g_stage("f64")
    ctx.load(x)
    w = rng.normal(size=(n, n)) / np.sqrt(n)
    mu = x.mean(axis=1)
    d = dens_of(pa, dens)
    got = ctx.eval(w, mu, d, False)
    assert ctx.int8_passes == 1
    want = po.pass_stats(w, mu, x, density_of(po, d), False)
    for k in want:
        assert rel_err(got[k], want[k]) <= TOL, (k, rel_err(got[k], want[k]))
    ctx.set_y_stage("f64")
    ref = ctx.eval(w, mu, d, False)
    assert ctx.int8_passes == 1
    for k in want:
        assert rel_err(got[k], ref[k]) <= TOL_MODES, (k, rel_err(got[k], ref[k]))


def test_int8_gram_stays_fp64(pa, rng):
    """The whitening Gram (LINEAR pass) never takes the int8 stage."""
    x = laplace_mix(rng, 100, 3000)
    ctx = pa.DeviceContext(0)
    ctx.load(x)
    g = ctx.gram(x.mean(axis=1))
    assert ctx.int8_passes == 0
    xc = x - x.mean(axis=1, keepdims=True)
    assert rel_err(g, xc @ xc.T) <= TOL


@pytest.mark.parametrize("n", [40, 64, 72, 128])
@pytest.mark.parametrize("dens", [("tanh", 1.0), ("tanh", 0.5), ("exp", 1.0), ("exp", 0.3)])
@pytest.mark.parametrize("dmax", ["2", "3"])
def test_screen_bound_holds(pa, rng, n, dens, dmax, monkeypatch):
    """The line-search screen's bound covers the exact pass: |Σℓ_exact − Σℓ_screen| ≤ bound
    for every row, over W of very different scales, from the first level D ≤ 2 (the default:
    tanh's fp32 screen; exp runs D ≤ 3) and from D ≤ 3; and at D ≤ 3 it is tight enough to
    decide (tanh: bound ≤ 2e-4 of Σ|ℓ| with its fp32 log-likelihood; the D ≤ 2 bound's size is
    checked on the bench mixture, tests/test_gpu_screen_stat.py — the loud sample here inflates
    its Σ_t 4^e_t)."""
    monkeypatch.setenv("PICARD_SCREEN_DMAX", dmax)
    x = laplace_mix(rng, n, 20011)
    x[:, 5] *= 1e3  # one loud sample: its exponent dominates its own column only
    ctx = pa.DeviceContext(0)
    ctx.load(x)
    mu = x.mean(axis=1)
    d = dens_of(pa, dens)
    xc = x - mu[:, None]
    k = np.linalg.cholesky(np.linalg.inv(xc @ xc.T / x.shape[1])).T
    for scale in (1e-3, 0.3, 1.0, 7.0):
        w = scale * (np.linalg.qr(rng.normal(size=(n, n)))[0] @ k)
        ll_s, bnd = ctx.eval_loss_screen(w, mu, d)
        lo, _, _ = ctx.eval_split(w, mu, d, False, need_y2=False)
        err = np.abs(lo["ll"] - ll_s)
        assert np.all(err <= bnd), (scale, np.max(err / bnd))
        assert np.all(bnd >= 0)
        if dens[0] == "tanh" and dmax == "3":  # (the loud sample keeps the worst-case tail here)
            assert np.max(bnd / np.abs(lo["ll"])) <= 2e-4, (scale, np.max(bnd / np.abs(lo["ll"])))
    _, ns = ctx.screen_stats()
    assert ns == 4


def test_screen_unavailable_shapes(pa, rng):
    x = laplace_mix(rng, 40, 3000)
    ctx = pa.DeviceContext(0)
    ctx.load(x)
    with pytest.raises(pa.ComputationError):  # nc ≤ 32: no int8 stage
        ctx.eval_loss_screen(np.eye(40)[:20], x.mean(axis=1), pa.DensityType.tanh())
    x = laplace_mix(rng, 80, 3000)
    ctx = pa.DeviceContext(0)
    ctx.load(x)
    with pytest.raises(pa.ComputationError):  # 32 < nc ≤ 64 needs nf ≤ 64
        ctx.eval_loss_screen(np.eye(80)[:50], x.mean(axis=1), pa.DensityType.tanh())
    x = laplace_mix(rng, 100, 3000)
    ctx = pa.DeviceContext(0)
    ctx.load(x)
    with pytest.raises(pa.ComputationError):  # cube: ℓ not Lipschitz
        ctx.eval_loss_screen(np.eye(100), x.mean(axis=1), pa.DensityType.cube())
    ctx.set_y_stage("int8-exact")
    with pytest.raises(pa.ComputationError):
        ctx.eval_loss_screen(np.eye(100), x.mean(axis=1), pa.DensityType.tanh())


@pytest.mark.parametrize("n,seed,model", [(128, 42, True), (96, 7, False), (64, 42, True), (48, 3, True)])
def test_screened_fit_bit_identical(pa, n, seed, model, capfd, monkeypatch):
    """A Picard-O fit with the line-search screen (default) and without it (int8-exact):
    identical iterations and bit-identical unmixing — the screen rejects only tries the
    exact pass would reject. The bench mixture (benches/benchmarks.rs) has line searches
    that fail all 10 tries, so the screen does reject some (counted in the trace). `model`:
    the fit also runs later tries as full passes by the quadratic-model policy ("[picard-model]",
    Solver::line_search), whose schedule must not change a bit either."""
    monkeypatch.setenv("PICARD_TRACE", "1")
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
    err = capfd.readouterr().err
    (r, ns), (r0, ns0) = res["auto"], res["int8-exact"]
    assert ns > 0 and ns0 == 0
    assert r.n_iterations == r0.n_iterations and r.converged == r0.converged
    assert np.array_equal(r.unmixing, r0.unmixing)
    rejected = [int(line.split("rejected ")[1].split()[0]) for line in err.splitlines() if "rejected " in line]
    assert rejected and max(rejected) > 0
    assert "[picard-model]" in err or not model


@pytest.mark.parametrize("t", [16 * 512 * 7 + 5, 1_000_003])
def test_int8_fused_many_blocks_per_workgroup(pa, po, rng, t):
    """Many 16-sample blocks per workgroup (the fused pass's pipeline runs its steady
    state: X staged two blocks ahead into a rotating third buffer): bit-identical to the
    loss-only pass, and the fp64 stage within 1e-13 (G on fp64 MFMA: the Y stage alone)."""
    n = 128
    x = laplace_mix(rng, n, t)
    ctx = pa.DeviceContext(0)
    ctx.set_g_stage("f64")
    ctx.load(x)
    w = rng.normal(size=(n, n)) / np.sqrt(n)
    mu = x.mean(axis=1)
    d = pa.DensityType.tanh()
    full = ctx.eval(w, mu, d, False)
    lo, _, done = ctx.eval_split(w, mu, d, False)
    assert np.array_equal(lo["ll"], full["ll"])
    for k in full:
        assert np.array_equal(done[k], full[k]), k
    ctx.set_y_stage("f64")
    ref = ctx.eval(w, mu, d, False)
    for k in full:
        assert rel_err(full[k], ref[k]) <= TOL_MODES, (k, rel_err(full[k], ref[k]))


def test_int8_non_finite_propagates(pa, rng):
    """A NaN in X or in W reaches the statistics as NaN on the int8 stage, as on the fp64
    stage (the digit image carries it in the sample / row scale)."""
    n = 100
    x = laplace_mix(rng, n, 3000)
    w = rng.normal(size=(n, n)) / np.sqrt(n)
    d = pa.DensityType.tanh()
    for mode in ("auto", "f64"):
        xb = x.copy()
        xb[3, 100] = np.nan
        ctx = pa.DeviceContext(0)
        ctx.load(xb)
        ctx.set_y_stage(mode)
        st = ctx.eval(w, None, d, False)
        assert np.isnan(st["ll"]).all() and np.isnan(st["G"]).any(), mode
        ctx = pa.DeviceContext(0)
        ctx.load(x)
        ctx.set_y_stage(mode)
        wb = w.copy()
        wb[5, 7] = np.inf
        st = ctx.eval(wb, None, d, False)
        assert np.isnan(st["ll"][5]) and np.isfinite(st["ll"][6]), mode


@pytest.mark.parametrize("nc,nf,t", [(128, 128, 5003), (100, 128, 20011), (72, 100, 1100003)])
def test_int8_sources(pa, rng, nc, nf, t):
    """Sources / transform (solver.rs:182,199-214) on the int8 stage (k_ystore_oz) once the
    context holds the digit image: against numpy's fp64 W·(X − μ) at 1e-12, against the
    fp64 MFMA store (k_ystore) at 1e-13; host copy and HBM copy bit-identical, padding zero.
    t = 1100003 crosses the 2^20-sample chunks of the host-copy path (b_first > 0)."""
    import ctypes
    x = laplace_mix(rng, nf, t)
    ctx = pa.DeviceContext(0)
    ctx.load(x)
    w = rng.normal(size=(nc, nf)) / np.sqrt(nf)
    mu = x.mean(axis=1)
    ctx.sources(w, mu)  # no digit image yet: the fp64 store, and no image is built for it
    assert ctx.int8_passes == 0
    loss_only(ctx, w, mu, pa.DensityType.tanh())  # builds the image
    n8 = ctx.int8_passes
    got = ctx.sources(w, mu)
    assert ctx.int8_passes == n8 + (t + (1 << 20) - 1) // (1 << 20)
    want = w @ (x - mu[:, None])
    assert rel_err(got, want) <= TOL, rel_err(got, want)
    ptr, ld, ms = ctx.sources_device(w, mu)
    assert ctx.int8_passes == n8 + (t + (1 << 20) - 1) // (1 << 20) + 1
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    dev = np.empty((nc, ld))
    assert hip.hipMemcpy(dev.ctypes.data, ptr, dev.nbytes, 2) == 0  # hipMemcpyDeviceToHost
    assert np.array_equal(dev[:, :t], got)
    assert not dev[:, t:].any()
    ctx.set_y_stage("f64")
    f64 = ctx.sources(w, mu)
    assert rel_err(got, f64) <= TOL_MODES, rel_err(got, f64)
    # per sample: each column against its own fp64 value (the stage's error follows the
    # sample's scale 2^e_t, not the whole matrix's)
    col = np.abs(got - f64).max(axis=0) / np.maximum(np.abs(f64).max(axis=0), 1e-300)
    assert col.max() <= 1e-13, col.max()


@pytest.mark.parametrize("n,t", [(40, 5003), (64, 100_003), (33, 777)])
@pytest.mark.parametrize("stage", ["auto", "f64"])
@pytest.mark.parametrize("dens", [("tanh", 1.0), ("exp", 0.5), ("cube", 1.0)])
def test_ws4_bit_identical_to_8wave(pa, rng, n, t, stage, dens, monkeypatch):
    """The warp-specialised NB = 4 fused pass (k_eval_fused_ws4) against the 8-wave
    k_eval_fused<4> (PICARD_NO_WS4=1), on either Y stage: every statistic bit for bit
    (same partition, G-tile map and k order, lane map, row-term order)."""
    x = laplace_mix(rng, n, t)
    w = rng.normal(size=(n, n)) / np.sqrt(n)
    mu = x.mean(axis=1)
    d = dens_of(pa, dens)
    out = []
    for no_ws4 in (False, True):
        if no_ws4:
            monkeypatch.setenv("PICARD_NO_WS4", "1")
        ctx = pa.DeviceContext(0)
        ctx.load(x)
        ctx.set_y_stage(stage)
        out.append((ctx.eval(w, mu, d, False), ctx.int8_passes, ctx.gram(mu)))
        ctx.close()
    (a, na, ga), (b, nb_, gb) = out
    assert na == nb_ and (na == 1) == (stage == "auto" and n > 32)
    for k in a:
        assert np.array_equal(a[k], b[k]), k
    assert np.array_equal(ga, gb)  # the whitening Gram takes the same kernels (fp64)


@pytest.mark.parametrize("nc,nf,h", [(256, 256, True), (256, 256, False), (200, 256, True), (150, 180, True),
                                     (100, 128, True), (40, 40, True)])
@pytest.mark.parametrize("dens", [("tanh", 1.0), ("exp", 0.5), ("cube", 1.0)])
def test_tiled_int8_vs_oracle_and_f64(pa, po, rng, nc, nf, h, dens):
    """The tiled two-phase pass (nc > 128, or H at nc > 64 — BASELINE C4's path) with phase 1
    on the int8 digit stage (k_tiled_yw_oz, nf ≤ 256): every statistic against the oracle
    (1e-12) and the fp64 stage (1e-13); its loss-only form (phase 1 alone) gives the full
    pass's Σℓ and Σy² bit for bit."""
    x = laplace_mix(rng, nf, 9001)
    ctx = pa.DeviceContext(0)
    ctx.load(x)
    w = rng.normal(size=(nc, nf)) / np.sqrt(nf)
    mu = x.mean(axis=1)
    d = dens_of(pa, dens)
    got = ctx.eval(w, mu, d, h)
    tiled = nc > 128 or (h and nc > 64)
    assert (ctx.int8_passes >= 1) == tiled or not tiled
    want = po.pass_stats(w, mu, x, density_of(po, d), h)
    for k in want:
        assert rel_err(got[k], want[k]) <= TOL, (k, rel_err(got[k], want[k]))
    lo, _, done = ctx.eval_split(w, mu, d, h)
    assert np.array_equal(lo["ll"], got["ll"]) and np.array_equal(lo["y2"], got["y2"])
    for k in got:
        assert np.array_equal(done[k], got[k]), k
    ctx.set_y_stage("f64")
    n8 = ctx.int8_passes
    ref = ctx.eval(w, mu, d, h)
    assert ctx.int8_passes == n8
    for k in want:
        assert rel_err(got[k], ref[k]) <= TOL_MODES, (k, rel_err(got[k], ref[k]))


@pytest.mark.parametrize("nc,nf", [(256, 256), (180, 200), (100, 128), (40, 64)])
@pytest.mark.parametrize("dens", [("tanh", 1.0), ("exp", 0.5), ("cube", 1.0)])
def test_multi_try_int8_vs_oracle_and_f64(pa, po, rng, nc, nf, dens):
    """The non-orthogonal one-pass line search with Y and Z = D·W on the int8 digit stage
    (k_multi_loss2_oz): Σℓ, Σy² of every Y + α_j·Z against the oracle at W + α_j·Z (1e-12,
    the per-try rounding) and against the fp64-stage pass (1e-13)."""
    x = laplace_mix(rng, nf, 7001)
    ctx = pa.DeviceContext(0)
    ctx.load(x)
    w = rng.normal(size=(nc, nf)) / np.sqrt(nf)
    z = 0.3 * rng.normal(size=(nc, nf)) / np.sqrt(nf)
    mu = x.mean(axis=1)
    d = dens_of(pa, dens)
    al = np.array([0.5 ** j for j in range(9)])
    ll, y2 = ctx.eval_loss_multi(w, z, al, mu, d)
    assert ctx.int8_passes >= 1
    for j in (0, 4, 8):
        want = po.pass_stats(w + al[j] * z, mu, x, density_of(po, d), True)
        assert rel_err(ll[j], want["ll"]) <= TOL and rel_err(y2[j], want["y2"]) <= TOL, j
    ctx.set_y_stage("f64")
    n8 = ctx.int8_passes
    ll64, y264 = ctx.eval_loss_multi(w, z, al, mu, d)
    assert ctx.int8_passes == n8
    assert rel_err(ll, ll64) <= TOL_MODES and rel_err(y2, y264) <= TOL_MODES
