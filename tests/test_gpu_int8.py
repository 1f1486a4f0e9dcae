"""GPU parity of the int8-slice Y stage (ozaki.inc) against the CPU oracle.

The loss-only line-search pass and the fused pass at 64 < nc ≤ 128, n_features ≤ 128
(no H) form Y = W·(X − μ)
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


@pytest.mark.parametrize("n", [65, 100, 128])
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


@pytest.mark.parametrize("nc,nf", [(128, 128), (80, 128), (72, 100), (65, 65)])
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


def test_int8_kept_y_completion_vs_oracle(pa, po, rng):
    """The loss-only pass keeps its (int8-stage) Y in HBM and the completion forms G,
    Σψ′ from it: G = ψ(Y)·Yᵀ checks Y itself element-wise against the oracle."""
    n, t = 128, 8191
    x = laplace_mix(rng, n, t)
    ctx = pa.DeviceContext(0)
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


@pytest.mark.parametrize("n", [100, 128])
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


@pytest.mark.parametrize("n", [65, 100, 128])
@pytest.mark.parametrize("dens", DENSITIES)
def test_int8_fused_vs_oracle_and_f64(pa, po, rng, n, dens):
    """The fused pass on the int8 stage (G, Σψ′, Σℓ, Σy²) against the oracle (1e-12) and
    against the fp64 Y stage of the same context (1e-13)."""
    x = laplace_mix(rng, n, 5003)
    ctx = pa.DeviceContext(0)
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
