"""GPU parity for the shapes beyond the register-resident kernels, all on MFMA:

  * n_components > 256 and n_features > 256 (the reference runs any N,
    core.rs:162-401 on generic ndarray): the tiled pass with feature chunks of
    256 (partial Y carried through the y buffer) and any number of 128-row roles;
  * tanh / exp at α ≤ 0 (density.rs:33-103 does not restrict α): the libm forms
    of the tiled pass;
  * sources / transform at any shape (solver.rs:182,199-214) through k_ystore,
    to the host and kept in HBM (pc_ctx_sources_device).

Same bounds as test_gpu_parity.py: statistics within 1e-12 × max|oracle|,
split evaluation bit-identical to the full pass, sources within 1e-12.
"""
import ctypes

import numpy as np
import pytest

from conftest import density_of, rel_err

pytestmark = pytest.mark.gpu

TOL = 1e-12


@pytest.fixture(scope="module")
def rng():
    return np.random.default_rng(4321)


def laplace_mix(rng, nf, t):
    s = rng.laplace(size=(nf, t))
    a = rng.uniform(-0.5, 0.5, size=(nf, nf)) + np.eye(nf)
    return a @ s + rng.normal(size=(nf, 1))


def ctx_with(pa, x):
    ctx = pa.DeviceContext(0)
    ctx.load(x)
    return ctx


@pytest.mark.parametrize("nc,nf", [(300, 300), (100, 300), (257, 260), (520, 520), (40, 513)])
@pytest.mark.parametrize("dens", [("tanh", 1.0), ("exp", 0.5), ("cube", 1.0)])
@pytest.mark.parametrize("need_h", [False, True])
def test_eval_wide_vs_oracle(pa, po, rng, nc, nf, dens, need_h):
    t = 2003  # ragged
    x = laplace_mix(rng, nf, t)
    ctx = ctx_with(pa, x)
    w = rng.normal(size=(nc, nf)) / np.sqrt(nf)
    mu = x.mean(axis=1)
    d = pa.DensityType(["tanh", "exp", "cube"].index(dens[0]), dens[1])
    got = ctx.eval(w, mu, d, need_h, need_y2=True)
    want = po.pass_stats(w, mu, x, density_of(po, d), need_h)
    for k in want:
        assert rel_err(got[k], want[k]) <= TOL, (k, rel_err(got[k], want[k]))


@pytest.mark.parametrize("n", [8, 64, 128, 300])
@pytest.mark.parametrize("dens", [("tanh", -0.5), ("tanh", -2.0), ("exp", -0.05), ("exp", -0.5)])
@pytest.mark.parametrize("need_h", [False, True])
def test_eval_nonpositive_alpha_vs_oracle(pa, po, rng, n, dens, need_h):
    """α < 0: the reference's formulas hold for any α (no validation in config.rs);
    the fused table paths assume α > 0, so these run the tiled libm forms."""
    t = 1999
    x = laplace_mix(rng, n, t) * 0.5
    ctx = ctx_with(pa, x)
    w = rng.normal(size=(n, n)) / np.sqrt(n)
    mu = x.mean(axis=1)
    d = pa.DensityType(["tanh", "exp", "cube"].index(dens[0]), dens[1])
    got = ctx.eval(w, mu, d, need_h, need_y2=True)
    want = po.pass_stats(w, mu, x, density_of(po, d), need_h)
    for k in want:
        assert np.isfinite(want[k]).all()
        assert rel_err(got[k], want[k]) <= TOL, (k, rel_err(got[k], want[k]))


@pytest.mark.parametrize("nc,nf", [(300, 300), (60, 700)])
@pytest.mark.parametrize("need_h", [False, True])
def test_split_eval_wide_bit_identical(pa, rng, nc, nf, need_h):
    """Loss-only try (tiled mode 1, feature chunks) + completion == the full pass, bit for bit."""
    x = laplace_mix(rng, nf, 2051)
    ctx = ctx_with(pa, x)
    w = rng.normal(size=(nc, nf)) / np.sqrt(nf)
    mu = x.mean(axis=1)
    d = pa.DensityType.tanh()
    full = ctx.eval(w, mu, d, need_h, need_y2=True)
    loss_only, kept, done = ctx.eval_split(w, mu, d, need_h, need_y2=True)
    assert np.array_equal(loss_only["ll"], full["ll"]) and np.array_equal(loss_only["y2"], full["y2"])
    for k in full:
        assert np.array_equal(done[k], full[k]), k


@pytest.mark.parametrize("nc,nf", [(5, 12), (128, 128), (300, 300), (70, 600)])
def test_sources_any_shape(pa, rng, nc, nf):
    x = laplace_mix(rng, nf, 4099)
    ctx = ctx_with(pa, x)
    mu = x.mean(axis=1)
    w = rng.normal(size=(nc, nf)) / np.sqrt(nf)
    want = w @ (x - mu[:, None])
    got = ctx.sources(w, mu)
    assert rel_err(got, want) <= TOL
    # kept in HBM: same bits as the host copy, zero padding past n_local
    ptr, ld, ms = ctx.sources_device(w, mu)
    assert ld >= x.shape[1] and ms > 0.0
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    dev = np.empty((nc, ld))
    assert hip.hipMemcpy(dev.ctypes.data, ptr, dev.nbytes, 2) == 0  # hipMemcpyDeviceToHost
    assert np.array_equal(dev[:, :x.shape[1]], got)
    assert not dev[:, x.shape[1]:].any()


def test_transform_wide(pa, po, rng):
    """Picard.transform (solver.rs:199-214) at N = 300 against the oracle's."""
    x = laplace_mix(rng, 300, 3000)
    r = pa.Picard.fit_with_config(x, pa.PicardConfig(w_init=np.eye(300), max_iter=2))
    y = pa.Picard.transform(x, r)
    want = r.full_unmixing() @ (x - r.mean[:, None])
    assert rel_err(y, want) <= 1e-11
    assert rel_err(y, r.sources) <= 1e-11


@pytest.mark.parametrize("ortho", [True, False])
def test_wide_fit_first_iterations_vs_oracle(pa, po, dg, ortho):
    """N = 300 > 256 end to end (tiled pass with a second 128-row role and
    feature chunks; non-ortho: per-try loss passes since the multi-try pass
    covers nc ≤ 256): the first iterations against core::run."""
    x, s, a = dg.generate_data(300, 6000, 42)
    kw = dict(ortho=ortho, extended=not ortho, max_iter=4)
    r = pa.Picard.fit_with_config(x, pa.PicardConfig(w_init=np.eye(300), **kw))
    ro = po.fit_with_config(x, po.PicardConfig(w_init=np.eye(300), **kw))
    assert r.n_iterations == ro.n_iterations == 4
    assert abs(r.gradient_norm - ro.gradient_norm) <= 1e-8 * max(ro.gradient_norm, 1e-300)
    assert np.max(np.abs(r.unmixing - ro.unmixing)) <= 1e-8
