"""Try 1's map of the orthogonal line search on the device (expm.inc k_expm_ps).

W ← expm(α·D)·W (core.rs:118-125, math.rs:38-74) is on every iteration's critical path; the
device forms expm with the host matrix_exp's arithmetic — the same scaling, the same
Paterson–Stockmeyer plan (expm_plan.hpp) from the same ∞-norms, every product summed over p in
increasing order by fma, every element-wise update unfused — so the tolerance is EXACT equality
with pc_matrix_exp (the host routine tests/test_host_expm.py pins against the reference series).
Shapes the device leaves to the host (n not a multiple of 32 in [32, 128], a series the
reference caps at 30 terms) raise Unsupported, and a fit with the device map is bit-identical
to one with the host map (PICARD_DEVICE_EXPM=0).
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def host_expm(pa, a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    out = np.empty_like(a)
    pa.lib.pc_matrix_exp(a.ctypes.data_as(C.POINTER(C.c_double)), a.shape[0], out.ctypes.data_as(C.POINTER(C.c_double)))
    return out


def skew(rng, n, scale):
    b = rng.normal(size=(n, n)) * scale / np.sqrt(n)
    return b - b.T


@pytest.fixture(scope="module")
def ctx(pa):
    import os
    os.environ["PICARD_DEVICE_EXPM_MIN_N"] = "32"  # every size the kernel supports (default: n ≥ 96)
    c = pa.DeviceContext(0)
    del os.environ["PICARD_DEVICE_EXPM_MIN_N"]
    c.load(np.random.default_rng(1).normal(size=(8, 64)))
    yield c
    c.close()


def series_converges(a):
    """expm_plan.hpp's test in numpy: does the reference's 30-term series converge (remainder
    bound < 1e-17 from ‖B^k‖∞, B = A / 2^s)? Where it does not, the host restates the capped loop
    and the device declines."""
    norm = np.max(np.abs(a))
    if norm < 1e-15:
        return True
    s = max(int(np.ceil(np.log2(norm))), 0)
    b = a / 2.0 ** s
    p, nu = b, [1.0]
    for _ in range(4):
        nu.append(np.max(np.sum(np.abs(p), axis=1)))
        p = p @ b
    terms, inv_fact, p4 = [0.0] * 91, 1.0, 1.0
    for k in range(1, 91):
        inv_fact /= k
        if k % 4 == 0:
            p4 *= nu[4]
        terms[k] = p4 * nu[k % 4] * inv_fact
    return np.isfinite(nu[4]) and sum(terms[31:]) < 1e-17


@pytest.mark.parametrize("n", [32, 64, 96, 128])
@pytest.mark.parametrize("scale", [1e-17, 1e-6, 1e-3, 0.05, 0.5, 2.0, 9.0])
def test_device_expm_equals_host(pa, ctx, n, scale):
    rng = np.random.default_rng(n * 1000 + int(scale * 100))
    a = skew(rng, n, scale)
    if not series_converges(a):  # the capped series: the host's path
        assert scale >= 2.0
        with pytest.raises(pa.Unsupported):
            ctx.matrix_exp(a)
        return
    dev = ctx.matrix_exp(a)
    assert np.array_equal(dev, host_expm(pa, a))


@pytest.mark.parametrize("n", [64, 128])
def test_device_expm_general_matrix(pa, ctx, n):
    """Not only skew directions: a general matrix (the routine is matrix_exp, any A)."""
    rng = np.random.default_rng(7)
    a = rng.normal(size=(n, n)) * 0.3 / np.sqrt(n)
    assert np.array_equal(ctx.matrix_exp(a), host_expm(pa, a))


def test_device_expm_repeated_calls(pa, ctx):
    """The grid barrier's tags continue across calls: many calls in a row stay exact."""
    rng = np.random.default_rng(11)
    done = 0
    for _ in range(40):
        a = skew(rng, 128, rng.uniform(0.01, 1.5))
        if series_converges(a):
            assert np.array_equal(ctx.matrix_exp(a), host_expm(pa, a))
            done += 1
    assert done >= 15


@pytest.mark.parametrize("n", [8, 48, 160])
def test_device_expm_shapes_left_to_host(pa, ctx, n):
    """n not a multiple of 32 in [32, 128]: the host's."""
    a = skew(np.random.default_rng(3), n, 0.5)
    with pytest.raises(pa.Unsupported):
        ctx.matrix_exp(a)


def test_device_expm_capped_series_left_to_host(pa, ctx):
    """A direction whose powers do not let the 30-term series converge (the host restates the
    reference's capped loop there): the device declines instead of guessing."""
    a = skew(np.random.default_rng(5), 64, 9.0)  # ‖B^k‖ bounds too large for 30 terms
    assert not series_converges(a)
    with pytest.raises(pa.Unsupported):
        ctx.matrix_exp(a)


def test_fit_with_device_map_bit_identical(pa, monkeypatch):
    """A Picard-O fit (N = 128: the int8 stage, the digit G stage, screens) with try 1's map on the
    device lands on the same unmixing bits as with the host map."""
    rng = np.random.default_rng(21)
    n, t = 128, 40000
    s = rng.laplace(size=(n, t))
    x = (rng.uniform(-0.5, 0.5, size=(n, n)) + np.eye(n)) @ s

    def fit():
        ctx = pa.DeviceContext(0)
        ctx.load(x)
        sv = pa.Solver(ctx, pa.PicardConfig(random_state=4, max_iter=100, want_sources=False))
        while not sv.step():
            pass
        r = sv.finish()
        sv.close()
        ctx.close()
        return r

    monkeypatch.delenv("PICARD_DEVICE_EXPM", raising=False)
    r_dev = fit()
    monkeypatch.setenv("PICARD_DEVICE_EXPM", "0")
    r_host = fit()
    assert r_dev.n_iterations == r_host.n_iterations and r_dev.converged == r_host.converged
    assert np.array_equal(r_dev.unmixing, r_host.unmixing)
