"""GPU properties at BASELINE config 3's full size (N = 128, T = 1e8: 102.4 GB of X
generated in HBM). The oracle cannot run at this size, so these are the
size-independent checks the domain offers:
  * whitening: with K from the device Gram, every row of Y = K·(X − μ) has
    Σy²/T = 1 (Y·Yᵀ/T = I) — to 1e-10;
  * orthogonal invariance: for Y = Q·K·(X − μ) with Q orthogonal,
    Σ_i Σ_t y_it² = N·T — to 1e-10 relative;
  * the split evaluation (loss-only try + completion) is bit-identical to the
    fused pass on either Y stage (int8 digits, the default here, and fp64), and
    the skipped-Σy² pass changes no other statistic;
  * the two Y stages agree to 1e-13 relative and both keep Σ y² = N·T to 1e-10.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, T = 128, 100_000_000


@pytest.fixture(scope="module")
def big(pa):
    ctx = pa.DeviceContext(0)
    ctx.generate(N, T, 42)
    mu = ctx.rowsum() / T
    c = ctx.gram(mu) / T
    ev, u = np.linalg.eigh(c)
    k = (u / np.sqrt(ev)).T  # K·C·Kᵀ = I
    return ctx, mu, k


def test_whitened_rows_have_unit_power(pa, big):
    ctx, mu, k = big
    st = ctx.eval(k, mu, pa.DensityType.tanh(), False, need_y2=True)
    assert np.max(np.abs(st["y2"] / T - 1.0)) < 1e-10


def test_orthogonal_invariance_and_split_identity(pa, big):
    ctx, mu, k = big
    q = np.linalg.qr(np.random.default_rng(7).normal(size=(N, N)))[0]
    w = q @ k
    d = pa.DensityType.tanh()
    full = ctx.eval(w, mu, d, False, need_y2=True)
    assert abs(full["y2"].sum() / (N * T) - 1.0) < 1e-10
    lean = ctx.eval(w, mu, d, False, need_y2=False)
    for key in ("G", "dpsi", "ll"):
        assert np.array_equal(lean[key], full[key]), key
    # the default (int8-digit) Y stage: loss-only try + completion == fused pass
    assert ctx.int8_passes >= 2
    loss_only, kept, done = ctx.eval_split(w, mu, d, False, need_y2=False)
    assert np.array_equal(loss_only["ll"], full["ll"])
    for key in ("G", "dpsi", "ll"):
        assert np.array_equal(done[key], full[key]), key
    # the fp64 Y stage: the same identities, and agreement with the int8 stage to 1e-13
    ctx.set_y_stage("f64")
    n8 = ctx.int8_passes
    full64 = ctx.eval(w, mu, d, False, need_y2=True)
    assert abs(full64["y2"].sum() / (N * T) - 1.0) < 1e-10
    lo64, _, done64 = ctx.eval_split(w, mu, d, False, need_y2=False)
    assert ctx.int8_passes == n8
    assert np.array_equal(lo64["ll"], full64["ll"])
    for key in ("G", "dpsi", "ll"):
        assert np.array_equal(done64[key], full64[key]), key
        assert np.max(np.abs(full64[key] - full[key])) <= 1e-13 * np.max(np.abs(full64[key])), key
    ctx.set_y_stage("auto")
    # tanh: 0 < ψ′ ≤ α and ℓ ≥ |y| ≥ 0 per sample, so the row sums are bounded
    assert np.all(full["dpsi"] > 0) and np.all(full["dpsi"] <= T)
    assert np.all(full["ll"] > 0)
