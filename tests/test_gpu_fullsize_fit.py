"""The headline workload's FIT at full size (BASELINE config 3: N = 128, T = 1e8, Picard-O
extended tanh, random_state 42 — the bench's configuration, generated in HBM).

The oracle cannot run at this size, so the check is the property that makes the bench's
schedule legitimate: the line-search screens (single and paired), the curvature rejections and
the quadratic-model schedule change no decision. The default mode ("auto") and the mode that
evaluates every try exactly on the same int8 digit stages ("int8-exact") must take the same
iterations to the same bits of the unmixing matrix; both converge to tol = 1e-7, and the fit
recovers the generated mixing (Amari distance < 1e-3). (core.rs:127-140 decides each try on
its exact loss; solver.rs:45-189.)
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N, T = 128, 100_000_000


def test_c3_fit_screened_equals_exact(pa):
    ctx = pa.DeviceContext(0)
    a = ctx.generate(N, T, 42)
    cfg = dict(ortho=True, max_iter=500, tol=1e-7, random_state=42, want_sources=False)

    def fit(mode):
        ctx.set_y_stage(mode)
        ctx.screen_stats(reset=True)
        n8 = ctx.int8_passes
        sv = pa.Solver(ctx, pa.PicardConfig(**cfg))
        while not sv.step():
            pass
        r = sv.finish()
        sv.close()
        return r, ctx.screen_stats()[1], ctx.int8_passes - n8

    r_auto, screens_auto, i8_auto = fit("auto")
    r_exact, screens_exact, i8_exact = fit("int8-exact")
    ctx.close()
    assert screens_auto > 0 and screens_exact == 0  # the schedule really differed
    assert i8_auto > 0 and i8_exact > 0
    assert r_auto.converged and r_exact.converged
    assert r_auto.n_iterations == r_exact.n_iterations
    assert np.array_equal(r_auto.unmixing, r_exact.unmixing)
    assert pa.utils.amari_distance(r_auto.full_unmixing(), a) < 1e-3


def test_c3_fit_digit_arithmetic_vs_fp64_stages(pa):
    """The shipped arithmetic (int8-digit Y, int8-digit G, screens) against the fp64 MFMA
    stages that the oracle pins at small sizes (PC_YSTAGE_F64 + PC_GSTAGE_F64), on the SAME
    generated X at the bench's full size. Tolerances: both converge; iterations within ±2; the
    first 5 per-iteration losses within 1e-9 relative; |ΔAmari| to the generated mixing
    ≤ 1e-6 (north_star's tolerance). (core.rs:211-293, solver.rs:45-189.)"""
    ctx = pa.DeviceContext(0)
    a = ctx.generate(N, T, 42)
    cfg = dict(ortho=True, max_iter=500, tol=1e-7, random_state=42, want_sources=False)

    def fit(y_stage, g_stage):
        ctx.set_y_stage(y_stage)
        ctx.set_g_stage(g_stage)
        n8, g8 = ctx.int8_passes, ctx.g8_passes
        sv = pa.Solver(ctx, pa.PicardConfig(**cfg))
        losses = []
        while not sv.step():
            losses.append(sv.last()[0])
        r = sv.finish()
        sv.close()
        return r, losses, ctx.int8_passes - n8, ctx.g8_passes - g8

    r_d, l_d, i8_d, g8_d = fit("auto", "auto")
    r_f, l_f, i8_f, g8_f = fit("f64", "f64")
    ctx.close()
    am_d = pa.utils.amari_distance(r_d.full_unmixing(), a)
    am_f = pa.utils.amari_distance(r_f.full_unmixing(), a)
    print(f"\ndigit stages: {r_d.n_iterations} iterations, Amari {am_d:.3e}, {i8_d} int8 / {g8_d} digit-G passes")
    print(f"fp64 stages : {r_f.n_iterations} iterations, Amari {am_f:.3e}, {i8_f} int8 / {g8_f} digit-G passes")
    print("first losses:", l_d[:5], l_f[:5])
    assert i8_d > 0 and g8_d > 0 and i8_f == 0 and g8_f == 0   # the two fits really ran different stages
    assert r_d.converged and r_f.converged
    assert abs(r_d.n_iterations - r_f.n_iterations) <= 2
    k = min(5, len(l_d), len(l_f))
    assert k == 5
    np.testing.assert_allclose(l_d[:k], l_f[:k], rtol=1e-9, atol=0)
    assert abs(am_d - am_f) <= 1e-6
