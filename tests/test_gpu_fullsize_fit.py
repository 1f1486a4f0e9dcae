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
