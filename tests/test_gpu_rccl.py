"""The RCCL transport of the multi-GPU run on ONE GPU: a one-rank RCCL
communicator (pc_ctx_create with an id at world_size 1).

RCCL refuses two ranks on one device, so a one-GPU box cannot host the 8-rank
communicator of bench.py --gpus 8. A one-rank communicator still runs every line
of RcclCollective on the hardware: ncclCommInitRank from an id made by
pc_rccl_unique_id, the shared-memory abort word, ncclAllReduce on the context's
stream at every call site, the polling wait (hipStreamQuery + abort word + peer
pids + watchdog), the capability agreement, ncclCommAbort and ncclCommDestroy.
The statistics of a one-rank sum are the rank's own, so the fit must equal the
communicator-free context bit for bit (core.rs:76,218,226,274: sums over t).
"""
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _fit(pa, ctx, cfg):
    s = pa.Solver(ctx, cfg)
    try:
        while not s.step():
            pass
        return s.finish()
    finally:
        s.close()


def test_rccl_one_rank_fit_bit_identical(pa):
    """Picard-O at N = 128 on the int8 Y stage with the screen (the bench's C3 path)
    through a one-rank RCCL communicator: the same unmixing bits and iterations as
    without a communicator; every pass went through ncclAllReduce and the screen
    branch was agreed through it."""
    nf, T = 128, 200003
    cfg = pa.PicardConfig(random_state=42, max_iter=40, want_sources=False)
    plain = pa.DeviceContext(0)
    plain.generate(nf, T, 42)
    ref = _fit(pa, plain, cfg)
    plain.close()

    ctx = pa.DeviceContext(0, 0, 1, pa.rccl_unique_id())
    try:
        ctx.generate(nf, T, 42)
        out = _fit(pa, ctx, cfg)
        st = ctx.comm_stats()
        n8 = ctx.int8_passes
    finally:
        ctx.close()
    assert st["kind"] == "rccl" and st["world_size"] == 1 and not st["aborted"]
    assert st["screen_agreed"] == 1 and st["agreements"] >= 1
    assert st["allreduces"] > out.n_iterations  # ≥ one per pass, plus setup and screens
    assert n8 > 0
    assert out.n_iterations == ref.n_iterations and out.converged == ref.converged
    assert np.array_equal(out.unmixing, ref.unmixing)
    assert np.array_equal(out.whitening, ref.whitening)


def test_rccl_one_rank_call_sites_match(pa):
    """Each all-reduce call site through RCCL equals the communicator-free context bit
    for bit: rowsum, Gram, the fused pass with and without H, the int8 screen."""
    nf, T = 96, 100003
    rng = np.random.default_rng(3)
    w = np.linalg.qr(rng.normal(size=(nf, nf)))[0]
    d = pa.DensityType.tanh()

    def calls(ctx):
        ctx.generate(nf, T, 7)
        mu = ctx.rowsum() / T
        out = {"rowsum": ctx.rowsum(), "gram": ctx.gram(mu)}
        for h in (False, True):
            for k, v in ctx.eval(w, mu, d, h).items():
                out[f"eval{int(h)}_{k}"] = v
        sl, sb = ctx.eval_loss_screen(w, mu, d)
        out["screen_ll"], out["screen_bound"] = sl, sb
        return out

    plain = pa.DeviceContext(0)
    want = calls(plain)
    plain.close()
    ctx = pa.DeviceContext(0, 0, 1, pa.rccl_unique_id())
    try:
        got = calls(ctx)
        assert ctx.comm_stats()["allreduces"] >= 6
    finally:
        ctx.close()
    for k in want:
        assert np.array_equal(got[k], want[k]), k


def test_rccl_one_rank_abort_ends_calls(pa):
    """pc_ctx_abort on an RCCL context: ncclCommAbort, then every later call raises
    instead of waiting on a dead communicator."""
    ctx = pa.DeviceContext(0, 0, 1, pa.rccl_unique_id())
    try:
        ctx.generate(16, 10007, 3)
        ctx.rowsum()
        ctx.abort("test abort")
        t0 = time.perf_counter()
        with pytest.raises(pa.ComputationError, match="aborted"):
            ctx.rowsum()
        assert time.perf_counter() - t0 < 10.0
        assert ctx.comm_stats()["aborted"]
    finally:
        ctx.close()


def test_rccl_one_rank_capability_loss_raises(pa):
    """The digit image the communicator agreed on is released mid-fit
    (pc_ctx_release_caches): the next screened try raises (no silent branch change
    that peers would not follow) and the communicator is aborted."""
    ctx = pa.DeviceContext(0, 0, 1, pa.rccl_unique_id())
    try:
        ctx.generate(128, 100003, 42)
        s = pa.Solver(ctx, pa.PicardConfig(random_state=42, max_iter=60, want_sources=False))
        released = False
        try:
            with pytest.raises(pa.ComputationError, match="lost it"):
                for _ in range(60):
                    if not released and ctx.comm_stats()["screen_agreed"] == 1:
                        ctx.release_caches()
                        released = True
                    if s.step():
                        break
        finally:
            s.close()
        assert released and ctx.comm_stats()["aborted"]
    finally:
        ctx.close()
