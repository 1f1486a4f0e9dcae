"""The communicator path of the multi-GPU run on ONE GPU.

An in-process rank group (pc_group_create_local) holds `world` rank contexts on
device 0; each rank is driven by its own host thread through the real
rank-replicated Solver (pc_solver_create / step / finish) — the structure of
bench.py --gpus N, one Solver per rank, with only the transport of the per-pass
all-reduce replaced (host memory, fixed rank-order sum, instead of RCCL/xGMI).
So every DeviceCtx branch that exists only with a communicator runs here: the
all-reduce at each call site, the capability agreements (DeviceCtx::agree_once)
that pick the screen branch, the pinned digit image, and the group abort that
turns one rank's error into an error on every rank instead of a hang.

Every statistic is a sum over t (core.rs:76,218,226,274; whitening.rs:25), so
the group must reproduce world = 1 up to the summation order: per-call sums to
1e-12, and a Picard-O fit on the int8 Y stage with the line-search screen and
the curvature rejection with the same iteration count and unmixing within 1e-10.
"""
import threading
import time

import numpy as np
import pytest

from conftest import rel_err

pytestmark = pytest.mark.gpu

TOL = 1e-12


class RankGroup:
    """`world` rank contexts of one in-process group on device 0, one thread per rank."""

    def __init__(self, pa, world, nf, T, seed=42):
        self.pa, self.world = pa, world
        self.g = pa.LocalGroup(world)
        self.ctxs = [pa.DeviceContext(0, r, world, group=self.g) for r in range(world)]
        self.a = [c.generate(nf, T, seed) for c in self.ctxs][0]  # local: no collective

    def run(self, fn, timeout=600):
        """fn(rank, ctx) on one thread per rank; returns (results, errors). A rank whose
        Python code raises aborts the group so that no peer is left waiting."""
        res, err = [None] * self.world, [None] * self.world

        def body(r):
            try:
                res[r] = fn(r, self.ctxs[r])
            except BaseException as e:  # noqa: BLE001 — reported to the test below
                err[r] = e
                self.ctxs[r].abort(f"rank {r} raised {e!r}")

        th = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(self.world)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout)
        assert not any(t.is_alive() for t in th), "a rank thread did not finish"
        return res, err

    def close(self):
        for c in self.ctxs:
            c.close()
        self.g.close()


def _no_errors(err):
    assert all(e is None for e in err), err


@pytest.mark.parametrize("world", [2, 8])
def test_group_call_sites_match_world1(pa, world):
    """Every all-reduce call site of DeviceCtx through the group equals world = 1:
    rowsum, gram, the fused pass (with and without H), the split loss + completion, the
    non-orthogonal multi-try pass, the int8 screen, moments4 — identical bits on every
    rank, within 1e-12 of world = 1."""
    nf, T = 96, 100003
    full = pa.DeviceContext(0)
    full.generate(nf, T, 7)
    rng = np.random.default_rng(world)
    w = np.linalg.qr(rng.normal(size=(nf, nf)))[0]
    mu = full.rowsum() / T
    z = rng.normal(size=(nf, nf)) / np.sqrt(nf)
    al = np.array([0.5 ** j for j in range(1, 6)])
    d = pa.DensityType.tanh()

    def calls(ctx):
        out = {"rowsum": ctx.rowsum(), "gram": ctx.gram(mu)}
        for h in (False, True):
            for k, v in ctx.eval(w, mu, d, h).items():
                out[f"eval{int(h)}_{k}"] = v
        lo, kept, done = ctx.eval_split(w, mu, d, False)
        out["split_ll"] = lo["ll"]
        out["split_G"] = done["G"]
        ll, y2 = ctx.eval_loss_multi(w, z, al, mu, d)
        out["multi_ll"], out["multi_y2"] = ll, y2
        sl, sb = ctx.eval_loss_screen(w, mu, d)
        out["screen_ll"], out["screen_bound"] = sl, sb
        out["moments4"] = ctx.moments4(w[:12], mu)
        return out

    want = calls(full)
    g = RankGroup(pa, world, nf, T, seed=7)
    try:
        res, err = g.run(lambda r, c: (calls(c), c.comm_stats()))
        _no_errors(err)
        for r in range(world):
            got, st = res[r]
            assert st["kind"] == "local" and st["world_size"] == world and not st["aborted"]
            assert st["screen_agreed"] == 1 and st["agreements"] >= 1
            for k in want:
                assert np.array_equal(got[k], res[0][0][k]), (r, k)  # lockstep: identical bits
                if k == "screen_bound":  # each shard bounds its own part: the worst-case tail adds
                    # up to world 1's, the statistical tail (per-shard Cauchy–Schwarz) to about it
                    assert np.all(got[k] >= want[k] * 0.5) and np.all(got[k] <= want[k] * 4.0), k
                    continue
                if k == "screen_ll":  # fp32 ℓ: shard-dependent grouping, within the two bounds
                    assert np.all(np.abs(got[k] - want[k]) <= got["screen_bound"] + want["screen_bound"])
                    continue
                assert rel_err(got[k], want[k]) <= TOL, (k, rel_err(got[k], want[k]))
    finally:
        g.close()


@pytest.mark.parametrize("world", [2, 8])
def test_group_fit_reproduces_world1(pa, world, capfd, monkeypatch):
    """The rank-replicated Solver over the group, Picard-O at N = 128 on the int8 Y stage
    with the line-search screen and the curvature rejection (the bench's C3 path):
    every rank bit-identical, and the same iteration count as world = 1 with the
    unmixing within 1e-10; the screen agreement ran, and so did the screen, the descent-search
    screen pairs and the curvature rejection."""
    monkeypatch.setenv("PICARD_TRACE", "1")
    nf, T = 128, 200003
    cfg = pa.PicardConfig(random_state=42, max_iter=40, want_sources=False)
    ref_ctx = pa.DeviceContext(0)
    ref_ctx.generate(nf, T, 42)
    sv = pa.Solver(ref_ctx, cfg)
    while not sv.step():
        pass
    ref = sv.finish()
    sv.close()
    ref_ctx.close()
    capfd.readouterr()

    g = RankGroup(pa, world, nf, T)

    def fit(r, ctx):
        s = pa.Solver(ctx, cfg)
        while not s.step():
            pass
        out = s.finish()
        s.close()
        return out, ctx.comm_stats(), ctx.int8_passes, ctx.screen_stats()[1]

    try:
        res, err = g.run(fit)
    finally:
        g.close()
    trace = capfd.readouterr().err
    _no_errors(err)
    r0 = res[0][0]
    for r in range(world):
        out, st, n8, nscreen = res[r]
        assert np.array_equal(out.unmixing, r0.unmixing) and out.n_iterations == r0.n_iterations
        assert st["screen_agreed"] == 1 and st["agreements"] >= 1 and not st["aborted"]
        assert n8 > 0 and nscreen > 0
        assert st["allreduces"] == res[0][1]["allreduces"]
    assert r0.n_iterations == ref.n_iterations and r0.converged == ref.converged
    assert np.max(np.abs(r0.unmixing - ref.unmixing)) <= 1e-10
    assert np.max(np.abs(r0.whitening - ref.whitening)) <= 1e-10
    assert "[picard-screen]" in trace and "[picard-curv]" in trace
    assert "(pair, descent)" in trace  # descent-search screen pairs ran on every rank alike


def test_group_nonortho_fit_rank_identical(pa):
    """C4's path over the group (world 2): non-orthogonal Picard at N = 100 — the tiled full
    pass with H and the multi-try pass reading Y back from it (k_multi_loss2_ozy) on every
    rank. Both ranks bit-identical (lockstep decisions from reduced sums), multi-try passes
    read Y back, and the fit converges to the fixed point world = 1 reaches: Amari distance to
    the generating mixing within 1e-6 of it. (Non-orthogonal trajectories are chaotic in the
    summation order — the shard split changes it — so the iteration counts differ: 124
    against 90 on the first run.)"""
    nf, T = 100, 60001
    cfg = pa.PicardConfig(ortho=False, extended=False, random_state=3, max_iter=200, want_sources=False)
    ref_ctx = pa.DeviceContext(0)
    a_mix = ref_ctx.generate(nf, T, 11)
    sv = pa.Solver(ref_ctx, cfg)
    while not sv.step():
        pass
    ref = sv.finish()
    sv.close()
    ref_ctx.close()
    g = RankGroup(pa, 2, nf, T, seed=11)

    def fit(r, ctx):
        s = pa.Solver(ctx, cfg)
        while not s.step():
            pass
        out = s.finish()
        s.close()
        return out, ctx.multi_ybuf_passes, ctx.comm_stats()

    try:
        res, err = g.run(fit)
    finally:
        g.close()
    _no_errors(err)
    (o0, n0, st0), (o1, n1, st1) = res
    assert np.array_equal(o0.unmixing, o1.unmixing) and o0.n_iterations == o1.n_iterations
    assert n0 == n1 and n0 > 0 and st0["allreduces"] == st1["allreduces"] and not st0["aborted"]
    assert o0.converged and ref.converged
    am0 = pa.utils.amari_distance(o0.full_unmixing(), a_mix)
    am_ref = pa.utils.amari_distance(ref.full_unmixing(), a_mix)
    assert abs(am0 - am_ref) <= 1e-6, (am0, am_ref)


@pytest.mark.parametrize("world", [2, 8])
def test_group_capability_loss_aborts_every_rank(pa, world):
    """One rank loses the int8 digit image the ranks agreed on (pc_ctx_release_caches)
    in the middle of a fit: its next screened try raises, the group is aborted, and every
    other rank — waiting in that pass's all-reduce — ends with an error within seconds
    instead of hanging."""
    nf, T = 128, 100003
    g = RankGroup(pa, world, nf, T)
    victim = world - 1
    t_release = [None]

    def fit(r, ctx):
        s = pa.Solver(ctx, pa.PicardConfig(random_state=42, max_iter=60, want_sources=False))
        try:
            for it in range(60):
                # the victim drops the image once the ranks have agreed on it (first screen)
                if r == victim and t_release[0] is None and ctx.comm_stats()["screen_agreed"] == 1:
                    t_release[0] = time.perf_counter()
                    ctx.release_caches()
                if s.step():
                    return "finished"
            return "max_iter"
        finally:
            s.close()

    try:
        res, err = g.run(fit, timeout=120)
        t_end = time.perf_counter()
        stats = [c.comm_stats() for c in g.ctxs]
    finally:
        g.close()
    assert all(isinstance(e, pa.ComputationError) for e in err), (res, err)
    assert "lost it" in str(err[victim])
    assert all(st["aborted"] for st in stats)
    assert t_release[0] is not None and t_end - t_release[0] < 30.0


def test_group_divergent_collectives_fail_fast(pa):
    """Ranks that issue different collectives in the same slot (a rowsum against a Gram)
    are caught by the group's call-site check and all end with an error."""
    g = RankGroup(pa, 2, 16, 10007)
    try:
        _, err = g.run(lambda r, c: c.rowsum() if r == 0 else c.gram(None), timeout=60)
    finally:
        g.close()
    assert all(isinstance(e, pa.ComputationError) for e in err), err
    assert any("diverged" in str(e) for e in err)


def test_group_unsupported_is_not_an_abort(pa, monkeypatch):
    """A capability miss (PC_ERR_UNSUPPORTED: the bounded multi-try pass without PICARD_MULTI_F32=1, a screen for a density
    without one, device JADE sweeps for a shape that does not fit) leaves the group usable: the documented fallback (pc_ctx_eval_loss_multi, an exact
    try) then runs on every rank and matches world = 1."""
    monkeypatch.setenv("PICARD_MULTI_F32", "0")
    nf, T = 96, 40009
    full = pa.DeviceContext(0)
    full.generate(nf, T, 11)
    rng = np.random.default_rng(3)
    w = np.linalg.qr(rng.normal(size=(nf, nf)))[0]
    z = rng.normal(size=(nf, nf)) / np.sqrt(nf)
    mu = full.rowsum() / T
    al = np.array([1.0, 0.5, 0.25])
    want_ll, want_y2 = full.eval_loss_multi(w, z, al, mu, pa.DensityType.tanh())
    full.close()

    def body(r, c):
        misses = 0
        for call in (lambda: c.eval_loss_multi_bound(w, z, al, mu, pa.DensityType.tanh()),
                     lambda: c.eval_loss_screen(w, mu, pa.DensityType.cube())):
            try:
                call()
            except pa.Unsupported:
                misses += 1
        ll, y2 = c.eval_loss_multi(w, z, al, mu, pa.DensityType.tanh())
        return misses, ll, y2, c.comm_stats()

    g = RankGroup(pa, 2, nf, T, seed=11)
    try:
        res, err = g.run(body, timeout=120)
    finally:
        g.close()
    _no_errors(err)
    for misses, ll, y2, st in res:
        assert misses == 2 and not st["aborted"]
        assert rel_err(ll, want_ll) <= TOL and rel_err(y2, want_y2) <= TOL


def test_group_refuses_bad_rank(pa):
    g = pa.LocalGroup(2)
    with pytest.raises(pa.InvalidDimensions):
        pa.DeviceContext(0, 2, 2, group=g)
    g.close()


def test_jade_refuses_detached_shard(pa):
    """A detached shard only holds its own fourth moments: pc_ctx_jade refuses it."""
    c = pa.DeviceContext(0, 1, 2)
    c.generate(8, 2000, 3)
    with pytest.raises(pa.InvalidConfig):
        c.jade(np.eye(8))
    c.close()
