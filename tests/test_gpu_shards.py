"""The T-sharded device path on ONE GPU, through detached shards.

A detached shard (pc_ctx_create with world_size > 1 and no RCCL id) is the
rank-r context of the multi-GPU run without its communicator: the same
per-shard generator jump-ahead, the same shard bounds (DeviceCtx::shard_t0 /
shard_n, shards whose n_local is not a multiple of 16), the same per-shard
resident centring and per-shard row constants (finalize_row with the shard's
n_local) — only the RCCL all-reduce is replaced by a host sum. Every
statistic is a sum over t (core.rs:76,218,226,274; whitening.rs:25), so:

  (a) each shard's generate() is bit-identical to its slice of the world=1 X;
  (b) host-summed per-shard eval / eval_split / eval_loss_multi / gram /
      rowsum / moments4 equal world=1 to 1e-12 (relative, summation order);
      per-shard sources are bit-identical to the world=1 slice;
  (c) the host driver (pc_fit_with_evaluator) over the shard contexts
      reproduces the world=1 GPU fit (pc_fit): Picard-O with the same
      iteration count and unmixing within 1e-10; non-orthogonal Picard (chaotic
      in the summation order, see the test) to the same separation.
"""
import numpy as np
import pytest

from conftest import rel_err

pytestmark = pytest.mark.gpu

TOL = 1e-12
T_SHARD = 100003  # ragged: shards of 50002/50001, 33335/33334/33334, 12501/12500 …


class ShardGroup:
    """`world` detached shard contexts on device 0; sums their statistics on the host."""

    def __init__(self, pa, world, nf, T, seed=42):
        self.pa, self.world, self.nf, self.T = pa, world, nf, T
        self.ctxs = [pa.DeviceContext(0, r, world) for r in range(world)]
        self.a = [c.generate(nf, T, seed) for c in self.ctxs][0]

    def sum(self, f):
        parts = [f(c) for c in self.ctxs]
        if isinstance(parts[0], dict):
            return {k: sum(p[k] for p in parts) for k in parts[0]}
        if isinstance(parts[0], tuple):
            return tuple(sum(p[i] for p in parts) for i in range(len(parts[0])))
        return sum(parts)

    def fit(self, cfg):
        pa = self.pa
        return pa.fit_with_host_evaluator(
            self.nf, self.T, cfg,
            rowsum=lambda: self.sum(lambda c: c.rowsum()),
            gram=lambda mu: self.sum(lambda c: c.gram(mu)),
            eval=lambda w, mu, d, h: self.sum(lambda c: c.eval(w, mu, d, h)),
            sources=lambda w, mu: np.concatenate([c.sources(w, mu) for c in self.ctxs], axis=1),
            moments4=lambda w, mu: self.sum(lambda c: c.moments4(w, mu)),
            eval_loss_multi=lambda w, z, al, mu, d: self.sum(lambda c: c.eval_loss_multi(w, z, al, mu, d)))


def shard_bounds(T, world, rank):
    base, rem = divmod(T, world)
    return rank * base + min(rank, rem), base + (1 if rank < rem else 0)


@pytest.fixture(scope="module")
def full16(pa):
    ctx = pa.DeviceContext(0)
    a = ctx.generate(16, T_SHARD, 42)
    return ctx, a, ctx.download()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_shard_generate_bit_identical(pa, full16, world):
    _, a, x = full16
    g = ShardGroup(pa, world, 16, T_SHARD)
    assert np.array_equal(g.a, a)
    for r, c in enumerate(g.ctxs):
        t0, nl = shard_bounds(T_SHARD, world, r)
        assert (c.t0, c.n_local) == (t0, nl)
        assert np.array_equal(c.download(), x[:, t0:t0 + nl]), r


def test_detached_shard_refuses_solver(pa):
    c = pa.DeviceContext(0, 1, 2)
    c.generate(8, 1000, 42)
    with pytest.raises(pa.PicardError):
        pa.Solver(c, pa.PicardConfig(w_init=np.eye(8)))


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("nf", [16, 64, 128, 256])
def test_shard_sums_match_world1(pa, world, nf):
    T = 40009 if nf >= 128 else T_SHARD
    full = pa.DeviceContext(0)
    full.generate(nf, T, 7)
    g = ShardGroup(pa, world, nf, T, seed=7)
    rng = np.random.default_rng(nf + world)
    w = np.linalg.qr(rng.normal(size=(nf, nf)))[0]
    mu = full.rowsum() / T
    assert rel_err(g.sum(lambda c: c.rowsum()), full.rowsum()) <= TOL
    assert rel_err(g.sum(lambda c: c.gram(mu)), full.gram(mu)) <= TOL
    for dens in [pa.DensityType.tanh(), pa.DensityType.exp(1.0), pa.DensityType.cube()]:
        for need_h in [False, True]:
            want = full.eval(w, mu, dens, need_h)
            got = g.sum(lambda c: c.eval(w, mu, dens, need_h))
            for k in want:
                assert rel_err(got[k], want[k]) <= TOL, (dens.kind, need_h, k)
    # split evaluation (line-search tries): loss-only stats, then the completion
    lo_w, _, full_w = full.eval_split(w, mu, pa.DensityType.tanh(), False)
    parts = [c.eval_split(w, mu, pa.DensityType.tanh(), False) for c in g.ctxs]
    for k in ("ll",):
        assert rel_err(sum(p[0][k] for p in parts), lo_w[k]) <= TOL
    for k in full_w:
        assert rel_err(sum(p[2][k] for p in parts), full_w[k]) <= TOL, k
    # non-orthogonal multi-try pass
    z = rng.normal(size=(nf, nf)) / np.sqrt(nf)
    al = np.array([0.5 ** j for j in range(1, 10)])
    ll_w, y2_w = full.eval_loss_multi(w, z, al, mu, pa.DensityType.tanh())
    ll_g, y2_g = g.sum(lambda c: c.eval_loss_multi(w, z, al, mu, pa.DensityType.tanh()))
    assert rel_err(ll_g, ll_w) <= TOL and rel_err(y2_g, y2_w) <= TOL
    if 64 < nf <= 128:  # these passes ran on each shard's own int8 digit image
        assert full.int8_passes > 0 and all(c.int8_passes > 0 for c in g.ctxs)
    # sources: per-sample, so every shard is bit-identical to its slice
    y_w = full.sources(w[: min(nf, 32)], mu)
    y_g = np.concatenate([c.sources(w[: min(nf, 32)], mu) for c in g.ctxs], axis=1)
    assert np.array_equal(y_g, y_w)


@pytest.mark.parametrize("world", [2, 8])
def test_shard_moments4(pa, world):
    nf, T = 12, 20011
    full = pa.DeviceContext(0)
    full.generate(nf, T, 3)
    g = ShardGroup(pa, world, nf, T, seed=3)
    w = np.eye(nf)
    mu = full.rowsum() / T
    assert rel_err(g.sum(lambda c: c.moments4(w, mu)), full.moments4(w, mu)) <= TOL


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("ortho", [True, False])
def test_sharded_fit_reproduces_world1(pa, world, ortho):
    """Picard-O: the sharded fit follows the world=1 trajectory (same iteration
    count, unmixing within 1e-10). Non-orthogonal Picard on this mixture is
    chaotic in the summation order — the CPU oracle itself, fed the same data
    as 1, 2 or 3 host-summed shards, converges in 70 / 60 / 76 iterations to
    solutions that differ by a signed row permutation — so there the check is
    the one that is order-free: both converge to the same separation
    (Amari distance against A within 1e-6, north_star) and the two unmixing
    matrices agree up to a signed permutation (Amari of one against the
    other's inverse ≤ 1e-6)."""
    nf, T = 16, 200003
    full = pa.DeviceContext(0)
    a = full.generate(nf, T, 42)
    x = full.download()
    cfg = pa.PicardConfig(ortho=ortho, w_init=np.eye(nf), max_iter=200)
    ref = pa.Picard.fit_with_config(x, cfg)  # world=1 GPU fit through pc_fit
    g = ShardGroup(pa, world, nf, T, seed=42)
    got = g.fit(cfg)
    assert got.converged and ref.converged
    if ortho:
        assert got.n_iterations == ref.n_iterations
        assert np.max(np.abs(got.unmixing - ref.unmixing)) <= 1e-10
        assert np.max(np.abs(got.sources - ref.sources)) <= 1e-9
    else:
        am = pa.utils.amari_distance
        assert abs(am(got.full_unmixing(), a) - am(ref.full_unmixing(), a)) <= 1e-6
        assert am(got.full_unmixing(), np.linalg.inv(ref.full_unmixing())) <= 1e-6
    assert np.max(np.abs(got.whitening - ref.whitening)) <= 1e-10


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_fit_int8_stage_reproduces_world1(pa, world):
    """Picard-O at N = 96 (the int8-digit Y stage: per-sample exponents, so every shard's
    y values are those of the world=1 context and only the summation order differs):
    same iteration count, unmixing within 1e-10."""
    nf, T = 96, 60013
    full = pa.DeviceContext(0)
    full.generate(nf, T, 42)
    x = full.download()
    cfg = pa.PicardConfig(w_init=np.eye(nf), max_iter=200)
    ref = pa.Picard.fit_with_config(x, cfg)
    g = ShardGroup(pa, world, nf, T, seed=42)
    got = g.fit(cfg)
    assert all(c.int8_passes > 0 for c in g.ctxs)
    assert got.converged and ref.converged
    assert got.n_iterations == ref.n_iterations
    assert np.max(np.abs(got.unmixing - ref.unmixing)) <= 1e-10
