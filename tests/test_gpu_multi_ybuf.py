"""Non-ortho multi-try pass with Y read back (k_multi_loss2_ozy).

The reference's line search forms every try from the Y it keeps between passes
(core.rs:117-141: y_new = transform.dot(y)). The tiled full pass on the int8 digit stage
leaves Y of the whole shard in HBM; the multi-try pass at the same W then reads it instead of
forming it again, and only forms Z. Both Y's come from the same digit products, scales and
combine, and the new kernel sums each lane's samples in the old kernel's order on the old
kernel's sample partition, so every Σℓ / Σy² — hence every line-search decision — is bit for
bit the one of the pass that forms Y (PICARD_MULTI_YBUF=0). Tolerance: exact equality.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rng():
    return np.random.default_rng(4242)


def laplace_mix(rng, nf, t):
    s = rng.laplace(size=(nf, t))
    a = rng.uniform(-0.5, 0.5, size=(nf, nf)) + np.eye(nf)
    return a @ s + rng.normal(size=(nf, 1))


def ctx_with(pa, x):
    ctx = pa.DeviceContext(0)
    ctx.load(x)
    return ctx


DENS = [("tanh", 1.0), ("tanh", 0.6), ("exp", 0.5), ("cube", 1.0)]


@pytest.mark.parametrize("nc,nf", [(256, 256), (100, 100), (128, 128), (20, 70)])
@pytest.mark.parametrize("dens", DENS)
def test_multi_ybuf_bit_identical(pa, rng, monkeypatch, nc, nf, dens):
    x = laplace_mix(rng, nf, 3001)  # ragged: the last 64-sample tile is partial
    w = rng.normal(size=(nc, nf)) / np.sqrt(nf)
    z = rng.normal(size=(nc, nf)) / np.sqrt(nf)
    mu = x.mean(axis=1)
    d = pa.DensityType(["tanh", "exp", "cube"].index(dens[0]), dens[1])
    alphas = 0.5 ** np.arange(0, 10)

    def run():
        ctx = ctx_with(pa, x)
        ctx.eval(w, mu, d, need_h=True)  # the tiled full pass at W (H: nc > 64 or nf > 16·NB)
        ll, y2 = ctx.eval_loss_multi(w, z, alphas, mu, d)
        return ll, y2, ctx.multi_ybuf_passes

    monkeypatch.delenv("PICARD_MULTI_YBUF", raising=False)
    ll1, y21, n1 = run()
    monkeypatch.setenv("PICARD_MULTI_YBUF", "0")
    ll0, y20, n0 = run()
    # pc_ctx_eval_loss_multi returns Σy²: tanh at 256 features then keeps the kernel that forms Y
    expect = 0 if (nf > 128 and dens[0] == "tanh") else 1
    assert (n1, n0) == (expect, 0)
    assert np.array_equal(ll1, ll0) and np.array_equal(y21, y20)


def test_multi_ybuf_only_for_the_same_w(pa, rng, monkeypatch):
    """Y is read back only for the W of the last full tiled pass; any other W forms it."""
    monkeypatch.delenv("PICARD_MULTI_YBUF", raising=False)
    nc = nf = 100
    x = laplace_mix(rng, nf, 4099)
    w1 = rng.normal(size=(nc, nf)) / np.sqrt(nf)
    w2 = w1.copy()
    w2[3, 7] = np.nextafter(w2[3, 7], 1.0)  # one ulp apart
    z = rng.normal(size=(nc, nf)) / np.sqrt(nf)
    mu = x.mean(axis=1)
    d = pa.DensityType(0, 1.0)
    alphas = 0.5 ** np.arange(0, 10)
    ctx = ctx_with(pa, x)
    ctx.eval(w1, mu, d, need_h=True)
    got2 = ctx.eval_loss_multi(w2, z, alphas, mu, d)
    assert ctx.multi_ybuf_passes == 0
    got1 = ctx.eval_loss_multi(w1, z, alphas, mu, d)
    assert ctx.multi_ybuf_passes == 1
    fresh = ctx_with(pa, x)
    ref2 = fresh.eval_loss_multi(w2, z, alphas, mu, d)
    ref1 = fresh.eval_loss_multi(w1, z, alphas, mu, d)
    assert fresh.multi_ybuf_passes == 0
    for a, b in ((got1, ref1), (got2, ref2)):
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_multi_ybuf_two_slots(pa, rng, monkeypatch):
    """Two full passes keep both Y's (the second W goes to the other slot); a third pass
    replaces the older one. Every read-back result equals the pass that forms Y."""
    monkeypatch.delenv("PICARD_MULTI_YBUF", raising=False)
    nc = nf = 128
    x = laplace_mix(rng, nf, 5003)
    ws = [rng.normal(size=(nc, nf)) / np.sqrt(nf) for _ in range(3)]
    z = rng.normal(size=(nc, nf)) / np.sqrt(nf)
    mu = x.mean(axis=1)
    d = pa.DensityType(1, 0.5)  # exp: the read-back kernel at any Σy² / try count
    alphas = 0.5 ** np.arange(0, 10)
    fresh = ctx_with(pa, x)
    ref = [fresh.eval_loss_multi(w, z, alphas, mu, d) for w in ws]
    assert fresh.multi_ybuf_passes == 0
    ctx = ctx_with(pa, x)
    ctx.eval(ws[0], mu, d, need_h=True)
    ctx.eval(ws[1], mu, d, need_h=True)
    got0 = ctx.eval_loss_multi(ws[0], z, alphas, mu, d)
    got1 = ctx.eval_loss_multi(ws[1], z, alphas, mu, d)
    assert ctx.multi_ybuf_passes == 2
    ctx.eval(ws[2], mu, d, need_h=True)  # replaces W0's slot
    got0b = ctx.eval_loss_multi(ws[0], z, alphas, mu, d)
    assert ctx.multi_ybuf_passes == 2
    got1b = ctx.eval_loss_multi(ws[1], z, alphas, mu, d)
    got2 = ctx.eval_loss_multi(ws[2], z, alphas, mu, d)
    assert ctx.multi_ybuf_passes == 4
    for a, b in ((got0, ref[0]), (got1, ref[1]), (got0b, ref[0]), (got1b, ref[1]), (got2, ref[2])):
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_multi_ybuf_slot0_dropped_when_buffer_grows(pa, rng, monkeypatch):
    """A full pass that grows the tiled pass's buffer (exp with H stores ψ′ as a third array,
    tanh forms it from ψ) frees slot 0's Y even when the allocator returns the same address:
    a multi-try pass at slot 0's old W must then form Y, and equal a fresh context's result."""
    monkeypatch.delenv("PICARD_MULTI_YBUF", raising=False)
    nc = nf = 128
    x = laplace_mix(rng, nf, 4099)
    w0, w1, w2 = (rng.normal(size=(nc, nf)) / np.sqrt(nf) for _ in range(3))
    z = rng.normal(size=(nc, nf)) / np.sqrt(nf)
    mu = x.mean(axis=1)
    th, ex = pa.DensityType(0, 1.0), pa.DensityType(1, 0.5)
    alphas = 0.5 ** np.arange(0, 10)
    fresh = ctx_with(pa, x)
    ref1 = fresh.eval_loss_multi(w1, z, alphas, mu, ex)
    ref2 = fresh.eval_loss_multi(w2, z, alphas, mu, ex)
    ctx = ctx_with(pa, x)
    ctx.eval(w0, mu, th, need_h=True)   # y, ψ: Y(w0) in slot 1 (the second y buffer)
    ctx.eval(w1, mu, th, need_h=True)   # Y(w1) in slot 0 (inside the tiled pass's buffer)
    ctx.eval(w2, mu, ex, need_h=True)   # y, ψ, ψ′: that buffer grows; Y(w2) replaces Y(w0) in slot 1
    got1 = ctx.eval_loss_multi(w1, z, alphas, mu, ex)   # slot 0 is gone: forms Y
    got2 = ctx.eval_loss_multi(w2, z, alphas, mu, ex)   # reads slot 1 back
    assert ctx.multi_ybuf_passes == 1
    for a, b in ((got1, ref1), (got2, ref2)):
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_release_caches_drops_y_fragments(pa, rng, monkeypatch):
    """pc_ctx_release_caches frees the second y buffer and invalidates both slots: a multi-try
    pass at a W whose Y was kept forms it again, with the bits of a context that never kept it
    (both without the digit image, which release_caches frees for good)."""
    monkeypatch.delenv("PICARD_MULTI_YBUF", raising=False)
    nc = nf = 128
    x = laplace_mix(rng, nf, 3001)
    ws = [rng.normal(size=(nc, nf)) / np.sqrt(nf) for _ in range(2)]
    z = rng.normal(size=(nc, nf)) / np.sqrt(nf)
    mu = x.mean(axis=1)
    d = pa.DensityType(1, 0.5)
    alphas = 0.5 ** np.arange(0, 10)
    fresh = ctx_with(pa, x)
    fresh.release_caches()
    ref = [fresh.eval_loss_multi(w, z, alphas, mu, d) for w in ws]
    ctx = ctx_with(pa, x)
    for w in ws:
        ctx.eval(w, mu, d, need_h=True)
    ctx.release_caches()
    got = [ctx.eval_loss_multi(w, z, alphas, mu, d) for w in ws]
    assert ctx.multi_ybuf_passes == 0
    for a, b in zip(got, ref):
        assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


@pytest.mark.parametrize("n", [100, 256])
def test_nonortho_fit_multi_ybuf_bit_identical(pa, rng, monkeypatch, n):
    """A non-ortho fit (C4's path: tiled full pass + one multi-try pass per search) lands on
    the same unmixing, bit for bit, with Y read back and with Y formed in every pass."""
    x = laplace_mix(rng, n, 20000)
    cfg = dict(ortho=False, extended=False, m=7, max_iter=30, random_state=2)

    def fit():
        ctx = ctx_with(pa, x)
        sv = pa.Solver(ctx, pa.PicardConfig(**cfg))
        while not sv.step():
            pass
        r = sv.finish()
        sv.close()
        return r, ctx.multi_ybuf_passes

    monkeypatch.delenv("PICARD_MULTI_YBUF", raising=False)
    r1, n1 = fit()
    monkeypatch.setenv("PICARD_MULTI_YBUF", "0")
    r0, n0 = fit()
    assert n1 > 0 and n0 == 0
    assert r1.n_iterations == r0.n_iterations and r1.converged == r0.converged
    assert np.array_equal(r1.unmixing, r0.unmixing)
