"""The non-orthogonal line search's tries with fp32 row terms and a rigorous bound
(k_multi_loss2_oz<…, F32>, DeviceCtx::eval_loss_multi_bound).

A non-extended fit's loss needs no Σy², so its multi-try pass may return, per try and row,
an fp32 estimate of Σℓ and a bound on its distance to the exact pass at W + α_j·Z; the
solver then rejects a try only when its lower bound cannot beat the current loss and takes
every acceptance on the exact loss of a full pass (core.rs:127-140 on exact values). Checked
here: the bound covers the exact loss-only pass at every try, over W of very different
scales, at the register-resident (nc ≤ 128) and the tiled (nc = 256) shapes; it is tight
(≤ 1e-5 of Σℓ); and a C4-shape fit takes the same decisions with it (opt-in,
PICARD_MULTI_F32=1: the solver then uses it until its first wasted full pass) as
with the exact multi-try pass (the default, PICARD_MULTI_F32=0): same iterations, bit-identical
unmixing."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _laplace_mix(rng, nf, t):
    s = rng.laplace(size=(nf, t))
    a = rng.uniform(-0.5, 0.5, size=(nf, nf)) + np.eye(nf)
    return a @ s + rng.normal(size=(nf, 1))


@pytest.mark.parametrize("nc,nf", [(256, 256), (100, 128), (60, 64)])
def test_multi_bound_covers_exact_tries(pa, nc, nf, monkeypatch):
    monkeypatch.setenv("PICARD_MULTI_F32", "1")
    rng = np.random.default_rng(nc)
    x = _laplace_mix(rng, nf, 12011)
    x[:, 9] *= 1e3  # one loud sample
    ctx = pa.DeviceContext(0)
    ctx.load(x)
    mu = x.mean(axis=1)
    d = pa.DensityType.tanh()
    al = np.array([0.5 ** j for j in range(9)])
    for scale in (1e-3, 1.0, 30.0):
        w = scale * rng.normal(size=(nc, nf)) / np.sqrt(nf)
        z = 0.3 * scale * rng.normal(size=(nc, nf)) / np.sqrt(nf)
        ll, bnd = ctx.eval_loss_multi_bound(w, z, al, mu, d)
        assert np.all(bnd > 0)
        for j in (0, 3, 8):
            lo, _, _ = ctx.eval_split(w + al[j] * z, mu, d, False, need_y2=False)
            err = np.abs(lo["ll"] - ll[j])
            assert np.all(err <= bnd[j]), (scale, j, np.max(err / bnd[j]))
            assert np.max(bnd[j] / np.abs(lo["ll"])) <= 1e-5, (scale, j, np.max(bnd[j] / np.abs(lo["ll"])))


def test_multi_bound_unavailable(pa, monkeypatch):
    monkeypatch.setenv("PICARD_MULTI_F32", "1")
    rng = np.random.default_rng(1)
    x = _laplace_mix(rng, 100, 3001)
    ctx = pa.DeviceContext(0)
    ctx.load(x)
    w = rng.normal(size=(100, 100)) / 10
    with pytest.raises(pa.ComputationError):  # exp: only tanh's ℓ has the fp32 form
        ctx.eval_loss_multi_bound(w, w, [1.0, 0.5], x.mean(axis=1), pa.DensityType.exp())


@pytest.mark.parametrize("n", [256, 96])
def test_bounded_multi_fit_matches_exact(pa, dg, n, monkeypatch):
    x, _, _ = dg.generate_data(n, 20011, 42)
    kw = dict(ortho=False, extended=False, m=7, max_iter=12)
    res = {}
    for mode in ("bound", "exact"):
        monkeypatch.setenv("PICARD_MULTI_F32", "1" if mode == "bound" else "0")
        ctx = pa.DeviceContext(0)
        ctx.load(x)
        sv = pa.Solver(ctx, pa.PicardConfig(w_init=np.eye(n), **kw))
        while not sv.step():
            pass
        res[mode] = sv.finish()
        sv.close()
        ctx.close()
    rb, re = res["bound"], res["exact"]
    assert rb.n_iterations == re.n_iterations
    assert np.array_equal(rb.unmixing, re.unmixing)
