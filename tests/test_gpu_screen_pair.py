"""The paired line-search screen (pc_ctx_eval_loss_screen2, k_screen_oz2<NB, ·, 2>): two tries'
screens in one pass over the digit image. Each try's rows must be exactly those of its own
screen (the same kernel arithmetic per W and the same bound terms), so the solver's decisions —
which take a paired try's rows in place of its single screen — cannot change: a fit with pairs
(default) and one without (PICARD_SCREEN_PAIRS=0) are bit-identical."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture
def rng():
    return np.random.default_rng(11)


@pytest.mark.parametrize("n,t", [(48, 20011), (64, 100003), (96, 20011), (128, 100003), (128, 16 * 512 * 7 + 5)])
def test_screen_pair_equals_single_screens(pa, rng, n, t):
    ctx = pa.DeviceContext(0)
    ctx.generate(n, t, 7)
    mu = ctx.rowsum() / t
    d = pa.DensityType.tanh()
    q = np.linalg.qr(rng.normal(size=(n, n)))[0]
    w1 = 0.8 * q
    w2 = 0.8 * np.linalg.qr(rng.normal(size=(n, n)))[0] @ q
    s1 = ctx.eval_loss_screen(w1, mu, d)
    s2 = ctx.eval_loss_screen(w2, mu, d)
    p1, p2 = ctx.eval_loss_screen2(w1, w2, mu, d)
    for single, paired in ((s1, p1), (s2, p2)):
        assert np.array_equal(single[0], paired[0]) and np.array_equal(single[1], paired[1])
    ctx.close()


def test_screen_pair_unsupported_density(pa):
    ctx = pa.DeviceContext(0)
    ctx.generate(64, 20011, 3)
    w = np.eye(64)
    with pytest.raises(pa.Unsupported):
        ctx.eval_loss_screen2(w, w, None, pa.DensityType.exp())
    ctx.close()


@pytest.mark.parametrize("n,seed", [(128, 42), (64, 7)])
def test_paired_fit_bit_identical(pa, n, seed, capfd, monkeypatch):
    """Picard-O on the bench mixture with paired screens (default) and without: identical
    iterations, bit-identical unmixing; the mixture has non-descent searches, so pairs ran."""
    monkeypatch.setenv("PICARD_TRACE", "1")
    res = {}
    for pairs in ("1", "0"):
        monkeypatch.setenv("PICARD_SCREEN_PAIRS", pairs)
        ctx = pa.DeviceContext(0)
        ctx.generate(n, 200003, seed)
        sv = pa.Solver(ctx, pa.PicardConfig(random_state=42, max_iter=60))
        while not sv.step():
            pass
        res[pairs] = sv.finish()
        sv.close()
        ctx.close()
        err = capfd.readouterr().err
        if pairs == "1":  # a try screened in a pair (its partner is used if the search gets there)
            assert "(pair)" in err
        else:
            assert "(pair)" not in err and "(paired)" not in err
    assert res["1"].n_iterations == res["0"].n_iterations and res["1"].converged == res["0"].converged
    assert np.array_equal(res["1"].unmixing, res["0"].unmixing)


@pytest.mark.parametrize("n,t,seed", [(128, 1000003, 42)])
def test_descent_paired_fit_bit_identical(pa, n, t, seed, capfd, monkeypatch):
    """Overshooting descent searches pair their screens (Solver::line_search: Picard's quadratic
    model and the previous try's margin decide, schedule only); with PICARD_DESCENT_PAIR=0 they
    run single screens. Identical iterations, bit-identical unmixing, and descent pairs ran."""
    monkeypatch.setenv("PICARD_TRACE", "1")
    res = {}
    for pairs in ("1", "0"):
        monkeypatch.setenv("PICARD_DESCENT_PAIR", pairs)
        ctx = pa.DeviceContext(0)
        ctx.generate(n, t, seed)
        sv = pa.Solver(ctx, pa.PicardConfig(random_state=42, max_iter=60))
        while not sv.step():
            pass
        res[pairs] = sv.finish()
        sv.close()
        ctx.close()
        err = capfd.readouterr().err
        print(pairs, err.count("(pair, descent)"))
        if pairs == "1":
            assert "(pair, descent)" in err
        else:
            assert "(pair, descent)" not in err
    assert res["1"].n_iterations == res["0"].n_iterations and res["1"].converged == res["0"].converged
    assert np.array_equal(res["1"].unmixing, res["0"].unmixing)
