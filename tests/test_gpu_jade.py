"""BASELINE config 5 (64 sources, jade_it = 50 warm start) under the GPU suite.

JADE (src/jade.rs:22-197) is three stages; each is checked at N = 64:
  * the fourth-moment pass (pc_ctx_moments4, MFMA) against numpy z·zᵀ of the
    pair products z = (y_i y_j)_{i≤j}, relative 1e-12 (summation order only);
  * the Jacobi sweeps — host (rotated cumulant matrices VᵀMV updated per Givens
    pair, O(n) per matrix) and device (one launch) — against the
    oracle's literal form (oracle.picard_oracle.jade_sweeps_batched: every
    b = v_pᵀ M v_q recomputed from V per pair, jade.rs:137-167, vectorised over
    the 2080 matrices, same cyclic pair order). The sweeps amplify rounding
    (chaotic over tens of sweeps), so the bounds are per
    sweep count and stated in the tests;
  * the full-size C5 run (64 × 1e7, jade_it = 50): the reference's own property
    (the warm start is orthogonal, jade.rs:245-255) and Picard converging after it.
"""
import numpy as np
import pytest

from conftest import rel_err

pytestmark = pytest.mark.gpu

N, T = 64, 20011


@pytest.fixture(scope="module")
def c5_small(pa, po):
    ctx = pa.DeviceContext(0)
    ctx.generate(N, T, 42)
    x = ctx.download()
    mu = x.mean(axis=1)
    x1, k = po.whiten(x - mu[:, None], N)
    pairs = [(i, j) for i in range(N) for j in range(i, N)]
    z = np.stack([x1[i] * x1[j] for i, j in pairs])
    m4 = z @ z.T
    mats = po.cumulants_from_moments(m4, N, float(T))
    return ctx, k, mu, m4, mats


def test_moments4_n64_vs_numpy(c5_small):
    ctx, k, mu, m4, _ = c5_small
    assert rel_err(ctx.moments4(k, mu), m4) <= 1e-12


# The sweeps amplify rounding exponentially: on this data a 1e-15 relative
# perturbation of the cumulant matrices moves V by 1.5e-14 / 9e-14 / 4e-12 /
# 1.3e-9 / 2e-4 after 63 / 200 / 500 / 1000 / 2016 Givens pairs (measured with
# the oracle). Parity is therefore checked on the first PREFIX = 500 pairs of
# the first sweep (rows p = 0 … 8 of the cyclic order), bound 1e-10 (25× the
# perturbation spread), through the PICARD_JADE_MAX_PAIRS hook.
PREFIX = 500


@pytest.mark.parametrize("where", ["host", "device"])
def test_jade_sweep_prefix_n64_vs_reference_order(po, c5_small, monkeypatch, where):
    ctx, k, mu, _, mats = c5_small
    monkeypatch.setenv("PICARD_JADE_MAX_PAIRS", str(PREFIX))
    w, sweeps, _, on_dev = ctx.jade(k, mu, max_iter=1, where=where)
    assert sweeps == 1 and on_dev == (where == "device")
    v, _, _ = po.jade_sweeps_batched(mats, 1, max_pairs=PREFIX)
    assert np.max(np.abs(w - po.sym_decorrelation(v))) <= 1e-10


@pytest.mark.parametrize("pairs", [PREFIX, 2016 + PREFIX])
def test_jade_device_sweeps_match_host_n64(c5_small, monkeypatch, pairs):
    """Device against host sweeps: a prefix of sweep 1 (1e-10) and, across the sweep
    boundary, a prefix of sweep 2 — where the chaos leaves only the reference's
    property (V orthogonal, both runs the same number of sweeps)."""
    ctx, k, mu, _, _ = c5_small
    monkeypatch.setenv("PICARD_JADE_MAX_PAIRS", str(pairs))
    wh, sh, _, dh = ctx.jade(k, mu, max_iter=3, where="host")
    wd, sd, _, dd = ctx.jade(k, mu, max_iter=3, where="device")
    assert sh == sd == pairs // 2016 + 1 and not dh and dd
    if pairs < 2016:
        assert np.max(np.abs(wd - wh)) <= 1e-10
    for w in (wh, wd):
        assert np.max(np.abs(w @ w.T - np.eye(N))) <= 1e-12


def test_jade_sequence_base_independent(c5_small, monkeypatch):
    """The device sweeps' granule sequence numbers started just below 2^32 (they are
    64-bit; PICARD_JADE_BAR_BASE presets the base): the sweeps must be unchanged
    (bit-identical) — the tags only gate, never feed, the arithmetic."""
    ctx, k, mu, _, _ = c5_small
    w0 = ctx.jade(k, mu, max_iter=2, where="device")[0]
    monkeypatch.setenv("PICARD_JADE_BAR_BASE", str(2 ** 32 - 5000))
    w1 = ctx.jade(k, mu, max_iter=2, where="device")[0]
    assert np.array_equal(w0, w1)


def test_jade_refused_launch_leaks_nothing(pa, c5_small, c1_data, monkeypatch):
    """The device sweeps' buffers are the context's (one ensure()d allocation, reused), so a
    refused launch (PICARD_TEST_JADE_REFUSE, a test hook) leaks nothing: where='device' then
    raises Unsupported — not an abort — and HBM free memory is the same after 1 and 10 such
    calls; a fit (device sweeps by default) falls back to the host sweeps, bit-identical to a
    fit that asked for them (PICARD_HOST_JADE)."""
    ctx, k, mu, _, _ = c5_small
    monkeypatch.setenv("PICARD_JADE_MAX_PAIRS", str(PREFIX))
    wh = ctx.jade(k, mu, max_iter=1, where="host")[0]
    monkeypatch.setenv("PICARD_TEST_JADE_REFUSE", "1")
    free = []
    for _ in range(10):
        with pytest.raises(pa.Unsupported):
            ctx.jade(k, mu, max_iter=1, where="device")
        free.append(pa.device_mem_info(0)[0])
    assert free[-1] == free[0], free
    w, _, _, on_dev = ctx.jade(k, mu, max_iter=1)
    assert not on_dev and np.array_equal(w, wh)
    x = c1_data[0]
    cfg = pa.PicardConfig(jade_it=5, max_iter=3, w_init=np.eye(x.shape[0]))
    refused = pa.Picard.fit_with_config(x, cfg)
    monkeypatch.delenv("PICARD_TEST_JADE_REFUSE")
    monkeypatch.setenv("PICARD_HOST_JADE", "1")
    host = pa.Picard.fit_with_config(x, cfg)
    assert np.array_equal(refused.unmixing, host.unmixing)


@pytest.mark.parametrize("stall_wg", [0, 5])
def test_jade_stalled_grid_aborts_and_falls_back(pa, c5_small, monkeypatch, stall_wg):
    """The device sweeps' bounded wait: a workgroup that never publishes a pair's
    partial sums (PICARD_TEST_JADE_STALL, with a low poll cap PICARD_TEST_JADE_POLL_CAP) must end
    the whole grid with the abort flag — every wave reaches it, the launch returns — and the
    context then runs the host sweeps: where='device' raises Unsupported, a default call gives
    the host sweeps' V bit for bit, and the device sweeps work again once the hook is cleared."""
    import time
    ctx, k, mu, _, _ = c5_small
    monkeypatch.setenv("PICARD_JADE_MAX_PAIRS", str(PREFIX))
    wh = ctx.jade(k, mu, max_iter=1, where="host")[0]
    wd = ctx.jade(k, mu, max_iter=1, where="device")[0]
    monkeypatch.setenv("PICARD_TEST_JADE_POLL_CAP", "20000")
    monkeypatch.setenv("PICARD_TEST_JADE_STALL", str(stall_wg))
    t0 = time.perf_counter()
    with pytest.raises(pa.Unsupported):
        ctx.jade(k, mu, max_iter=1, where="device")
    w, _, _, on_dev = ctx.jade(k, mu, max_iter=1)
    assert time.perf_counter() - t0 < 30.0
    assert not on_dev and np.array_equal(w, wh)
    monkeypatch.delenv("PICARD_TEST_JADE_STALL")
    monkeypatch.delenv("PICARD_TEST_JADE_POLL_CAP")
    w2, _, _, on_dev2 = ctx.jade(k, mu, max_iter=1, where="device")
    assert on_dev2 and np.array_equal(w2, wd)


@pytest.mark.parametrize("host", [False, True])
def test_jade_verbose_lines(pa, c1_data, capfd, monkeypatch, host):
    """jade.rs:57-66: the 'JADE iteration N: max angle' line every 10 sweeps, from the
    device sweeps (default) and the host sweeps (PICARD_HOST_JADE)."""
    x, s, a = c1_data
    monkeypatch.setenv("PICARD_TRACE", "1")
    if host:
        monkeypatch.setenv("PICARD_HOST_JADE", "1")
    pa.Picard.fit_with_config(x, pa.PicardConfig(jade_it=20, max_iter=1, w_init=np.eye(8), verbose=True))
    cap = capfd.readouterr()
    assert "JADE iteration 10: max angle = " in cap.out and "JADE iteration 20: max angle = " in cap.out
    assert ("host sweeps" if host else "device sweeps") in cap.err


@pytest.mark.timeout(300)
def test_c5_fullsize_warm_start_and_fit(pa):
    """C5 at full size: 64 × 1e7, jade_it = 50 (jade.rs runs all 50 sweeps on this data)."""
    n, t = 64, 10 ** 7
    ctx = pa.DeviceContext(0)
    ctx.generate(n, t, 42)
    # the warm start on its own, on the whitened data (as solver.rs:124-128 does)
    mu = ctx.rowsum() / t
    c = ctx.gram(mu) / t
    ev, u = np.linalg.eigh(c)
    k = (u / np.sqrt(ev)).T
    w0, sweeps, conv, _ = ctx.jade(k, mu, max_iter=50)
    assert sweeps == 50 or conv
    assert np.max(np.abs(w0 @ w0.T - np.eye(n))) <= 1e-10
    # the whole C5 fit
    sv = pa.Solver(ctx, pa.PicardConfig(jade_it=50, random_state=0, want_sources=False))
    while not sv.step():
        pass
    r = sv.finish()
    assert r.converged and r.gradient_norm < 1e-7
    wt = r.unmixing
    assert np.max(np.abs(wt @ wt.T - np.eye(n))) <= 1e-8  # Picard-O keeps W orthogonal
