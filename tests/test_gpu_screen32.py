"""The tanh line-search screen with its log-likelihood in fp32 (loss_acc4_f32).

The screen's bound (DeviceCtx::screen_f32_block_bound) rests on three hardware
constants: the relative error of v_exp_f32 on [−126, 0], its absolute error below,
and the absolute error of v_log_f32 on [2^-4, 1]. They are checked here
exhaustively — every fp32 input of those ranges against fp64 libm, on this device —
so the bound is rigorous on the hardware the tests run on. Then: the bound covers
the exact pass on hard inputs, it stays small (≤ 1e-4 of Σℓ on the default D ≤ 3
digit diagonals, 1e-5 on D ≤ 4; whether it decides is measured on C3), and the fp64-ℓ screen (PICARD_SCREEN_F64=1) agrees within
both bounds. Both screen depths (PICARD_SCREEN_DMAX = 3, 4) are covered."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# DeviceCtx::SCREEN_EXP2_REL, SCREEN_EXP2_TINY, SCREEN_LOG2_ABS
EXP2_REL, EXP2_TINY, LOG2_ABS = 2.0 ** -23, 2.0 ** -124, 2.0 ** -21


def test_fp32_transcendental_constants_hold(pa):
    import ctypes as C
    out = (C.c_double * 4)()
    assert pa.lib.pc_device_check_fp32_transcendentals(0, out) == 0
    rel, tiny, lg, exact = list(out)
    print(f"v_exp_f32 rel {rel / 2 ** -24:.3f} x 2^-24, tiny abs {tiny:.3e}, v_log_f32 abs {lg / 2 ** -24:.3f} x 2^-24")
    assert rel <= EXP2_REL and tiny <= EXP2_TINY and lg <= LOG2_ABS
    assert exact == 1.0  # 2^0 = 1 and log2 1 = 0: padded samples contribute exactly 0


def _laplace_mix(rng, n, t):
    s = rng.laplace(size=(n, t))
    a = rng.uniform(-0.5, 0.5, size=(n, n))
    return a @ s


@pytest.mark.parametrize("n", [72, 128])
@pytest.mark.parametrize("alpha", [1.0, 0.5, 2.0])
@pytest.mark.parametrize("dmax", ["3", "4"])
def test_f32_screen_bound_covers_exact(pa, n, alpha, dmax, monkeypatch):
    monkeypatch.setenv("PICARD_SCREEN_DMAX", dmax)
    rng = np.random.default_rng(n)
    x = _laplace_mix(rng, n, 30011)
    x[:, 7] *= 1e4  # one loud sample
    x[:, 11] = 0.0  # one silent sample
    mu = x.mean(axis=1)
    xc = x - mu[:, None]
    k = np.linalg.cholesky(np.linalg.inv(xc @ xc.T / x.shape[1])).T
    d = pa.DensityType.tanh(alpha)
    monkeypatch.setenv("PICARD_SCREEN_F64", "1")
    c64 = pa.DeviceContext(0)
    c64.load(x)
    monkeypatch.delenv("PICARD_SCREEN_F64")
    c32 = pa.DeviceContext(0)
    c32.load(x)
    for scale in (1e-4, 0.3, 1.0, 10.0, 300.0):
        w = scale * (np.linalg.qr(rng.normal(size=(n, n)))[0] @ k)
        ll32, b32 = c32.eval_loss_screen(w, mu, d)
        ll64, b64 = c64.eval_loss_screen(w, mu, d)
        lo, _, _ = c32.eval_split(w, mu, d, False, need_y2=False)
        exact = lo["ll"]
        assert np.all(np.abs(exact - ll32) <= b32), (scale, np.max(np.abs(exact - ll32) / b32))
        assert np.all(np.abs(exact - ll64) <= b64)
        assert np.all(b32 >= b64)  # the fp32 bound adds to the digit tail
        tight = 1e-4 if dmax == "3" else 1e-5  # the dropped digit diagonals dominate the bound
        assert np.max(b32 / np.abs(exact)) <= tight, (scale, np.max(b32 / np.abs(exact)))


@pytest.mark.parametrize("tiny", [1e-35, 1e-25])
def test_f32_screen_scale_range(pa, tiny, monkeypatch):
    """The fp32 screen forms |ỹ| = |Y'|·2^(f_i+e_t−20) in fp32, which needs every scale in the
    normal fp32 range (DeviceCtx::screen_at checks the digit image's exponent range): a sample
    of size 1e-35 takes the rank to the fp64-ℓ screen, one of 1e-25 keeps the fp32 screen; the
    bound covers the exact pass either way."""
    monkeypatch.setenv("PICARD_SCREEN_DMAX", "3")  # the D ≤ 3 bound's tightness is asserted
    rng = np.random.default_rng(5)
    n = 96
    x = _laplace_mix(rng, n, 20011)
    x[:, 3] *= tiny
    mu = x.mean(axis=1)
    xc = x - mu[:, None]
    k = np.linalg.cholesky(np.linalg.inv(xc @ xc.T / x.shape[1])).T
    d = pa.DensityType.tanh()
    ctx = pa.DeviceContext(0)
    ctx.load(x)
    for scale in (0.1, 1.0, 30.0):
        w = scale * (np.linalg.qr(rng.normal(size=(n, n)))[0] @ k)
        ll, b = ctx.eval_loss_screen(w, mu, d)
        lo, _, _ = ctx.eval_split(w, mu, d, False, need_y2=False)
        assert np.all(np.abs(lo["ll"] - ll) <= b), (scale, np.max(np.abs(lo["ll"] - ll) / b))
        assert np.max(b / np.abs(lo["ll"])) <= 1e-4
