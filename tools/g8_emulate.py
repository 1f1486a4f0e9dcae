"""numpy emulation of the digit G stage's arithmetic (picard-ica_amd/csrc/fused_g8.inc): ψ and y
rounded to one fixed-point scale per row and pass (ψ̌ = rne(ψ·2^(46−Fψ)), ỹ = rne(y·2^(46−F_j)),
F_j from Σ_k|W_jk| and the largest sample exponent), split into 6 signed radix-256 digits each,
and only the digit products of diagonals qa + qb ≥ 4 summed. Prints the relative error of
G = ψ·Yᵀ against the fp64 product for the test mixtures of tests/test_gpu_g8.py.
Usage: python tools/g8_emulate.py [T …]"""
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from oracle import picard_oracle as po  # noqa: E402


def digits(v, nd):
    """balanced radix-256 digits of the int64 array v, q = 0 least significant (the kernel's
    shifter: bytes of v + Σ 128·256^q, each XOR 0x80)"""
    u = v + sum(128 * 256 ** q for q in range(nd))
    return [((u >> (8 * q)) & 0xFF).astype(np.int64) - 128 for q in range(nd)]


def g_digits(psi, y, psc, ysc, nd=6, emin=4):
    pv = np.rint(psi * psc).astype(np.int64)
    yv = np.rint(y * ysc[:, None]).astype(np.int64)
    a, b = digits(pv, nd), digits(yv, nd)
    g = np.zeros((psi.shape[0], y.shape[0]))
    for qa in range(nd):
        for qb in range(nd):
            if qa + qb >= emin:
                g += float(256.0 ** (qa + qb)) * (a[qa].astype(np.float64) @ b[qb].T.astype(np.float64))
    return g / psc / ysc[None, :]


def laplace_mix(rng, nf, t):
    s = rng.laplace(size=(nf, t))
    a = rng.uniform(-0.5, 0.5, size=(nf, nf)) + np.eye(nf)
    return a @ s + rng.normal(size=(nf, 1))


def main():
    ts = [int(float(a)) for a in sys.argv[1:]] or [5003, 50_000, 500_000]
    rng = np.random.default_rng(8642)
    for t in ts:
        for n, dens in [(65, po.Density("exp", 1.0)), (100, po.Density("tanh", 1.0)), (128, po.Density("exp", 0.1)),
                        (128, po.Density("tanh", 0.7))]:
            x = laplace_mix(rng, n, t)
            w = rng.normal(size=(n, n)) / np.sqrt(n)
            y = w @ (x - x.mean(axis=1, keepdims=True))
            psi, _ = dens.score_and_der(y)
            g = psi @ y.T
            emax = int(np.frexp(np.max(np.abs(x - x.mean(axis=1, keepdims=True))))[1])  # max|x| < 2^emax
            f = np.array([np.frexp(s * (1 + 1e-12))[1] for s in np.abs(w).sum(axis=1)]) + emax
            bound = 1.0 if dens.kind == "tanh" else 1.0 / np.sqrt(dens.alpha * np.e)
            psc = 2.0 ** (46 - (0 if dens.kind == "tanh" else int(np.frexp(bound * (1 + 1e-12))[1])))
            gq = g_digits(psi, y, psc, 2.0 ** (46 - f))
            print(f"T={t} n={n} {dens.kind}({dens.alpha}): rel err {np.max(np.abs(gq - g)) / np.max(np.abs(g)):.2e}, "
                  f"bound slack {np.mean(f - np.log2(np.max(np.abs(y), axis=1))):.1f} bits", flush=True)


if __name__ == "__main__":
    main()
