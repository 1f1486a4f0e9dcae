"""CPU ORACLE — test infrastructure only (see oracle/picard_oracle.py header).

Restates the reference's synthetic-mixture generator, benches/benchmarks.rs:8-35:
a 64-bit LCG ``state = state·6364136223846793005 + 1`` consumed in row-major
(feature i, sample j) order, ``u = (state >> 33) / 2^31``, Laplace sources by
inverse CDF (benchmarks.rs:17-21), then the mixing matrix A_ij = u − 0.5 from
the following states (benchmarks.rs:26-32), and X = A·S (benchmarks.rs:34).

One documented deviation (DESIGN.md §Synthetic inputs): u == 0 happens when
state < 2^33 (p = 2^-31 per draw) and the reference then yields ln(0) = −inf.
At the 1.28e10 draws of N=128 × T=1e8 that is expected ≈6 times and would
turn every statistic into NaN, so ``guard_zero=True`` (the default, and what
the HIP generator does) substitutes u = 2^-32. ``guard_zero=False`` restates
the reference exactly. All other values are bit-identical to the reference.
"""
from __future__ import annotations

import numpy as np

LCG_A = np.uint64(6364136223846793005)
LCG_C = np.uint64(1)
MASK = (1 << 64) - 1


def lcg_jump(n: int):
    """Affine map (A_n, C_n) with state_{k+n} = A_n·state_k + C_n (mod 2^64)."""
    a, c = 6364136223846793005, 1
    ra, rc = 1, 0
    while n:
        if n & 1:
            ra, rc = (ra * a) & MASK, (rc * a + c) & MASK
        a, c = (a * a) & MASK, (c * a + c) & MASK
        n >>= 1
    return ra, rc


def lcg_states(seed: int, start: int, count: int) -> np.ndarray:
    """States number start+1 … start+count after ``seed`` (state_0 = seed)."""
    block = 4096
    nblk = (count + block - 1) // block
    # per-offset affine maps inside a block
    aj = np.empty(block, dtype=np.uint64)
    cj = np.empty(block, dtype=np.uint64)
    a, c = 1, 0
    for j in range(block):
        a, c = (a * 6364136223846793005) & MASK, (c * 6364136223846793005 + 1) & MASK
        aj[j], cj[j] = a, c
    ja, jc = lcg_jump(start)
    s = (ja * seed + jc) & MASK
    ba, bc = lcg_jump(block)
    starts = np.empty(nblk, dtype=np.uint64)
    for b in range(nblk):
        starts[b] = s
        s = (ba * s + bc) & MASK
    with np.errstate(over="ignore"):
        st = starts[:, None] * aj[None, :] + cj[None, :]
    return st.reshape(-1)[:count]


def uniform_from_state(st: np.ndarray) -> np.ndarray:
    """benchmarks.rs:16: u = (state >> 33) as f64 / (1u64 << 31) as f64."""
    return (st >> np.uint64(33)).astype(np.float64) / float(1 << 31)


def laplace_from_uniform(u: np.ndarray, guard_zero: bool = True) -> np.ndarray:
    """benchmarks.rs:17-21."""
    if guard_zero:
        u = np.where(u == 0.0, 2.0 ** -32, u)
    with np.errstate(divide="ignore"):
        return np.where(u < 0.5, np.log(2.0 * u), -np.log(2.0 * (1.0 - u)))


def generate_sources_and_mixing(n_features: int, n_samples: int, seed: int = 42,
                                guard_zero: bool = True):
    """Returns (S, A) exactly as benchmarks.rs:8-32 draws them."""
    st = lcg_states(seed, 0, n_features * n_samples + n_features * n_features)
    u = uniform_from_state(st)
    s = laplace_from_uniform(u[: n_features * n_samples], guard_zero).reshape(n_features, n_samples)
    a = (u[n_features * n_samples:] - 0.5).reshape(n_features, n_features)
    return s, a


def generate_data(n_features: int, n_samples: int, seed: int = 42, guard_zero: bool = True):
    """benchmarks.rs:8-35 → X = A·S (plus S and A for Amari checks)."""
    s, a = generate_sources_and_mixing(n_features, n_samples, seed, guard_zero)
    return a @ s, s, a
