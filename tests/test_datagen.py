"""The synthetic-mixture generator (benches/benchmarks.rs:8-35) restated in oracle/datagen.py."""
import numpy as np


def test_lcg_jump_matches_sequential(dg):
    st, seq = 42, []
    for _ in range(5000):
        st = (st * 6364136223846793005 + 1) & ((1 << 64) - 1)
        seq.append(st)
    assert [int(v) for v in dg.lcg_states(42, 0, 5000)] == seq
    assert [int(v) for v in dg.lcg_states(42, 777, 1000)] == seq[777:1777]


def test_generator_sequential_restatement(dg):
    """Bit-exact against a literal loop over benchmarks.rs:13-32."""
    nf, ns, seed = 3, 50, 7
    state = seed
    data = np.zeros((nf, ns))
    for i in range(nf):
        for j in range(ns):
            state = (state * 6364136223846793005 + 1) & ((1 << 64) - 1)
            u = (state >> 33) / float(1 << 31)
            data[i, j] = np.log(2 * u) if u < 0.5 else -np.log(2 * (1 - u))
    mix = np.zeros((nf, nf))
    for i in range(nf):
        for j in range(nf):
            state = (state * 6364136223846793005 + 1) & ((1 << 64) - 1)
            mix[i, j] = (state >> 33) / float(1 << 31) - 0.5
    s, a = dg.generate_sources_and_mixing(nf, ns, seed)
    assert np.array_equal(s, data) and np.array_equal(a, mix)


def test_zero_guard(dg):
    u = np.array([0.0, 0.25, 0.75])
    assert np.isneginf(dg.laplace_from_uniform(u, guard_zero=False)[0])
    g = dg.laplace_from_uniform(u, guard_zero=True)
    assert np.isfinite(g).all() and g[0] == np.log(2.0 ** -31)


def test_shards_are_slices(dg):
    """A shard [t0, t0+n) of sample columns uses LCG states i·T + t + 1 (what the HIP generator does)."""
    nf, T, t0, n = 4, 1000, 300, 200
    s, _ = dg.generate_sources_and_mixing(nf, T, 42)
    for i in range(nf):
        st = dg.lcg_states(42, i * T + t0, n)
        assert np.array_equal(dg.laplace_from_uniform(dg.uniform_from_state(st)), s[i, t0:t0 + n])
