"""The seeded random w_init stream (src/solver.rs:56-60, :112-118): rand 0.9.2
StdRng (ChaCha12Rng, seed_from_u64) + rand_distr 0.5.1 StandardNormal.

The crates are not under /root/reference and cannot be fetched, so
oracle/rust_rand.py restates their published algorithms. Pinned here:
  * the ChaCha block function against the RFC 8439 §2.3.2 known answer;
  * the ziggurat tables against the values the generated rand_distr source holds
    (first entries of ZIG_NORM_X / ZIG_NORM_F and ZIG_NORM_R as printed there);
  * the normal draws' moments.
The composition (seed expansion, word order, ziggurat branches) has no
reference-held vector offline: parity unpinned. The product's C++ stream
(host_rng.cpp) is checked against the restatement bit for bit through seeded fits
(pc_fit_with_evaluator with the oracle's pass statistics, CPU only).
"""
import struct

import numpy as np
import pytest

from oracle import rust_rand as rr
from test_host_driver import host_fit


def test_chacha20_rfc8439_block():
    key = list(struct.unpack("<8I", bytes(range(32))))
    out = rr.chacha_block(key, [1, 0x09000000, 0x4A000000, 0], 20)
    want = [0xE4E7F110, 0x15593BD1, 0x1FDD0F50, 0xC47120A3, 0xC7F4D1C7, 0x0368C033, 0x9AAA2204, 0x4E6CD4C3,
            0x466482D2, 0x09AA9F07, 0x05D7C214, 0xA2028BD9, 0xD19C12B5, 0xB94E16DE, 0xE883D0CB, 0x4E3C50A2]
    assert out == want


def test_ziggurat_table_literals():
    assert "%.18f" % rr.ZIG_NORM_R == "3.654152885361008796"
    assert ["%.18f" % v for v in rr.ZIG_NORM_X[:3]] == ["3.910757959537090045", "3.654152885361008796",
                                                       "3.449278298560964462"]
    assert ["%.18f" % v for v in rr.ZIG_NORM_F[:2]] == ["0.000477467764586655", "0.001260285930498598"]
    assert rr.ZIG_NORM_X[256] == 0.0 and rr.ZIG_NORM_F[256] == 1.0


def test_product_table_literals_pin_every_entry():
    """host_rng.cpp takes the tables from zig_tables.inc (hex-float literals, no libm at
    run time): every one of the 1 + 257 + 257 entries equals the restatement's recipe."""
    import os
    import re
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "picard-ica_amd", "csrc", "zig_tables.inc")).read()
    def arr(name):
        body = re.search(name + r"\[257\] = \{(.*?)\};", src, re.S).group(1)
        return [float.fromhex(v) for v in re.findall(r"-?0x[0-9a-fp.+-]+", body)]
    r = float.fromhex(re.search(r"ZIG_R = (0x[0-9a-fp.+-]+);", src).group(1))
    assert r == rr.ZIG_NORM_R
    assert arr("ZIG_X") == list(rr.ZIG_NORM_X) and arr("ZIG_F") == list(rr.ZIG_NORM_F)


def test_standard_normal_moments():
    g = rr.StdRng(42)
    xs = np.array([rr.standard_normal(g) for _ in range(50000)])
    assert abs(xs.mean()) < 0.02 and abs(xs.var() - 1.0) < 0.03
    assert np.mean(np.abs(xs) > 3.0) == pytest.approx(0.0027, abs=0.0015)  # the tail branch runs


@pytest.mark.parametrize("seed", [0, 7, 42, 2 ** 63 + 5])
def test_seeded_w_init_matches_restatement(pa, po, c1_data, seed):
    """Orthogonal fits from the seeded random w_init: the C++ driver and the oracle
    (w_init from oracle/rust_rand.py) follow the same trajectory, which they only can
    from the same draws (W differs O(1) otherwise)."""
    x, s, a = c1_data
    r = host_fit(pa, po, x, pa.PicardConfig(random_state=seed, max_iter=5))
    ro = po.fit_with_config(x, po.PicardConfig(random_state=seed, max_iter=5))
    assert r.n_iterations == ro.n_iterations
    # rounding only (host vs numpy eigh in sym_decorrelation, five iterations); a
    # different draw would move W by O(1)
    assert np.max(np.abs(r.unmixing - ro.unmixing)) < 1e-8
