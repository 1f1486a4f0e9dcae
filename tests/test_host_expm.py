"""The host matrix exponential of the orthogonal line search (host_linalg.cpp matrix_exp,
restating math.rs:38-74): Paterson–Stockmeyer evaluation where the reference's term-by-term
Taylor series converges within its 30 terms, the reference's own loop where it does not.

The routine is internal (no C-ABI symbol), so the test compiles host_linalg.cpp with a small
driver (g++, as the library build does) and checks it against the oracle's restatement of the
reference series and against scipy's expm for skew-symmetric directions of every size the
fits use, from 1e-6 to beyond the 30-term cap: never further from exp(A) than 1e-15 + twice the
reference series' own error (which grows with its squarings), orthogonal to the same bound, and
where the fast path is not taken bit-for-bit equal to a direct restatement of the 30-term loop in
the same C++ arithmetic.
"""
import os
import shutil
import subprocess
import tempfile

import numpy as np
import pytest
from scipy.linalg import expm

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "picard-ica_amd", "csrc")

DRIVER = r"""
#include "host_linalg.hpp"
#include <cmath>
#include <cstdio>
#include <vector>
using namespace pcamd;
// the 30-term loop of math.rs:38-74, term by term (the capped region's expected value)
static Mat series(const Mat& a) {
  const size_t n = a.rows;
  const double norm = max_abs(a);
  if (norm < 1e-15) return Mat::eye(n);
  const int s = (int)std::fmax(std::ceil(std::log2(norm)), 0.0);
  Mat as = a;
  for (double& v : as.a) v /= std::ldexp(1.0, s);
  Mat r = Mat::eye(n), t = Mat::eye(n);
  for (int k = 1; k <= 30; ++k) {
    t = matmul(t, as);
    double m = 0.0;
    for (double& v : t.a) { v /= (double)k; m = std::fabs(v) > m ? std::fabs(v) : m; }
    for (size_t i = 0; i < r.a.size(); ++i) r.a[i] += t.a[i];
    if (m < 1e-16) break;
  }
  for (int i = 0; i < s; ++i) r = matmul(r, r);
  return r;
}
int main(int argc, char** argv) {
  FILE* f = std::fopen(argv[1], "rb");
  FILE* g = std::fopen(argv[2], "wb");
  unsigned long long n;
  while (std::fread(&n, sizeof n, 1, f) == 1) {
    Mat a(n, n);
    if (std::fread(a.data(), sizeof(double), n * n, f) != n * n) return 1;
    const Mat e = matrix_exp(a), r = series(a);
    std::fwrite(e.data(), sizeof(double), n * n, g);
    std::fwrite(r.data(), sizeof(double), n * n, g);
  }
  std::fclose(g);
  return 0;
}
"""


@pytest.fixture(scope="module")
def run_expm():
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    tmp = tempfile.mkdtemp(prefix="pc_expm_")
    src = os.path.join(tmp, "drv.cpp")
    exe = os.path.join(tmp, "drv")
    with open(src, "w") as fh:
        fh.write(DRIVER)
    subprocess.run([gxx, "-O3", "-std=c++17", "-fopenmp", "-I", CSRC, src, os.path.join(CSRC, "host_linalg.cpp"),
                    "-o", exe], check=True)

    def run(mats):
        fin, fout = os.path.join(tmp, "in.bin"), os.path.join(tmp, "out.bin")
        with open(fin, "wb") as fh:
            for a in mats:
                fh.write(np.uint64(a.shape[0]).tobytes())
                fh.write(np.ascontiguousarray(a, dtype=np.float64).tobytes())
        subprocess.run([exe, fin, fout], check=True, env=dict(os.environ, OMP_NUM_THREADS="4"))
        out = np.fromfile(fout, dtype=np.float64)
        res, off = [], 0
        for a in mats:
            k = a.size
            res.append((out[off:off + k].reshape(a.shape), out[off + k:off + 2 * k].reshape(a.shape)))
            off += 2 * k
        return res

    yield run
    shutil.rmtree(tmp, ignore_errors=True)


def skew(rng, n, scale):
    a = rng.normal(size=(n, n)) * scale / np.sqrt(n)
    return a - a.T


@pytest.mark.parametrize("n", [2, 8, 64, 100, 128])
def test_expm_matches_series_and_scipy(po, run_expm, n):
    rng = np.random.default_rng(n)
    scales = [1e-6, 1e-3, 0.02, 0.2, 0.7, 2.0, 6.0]
    mats = [skew(rng, n, sc) for sc in scales]
    for a, (e, r) in zip(mats, run_expm(mats)):
        want = expm(a)
        ref = po.matrix_exp(a)
        err_ref = np.max(np.abs(ref - want))
        if not np.array_equal(e, r):
            # Paterson–Stockmeyer: exp(A) to rounding, never further off than the reference's
            # series (whose error grows with its squarings, ≈ 3e-14 at n = 8, |A| ≈ 6)
            tol = 1e-15 + 2.0 * err_ref
            assert np.max(np.abs(e - want)) <= tol, (np.max(np.abs(e - want)), err_ref)
            assert np.max(np.abs(e - ref)) <= tol + err_ref
            orth_ref = np.max(np.abs(ref @ ref.T - np.eye(n)))
            assert np.max(np.abs(e @ e.T - np.eye(n))) <= 2e-15 + 2.0 * orth_ref
        else:  # the series' own value (its 30-term cap, or no halving needed), bit for bit
            assert np.max(np.abs(e - ref)) < 1e-12 * max(1.0, np.max(np.abs(ref)))


def test_expm_general_and_edge(po, run_expm):
    rng = np.random.default_rng(5)
    mats = [np.zeros((4, 4)), np.full((3, 3), 1e-16), rng.normal(size=(16, 16)) * 0.05,
            rng.normal(size=(16, 16)) * 0.5, np.diag([0.3, -0.2, 1.5])]
    for a, (e, r) in zip(mats, run_expm(mats)):
        want = expm(a) if np.max(np.abs(a)) >= 1e-15 else np.eye(a.shape[0])
        assert np.max(np.abs(e - want)) <= 1e-14 * max(1.0, np.max(np.abs(want)))
