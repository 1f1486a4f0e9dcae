"""The host team size (PICARD_HOST_THREADS) must not change a fit: the host N×N work —
blocked products whose tiles are summed independently of the thread that owns them, the
Taylor series' max reduction (exact in any order), the digit split per row — gives the same
bits for any team. Checked at N = 128 (where the products are threaded) through
pc_fit_with_evaluator with the oracle's pass statistics, one subprocess per team size
(the cap is read once per process)."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import picard_ica_amd as pa
from oracle import datagen as dg, picard_oracle as po

x, _, _ = dg.generate_data(128, 3000, 5)

def ev(w, mu, d, need_h):
    return po.pass_stats(w, mu, x, po.Density(["tanh", "exp", "cube"][d.kind], d.alpha), need_h)

def gram(mu):
    xc = x - mu[:, None] if mu is not None else x
    return xc @ xc.T

r = pa.fit_with_host_evaluator(128, 3000, pa.PicardConfig(random_state=3, max_iter=8), rowsum=lambda: x.sum(axis=1),
                               gram=gram, eval=ev, sources=lambda w, mu: w @ (x - mu[:, None]))
np.save(sys.argv[2], np.concatenate([r.unmixing.ravel(), r.whitening.ravel(), [r.n_iterations]]))
"""


def _fit(tmp_path, threads):
    out = tmp_path / f"w{threads}.npy"
    env = dict(os.environ, PICARD_HOST_THREADS=str(threads), OMP_NUM_THREADS="8")
    subprocess.run([sys.executable, "-c", SCRIPT, ROOT, str(out)], env=env, check=True, timeout=600)
    return np.load(out)


def test_fit_bits_independent_of_host_team(tmp_path):
    a = _fit(tmp_path, 1)
    b = _fit(tmp_path, 8)
    assert a[-1] >= 2  # iterations ran (line searches, Taylor series)
    assert np.array_equal(a, b)


def test_solver_leaves_the_callers_openmp_team(pa, po, c1_data):
    """The solver runs its host work on its own team size (PICARD_HOST_THREADS cap) and gives the
    calling thread back its OpenMP setting: a library call must not change the caller's team."""
    import ctypes

    gomp = ctypes.CDLL("libgomp.so.1")  # the runtime the library links (one per process)
    x, _, _ = c1_data

    def ev(w, mu, d, need_h):
        return po.pass_stats(w, mu, x, po.Density(["tanh", "exp", "cube"][d.kind], d.alpha), need_h)

    gomp.omp_set_num_threads(3)
    r = pa.fit_with_host_evaluator(8, x.shape[1], pa.PicardConfig(w_init=np.eye(8), max_iter=20),
                                   rowsum=lambda: x.sum(axis=1), gram=lambda mu: (x - mu[:, None]) @ (x - mu[:, None]).T,
                                   eval=ev, sources=lambda w, mu: w @ (x - mu[:, None]))
    assert r.n_iterations > 1
    assert gomp.omp_get_max_threads() == 3
