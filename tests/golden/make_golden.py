"""Regenerate the golden fixtures in tests/golden/ from the CPU oracle.

The reference (Rust) cannot be built in this image and ships no fixtures, so these
vectors come from oracle/picard_oracle.py, itself pinned by the reference's KATs
(tests/test_oracle_kats.py). They freeze the oracle's behaviour so the GPU path is
checked against committed data, and record the synthetic-input generator's output.
Run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import datagen, picard_oracle as po  # noqa: E402

GRID = np.array([-2.0, -1.0, -0.5, 0.0, 0.5, 1.0, 2.0])  # utils.rs:113


def main():
    out = {}
    for name, d in [("tanh1", po.Density("tanh", 1.0)), ("exp01", po.Density("exp", 0.1)),
                    ("cube", po.Density("cube", 1.0))]:
        psi, dpsi = d.score_and_der(GRID[None, :])
        out[f"{name}_psi"], out[f"{name}_dpsi"], out[f"{name}_ll"] = psi[0], dpsi[0], d.log_lik(GRID)
    out["grid"] = GRID
    np.savez(os.path.join(HERE, "density_kats.npz"), **out)

    x, s, a = datagen.generate_data(8, 10000, 42)
    np.savez(os.path.join(HERE, "c1_data_digest.npz"), a=a, x_first=x[:, :64], x_last=x[:, -64:],
             x_rowsum=x.sum(axis=1), s_rowsum=s.sum(axis=1))

    rng = np.random.default_rng(20261015)
    w = np.linalg.qr(rng.normal(size=(8, 8)))[0]
    mu = x.sum(axis=1) / x.shape[1]
    st = po.pass_stats(w, mu, x, po.Density("tanh", 1.0), True)
    np.savez(os.path.join(HERE, "c1_pass_stats.npz"), w=w, mu=mu, **st)

    traj = {}
    for tag, kw in [("ortho_ext", dict(ortho=True, extended=True)), ("ortho", dict(ortho=True, extended=False)),
                    ("nonortho_ext", dict(ortho=False, extended=True)), ("nonortho", dict(ortho=False, extended=False))]:
        r = po.fit_with_config(x, po.PicardConfig(w_init=np.eye(8), **kw))
        traj[f"{tag}_loss"] = np.array(r.info.trace_loss)
        traj[f"{tag}_gnorm"] = np.array(r.info.trace_gnorm)
        traj[f"{tag}_unmixing"] = r.unmixing
        traj[f"{tag}_whitening"] = r.whitening
        traj[f"{tag}_n_iter"] = np.array(r.n_iterations)
        traj[f"{tag}_n_evals"] = np.array(r.info.n_evals)
        traj[f"{tag}_amari"] = np.array(po.amari_distance(r.full_unmixing(), a))
    np.savez(os.path.join(HERE, "c1_trajectories.npz"), **traj)
    c2_fit()
    print("wrote", sorted(os.listdir(HERE)))


def c2_fit():
    """BASELINE config 2 whole (64 sources × 1e6 samples of the bench mixture, seed 42),
    Picard-O extended tanh with w_init = I: the one GPU config the oracle can fit entirely
    (≈ a minute of numpy). tests/test_gpu_golden.py fits the same data on the device."""
    x, _, a = datagen.generate_data(64, 1_000_000, 42)
    r = po.fit_with_config(x, po.PicardConfig(w_init=np.eye(64)))
    np.savez(os.path.join(HERE, "c2_fit.npz"), n_iter=np.array(r.n_iterations), converged=np.array(r.converged),
             unmixing=r.unmixing, whitening=r.whitening, mean=r.mean, a=a,
             amari=np.array(po.amari_distance(r.full_unmixing(), a)),
             loss=np.array(r.info.trace_loss), gnorm=np.array(r.info.trace_gnorm),
             n_evals=np.array(r.info.n_evals))


if __name__ == "__main__":
    if sys.argv[1:] == ["c2"]:
        c2_fit()
    else:
        main()
