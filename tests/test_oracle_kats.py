"""The oracle pinned against the reference's own known-answer unit tests.

Each test restates one #[test] of the Rust reference (file:line cited); the
reference ships no other fixtures, so these are the pins."""
import math

import numpy as np
import pytest


def test_sym_decorrelation_kat(po):
    """math.rs:101-111."""
    w = po.sym_decorrelation(np.array([[1.0, 0.5], [0.5, 1.0]]))
    ww = w @ w.T
    assert abs(ww[0, 0] - 1) < 1e-10 and abs(ww[1, 1] - 1) < 1e-10
    assert abs(ww[0, 1]) < 1e-10 and abs(ww[1, 0]) < 1e-10


def test_matrix_exp_zero_kat(po):
    """math.rs:114-124."""
    assert np.allclose(po.matrix_exp(np.zeros((3, 3))), np.eye(3), atol=1e-10)


def test_sln_det_kats(po):
    """math.rs:127-141."""
    s, l = po.sln_det(np.array([[1.0, 2.0], [3.0, 4.0]]))
    assert abs(s + 1) < 1e-10 and abs(l - math.log(2)) < 1e-10
    s, l = po.sln_det(np.array([[1e150, 0.0], [0.0, 1e150]]))
    assert abs(s - 1) < 1e-10 and abs(l - 2 * 150 * math.log(10)) < 1e-6


def test_skew_kat(po):
    """math.rs:144-152."""
    k = po.skew_symmetric(np.array([[1.0, 2.0], [3.0, 4.0]]))
    assert abs(k[0, 0]) < 1e-10 and abs(k[1, 1]) < 1e-10 and abs(k[0, 1] + k[1, 0]) < 1e-10


def test_center_kat(po):
    """whitening.rs:124-135."""
    xc, mean = po.center(np.array([[1.0, 2.0, 3.0], [4.0, 5.0, 6.0]]))
    assert abs(mean[0] - 2) < 1e-10 and abs(mean[1] - 5) < 1e-10
    assert np.all(np.abs(xc.mean(axis=1)) < 1e-10)


def test_whiten_shapes_kat(po):
    """whitening.rs:138-150."""
    x = np.array([[1.0, 2.0, 3.0, 4.0], [2.0, 4.0, 6.0, 8.0], [1.0, 3.0, 2.0, 4.0]])
    xc, _ = po.center(x)
    data, k = po.whiten(xc, 2)
    assert data.shape == (2, 4) and k.shape == (2, 3)


def test_amari_kats(po):
    """utils.rs:147-171."""
    a = np.array([[1.0, 0.5, 0.2], [0.3, 1.0, 0.4], [0.1, 0.2, 1.0]])
    assert po.amari_distance(np.linalg.inv(a), a) < 1e-10
    a2 = np.array([[1.0, 0.5], [0.3, 1.0]])
    wi = np.linalg.inv(a2)
    assert po.amari_distance(wi[::-1].copy(), a2) < 1e-10


def test_permute_kat(po):
    """utils.rs:174-190."""
    p = po.permute(np.array([[0.1, 0.9], [0.95, 0.05]]), True)
    assert abs(p[0, 0] - 1) < 1e-6 and abs(p[1, 1] - 1) < 1e-6


@pytest.mark.parametrize("dens", [("tanh", 1.0), ("exp", 0.1), ("cube", 1.0)])
def test_density_score_is_derivative(po, dens):
    """utils.rs:192-208 via check_density (utils.rs:110-137)."""
    assert po.check_density(po.Density(*dens), 1e-5)


def test_lbfgs_memory_kats(po):
    """lbfgs.rs:178-202."""
    m = po.LbfgsMemory(3)
    assert m.is_empty()
    m.update(np.eye(2), 0.5 * np.eye(2))
    assert len(m) == 1
    m = po.LbfgsMemory(2)
    for i in range(5):
        m.update(np.full((2, 2), i + 1.0), np.ones((2, 2)))
    assert len(m) == 2


def test_config_validation(po):
    """config.rs:104-142 and solver.rs:401-408."""
    for kw, param in [(dict(max_iter=0), "max_iter"), (dict(tol=0.0), "tol"), (dict(lambda_min=-1.0), "lambda_min"),
                      (dict(m=0), "m"), (dict(fastica_it=10, jade_it=10), "jade_it")]:
        with pytest.raises(po.InvalidConfig) as e:
            po.PicardConfig(**kw).validate()
        assert e.value.parameter == param
    po.PicardConfig().validate()
    assert po.PicardConfig().effective_extended() is True
    assert po.PicardConfig(ortho=False).effective_extended() is False


def test_rust_e4_format(po):
    """core.rs:385 `{:.4e}` formatting of the verbose line."""
    assert po.rust_e4(1.23456e-5) == "1.2346e-5"
    assert po.rust_e4(8.24883985) == "8.2488e0"
    assert po.rust_e4(-1234.5) == "-1.2345e3"


def test_batched_jade_sweeps_match_literal_form(po, dg):
    """oracle.jade_sweeps_batched (the matrix loop of jade.rs:137-167 vectorised, used
    by the N = 64 GPU tests) against the literal per-matrix loop (po.jade) at C1 size,
    and cumulants_from_moments against compute_cumulant_matrices (jade.rs:78-131)."""
    x, _, _ = dg.generate_data(8, 10000, 42)
    xc, _ = po.center(x)
    x1, _ = po.whiten(xc, 8)
    mats = np.stack(po.compute_cumulant_matrices(x1))
    pairs = [(i, j) for i in range(8) for j in range(i, 8)]
    z = np.stack([x1[i] * x1[j] for i, j in pairs])
    assert np.max(np.abs(po.cumulants_from_moments(z @ z.T, 8, x1.shape[1]) - mats)) <= 1e-12
    for it in (1, 3):
        v, sweeps, _ = po.jade_sweeps_batched(mats, it)
        assert sweeps == it
        assert np.max(np.abs(po.sym_decorrelation(v) - po.jade(x1, it))) <= 1e-12
    v, _, _ = po.jade_sweeps_batched(mats, 1, max_pairs=0)
    assert np.array_equal(v, np.eye(8))
