"""The C-ABI library: loads on a CPU-only host and exports every symbol that
include/picard_mi355x.h declares. No compute call needs a GPU here."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "picard_mi355x.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set(re.findall(r"\b(pc_[a-z0-9_]+)\s*\(", src))
    return sorted(names)


def test_every_declared_symbol_is_exported(pa):
    lib = ctypes.CDLL(pa.LIB_PATH)
    missing = [n for n in header_functions() if not hasattr(lib, n)]
    assert not missing, missing
    assert set(header_functions()) == set(pa.EXPORTED)


def test_no_cpu_fallback_in_package(pa):
    """The product package (Python binding, C++/HIP sources, Makefile) never names the
    oracle: no import, include, link or path (it is the checker only)."""
    for root, _, files in os.walk(os.path.join(ROOT, "picard-ica_amd")):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".hpp", ".inc", ".h")) or f == "Makefile":
                assert "oracle" not in open(os.path.join(root, f)).read().lower(), f


def test_config_defaults(pa):
    """config.rs:64-85."""
    c, _ = pa.PicardConfig()._c()
    assert (c.density.kind, c.density.alpha) == (0, 1.0)
    assert c.ortho == 1 and c.has_extended == 0 and c.whiten == 1 and c.centering == 1
    assert (c.max_iter, c.tol, c.m, c.ls_tries, c.lambda_min) == (500, 1e-7, 7, 10, 0.01)
    assert not c.w_init and c.has_fastica_it == 0 and c.has_jade_it == 0 and c.has_random_state == 0
    cd = type(c)()
    pa.lib.pc_config_default(ctypes.byref(cd))
    assert bytes(cd) == bytes(type(c).from_buffer_copy(bytes(cd)))


@pytest.mark.parametrize("kw,param,msg", [
    (dict(max_iter=0), "max_iter", "must be greater than 0"),
    (dict(tol=0.0), "tol", "must be positive"),
    (dict(lambda_min=0.0), "lambda_min", "must be positive"),
    (dict(m=0), "m", "L-BFGS memory size must be at least 1"),
    (dict(fastica_it=10, jade_it=10), "jade_it", "cannot use both fastica_it and jade_it; choose one warm start method"),
])
def test_validate_messages(pa, kw, param, msg):
    """config.rs:104-142 with the Display text of error.rs:69."""
    with pytest.raises(pa.InvalidConfig) as e:
        pa.PicardConfig(**kw).validate()
    assert str(e.value) == f"Invalid configuration for '{param}': {msg}"


def test_builder(pa):
    """config.rs:147-273 (solver.rs:401-408)."""
    c = pa.PicardConfig.builder().fastica_it(10).jade_it(10).build()
    with pytest.raises(pa.InvalidConfig):
        c.validate()
    c = pa.PicardConfig.builder().n_components(5).max_iter(200).ortho(True).build_validated()
    assert c.n_components == 5 and c.max_iter == 200


def test_amari_and_permute_match_oracle(pa, po):
    rng = np.random.default_rng(3)
    for n in [2, 3, 8, 20]:
        w, a = rng.normal(size=(n, n)), rng.normal(size=(n, n))
        assert abs(pa.utils.amari_distance(w, a) - po.amari_distance(w, a)) < 1e-12
        m = rng.normal(size=(n, n))
        assert np.allclose(pa.utils.permute(m, True), po.permute(m, True))
        assert np.allclose(pa.utils.permute(m, False), po.permute(m, False))
    a = np.array([[1.0, 0.5, 0.2], [0.3, 1.0, 0.4], [0.1, 0.2, 1.0]])
    assert pa.utils.amari_distance(np.linalg.inv(a), a) < 1e-10  # utils.rs:147-156


def test_result_helpers_match_oracle(pa, po):
    """result.rs:39-64 (full_unmixing, mixing via Gauss-Jordan)."""
    rng = np.random.default_rng(5)
    k, w, mu = rng.normal(size=(3, 3)), rng.normal(size=(3, 3)), rng.normal(size=3)
    r = pa.PicardResult(k, w, None, mu, 3, True, 1e-8, None)
    ro = po.PicardResult(k, w, None, mu, 3, True, 1e-8, None)
    assert np.allclose(r.full_unmixing(), ro.full_unmixing())
    assert np.allclose(r.mixing(), ro.mixing())
    r2 = pa.PicardResult(None, w, None, None, 3, True, 1e-8, None)
    assert np.allclose(r2.mixing(), po.PicardResult(None, w, None, None, 3, True, 1e-8, None).mixing())


def test_error_names(pa):
    assert [pa.lib.pc_error_name(i).decode() for i in range(7)] == [
        "Ok", "InvalidDimensions", "SingularMatrix", "ComputationError", "InvalidConfig", "NotConverged",
        "Unsupported"]
    assert pa.lib.pc_abi_version() == 8
    assert issubclass(pa.Unsupported, pa.ComputationError) and pa.Unsupported.code == 6
