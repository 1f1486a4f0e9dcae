"""Shared fixtures. `-m gpu` tests need an MI355X; everything else runs on CPU."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD Instinct MI355X (HIP device)")


@pytest.fixture(scope="session")
def pa():
    import picard_ica_amd
    return picard_ica_amd


@pytest.fixture(scope="session")
def po():
    from oracle import picard_oracle
    return picard_oracle


@pytest.fixture(scope="session")
def dg():
    from oracle import datagen
    return datagen


@pytest.fixture(scope="session")
def c1_data(dg):
    """BASELINE config 1: 8 sources × 10k samples from the bench LCG (benchmarks.rs:8-35)."""
    x, s, a = dg.generate_data(8, 10000, 42)
    return x, s, a


def density_of(po, d):
    return po.Density(["tanh", "exp", "cube"][d.kind], d.alpha)


def rel_err(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))
