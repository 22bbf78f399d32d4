import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import torch  # noqa: E402,F401  (before libcfk_als.so: one HIP runtime per process)

import __graft_entry__  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libcfk_als.so on cuda:0)")


@pytest.fixture(scope="session")
def cfk():
    # content-addressed (BUILD_INFO.json): compiles nothing when the libraries were built from these sources, and
    # rebuilds them from scratch when not -- the session always tests a library built from the tree it runs on
    __graft_entry__.build()
    return __graft_entry__.load_package()


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def tiny_path():
    return os.path.join(GOLDEN, "data_sample_tiny.txt")


@pytest.fixture(scope="session")
def medium_path():
    return os.path.join(GOLDEN, "data_sample_medium.txt")


def max_rel(a, b):
    """Element-wise max relative error with the SURVEY §8c denominator floor max(|b|, 1e-12 * ||row||)."""
    import numpy as np
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    denom = np.maximum(np.abs(b), 1e-12 * np.linalg.norm(b, axis=1, keepdims=True))
    denom = np.where(denom == 0, 1.0, denom)
    return float(np.max(np.abs(a - b) / denom)) if a.size else 0.0
