import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libqdyn)")


def load_golden(name):
    path = os.path.join(GOLDEN, name + ".npz")
    return dict(np.load(path, allow_pickle=False))


@pytest.fixture
def golden():
    return load_golden


def relerr(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    den = max(np.linalg.norm(b.ravel()), 1e-300)
    return np.linalg.norm((a - b).ravel()) / den


# spectral functions used by the Redfield golden vectors (tests/golden/make_golden.py SPECTRA)
SPECTRA = {
    "flat005": lambda w: 0.05,
    "tanh": lambda w: 0.02 * (1.0 + np.tanh(2.0 * w)),
}
