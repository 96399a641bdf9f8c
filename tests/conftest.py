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


import contextlib  # noqa: E402


@contextlib.contextmanager
def qd_option(name, value):
    """Set a libqdyn process option (include/qdyn.h QD_OPT_*: "coop", "fake_timeout", "glf_path", "idle_cap") for the
    block and
    restore it after."""
    from pyqed_amd import _lib
    opt = {"coop": _lib.QD_OPT_COOP_LAUNCH, "fake_timeout": _lib.QD_OPT_FAKE_TIMEOUT,
           "glf_path": _lib.QD_OPT_GLF_PATH, "idle_cap": _lib.QD_OPT_IDLE_CAP_MIB}[name]
    if isinstance(value, str):
        value = _lib.GLF_PATHS[value]
    prev = _lib.set_option(opt, value)
    try:
        yield
    finally:
        _lib.set_option(opt, prev)


def took(path_name):
    """True when the library calls since the last check took a kernel path whose name starts with path_name
    (qd_take_path; clears the record)."""
    from pyqed_amd import _lib
    got = _lib.take_path().split()
    return any(p.startswith(path_name) for p in got), got
