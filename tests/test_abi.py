"""The C-ABI library loads and exports every symbol include/qdyn.h declares (no GPU calls)."""
import ctypes
import os
import re

from conftest import ROOT


def declared_symbols():
    syms = set()
    inc = os.path.join(ROOT, "include")
    for f in os.listdir(inc):
        if f.endswith(".h"):
            txt = open(os.path.join(inc, f)).read()
            txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
            syms |= set(re.findall(r"\b(qd_[a-z0-9_]+)\s*\(", txt))
    return syms


def test_library_exports_every_declared_symbol():
    from pyqed_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    syms = declared_symbols()
    assert "qd_lindblad_rk4" in syms
    missing = [s for s in sorted(syms) if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_covers_header():
    from pyqed_amd import _lib
    assert declared_symbols() == set(_lib.SIGNATURES)


def test_version_and_error_string():
    from pyqed_amd import _lib
    lib = _lib.load()
    assert lib.qd_version() >= 100
    # argument validation happens before any HIP call -> safe without a GPU
    rc = lib.qd_lindblad_rk4(None, None, 0, None, 1, 4, 0.1, 1, None, 0, None, None, 0, None)
    assert rc == _lib.QD_EINVAL
    assert "non-null" in _lib.last_error()
