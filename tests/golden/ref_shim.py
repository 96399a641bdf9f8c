"""Import shim for the read-only reference (generation-time only).

Used ONLY by tests/golden/make_golden.py in the build container to import the
reference pyqed (pure Python) and produce golden .npz vectors.  It installs
identity/dummy stubs for packages the reference imports but which are absent
here or out of scope (SURVEY.md §8(c) "Import recipe").  Nothing in the
product, the GPU tests, smoke() or bench.py imports this module.
"""
import os
import sys
import types

import numpy as np

REF = "/root/reference"


def _identity_decorator(*args, **kwargs):
    if len(args) == 1 and callable(args[0]) and not kwargs:
        return args[0]

    def wrap(f):
        return f
    return wrap


class _Permissive(types.ModuleType):
    """A module whose every attribute is a harmless dummy."""

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return _Dummy()


class _Dummy:
    def __call__(self, *a, **k):
        return _Dummy()

    def __getattr__(self, name):
        return _Dummy()

    def __mro_entries__(self, bases):
        return (object,)


def install():
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    numba = types.ModuleType("numba")
    numba.jit = numba.njit = numba.autojit = _identity_decorator
    numba.prange = range
    sys.modules.setdefault("numba", numba)

    oe = types.ModuleType("opt_einsum")
    oe.contract = np.einsum
    sys.modules.setdefault("opt_einsum", oe)

    sys.modules.setdefault("proplot", plt)

    for name in ["pyqed.qchem", "pyqed.qchem.mol", "tensorly", "tensorly.tenalg",
                 "tensorly.decomposition", "gbasis", "pyscf", "periodictable"]:
        sys.modules.setdefault(name, _Permissive(name))
    if REF not in sys.path:
        sys.path.insert(0, REF)


def lib_versions():
    import scipy
    out = {"numpy": np.__version__, "scipy": scipy.__version__}
    try:
        import sympy
        out["sympy"] = sympy.__version__
    except Exception:
        pass
    return out
