"""Generate golden vectors by running the REAL reference (ShuoyiHU/pyqed) here.

Run in the build container only (the reference does not exist on the GPU box):
    python tests/golden/make_golden.py [name ...]
Writes tests/golden/<name>.npz (inputs + reference outputs + library versions).
The reference is imported read-only through ref_shim.
Fixtures are data; no reference source is copied.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ref_shim  # noqa: E402

ref_shim.install()

from scipy.sparse import csr_matrix  # noqa: E402

GENERATORS = {}


def golden(fn):
    GENERATORS[fn.__name__] = fn
    return fn


def save(name, **arrays):
    arrays["lib_versions"] = np.array(str(ref_shim.lib_versions()))
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **arrays)
    print("wrote", path, f"{os.path.getsize(path)/1024:.1f} KiB")


def _herm(rng, n, scale=1.0):
    a = rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n))
    return scale * (a + a.conj().T) / 2


def _ginibre(rng, n, scale=1.0):
    return scale * (rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n)))


# ----------------------------------------------------------------- Lindblad
def _lindblad_case(name, N, nc, ne, Nt, dt, seed, keep_all=True):
    import pyqed.oqs as oqs
    rng = np.random.default_rng(seed)
    H = _herm(rng, N, 1 / np.sqrt(N))
    C = np.array([_ginibre(rng, N, 0.3 / np.sqrt(N)) for _ in range(nc)]).reshape(nc, N, N)
    E = np.array([_herm(rng, N) for _ in range(ne)]).reshape(ne, N, N)
    psi = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    psi /= np.linalg.norm(psi)
    rho0 = np.outer(psi, psi.conj())
    solver = oqs.LindbladSolver(csr_matrix(H), [csr_matrix(c) for c in C])
    r = solver.run(rho0, dt=dt, Nt=Nt, e_ops=[csr_matrix(e) for e in E])
    rholist = np.array([x.toarray() for x in r.rholist])
    out = dict(H=H, C=C, E=E, rho0=rho0, dt=dt, Nt=Nt, observables=r.observables, times=r.times)
    if keep_all:
        out["rholist"] = rholist
    else:
        out["rho_final"] = rholist[-1]
    save(name, **out)


@golden
def lindblad_n4():
    _lindblad_case("lindblad_n4", N=4, nc=2, ne=2, Nt=10, dt=0.01, seed=11)


@golden
def lindblad_n16():
    _lindblad_case("lindblad_n16", N=16, nc=1, ne=3, Nt=10, dt=0.005, seed=12)


@golden
def lindblad_n40_noc():
    # no collapse operators, N not a multiple of 32 (exercises padding)
    _lindblad_case("lindblad_n40_noc", N=40, nc=0, ne=1, Nt=5, dt=0.01, seed=13)


@golden
def lindblad_n128():
    # BASELINE config d1 size (few steps: the reference does ~5.6 steps/s here)
    _lindblad_case("lindblad_n128", N=128, nc=1, ne=1, Nt=3, dt=1e-3, seed=14, keep_all=False)


if __name__ == "__main__":
    names = sys.argv[1:] or list(GENERATORS)
    for n in names:
        GENERATORS[n]()
