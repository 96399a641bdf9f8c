"""Result container (mirror of pyqed/mol.py:98-171)."""
from __future__ import annotations

import pickle

import numpy as np


class Result:
    """Same fields and `times` convention as pyqed.mol.Result (mol.py:98-119):
    times = t0 + arange(Nt//nout + 1) * dt * nout."""

    def __init__(self, description=None, psi0=None, rho0=None, dt=None, Nt=None, times=None, t0=0, nout=1):
        self.description = description
        self.dt = dt
        self.timesteps = self.nt = Nt
        self.observables = None
        self.rholist = None
        self.psilist = []
        self.psi = None
        self.rho0 = rho0
        self.psi0 = psi0
        self.nout = nout
        self.times = t0 + np.arange(Nt // nout + 1) * dt * nout
        return

    def expect(self):
        return self.observables

    def dump(self, fname):
        """Pickle the result (mol.py:146-162)."""
        with open(fname, "wb") as f:
            pickle.dump(self, f)

    def save(self, fname):
        self.dump(fname)


def load_result(fname):
    """Counterpart of mol.load_result (mol.py:173-179); loads a file this package wrote."""
    with open(fname, "rb") as f:
        return pickle.load(f)
