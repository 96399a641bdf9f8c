"""Sum-over-states nonlinear spectra (drop-in for pyqed/signal/sos.py photon_echo)."""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from ._util import default_device


def _photon_echo(evals, edip, omega1, omega3, t2, g_idx, e_idx, f_idx, gamma):
    """GSB + SE + ESA on the (omega3, omega1) grid (sos.py:845-879), computed on the GPU.
    Returns S [len(omega3), len(omega1)]."""
    dev = default_device()
    _lib.ensure_device(dev)
    E = torch.from_numpy(np.ascontiguousarray(np.asarray(evals, dtype=complex))).to(dev)
    D = torch.from_numpy(np.ascontiguousarray(np.asarray(edip, dtype=complex))).to(dev)
    G = torch.from_numpy(np.ascontiguousarray(np.asarray(gamma, dtype=float))).to(dev)
    idx = [torch.from_numpy(np.ascontiguousarray(np.asarray(list(x), dtype=np.int32).reshape(-1))).to(dev)
           for x in (g_idx, e_idx, f_idx)]
    pump = torch.from_numpy(np.ascontiguousarray(-np.asarray(omega1, dtype=float))).to(dev)
    probe = torch.from_numpy(np.ascontiguousarray(np.asarray(omega3, dtype=float))).to(dev)
    N = E.numel()
    S = torch.empty((probe.numel(), pump.numel()), dtype=torch.complex128, device=dev)
    with torch.cuda.device(dev):
        rc = _lib.load().qd_photon_echo(E.data_ptr(), D.data_ptr(), G.data_ptr(), N, idx[0].data_ptr(),
                                        idx[0].numel(), idx[1].data_ptr(), idx[1].numel(), idx[2].data_ptr(),
                                        idx[2].numel(), pump.data_ptr(), pump.numel(), probe.data_ptr(),
                                        probe.numel(), float(t2), S.data_ptr(), _lib.stream_ptr(dev))
    _lib.check(rc, "qd_photon_echo")
    return S.cpu().numpy()


def photon_echo(mol, pump, probe, t2=0., g_idx=[0], e_idx=None, f_idx=None, fname='signal', plt_signal=False,
                pol=None):
    """sos.py:962-1052: S = GSB + SE + ESA with omega1 = -pump; writes `fname`.npz as the reference."""
    E = mol.eigvals()
    dip = mol.edip_rms
    gamma = mol.gamma
    if gamma is None:
        raise ValueError('Please set the decay constants gamma first.')
    N = mol.nstates
    if e_idx is None:
        e_idx = range(N)
    if f_idx is None:
        f_idx = range(N)
    S = _photon_echo(E, dip, omega1=-np.asarray(pump), omega3=probe, t2=t2, g_idx=g_idx, e_idx=e_idx, f_idx=f_idx,
                     gamma=gamma)
    if fname is not None:
        np.savez(fname, pump, probe, S)
    return S
