"""Quantum-regression correlation functions on MI355X (drop-in for pyqed/correlation.py).

correlation_3p_1t (correlation.py:17-70): <A B(t) C> = Tr[B U(t) (C rho0 A) U^+(t)] with the
propagation on the Lindblad RK4 kernel (qd_lindblad_rk4).  Like the reference it returns None and
writes 'cor.dat' (t, cor) and 'dm.dat' (t, ravel rho) in the current directory.
"""
from __future__ import annotations

import numpy as np
import torch

from ._util import default_device, stack_ops, to_numpy
from .oqs import lindblad_rk4


def _is_lindblad(dyn) -> bool:
    """dyn the reference passes for Lindblad dynamics: pyqed.oqs.liouvillian(rho, H, c_ops)
    (oqs.py:697-704), or the string 'lindblad'."""
    if dyn is None or (isinstance(dyn, str) and dyn.lower() in ("lindblad", "liouvillian")):
        return True
    return getattr(dyn, "__name__", "") == "liouvillian"


def correlation_3p_1t(H, rho0, ops, c_ops, tlist, dyn=None, *args):
    """<A B(t) C> by the quantum regression theorem (correlation.py:17-70).

    rho <- C rho0 A; len(tlist) RK4 steps of dt = tlist[1] - tlist[0]; after each step
    t += dt, cor = Tr(B rho).  Only Lindblad dynamics (dyn = oqs.liouvillian) run here: any other
    `dyn` is an arbitrary host callable and raises NotImplementedError (no CPU fallback).
    """
    if not _is_lindblad(dyn):
        raise NotImplementedError(f"correlation_3p_1t: dynamics {dyn!r} is not supported on the GPU; "
                                  "use dyn=pyqed.oqs.liouvillian (Lindblad)")
    A, B, C = (np.ascontiguousarray(to_numpy(o, np.complex128)) for o in ops)
    Hn = np.ascontiguousarray(to_numpy(H, np.complex128))
    nstates = Hn.shape[-1]
    r0 = C @ (np.ascontiguousarray(to_numpy(rho0, np.complex128)) @ A)
    Nt = len(tlist)
    dt = tlist[1] - tlist[0]
    dev = default_device()
    rho = torch.from_numpy(r0).to(dev).reshape(1, nstates, nstates).contiguous()
    obs, snap = lindblad_rk4(torch.from_numpy(Hn).to(dev), stack_ops(c_ops or [], nstates, dev), rho, float(dt), Nt,
                             stack_ops([B], nstates, dev), save_every=1, hermitian=False)
    torch.cuda.synchronize(dev)
    cor = obs[0, 1:, 0].cpu().numpy()
    rhos = snap[0].cpu().numpy()
    fmt = '{} ' * (nstates ** 2 + 1) + '\n'
    with open('cor.dat', 'w') as f, open('dm.dat', 'w') as f_dm:
        t = 0.0
        for k in range(Nt):
            t += dt
            f.write('{} {} \n'.format(t, cor[k]))
            f_dm.write(fmt.format(t, *np.ravel(rhos[k])))
    return
