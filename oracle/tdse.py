"""NumPy restatement of the TDSE RK4 paths (test infrastructure only).

Follows:
  pyqed/phys.py:1051-1064   rk4 (k1 + 2k2 + 2k3 + k4)/6 dt
  pyqed/phys.py:1322        tdse = -1j H psi
  pyqed/phys.py:1266-1283   obs = <psi|a|psi>
  pyqed/mol.py:1603-1691    _quantum_dynamics (store_states=True): (Nt//nout - 1)*nout steps,
                            observables (Nt//nout, n_e) incl. t0, psilist [psi0] + per block
  pyqed/mol.py:1862-1958    driven_dynamics (return_result=True): H(t) = H0 - sum_d f_d(t) Hd_d
                            evaluated at the block start time t (advanced by nout dt per block);
                            result.psi = psit [nstates, Nt//nout]
Dense NumPy instead of scipy.sparse csr; same operation order.
"""
import numpy as np


def _rk4(psi, H, dt):
    f = lambda p: -1j * (H @ p)  # noqa: E731
    dt2 = dt / 2.0
    k1 = f(psi)
    k2 = f(psi + k1 * dt2)
    k3 = f(psi + k2 * dt2)
    k4 = f(psi + k3 * dt)
    return psi + (k1 + 2 * k2 + 2 * k3 + k4) / 6. * dt


def _obs(psi, a):
    return np.conj(psi) @ a @ psi


def quantum_dynamics(H, psi0, dt, Nt, e_ops, nout=1):
    psi = np.array(psi0, dtype=complex)
    observables = np.zeros((Nt // nout, len(e_ops)), dtype=complex)
    observables[0, :] = [_obs(psi, e) for e in e_ops]
    psilist = [psi.copy()]
    for k1 in range(1, Nt // nout):
        for _ in range(nout):
            psi = _rk4(psi, H, dt)
        observables[k1, :] = [_obs(psi, e) for e in e_ops]
        psilist.append(psi.copy())
    return observables, np.array(psilist)


def driven_dynamics(H0, drives, psi0, dt, Nt, e_ops, nout=1, t0=0.0):
    """drives: list of (Hd, f) with H(t) = H0 - sum f(t) Hd.  Returns (observables, psit, psilist)."""
    psi = np.array(psi0, dtype=complex)
    nstates = len(psi)
    nrec = Nt // nout
    observables = np.zeros((nrec, len(e_ops)), dtype=complex)
    psit = np.zeros((nstates, nrec), dtype=complex)
    observables[0, :] = [_obs(psi, e) for e in e_ops]
    psit[:, 0] = psi
    psilist = [psi.copy()]
    t = t0
    for k1 in range(1, nrec):
        for _ in range(nout):
            Ht = np.array(H0, dtype=complex)
            for Hd, f in drives:
                Ht = Ht + (-f(t) * Hd)
            psi = _rk4(psi, Ht, dt)
        t += dt * nout
        observables[k1, :] = [_obs(psi, e) for e in e_ops]
        psilist.append(psi.copy())
        psit[:, k1] = psi
    return observables, psit, np.array(psilist)


def gaussian_efield(omegac, tau, tc, amplitude):
    """optics.py:293-318 Pulse.efield: Re[A exp(-(t-tc)^2/2tau^2) exp(-i omegac (t-tc))]."""
    return lambda t: np.real(amplitude * np.exp(-(t - tc) ** 2 / 2. / tau ** 2) * np.exp(-1j * omegac * (t - tc)))
