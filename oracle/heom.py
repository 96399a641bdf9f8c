"""NumPy restatement of the single-exponential HEOM chains (test infrastructure only).

Follows:
  pyqed/HEOM/heom.py:275-347  _heom: RK4 (phys.rk4, phys.py:1051-1064) of the chain
        rhs_0 = -i[H, r_0] - [Q, r_1]
        rhs_n = -i[H, r_n] - [Q, r_{n+1}] - n gamma r_n + n (Re D0 [Q, r_{n-1}] + i Im D0 {Q, r_{n-1}}),
        n = 1 .. nado-2 (ADO nado-1 never updated), D0 = reorg (2T - i gamma)
  pyqed/oqs.py:1808-1875      _heom: explicit in-place sweep (ADO n sees the already-updated n-1),
        D0 = reorg gamma (coth(gamma / 2T) - i)
Observables Tr(r_0 e) after every step, shape (n_e, nt).
"""
import numpy as np


def _comm(a, b):
    return a @ b - b @ a


def _acomm(a, b):
    return a @ b + b @ a


def _obs(r, e):
    return np.trace(r @ e)


def chain_rk4(H, Q, rho0, e_ops, temperature, cutoff, reorg, nado, dt, nt):
    ns = H.shape[0]
    gamma, T = cutoff, temperature
    D0 = reorg * (2.0 * T - 1j * gamma)
    ado = np.zeros((nado, ns, ns), complex)
    ado[0] = rho0

    def L(a):
        r = np.zeros_like(a)
        r[0] = -1j * _comm(H, a[0]) - _comm(Q, a[1])
        for n in range(1, nado - 1):
            r[n] = (-1j * _comm(H, a[n]) - _comm(Q, a[n + 1]) - n * gamma * a[n]
                    + n * (D0.real * _comm(Q, a[n - 1]) + 1j * D0.imag * _acomm(Q, a[n - 1])))
        return r

    out = np.zeros((len(e_ops), nt), complex)
    for k in range(nt):
        k1 = L(ado)
        k2 = L(ado + k1 * dt / 2)
        k3 = L(ado + k2 * dt / 2)
        k4 = L(ado + k3 * dt)
        ado = ado + (k1 + 2 * k2 + 2 * k3 + k4) / 6.0 * dt
        out[:, k] = [_obs(ado[0], e) for e in e_ops]
    return out


def chain_euler(H, Q, rho0, e_ops, temperature, cutoff, reorg, nado, dt, nt):
    ns = H.shape[0]
    gamma, T = cutoff, temperature
    D0 = reorg * gamma * (1.0 / np.tanh(gamma / (2.0 * T)) - 1j)
    ado = np.zeros((nado, ns, ns), complex)
    ado[0] = rho0
    out = np.zeros((len(e_ops), nt), complex)
    for k in range(nt):
        ado[0] = ado[0] - 1j * _comm(H, ado[0]) * dt - _comm(Q, ado[1]) * dt
        for n in range(1, nado - 1):
            ado[n] = ado[n] + (-1j * _comm(H, ado[n]) * dt
                               + (-_comm(Q, ado[n + 1]) - n * gamma * ado[n]
                                  + n * (D0.real * _comm(Q, ado[n - 1]) + 1j * D0.imag * _acomm(Q, ado[n - 1]))) * dt)
        out[:, k] = [_obs(ado[0], e) for e in e_ops]
    return out
