"""NumPy restatement of the Lindblad RK4 path (test infrastructure only).

Follows:
  pyqed/phys.py:1051-1064      rk4 (in-place `rho += (k1+2k2+2k3+k4)/6*dt`)
  pyqed/phys.py:1161-1168      comm / anticomm
  pyqed/oqs.py:697-714         liouvillian / lindbladian
  pyqed/oqs.py:1596-1696       _lindblad (observables incl. t0, rholist excl. rho0)
  pyqed/phys.py:1257-1264      obs_dm = Tr(d rho)
Dense NumPy instead of scipy.sparse csr; same operation order.
"""
import numpy as np


def comm(A, B):
    return A @ B - B @ A                                    # phys.py:1161-1163


def anticomm(A, B):
    return A @ B + B @ A                                    # phys.py:1166-1168


def dag(a):
    return a.conj().T


def lindbladian(l, rho):
    # oqs.py:707-714
    return l @ (rho @ dag(l)) - 0.5 * anticomm(dag(l) @ l, rho)


def liouvillian(rho, H, c_ops):
    # oqs.py:697-704
    rhs = -1j * comm(H, rho)
    for c in c_ops:
        rhs = rhs + lindbladian(c, rho)
    return rhs


def rk4(rho, fun, dt, *args):
    # phys.py:1051-1064
    dt2 = dt / 2.0
    k1 = fun(rho, *args)
    k2 = fun(rho + k1 * dt2, *args)
    k3 = fun(rho + k2 * dt2, *args)
    k4 = fun(rho + k3 * dt, *args)
    return rho + (k1 + 2 * k2 + 2 * k3 + k4) / 6. * dt


def obs_dm(rho, d):
    return (d @ rho).diagonal().sum()                       # phys.py:1257-1264


def lindblad(H, rho0, c_ops, e_ops, Nt, dt, keep_states=True):
    """oqs._lindblad: returns (observables (Nt+1, ne), rholist [Nt], rho_final)."""
    H = np.asarray(H, complex)
    c_ops = [np.asarray(c, complex) for c in c_ops]
    e_ops = [np.asarray(e, complex) for e in e_ops]
    rho = np.asarray(rho0, complex).copy()
    obs = np.zeros((Nt + 1, len(e_ops)), dtype=complex)
    obs[0, :] = [obs_dm(rho, e) for e in e_ops]
    rholist = []
    for k in range(Nt):
        rho = rk4(rho, liouvillian, dt, H, c_ops)
        if keep_states:
            rholist.append(rho.copy())
        obs[k + 1, :] = [obs_dm(rho, e) for e in e_ops]
    return obs, rholist, rho


def lindblad_batch(H, c_ops, rho_b, dt, Nt):
    """Batched variant (same arithmetic per member) used for the CPU baseline: rho_b [B,N,N]."""
    H = np.asarray(H, complex)
    c_ops = [np.asarray(c, complex) for c in c_ops]
    rho = np.asarray(rho_b, complex).copy()

    def rhs(r):
        out = -1j * (H @ r - r @ H)
        for c in c_ops:
            cd = dag(c)
            cdc = cd @ c
            out = out + c @ (r @ cd) - 0.5 * (cdc @ r + r @ cdc)
        return out

    for _ in range(Nt):
        rho = rk4(rho, lambda r: rhs(r), dt)
    return rho


def synthetic_lindblad(N, seed_h=0, seed_c=1, nc=1, gamma=0.1):
    """BASELINE config d1: GUE H/sqrt(N), dense Ginibre c_op * 0.1/sqrt(N)."""
    rng = np.random.default_rng(seed_h)
    A = rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N))
    H = (A + A.conj().T) / 2 / np.sqrt(N)
    rng = np.random.default_rng(seed_c)
    cs = []
    for _ in range(nc):
        C = rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N))
        cs.append(gamma * C / np.sqrt(N))
    return H, cs


def random_pure_states(B, N, seed=2):
    rng = np.random.default_rng(seed)
    psi = rng.standard_normal((B, N)) + 1j * rng.standard_normal((B, N))
    psi /= np.linalg.norm(psi, axis=1, keepdims=True)
    return np.einsum("bi,bj->bij", psi, psi.conj())


def lindblad_csr(H, rho0, c_ops, e_ops, Nt, dt):
    """Reference-faithful scipy.sparse csr path (oqs.py:1617-1690: H, c_ops, e_ops, rho all csr).

    Used as the timed CPU baseline (`cpu_baseline.kind = "port"`): the same
    csr x csr products the reference performs per RHS.
    """
    from scipy.sparse import csr_matrix

    H = csr_matrix(H)
    c_ops = [csr_matrix(c) for c in c_ops]
    e_ops = [csr_matrix(e) for e in e_ops]
    rho = csr_matrix(np.asarray(rho0, complex))

    def rhs(r, H, c_ops):
        out = -1j * (H @ r - r @ H)
        for l in c_ops:
            ld = l.conj().T
            out = out + (l @ (r @ ld) - 0.5 * ((ld @ l) @ r + r @ (ld @ l)))
        return out

    obs = np.zeros((Nt + 1, len(e_ops)), dtype=complex)
    obs[0, :] = [(e @ rho).diagonal().sum() for e in e_ops]
    for k in range(Nt):
        rho = rk4(rho, rhs, dt, H, c_ops)
        obs[k + 1, :] = [(e @ rho).diagonal().sum() for e in e_ops]
    return obs, rho


def correlation_3p_1t(H, rho0, ops, c_ops, tlist, dyn=None):
    """correlation.correlation_3p_1t (pyqed/correlation.py:17-70) with dyn = oqs.liouvillian by default, or any
    dyn(rho, H, c_ops) (:62 rk4(rho, dyn, dt, H, c_ops)).

    rho <- C rho0 A (:41), then len(tlist) RK4 steps of dt = tlist[1]-tlist[0] (:50-57); after each
    step t += dt and cor = Tr(B rho) (:59).  Returns (t [Nt], cor [Nt], rho_k [Nt,N,N]) -- the values
    the reference writes to cor.dat / dm.dat (it returns None)."""
    A, B, C = (np.asarray(o, complex) for o in ops)
    H = np.asarray(H, complex)
    c_ops = [np.asarray(c, complex) for c in c_ops]
    rho = C @ (np.asarray(rho0, complex) @ A)
    dt = tlist[1] - tlist[0]
    t, ts, cor, rhos = 0.0, [], [], []
    for _ in range(len(tlist)):
        t += dt
        rho = rk4(rho, dyn or liouvillian, dt, H, c_ops)
        ts.append(t)
        cor.append((B @ rho).diagonal().sum())
        rhos.append(rho.copy())
    return np.array(ts), np.array(cor), np.array(rhos)
