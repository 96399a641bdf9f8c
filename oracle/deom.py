"""NumPy restatement of the DEOM/HEOM hierarchy propagation (test infrastructure only).

Follows pyqed/heom/deom.py:
  :1048-1064  init_      Pascal table comb_list, nmax = comb[L+K, L]
  :555-566    gen_hash_value(key) = sum_i comb[S_i + i, i + 1], S_i = key[0] + ... + key[i]
  :609-638    gen_keys / gen_keys_element (tier-by-tier expansion, keys[hash] = key)
  :641-673    generate_dot_element / rem_cal (the ADO stencil)
  :676-688    generate_time (H(t) = H + Hdip f(t), Q(t) = Q + Qdip g(t))
  :725-766    rk4 (stages at t, t+dt/2, t+dt/2, t+dt)
  :1072-1114  DEOMSolver.run (t_save, Tr(p1 rho_0) or rho_0 per step)
  :769-893    generate_propgator / generate_actions (dense ADO Liouvillian, element by element)
  :1127-1209  DEOMSolver.correlation_4op_3t (eig + pinv, trace per (w_x, w_y) point)
"""
import numpy as np


def comb_table(L, K):
    n = K + L + 1
    comb = np.zeros((n, n), dtype=np.int64)
    comb[0, 0] = 1
    for i in range(1, n):
        for j in range(1, n):
            comb[i, j] = comb[i - 1, j] + comb[i - 1, j - 1]
        comb[i, 0] = 1
    return comb


def gen_hash_value(key, comb):
    s, h = 0, 0
    for i in range(len(key)):
        s += key[i]
        h += comb[s + i, i + 1]
    return h


def gen_keys(L, K):
    comb = comb_table(L, K)
    nmax = comb[L + K, L]
    keys = np.zeros((nmax, K), dtype=np.int64)
    lo, hi = 0, 1
    for tier in range(L + 1):
        for n in range(lo, hi):
            for k in range(K):
                if keys[n].sum() < L:
                    kp = keys[n].copy(); kp[k] += 1
                    keys[gen_hash_value(kp, comb)] = kp
                if keys[n, k] > 0:
                    km = keys[n].copy(); km[k] -= 1
                    keys[gen_hash_value(km, comb)] = km
        lo, hi = hi, comb[K + tier, K]
    return keys, comb


def rem_cal(ddos, keys, comb, L, expn, etal, etar, etaa, mode, H, Q):
    K = keys.shape[1]
    dot = np.zeros_like(ddos)
    for n in range(len(keys)):
        key = keys[n]
        r = ddos[n]
        d = -np.sum(key * expn) * r
        d = d - 1j * (H @ r - r @ H)
        for k in range(K):
            m = mode[k]
            if key[k] > 0:
                km = key.copy(); km[k] -= 1
                rm = ddos[gen_hash_value(km, comb)]
                d = d - 1j * np.sqrt(key[k]) / np.sqrt(etaa[k]) * (etal[k] * Q[m] @ rm - etar[k] * rm @ Q[m])
            if key.sum() < L:
                kp = key.copy(); kp[k] += 1
                rp = ddos[gen_hash_value(kp, comb)]
                d = d - 1j * np.sqrt(key[k] + 1) * np.sqrt(etaa[k]) * (Q[m] @ rp - rp @ Q[m])
        dot[n] = d
    return dot


def run(H, Hdip, fs, Q, Qdip, fc, bath, L, rho0, dt, nt, p1=None, mode=None):
    """DEOMSolver.run: returns (t_save, saved) with saved = Tr(p1 rho_0) (p1 given) or rho_0 copies."""
    etal, etar, etaa, expn = (np.asarray(x, complex) for x in bath)
    K = len(expn)
    mode = np.zeros(K, dtype=int) if mode is None else np.asarray(mode)
    keys, comb = gen_keys(L, K)
    nsys = H.shape[0]
    ddos = np.zeros((len(keys), nsys, nsys), dtype=complex)
    ddos[0] = rho0
    Q = np.asarray(Q, complex)
    Qdip = np.asarray(Qdip, complex)

    def at(t):
        return H + Hdip * fs(t), np.array([Q[i] + Qdip[i] * fc(t) for i in range(len(Q))])

    def rhs(x, t):
        Ht, Qt = at(t)
        return rem_cal(x, keys, comb, L, expn, etal, etar, etaa, mode, Ht, Qt)

    t_save = np.zeros(nt + 1)
    saved = [np.trace(p1 @ ddos[0]) if p1 is not None else ddos[0].copy()]
    for i in range(nt):
        t = i * dt
        k1 = rhs(ddos, t)
        k2 = rhs(ddos + k1 * dt / 2, t + dt / 2)
        acc = k1 + k2 * 2
        k3 = rhs(ddos + k2 * dt / 2, t + dt / 2)
        acc = acc + k3 * 2
        k4 = rhs(ddos + k3 * dt, t + dt)
        acc = acc + k4
        ddos = ddos + acc * dt / 6
        t_save[i + 1] = (i + 1) * dt
        saved.append(np.trace(p1 @ ddos[0]) if p1 is not None else ddos[0].copy())
    return t_save, np.array(saved), ddos


def _idx(iado, i, j, ns):
    return iado * ns * ns + i * ns + j                       # gen_index2 (:769-771)


def propagator(keys, comb, L, expn, etal, etar, etaa, mode, H, Q):
    """generate_propgator (:856-882): dense P with P vec(ddos) = rem_cal, element by element."""
    nmax, K = keys.shape
    ns = H.shape[0]
    P = np.zeros((nmax * ns * ns, nmax * ns * ns), dtype=complex)
    for a in range(nmax):
        key = keys[a]
        for i in range(ns):
            for j in range(ns):
                P[_idx(a, i, j, ns), _idx(a, i, j, ns)] -= np.sum(key * expn)
        for i in range(ns):
            for j in range(ns):
                if np.abs(H[i, j]) > 1e-10:                       # allcator_H (:774-782)
                    for k in range(ns):
                        P[_idx(a, i, k, ns), _idx(a, j, k, ns)] -= 1j * H[i, j]
                        P[_idx(a, k, j, ns), _idx(a, k, i, ns)] += 1j * H[i, j]
        for mp in range(K):
            n, q = key[mp], Q[mode[mp]]
            if n > 0:                                             # allcator_Q_m (:799-810)
                km = key.copy(); km[mp] -= 1
                pos = gen_hash_value(km, comb)
                for i in range(ns):
                    for j in range(ns):
                        for k in range(ns):
                            P[_idx(a, i, k, ns), _idx(pos, j, k, ns)] -= \
                                1j * np.sqrt(n) / np.sqrt(etaa[mp]) * etal[mp] * q[i, j]
                            P[_idx(a, k, j, ns), _idx(pos, k, i, ns)] += \
                                1j * np.sqrt(n) / np.sqrt(etaa[mp]) * etar[mp] * q[i, j]
            if key.sum() < L:                                     # allcator_Q_p (:813-823)
                kp = key.copy(); kp[mp] += 1
                pos = gen_hash_value(kp, comb)
                for i in range(ns):
                    for j in range(ns):
                        for k in range(ns):
                            P[_idx(a, i, k, ns), _idx(pos, j, k, ns)] -= 1j * np.sqrt(n + 1) * np.sqrt(etaa[mp]) * q[i, j]
                            P[_idx(a, k, j, ns), _idx(pos, k, i, ns)] += 1j * np.sqrt(n + 1) * np.sqrt(etaa[mp]) * q[i, j]
    return P


def actions(A, nmax, lcr):
    """generate_actions (:885-892) / actions_element (:826-838)."""
    ns = A.shape[0]
    X = np.zeros((nmax * ns * ns, nmax * ns * ns), dtype=complex)
    for a in range(nmax):
        for i in range(ns):
            for j in range(ns):
                if np.abs(A[i, j]) > 1e-10:
                    for k in range(ns):
                        if lcr in ('l', 'c'):
                            X[_idx(a, i, k, ns), _idx(a, j, k, ns)] += A[i, j]
                        if lcr in ('r', 'c'):
                            X[_idx(a, k, j, ns), _idx(a, k, i, ns)] += A[i, j]
    return X


def correlation_4op_3t(P, nmax, ns, ops, rho0, T, w_x, w_y, if_full=True, cut_off_min=0.5, cut_off_max=1.1,
                       lcr='llll'):
    """DEOMSolver.correlation_4op_3t (:1127-1209) with ops = (a, b, c, d), evaluated as the reference does:
    one trace per (w_x, w_y) point."""
    import scipy.linalg as la
    lam, V = la.eig(P)
    Vi = la.pinv(V)
    a, b, c, d = ops
    A1, A2, A3, A4 = actions(d, nmax, lcr[3]), actions(c, nmax, lcr[2]), actions(b, nmax, lcr[1]), \
        actions(a, nmax, lcr[0])
    rho = np.zeros((nmax * ns * ns, 1), dtype=complex)
    rho[:ns * ns, 0] = np.asarray(rho0).flatten()
    if not if_full:
        lo, hi = np.min(np.real(lam)) * cut_off_min, np.max(np.real(lam)) * cut_off_max
        sel = (np.real(lam) > lo) & (np.real(lam) < hi)
        V, Vi, lam = V[:, sel], Vi[sel, :], lam[sel]
    A1V = A1 @ V
    G = (Vi @ A2 @ V) @ (np.diag(np.exp(lam * T)) @ (Vi @ A3 @ V))
    VA4 = Vi @ (A4 @ rho)
    cw = np.zeros((len(w_x), len(w_y)), dtype=complex)
    for i in range(len(w_x)):
        for j in range(len(w_y)):
            y = A1V @ ((1 / (-lam - 1j * w_x[i])).reshape(-1, 1) * (G @ ((1 / (-lam - 1j * w_y[j])).reshape(-1, 1) * VA4)))
            cw[i, j] = np.trace(y[:ns * ns, 0].reshape(ns, ns))
    return cw


def band_rhs(x_loc, n_own, minus, plus, coef, damp, mode, H, Q):
    """rem_cal (:641-673) for the owned rows of a band with precomputed prefactors: x_loc [n_loc, ns, ns] holds the
    owned rows then the halo rows, minus / plus [n_own, K] local rows (-1 absent), coef [n_own, K, 3] =
    (cL, cR, cP) = (-i sqrt(n_k) etal_k / sqrt(etaa_k), +i sqrt(n_k) etar_k / sqrt(etaa_k), -i sqrt(n_k + 1)
    sqrt(etaa_k)), damp [n_own] = -sum_k n_k expn_k."""
    K = minus.shape[1]
    d = np.empty((n_own,) + x_loc.shape[1:], dtype=complex)
    for n in range(n_own):
        r = x_loc[n]
        v = damp[n] * r - 1j * (H @ r - r @ H)
        for k in range(K):
            q = Q[mode[k]]
            if minus[n, k] >= 0:
                y = x_loc[minus[n, k]]
                v = v + coef[n, k, 0] * (q @ y) + coef[n, k, 1] * (y @ q)
            if plus[n, k] >= 0:
                y = x_loc[plus[n, k]]
                v = v + coef[n, k, 2] * (q @ y - y @ q)
        d[n] = v
    return d
