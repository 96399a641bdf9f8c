"""NumPy restatement of the DEOM/HEOM hierarchy propagation (test infrastructure only).

Follows pyqed/heom/deom.py:
  :1048-1064  init_      Pascal table comb_list, nmax = comb[L+K, L]
  :555-566    gen_hash_value(key) = sum_i comb[S_i + i, i + 1], S_i = key[0] + ... + key[i]
  :609-638    gen_keys / gen_keys_element (tier-by-tier expansion, keys[hash] = key)
  :641-673    generate_dot_element / rem_cal (the ADO stencil)
  :676-688    generate_time (H(t) = H + Hdip f(t), Q(t) = Q + Qdip g(t))
  :725-766    rk4 (stages at t, t+dt/2, t+dt/2, t+dt)
  :1072-1114  DEOMSolver.run (t_save, Tr(p1 rho_0) or rho_0 per step)
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
