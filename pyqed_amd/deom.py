"""DEOM / HEOM hierarchy on MI355X (drop-in for pyqed/heom/deom.py Bath, DEOMSolver).

Host (setup, as the reference): Pade decomposition of the bath correlation
function (sympy), the graded ADO index and its neighbour tables.  Propagation:
libqdyn qd_deom_rk4 (one kernel launch per RK4 stage).
"""
from __future__ import annotations

import functools
import math
import os

import numpy as np
import torch

from . import _lib
from ._util import default_device, to_numpy


# --------------------------------------------------------------------------- bath
def _tridiag_eigs_desc(offdiag, size):
    m = np.diag(offdiag, -1) + np.diag(offdiag, 1) if size > 1 else np.zeros((1, 1))
    return np.sort(np.linalg.eigvalsh(m))[::-1]


def matsubara_approximation_distribution(N, BoseFermi=1):
    """Matsubara poles/residues (heom/deom.py:84-101)."""
    if BoseFermi == 1:
        return np.array([2 * (i + 1) * np.pi for i in range(N)]), np.ones(N)
    return np.array([(2 * i + 1) * np.pi for i in range(N)]), np.ones(N)


def pade_approximation_distribution(N, BoseFermi=1, pade=1):
    """[N-1/N] (pade=1) or [N/N] (pade=2) Pade spectrum decomposition of the Bose/Fermi
    function (Hu, Xu, Yan, JCP 133, 101106 (2010)); same poles/residues as heom/deom.py:104-206.

    Poles xi_j = 2/eps_j from the N largest eigenvalues of the tridiagonal matrix with
    off-diagonals 1/sqrt((a+2i)(a+2i+2)), a = 3 (Bose) or 1 (Fermi); zeta from the second
    matrix (a+2); residue_j = (s/2) prod_k (zeta_k^2 - xi_j^2) / prod_{k != j} (xi_k^2 - xi_j^2).
    """
    if N < 0 or BoseFermi not in (1, 2) or pade not in (0, 1, 2, 3):
        raise ValueError("N or BoseFermi or pade has wrong value!")
    if pade == 0:
        return matsubara_approximation_distribution(N, BoseFermi)
    if pade == 3:
        return _extended_psd(N, BoseFermi)
    if N == 0:
        return [], []
    M = 2 * N + pade // 2
    a = 3.0 if BoseFermi == 1 else 1.0
    off = np.array([1.0 / math.sqrt((a + 2.0 * i) * (a + 2.0 * i + 2.0)) for i in range(M - 1)])
    xi = 2.0 / _tridiag_eigs_desc(off, M)[:N]
    xi2 = xi * xi
    M2 = M - 1
    a2 = a + 2.0
    off2 = np.array([1.0 / math.sqrt((a2 + 2.0 * i) * (a2 + 2.0 * i + 2.0)) for i in range(M2 - 1)])
    nz = M2 // 2
    zeta2 = (2.0 / _tridiag_eigs_desc(off2, M2)[:nz]) ** 2
    if BoseFermi == 1:
        s = N * (2.0 * N + 3.0) if pade == 1 else 1.0 / (4.0 * (N + 1.0) * (2.0 * N + 3.0))
    else:
        s = N * (2.0 * N + 1.0) if pade == 1 else 1.0 / (4.0 * (N + 1.0) * (2.0 * N + 1.0))
    resi = np.zeros(N)
    for j in range(N):
        num = np.prod([zeta2[k] - xi2[j] for k in range(nz)]) if nz else 1.0
        den = np.prod([xi2[k] - xi2[j] for k in range(N) if k != j]) if N > 1 else 1.0
        resi[j] = 0.5 * s * num / den
    return xi, resi


def _extended_psd(N, BoseFermi):
    """Extended [N/N] Pade spectrum decomposition (pade=3; heom/deom.py:163-206; Hu, Xu, Yan, JCP 134,
    244106 (2011)): the Bose/Fermi function as a continued fraction whose 2N+2 coefficients d_k are closed
    forms in k.  Poles xi_j = 2 / eps_j from the N largest eigenvalues of the symmetric tridiagonal matrix with
    off-diagonals 1/sqrt(d_{k+1} d_{k+2}), k < 2N; the residue at xi_j is the last term of the three-term
    recurrence that evaluates the continued fraction's numerator at z^2 = xi_j^2, with the partial fractions
    scaled so that the recurrence stays bounded (factor t_i / (xi_i^2 - xi_j^2), t_i the ratio of consecutive
    partial sums of the odd coefficients)."""
    a = 3.0 if BoseFermi == 1 else 1.0
    n1 = N + 1
    i = np.arange(1, n1, dtype=float)
    d = np.empty(2 * n1)
    d[0] = 0.25 / a
    d[1:2 * n1 - 1:2] = -4.0 * i * i * (a + 2.0 * i - 2.0) ** 2 * (a + 4.0 * i - 2.0)
    d[2:2 * n1 - 1:2] = -0.25 * (a + 4.0 * i) / (i * (i + 1.0) * (a + 2.0 * i - 2.0) * (a + 2.0 * i))
    d[-1] = -4.0 * (N + 1.0) ** 2 * (a + 2.0 * N) ** 2 * (a + 4.0 * N + 2.0)
    odd_cum = np.cumsum(d[1::2])  # sum_{k <= i} d_{2k+1}, i = 0 .. N
    M = 2 * N + 1
    off = 1.0 / np.sqrt(d[1:M] * d[2:M + 1])
    xi = 2.0 / _tridiag_eigs_desc(off, M)[:N]
    xi2 = xi * xi
    resi = np.zeros(N)
    for j in range(N):
        z2 = xi2[j]
        prev2, prev1 = 0.0, 0.5  # eta_{-1}, eta_0
        r_prev = 0.0
        t = 0.25 / d[1]
        for k in range(n1):
            q = t if (k == j or k == N) else t / (xi2[k] - z2)
            g = 2.0 * math.sqrt(abs(q))   # magnitude factor of the even coefficient
            h = g if q > 0 else -g        # signed factor of the odd coefficient
            e_even = d[2 * k] * g * prev1 - 0.25 * g * r_prev * z2 * prev2
            e_odd = d[2 * k + 1] * h * e_even - 0.25 * h * g * z2 * prev1
            prev2, prev1 = e_even, e_odd
            r_prev = h
            if k != N:
                t = odd_cum[k] / odd_cum[k + 1]
        resi[j] = prev1
    return xi, resi


def function_bose(x, pole, resi):
    """Pade-approximated Bose function x n(x) / ... (heom/deom.py:67-72)."""
    return 1 / x + 0.5 + sum(2.0 * resi[i] * x / (x ** 2 + pole[i] ** 2) for i in range(len(pole)))


def decompose_spectrum_pade(spe, w_sp, beta, npsd, pade=1, bose_fermi=1):
    """Bath correlation as a sum of exponentials (heom/deom.py:226-307): (etal, etar, etaa, expn).

    Poles of the spectral density in the lower half plane give the 'physical' exponents
    expn = i*pole (sorted by |Im| descending; complex pairs first, then real ones), each
    weighted by its residue times the Pade Bose function; the npsd Pade poles of the Bose
    function give the remaining exponents pole*T."""
    import sympy as sp
    re_part, im_part = sp.cancel(spe).as_real_imag()
    part = re_part if im_part == 0 else im_part
    numer, denom = sp.cancel(sp.factor(part)).as_numer_denom()
    roots = np.array([complex(z) for z in sp.nroots(denom)])
    expn = np.array([1j * z for z in roots if z.imag < 0])
    order = np.argsort(np.abs(np.imag(expn)))[::-1]
    mag = np.sort(np.abs(np.imag(expn)))[::-1]
    cc = expn[order[mag != 0]]
    real = expn[order[mag == 0]]
    expn_all = list(expn[order])
    pole, resi = pade_approximation_distribution(npsd, bose_fermi, pade)
    T = 1.0 / beta
    num_f = sp.lambdify(w_sp, numer, "numpy")

    def residue_weight(x):
        w = -1j * x
        others = roots[np.abs(roots + 1j * x) > 1e-14]
        val = -2j * complex(num_f(w)) / np.prod(w - others)
        return complex(val * function_bose(-1j * x / T, pole, resi))

    etal, etar, etaa = [], [], []
    for ii in range(0, len(cc), 2):
        e0, e1 = residue_weight(cc[ii]), residue_weight(cc[ii + 1])
        etal += [e0, e1]
        etar += [np.conj(e1), np.conj(e0)]
        etaa += [np.sqrt(abs(e0) * abs(np.conj(e1))), np.sqrt(abs(e1) * abs(np.conj(e0)))]
    for x in real:
        e = residue_weight(x)
        etal.append(e)
        etar.append(np.conj(e))
        etaa.append(np.sqrt(abs(e) * abs(np.conj(e))))
    for j in range(len(pole)):
        z = -1j * pole[j] * T
        fz = complex(num_f(z)) / np.prod(z - roots)
        expn_all.append(pole[j] * T)
        e = -2j * resi[j] * T * fz
        etal.append(e)
        etar.append(np.conj(e))
        etaa.append(abs(e))
    return np.array(etal), np.array(etar), np.array(etaa), np.array(expn_all)


class Bath:
    """Drop-in for pyqed.heom.deom.Bath (heom/deom.py:895-942), list form:
    Bath([spe_1, ...], w_sp, [beta_1, ...], [npsd_1, ...], mode, function)."""

    def __init__(self, spectrum_sp=None, w_sp=None, beta=None, npsd=None, mode=None, function=None):
        self.bath = spectrum_sp
        self.w_sp = w_sp
        self.beta = beta
        self.npsd = npsd
        self.mode = mode
        if isinstance(self.bath, list) and isinstance(self.beta, list) and isinstance(self.npsd, list):
            if function is None:
                function = [decompose_spectrum_pade] * len(self.bath)
            parts = [function[i](self.bath[i], self.w_sp, self.beta[i], self.npsd[i]) for i in range(len(self.bath))]
            self.etal, self.etar, self.etaa, self.expn = (
                np.concatenate([np.asarray(p[c], dtype=np.complex128) for p in parts]) for c in range(4))
            if self.mode is None:
                raise ValueError("mode is not set!")
            if len(self.mode) != len(self.expn):
                raise ValueError("the length of mode is not equal to the number of dissipatons!")
            self.mode = np.asarray(self.mode, dtype=np.int64)
        else:
            self.etal, self.etar, self.etaa, self.expn = decompose_spectrum_pade(self.bath, self.w_sp, self.beta,
                                                                                 self.npsd)
            self.mode = np.zeros_like(self.expn, dtype=np.int64)


# --------------------------------------------------------------------------- ADO index
def comb_table(L, K):
    n = K + L + 1
    c = np.zeros((n, n), dtype=np.int64)
    c[:, 0] = 1
    for i in range(1, n):
        c[i, 1:] = c[i - 1, 1:] + c[i - 1, :-1]
    return c


def ado_hash(keys, comb):
    """heom/deom.py:555-566 vectorised: h = sum_i comb[S_i + i, i + 1], S = cumsum(key)."""
    keys = np.atleast_2d(keys)
    S = np.cumsum(keys, axis=1)
    idx = np.arange(keys.shape[1])
    return comb[S + idx, idx + 1].sum(axis=1)


def ado_tables(L, K):
    """(keys [nmax, K] int64 bit-identical to gen_keys, minus/plus [nmax, K] int32, comb).  Built once per (L, K)
    per process (the reference rebuilds them in every run's init_; they are a function of L and K only), returned as
    copies."""
    return tuple(a.copy() for a in _ado_tables_cached(int(L), int(K)))


@functools.lru_cache(maxsize=16)
def _ado_tables_cached(L, K):
    comb = comb_table(L, K)
    nmax = int(comb[L + K, L])
    tier = np.zeros((1, K), dtype=np.int64)
    keys = np.zeros((nmax, K), dtype=np.int64)
    for _ in range(L):
        keys[ado_hash(tier, comb)] = tier
        tier = np.unique((tier[:, None, :] + np.eye(K, dtype=np.int64)[None]).reshape(-1, K), axis=0)
    keys[ado_hash(tier, comb)] = tier
    tiers = keys.sum(axis=1)
    eye = np.eye(K, dtype=np.int64)
    minus = np.full((nmax, K), -1, dtype=np.int32)
    plus = np.full((nmax, K), -1, dtype=np.int32)
    for k in range(K):
        has = keys[:, k] > 0
        minus[has, k] = ado_hash(keys[has] - eye[k], comb)
        up = tiers < L
        plus[up, k] = ado_hash(keys[up] + eye[k], comb)
    return keys, minus, plus, comb


def ado_coefficients(keys, etal, etar, etaa, expn, L):
    """Per-(ADO, dissipaton) prefactors of generate_dot_element (heom/deom.py:641-664)."""
    n = keys.astype(float)
    sq_e = np.sqrt(np.asarray(etaa, dtype=complex))
    cm = 1j * np.sqrt(n) / sq_e[None, :]
    coef = np.empty(keys.shape + (3,), dtype=complex)
    coef[..., 0] = -cm * etal[None, :]
    coef[..., 1] = cm * etar[None, :]
    coef[..., 2] = -1j * np.sqrt(n + 1) * sq_e[None, :]
    damp = -np.sum(keys * np.asarray(expn)[None, :], axis=1)
    return coef, damp


# --------------------------------------------------------------------------- ADO Liouvillian
def _thresh(A, tol=1e-10):
    """Elements with |A_ij| <= 1e-10 are skipped by the reference's assembly (allcator_H / actions_element)."""
    A = np.asarray(A, dtype=complex)
    return np.where(np.abs(A) > tol, A, 0)


def ado_liouvillian(keys, minus, plus, coef, damp, H, Q, mode):
    """Dense ADO-space generator P, (nmax ns^2)^2, with P vec(ados) = rem_cal (generate_propgator,
    heom/deom.py:769-893): index (ado, i, j) -> ado ns^2 + i ns + j.  Per ADO block:
      diag:  damp_n I - i (H (x) I) + i (I (x) H^T)                    (allcator_H, |H_ij| > 1e-10)
      n-e_k: coef0 (Q_m (x) I) + coef1 (I (x) Q_m^T)                    (allcator_Q_m)
      n+e_k: coef2 ((Q_m (x) I) - (I (x) Q_m^T))                        (allcator_Q_p)
    Host setup (like the reference); vectorised over ADOs instead of its per-element loops."""
    nmax, K = keys.shape
    ns = H.shape[0]
    n2 = ns * ns
    I = np.eye(ns)
    Ht = _thresh(H)
    P4 = np.zeros((nmax, n2, nmax, n2), dtype=complex)
    ar = np.arange(nmax)
    blkH = -1j * np.kron(Ht, I) + 1j * np.kron(I, Ht.T)
    P4[ar, :, ar, :] += damp[:, None, None] * np.eye(n2)[None] + blkH[None]
    Q = np.asarray(Q, dtype=complex).reshape(-1, ns, ns)
    for k in range(K):
        q = Q[mode[k]]
        ql, qr = np.kron(q, I), np.kron(I, q.T)
        has = minus[:, k] >= 0
        a = ar[has]
        P4[a, :, minus[has, k], :] += coef[has, k, 0][:, None, None] * ql[None] + coef[has, k, 1][:, None, None] * qr[None]
        up = plus[:, k] >= 0
        a = ar[up]
        P4[a, :, plus[up, k], :] += coef[up, k, 2][:, None, None] * (ql - qr)[None]
    return P4.reshape(nmax * n2, nmax * n2)


def _action_block(A, lcr):
    """One ADO block of generate_actions (heom/deom.py:830-846, 885-892): 'l' A rho, 'r' rho A, 'c' both."""
    At = _thresh(A)
    ns = At.shape[0]
    I = np.eye(ns)
    blk = np.zeros((ns * ns, ns * ns), dtype=complex)
    if lcr in ('l', 'c'):
        blk += np.kron(At, I)
    if lcr in ('r', 'c'):
        blk += np.kron(I, At.T)
    return blk


# --------------------------------------------------------------------------- solver
BANDS_MAX = 256   # one workgroup per CU at most (the bands must be co-resident)
# correlation_4op_3t(if_full=True) runs the Krylov form (deom_krylov.py) from this ADO-space dimension nmax ns^2 on:
# the host eig of P is O(n^3) (n = 1024: seconds; the bench hierarchy's 24,752: beyond the reference itself)
KRYLOV_MIN_DIM = 1024


class _BandTables:
    """Device copies of the tier-band partition (deom_shard.make_plans) in qd_deom_rk4_banded's layout."""

    def __init__(self, plans, dev, max_own, max_loc):
        i32 = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.int32))).to(dev)
        self.nbands, self.max_own, self.max_loc = len(plans), max_own, max_loc
        self.band_lo = i32([p.lo for p in plans] + [plans[-1].hi])
        self.halo_off = i32(np.concatenate([[0], np.cumsum([len(p.halo) for p in plans])]))
        halo = np.concatenate([p.halo for p in plans]) if self.halo_off[-1].item() else np.zeros(1)
        self.halo_idx = i32(halo)
        srcs = [sorted(p.recv) for p in plans]
        self.src_off = i32(np.concatenate([[0], np.cumsum([len(s) for s in srcs])]))
        self.src = i32(np.concatenate([np.asarray(s, dtype=np.int64) for s in srcs]) if sum(map(len, srcs)) else
                       np.zeros(1))
        self.lminus = i32(np.concatenate([p.minus for p in plans]))
        self.lplus = i32(np.concatenate([p.plus for p in plans]))

    def args(self):
        """lminus, lplus, band_lo, halo_off, halo_idx, src_off, src, nbands, max_own, max_loc."""
        return (self.lminus.data_ptr(), self.lplus.data_ptr(), self.band_lo.data_ptr(), self.halo_off.data_ptr(),
                self.halo_idx.data_ptr(), self.src_off.data_ptr(), self.src.data_ptr(), self.nbands, self.max_own,
                self.max_loc)


class DEOMSolver:
    """Drop-in for pyqed.heom.deom.DEOMSolver (heom/deom.py:953-1125)."""

    def __init__(self, system=None, system_dipole=None, bath=None, coupling=None, coupling_dipole=None,
                 pulse_system_func=None, pulse_coupling_func=None, lmax=None):
        self.system = system
        self.system_dipole = system_dipole
        self.coupling = coupling
        self.coupling_dipole = coupling_dipole
        self.pulse_system_func = pulse_system_func
        self.pulse_coupling_func = pulse_coupling_func
        self.lmax = lmax
        self.nsys = 0
        self.nmax = 1
        self.nind = 0
        self.nmod = 0
        self.bath = bath
        self.comb_list = []
        self.keys = None
        self.ddos = None
        self.Δ = None
        self.V = None
        self.V_inv = None
        self.propgator = None
        # extensions (not in the reference): run_batch's ADO layout ("ado_major" / "element_major"; None = by batch
        # size), the one-hierarchy banded launch (False = the stage launches; None = where it applies) and its band
        # count (None = by hierarchy size, band_tables)
        self.layout = None
        self.banded = None
        self.bands = None
        # correlation_4op_3t's method: None = the eigen form (as the reference) below KRYLOV_MIN_DIM, the Krylov form
        # above; "eig" / "krylov" force one (last_corr4 records what ran)
        self.corr4_method = None
        self.last_corr4 = None

    def set_hierarchy(self, lmax):
        self.lmax = lmax

    def set_system(self, system):
        self.system = np.array(system, dtype=np.complex128)

    def set_system_dipole(self, system_dipole):
        self.system_dipole = np.array(system_dipole, dtype=np.complex128)

    def set_coupling(self, coupling):
        self.coupling = np.array(coupling, dtype=np.complex128)

    def set_coupling_dipole(self, coupling_dipole):
        self.coupling_dipole = np.array(coupling_dipole, dtype=np.complex128)

    def set_pulse_system_func(self, f):
        self.pulse_system_func = f

    def set_pulse_coupling_func(self, f):
        self.pulse_coupling_func = f

    def check_(self):
        if self.system is None:
            raise ValueError('System Hamiltonian is not set.')
        if self.coupling is None:
            raise ValueError('system bath interaction operator is not set.')
        self.nsys = np.shape(self.system)[0]
        self.nind = len(self.bath.expn)
        self.nmod = int(np.max(self.bath.mode)) + 1

    def init_(self):
        keys, minus, plus, comb = ado_tables(self.lmax, self.nind)
        self.keys, self._minus, self._plus, self.comb_list = keys, minus, plus, comb
        self.nmax = len(keys)

    @staticmethod
    def _dip_values(dip, func, nt, dt, shape):
        if dip is None or func is None or not np.any(np.asarray(dip)):
            return None, None
        f = np.empty((nt, 3), dtype=complex)
        for s in range(nt):
            t = s * dt
            f[s] = [func(t), func(t + dt / 2), func(t + dt)]
        return np.asarray(dip, dtype=complex).reshape(shape), f

    def run(self, rho0, dt, nt, p1=None):
        """heom/deom.py:1072-1114: returns (t_save (nt+1,), ddos_save) with ddos_save the
        Tr(p1 rho_0) values (p1 given) or the list of rho_0 copies.  As in the reference,
        a complex ndarray rho0 is overwritten with the final system density matrix."""
        self.check_()
        self.init_()
        out = self.run_batch(np.asarray(rho0)[None], dt, nt, p1)
        t_save, saved = out
        saved = saved[0]
        if isinstance(rho0, np.ndarray) and np.iscomplexobj(rho0) and rho0.flags.writeable:
            rho0[...] = self.ddos[0][0]
        self.ddos = self.ddos[0]
        if p1 is None:
            return t_save, [saved[k] for k in range(nt + 1)]
        return t_save, saved

    def run_batch(self, rho0, dt, nt, p1=None):
        """Extension: B independent hierarchies (rho0 [B, ns, ns]) in one launch sequence."""
        if self.keys is None:
            self.check_()
            self.init_()
        dev = default_device()
        _lib.ensure_device(dev)
        ns, K, nmax = self.nsys, self.nind, self.nmax
        rho0 = np.asarray(rho0, dtype=complex)
        B = rho0.shape[0]
        b = self.bath
        c128 = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=complex))).to(dev)
        # batches of >= 16 hierarchies run ADO-major ([nmax][B]: coalesced neighbour reads across
        # hierarchies, wave-uniform index / prefactor loads); self.layout picks the layout explicitly
        if self.layout not in (None, "ado_major", "element_major"):
            raise ValueError(f"DEOMSolver.layout must be None, 'ado_major' or 'element_major', got {self.layout!r}")
        want_am = B >= 16 if self.layout is None else self.layout == "ado_major"
        ado_major = want_am and ns * ns <= 64 and K <= 8
        if ado_major:
            ados = torch.zeros((nmax, B, ns, ns), dtype=torch.complex128, device=dev)
            ados[0] = c128(rho0)
        else:
            ados = torch.zeros((B, nmax, ns, ns), dtype=torch.complex128, device=dev)
            ados[:, 0] = c128(rho0)
        H = c128(self.system)
        Q = c128(np.asarray(self.coupling, dtype=complex).reshape(-1, ns, ns))
        nmod = Q.shape[0]
        Hdip, fs = self._dip_values(self.system_dipole, self.pulse_system_func, nt, dt, (ns, ns))
        Qdip, fc = self._dip_values(self.coupling_dipole, self.pulse_coupling_func, nt, dt, (nmod, ns, ns))
        Hdip_t = c128(Hdip) if Hdip is not None else None
        Qdip_t = c128(Qdip) if Qdip is not None else None
        fs = np.ascontiguousarray(fs) if fs is not None else None
        fc = np.ascontiguousarray(fc) if fc is not None else None
        rho_sys = torch.empty((B, nt + 1, ns, ns), dtype=torch.complex128, device=dev)
        p1_t = c128(np.asarray(p1, dtype=complex).reshape(1, ns, ns)) if p1 is not None else None
        trace = torch.empty((B, nt + 1, 1), dtype=torch.complex128, device=dev) if p1 is not None else None
        tabs = self.device_tables(dev)
        bands = self.band_tables(dev) if B == 1 else None
        self.last_run_banded = False
        if bands is not None:
            # The bands wait on each other inside one launch: if the device cannot hold them all at once
            # (QD_EBUSY from the cooperative launch, nothing ran) or a hand-off timed out (status, e.g. work on
            # another stream delayed a band; ados was overwritten), the run is repeated on the stage launches,
            # which need no co-residency and give the same results (bit-identical with one band, within 1e-13
            # with several: the halo hand-off tags, qdyn.h).
            ados0 = ados.clone()
            status = torch.zeros(1, dtype=torch.int32, device=dev)
            with torch.cuda.device(dev):
                rc = _lib.load().qd_deom_rk4_banded(
                    ados.data_ptr(), nmax, K, ns, *bands.args(), tabs[2].data_ptr(), tabs[3].data_ptr(),
                    tabs[4].data_ptr(), nmod, H.data_ptr(), _lib.ptr(Hdip_t), Q.data_ptr(), _lib.ptr(Qdip_t),
                    fs.ctypes.data if fs is not None else None, fc.ctypes.data if fc is not None else None, float(dt),
                    int(nt), rho_sys.data_ptr(), _lib.ptr(p1_t), 1 if p1 is not None else 0, _lib.ptr(trace),
                    status.data_ptr(), _lib.stream_ptr(dev))
            if rc != _lib.QD_EBUSY:
                _lib.check(rc, "qd_deom_rk4_banded")
            if rc == _lib.QD_EBUSY or int(status.item()) != 0:
                import warnings
                warnings.warn("qd_deom_rk4_banded: " + ("bands cannot be co-resident" if rc else
                                                         "a band hand-off timed out") +
                              "; re-running on the stage launches", RuntimeWarning)
                ados.copy_(ados0)
                bands = None
            else:
                self.last_run_banded = True
        if bands is None:
            with torch.cuda.device(dev):
                rc = getattr(_lib.load(), "qd_deom_rk4_ado_major" if ado_major else "qd_deom_rk4")(
                    ados.data_ptr(), B, nmax, K, ns, tabs[0].data_ptr(), tabs[1].data_ptr(), tabs[2].data_ptr(),
                    tabs[3].data_ptr(), tabs[4].data_ptr(), nmod, H.data_ptr(), _lib.ptr(Hdip_t), Q.data_ptr(),
                    _lib.ptr(Qdip_t), fs.ctypes.data if fs is not None else None,
                    fc.ctypes.data if fc is not None else None, float(dt), int(nt), rho_sys.data_ptr(),
                    _lib.ptr(p1_t), 1 if p1 is not None else 0, _lib.ptr(trace), _lib.stream_ptr(dev))
            _lib.check(rc, "qd_deom_rk4_ado_major" if ado_major else "qd_deom_rk4")
        torch.cuda.synchronize(dev)
        self.ddos = (ados.transpose(0, 1) if ado_major else ados).cpu().numpy()   # [B][nmax][ns][ns]
        t_save = np.arange(nt + 1) * dt
        t_save[0] = 0
        if p1 is not None:
            return t_save, trace[..., 0].cpu().numpy()
        return t_save, rho_sys.cpu().numpy()

    def device_tables(self, dev):
        """(minus, plus, coef, damp, mode) of the hierarchy on `dev`, cached per (device, L, K, bath) so that repeated
        runs upload them once."""
        b = self.bath
        key = (str(dev), self.lmax, self.nind) + tuple(np.asarray(x).tobytes() for x in
                                                         (b.etal, b.etar, b.etaa, b.expn, b.mode))
        cache = getattr(self, "_dev_tab_cache", None)
        if cache is not None and cache[0] == key:
            return cache[1]
        coef, damp = ado_coefficients(self.keys, np.asarray(b.etal), np.asarray(b.etar), np.asarray(b.etaa),
                                      np.asarray(b.expn), self.lmax)
        c128 = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=complex))).to(dev)
        i32 = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.int32))).to(dev)
        tabs = (i32(self._minus), i32(self._plus), c128(coef), c128(damp), i32(b.mode))
        self._dev_tab_cache = (key, tabs)
        return tabs

    def band_tables(self, dev, nbands=None):
        """Band tables of qd_deom_rk4_banded (one hierarchy as one persistent launch over tier bands), or None
        when the hierarchy does not qualify (ns outside [2, 4], K > 8, rows beyond one workgroup's lanes / LDS)
        or self.banded is False.  Default band count: ~24 ADOs per band (ns = 2; 8 for ns = 3, 4), at most one band
        per CU (the bands must be co-resident); hierarchies that would then need more than 80 (20) rows per band
        stay on the stage launches.  Measured at 6188 ADOs: 256 bands 94.7k steps/s against 51.7k for the stage
        launches; 18,564 ADOs on 256 bands 68k against 42.1k (tools/deom_band_sweep.py,
        profiles/r03/deom/band_sweep.txt).  self.bands sets the count.  Cached per (device, count)."""
        if self.banded is False:
            return None
        ns, K, nmax = self.nsys, self.nind, self.nmax
        if not (2 <= ns <= 4) or K > 8:
            return None
        G = 4 if ns == 2 else 16
        per, fat = (24, 80) if G == 4 else (8, 20)
        cap = min(BANDS_MAX, torch.cuda.get_device_properties(dev).multi_processor_count)
        if nbands is None:
            if self.bands:
                nbands = int(self.bands)
            else:
                nbands = min(cap, max(1, -(-nmax // per)))
                if -(-nmax // nbands) > fat:   # fat bands lose to the stage launches (146 rows: 0.78x)
                    return None
        nbands = max(1, min(int(nbands), nmax, cap))
        nmod = int(np.max(self.bath.mode)) + 1
        # the keys are a function of (lmax, K); ns and nmod enter the eligibility checks below
        key = (str(dev), nbands, self.lmax, K, nmax, ns, nmod)
        cache = getattr(self, "_band_cache", None)
        if cache is not None and cache[0] == key:
            return cache[1]
        from .deom_shard import make_plans
        plans = make_plans(self._minus, self._plus, nbands)
        own = np.array([p.n_own for p in plans])
        loc = np.array([p.n_loc for p in plans])
        if own.max() * G > 1024 or (2 + nmod + loc.max()) * ns * ns * 16 > 160 * 1024 or \
                max(len(p.recv) for p in plans) > 64:
            return None
        tabs = _BandTables(plans, dev, int(own.max()), int(loc.max()))
        self._band_cache = (key, tabs)
        return tabs

    # ------------------------------------------------------------------ frequency-domain 2D signal
    def gen_generate_propgator(self):
        """heom/deom.py:1116-1125: the dense ADO Liouvillian (host assembly, ado_liouvillian)."""
        self.check_()
        self.init_()
        b = self.bath
        coef, damp = ado_coefficients(self.keys, np.asarray(b.etal), np.asarray(b.etar), np.asarray(b.etaa),
                                      np.asarray(b.expn), self.lmax)
        self.propgator = ado_liouvillian(self.keys, self._minus, self._plus, coef, damp,
                                         np.asarray(self.system, dtype=complex), self.coupling, np.asarray(b.mode))

    def correlation_4op_3t(self, operator_a, operator_b, operator_c, operator_d, rho0, T, w_x, w_y, if_full=True,
                           cut_off_min=0.5, cut_off_max=1.1, if_load=False, if_save=False, lcr='llll'):
        """heom/deom.py:1127-1209: c_w[i, j] = Tr_sys[A1 V r(w_x_i) (V^-1 A2 V) e^{Delta T} (V^-1 A3 V)
        r(w_y_j) V^-1 A4 rho], r(w) = diag(1 / (-Delta - i w)).

        Eigen form (as the reference; ADO dimension n = nmax ns^2 below KRYLOV_MIN_DIM, if_full=False, if_load,
        if_save): host P, eig + pinv, the O(n^3) basis changes; the (w_x, w_y) grid, which the reference evaluates
        with a matrix-vector trace per grid point, as two split-K MFMA GEMMs (qd_resolvent_grid2d).
        if_full=False keeps the eigenvalues with min(Re) * cut_off_min < Re < max(Re) * cut_off_max; if_load /
        if_save use correlation_4op_3t.npz.
        Krylov form (if_full=True from n = KRYLOV_MIN_DIM, e.g. the bench hierarchy's 24,752 whose dense P the
        reference cannot diagonalise): the same quantity u^T R(w_x) A2 e^{PT} A3 R(w_y) v with R(w) = (-P - i w)^-1
        from multi-shift Krylov solves of P and P^T on the GPU stencil kernel (pyqed_amd/deom_krylov.py); agrees with
        the eigen form to ~1e-12 (tests/test_deom_krylov_*.py).  self.corr4_method forces either."""
        import os
        import scipy.linalg as la
        self.check_()
        self.init_()
        n = self.nmax * self.nsys ** 2
        if self.corr4_method not in (None, "eig", "krylov"):
            raise ValueError(f"DEOMSolver.corr4_method must be None, 'eig' or 'krylov', got {self.corr4_method!r}")
        krylov_ok = if_full and not if_load and not if_save
        if self.corr4_method == "krylov" and not krylov_ok:
            raise ValueError("correlation_4op_3t: the Krylov form serves if_full=True without if_load / if_save "
                             "(the eigen cut and the eigendecomposition cache need P's eigenvectors)")
        if krylov_ok and (self.corr4_method == "krylov" or (self.corr4_method is None and n >= KRYLOV_MIN_DIM)):
            return self._corr4_krylov(operator_a, operator_b, operator_c, operator_d, rho0, T, w_x, w_y, lcr)
        self.last_corr4 = {"method": "eig", "n": n}
        if self.propgator is None:
            self.gen_generate_propgator()
        if if_load and os.path.exists('correlation_4op_3t.npz'):
            data = np.load('correlation_4op_3t.npz')
            self.Δ, self.V, self.V_inv = data['Δ'], data['V'], data['V_inv']
        if self.Δ is None:
            self.Δ, self.V = la.eig(self.propgator)
            self.V_inv = la.pinv(self.V)
        if if_save:
            np.savez('correlation_4op_3t.npz', Δ=self.Δ, V=self.V, V_inv=self.V_inv)
        ns, nmax = self.nsys, self.nmax
        n2 = ns * ns
        # actions1..4 of the reference: operator_d (lcr[3]) detects, operator_a (lcr[0]) acts first on rho
        A1, A2, A3, A4 = (_action_block(op, c) for op, c in
                          zip((operator_d, operator_c, operator_b, operator_a), (lcr[3], lcr[2], lcr[1], lcr[0])))
        lam, V, Vi = self.Δ, self.V, self.V_inv
        if not if_full:
            lo = np.min(np.real(lam)) * cut_off_min
            hi = np.max(np.real(lam)) * cut_off_max
            sel = (np.real(lam) > lo) & (np.real(lam) < hi)
            lam, V, Vi = lam[sel], V[:, sel], Vi[sel, :]

        def act(b, X):  # (I_nmax (x) b) @ X
            return np.einsum('xy,ayp->axp', b, X.reshape(nmax, n2, -1)).reshape(nmax * n2, -1)

        diag = np.arange(ns) * (ns + 1)
        a = (A1 @ V[:n2])[diag].sum(axis=0)                        # Tr_sys of the ADO-0 rows of actions1 @ V
        M = (Vi @ act(A2, V)) @ (np.exp(lam * T)[:, None] * (Vi @ act(A3, V)))
        v = Vi[:, :n2] @ (A4 @ np.asarray(rho0, dtype=complex).flatten())   # rho: ADO 0 only
        dev = default_device()
        _lib.ensure_device(dev)
        t = lambda x, dt=torch.complex128: torch.from_numpy(np.ascontiguousarray(x)).to(device=dev, dtype=dt)
        wx = np.asarray(w_x, dtype=float)
        wy = np.asarray(w_y, dtype=float)
        out = torch.empty((len(wx), len(wy)), dtype=torch.complex128, device=dev)
        args = [t(a), t(M), t(v), t(lam)]
        wxt, wyt = t(wx, torch.float64), t(wy, torch.float64)
        with torch.cuda.device(dev):
            rc = _lib.load().qd_resolvent_grid2d(*(x.data_ptr() for x in args), len(lam), wxt.data_ptr(), len(wx),
                                                 wyt.data_ptr(), len(wy), out.data_ptr(), _lib.stream_ptr(dev))
        _lib.check(rc, "qd_resolvent_grid2d")
        return out.cpu().numpy()

    def _corr4_krylov(self, operator_a, operator_b, operator_c, operator_d, rho0, T, w_x, w_y, lcr):
        """correlation_4op_3t(if_full=True) as u^T R(w_x) A2 e^{PT} A3 R(w_y) v: multi-shift Krylov solves of P and
        P^T and a Taylor-substep exponential, every generator application the DEOM stencil kernel (qd_deom_apply;
        pyqed_amd/deom_krylov.py).  P is never formed: the bench hierarchy's would be 9.8 GB."""
        from .deom_krylov import DeomOperator, corr4_krylov, transposed_tables
        dev = default_device()
        _lib.ensure_device(dev)
        b = self.bath
        ns = self.nsys
        coef, damp = ado_coefficients(self.keys, np.asarray(b.etal), np.asarray(b.etar), np.asarray(b.etaa),
                                      np.asarray(b.expn), self.lmax)
        H = _thresh(np.asarray(self.system, dtype=complex))   # the P of generate_propgator (ado_liouvillian)
        Q = np.asarray(self.coupling, dtype=complex).reshape(-1, ns, ns)
        mode = np.asarray(b.mode)
        op = DeomOperator(dev, self._minus, self._plus, coef, damp, mode, H, Q, ns)
        mT, pT, cT = transposed_tables(self._minus, self._plus, coef)
        opT = DeomOperator(dev, mT, pT, cT, damp, mode, H.T, np.swapaxes(Q, 1, 2), ns)
        A1, A2, A3, A4 = (_action_block(o, c) for o, c in
                          zip((operator_d, operator_c, operator_b, operator_a), (lcr[3], lcr[2], lcr[1], lcr[0])))
        c, info = corr4_krylov(op, opT, A1, A2, A3, A4, rho0, float(T), w_x, w_y, self.nmax, ns)
        info["n"] = self.nmax * ns * ns
        self.last_corr4 = info
        return c
