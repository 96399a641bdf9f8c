"""Host check of deom.hip's tiled stage kernel (and the any-ns Euler HEOM chain) through the flat-loop emulation
(tools/cpu_emu/libemu_deom.so) against oracle/deom.py and oracle/heom.py.  Debug tool."""
import ctypes
import os
import sys

import numpy as np
import sympy as sp

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from oracle import deom as od  # noqa: E402
from oracle import heom as oh  # noqa: E402
from pyqed_amd.deom import ado_coefficients, ado_tables  # noqa: E402
from test_deom_large_gpu import _model  # noqa: E402

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libemu_deom.so"))
P = ctypes.c_void_p


def p(a):
    return None if a is None else a.ctypes.data_as(P)


def rel(a, b):
    return np.linalg.norm(a - b) / np.linalg.norm(b)


def deom_case(ns, L, nbath=1, npsd=2, nt=3, dt=0.01):
    sol, bath, H, Q, sdip, cdip, fs, fc, rho0 = _model(ns, L, nbath, npsd)
    K = len(bath.expn)
    keys, minus, plus, comb = ado_tables(L, K)
    coef, damp = ado_coefficients(keys, np.asarray(bath.etal), np.asarray(bath.etar), np.asarray(bath.etaa),
                                  np.asarray(bath.expn), L)
    nmax = len(keys)
    ados = np.zeros((1, nmax, ns, ns), complex)
    ados[0, 0] = rho0
    f = lambda fn: np.array([[fn(s * dt), fn(s * dt + dt / 2), fn(s * dt + dt)] for s in range(nt)], complex)
    fsv, fcv = f(fs), f(fc)
    rho_sys = np.zeros((1, nt + 1, ns, ns), complex)
    i32 = lambda a: np.ascontiguousarray(a, dtype=np.int32)
    c = lambda a: np.ascontiguousarray(a, dtype=complex)
    tabs = [i32(minus), i32(plus), c(coef), c(damp), i32(bath.mode)]
    Hc, Hd, Qc, Qd = c(H), c(sdip), c(Q), c(cdip)
    fn = lib.qd_deom_rk4
    fn.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, P, P, P, ctypes.c_int, P, P, P,
                   P, P, P, ctypes.c_double, ctypes.c_int, P, P, ctypes.c_int, P, P]
    rc = fn(p(ados), 1, nmax, K, ns, *[p(t) for t in tabs], Q.shape[0], p(Hc), p(Hd), p(Qc), p(Qd), p(fsv), p(fcv),
            dt, nt, p(rho_sys), None, 0, None, None)
    assert rc == 0, rc
    _, saved, ados_ref = od.run(H, sdip, fs, Q, cdip, fc, (bath.etal, bath.etar, bath.etaa, bath.expn), L, rho0, dt, nt,
                                mode=bath.mode)
    return rel(rho_sys[0], saved), rel(ados[0], ados_ref)


def chain_case(ns, nado=5, nt=6, dt=0.01):
    rng = np.random.default_rng(ns)
    a = rng.standard_normal((ns, ns)) + 1j * rng.standard_normal((ns, ns))
    H = (a + a.conj().T) / 2 / np.sqrt(ns)
    Q = np.diag(np.linspace(-1, 1, ns)).astype(complex)
    rho0 = np.zeros((ns, ns), complex); rho0[0, 0] = 1
    E = np.array([Q])
    T, gam, lam = 2.0, 1.0, 0.1
    D0 = lam * gam * (1.0 / np.tanh(gam / (2 * T)) - 1j)
    ados = np.zeros((1, nado, ns, ns), complex); ados[0, 0] = rho0
    obs = np.zeros((1, nt + 1, 1), complex)
    fn = lib.qd_heom_chain_euler
    fn.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, ctypes.c_double, ctypes.c_double,
                   ctypes.c_double, ctypes.c_double, ctypes.c_int, P, P, ctypes.c_int, P, P]
    rc = fn(p(ados), 1, nado, ns, p(np.ascontiguousarray(H)), p(Q), gam, D0.real, D0.imag, dt, nt, None, p(E), 1,
            p(obs), None)
    assert rc == 0
    ref = oh.chain_euler(H, Q, rho0, [Q], T, gam, lam, nado, dt, nt)
    return rel(obs[0, 1:, 0], ref[0])


if __name__ == "__main__":
    for args in [(24, 3), (17, 2), (40, 2)]:
        print("deom", args, deom_case(*args))
    print("deom 10 modes", deom_case(3, 2, nbath=10, npsd=0))
    print("chain 20", chain_case(20))
