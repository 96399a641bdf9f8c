"""Generate golden vectors by running the REAL reference (ShuoyiHU/pyqed) here.

Run in the build container only (the reference does not exist on the GPU box):
    python tests/golden/make_golden.py [name ...]
Writes tests/golden/<name>.npz (inputs + reference outputs + library versions).
The reference is imported read-only through ref_shim.
Fixtures are data; no reference source is copied.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ref_shim  # noqa: E402

ref_shim.install()

from scipy.sparse import csr_matrix  # noqa: E402

GENERATORS = {}


def golden(fn):
    GENERATORS[fn.__name__] = fn
    return fn


def save(name, **arrays):
    arrays["lib_versions"] = np.array(str(ref_shim.lib_versions()))
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **arrays)
    print("wrote", path, f"{os.path.getsize(path)/1024:.1f} KiB")


def _herm(rng, n, scale=1.0):
    a = rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n))
    return scale * (a + a.conj().T) / 2


def _ginibre(rng, n, scale=1.0):
    return scale * (rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n)))


# ----------------------------------------------------------------- Lindblad
def _lindblad_case(name, N, nc, ne, Nt, dt, seed, keep_all=True):
    import pyqed.oqs as oqs
    rng = np.random.default_rng(seed)
    H = _herm(rng, N, 1 / np.sqrt(N))
    C = np.array([_ginibre(rng, N, 0.3 / np.sqrt(N)) for _ in range(nc)]).reshape(nc, N, N)
    E = np.array([_herm(rng, N) for _ in range(ne)]).reshape(ne, N, N)
    psi = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    psi /= np.linalg.norm(psi)
    rho0 = np.outer(psi, psi.conj())
    solver = oqs.LindbladSolver(csr_matrix(H), [csr_matrix(c) for c in C])
    r = solver.run(rho0, dt=dt, Nt=Nt, e_ops=[csr_matrix(e) for e in E])
    rholist = np.array([x.toarray() for x in r.rholist])
    out = dict(H=H, C=C, E=E, rho0=rho0, dt=dt, Nt=Nt, observables=r.observables, times=r.times)
    if keep_all:
        out["rholist"] = rholist
    else:
        out["rho_final"] = rholist[-1]
    save(name, **out)


@golden
def lindblad_n4():
    _lindblad_case("lindblad_n4", N=4, nc=2, ne=2, Nt=10, dt=0.01, seed=11)


@golden
def lindblad_n16():
    _lindblad_case("lindblad_n16", N=16, nc=1, ne=3, Nt=10, dt=0.005, seed=12)


@golden
def lindblad_n40_noc():
    # no collapse operators, N not a multiple of 32 (exercises padding)
    _lindblad_case("lindblad_n40_noc", N=40, nc=0, ne=1, Nt=5, dt=0.01, seed=13)


@golden
def lindblad_n128():
    # BASELINE config d1 size (few steps: the reference does ~5.6 steps/s here)
    _lindblad_case("lindblad_n128", N=128, nc=1, ne=1, Nt=3, dt=1e-3, seed=14, keep_all=False)


@golden
def lindblad_driven():
    """LindbladSolver.run with H = [H0, [H1, f]] -> _lindblad_driven (oqs.py:1699-1806)."""
    import pyqed.oqs as oqs
    rng = np.random.default_rng(16)
    N = 6
    H0 = _herm(rng, N, 1 / np.sqrt(N))
    H1 = _herm(rng, N, 0.3)
    H2 = _herm(rng, N, 0.2)
    C = _ginibre(rng, N, 0.2 / np.sqrt(N))
    E = _herm(rng, N)
    psi = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    psi /= np.linalg.norm(psi)
    rho0 = np.outer(psi, psi.conj())
    f1 = lambda t: np.cos(2.0 * t) * np.exp(-(t - 0.3) ** 2)
    f2 = lambda t: 0.5 * np.sin(t)
    H0c = csr_matrix(H0)
    H0_before = H0c.toarray().copy()
    sol = oqs.LindbladSolver([H0c, [csr_matrix(H1), f1], [csr_matrix(H2), f2]], [csr_matrix(C)])
    r = sol.run(rho0, dt=0.02, Nt=25, t0=0.1, e_ops=[csr_matrix(E)])
    h0_mutated = not np.array_equal(H0c.toarray(), H0_before)
    save("lindblad_driven", H0=H0, H1=H1, H2=H2, C=C, E=E, rho0=rho0, dt=0.02, Nt=25, t0=0.1,
         observables=r.observables, rholist=np.array([x.toarray() for x in r.rholist]), h0_mutated=h0_mutated)


@golden
def lindblad_corr():
    """LindbladSolver correlation functions (oqs.py:1193-1329, _correlation_2p_1t oqs.py:717-791)."""
    import tempfile
    import pyqed.oqs as oqs
    rng = np.random.default_rng(15)
    N = 5
    H = _herm(rng, N, 1 / np.sqrt(N))
    C = _ginibre(rng, N, 0.3 / np.sqrt(N))
    A, B, Cop, D = (_ginibre(rng, N) for _ in range(4))
    psi = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    psi /= np.linalg.norm(psi)
    rho0 = np.outer(psi, psi.conj())
    sol = oqs.LindbladSolver(csr_matrix(H), [csr_matrix(C)])
    dt, Nt = 0.02, 12
    with tempfile.TemporaryDirectory() as d:
        cwd = os.getcwd()
        os.chdir(d)
        try:
            c2 = sol.correlation_2op_1t(rho0, csr_matrix(A), csr_matrix(B), dt, Nt)
            cordat = open("cor.dat").read()
        finally:
            os.chdir(cwd)
    c3 = sol.correlation_3op_1t(rho0, [csr_matrix(A), csr_matrix(B), csr_matrix(Cop)], dt=dt, Nt=Nt)
    c4 = sol.correlation_4op_1t(rho0, [csr_matrix(A), csr_matrix(B), csr_matrix(Cop), csr_matrix(D)], dt, Nt)
    # correlation_3op_2t is broken at oqs.py:1292 (Nt+1 vs Ntau); build its intended matrix
    # from the reference's own _lindblad exactly as the method does
    Ntau = 7
    rho_t = oqs._lindblad(csr_matrix(H), rho0, [csr_matrix(C)], dt=dt, Nt=Nt).rholist
    c32 = np.zeros((Nt, Ntau), dtype=complex)
    for k, r in enumerate(rho_t):
        c32[k] = oqs._lindblad(csr_matrix(H), rho0=csr_matrix(Cop) @ r @ csr_matrix(A), dt=dt, Nt=Ntau,
                               c_ops=[csr_matrix(C)], e_ops=[csr_matrix(B)]).observables[:Ntau, 0]
    save("lindblad_corr", H=H, C=C, A=A, B=B, Cop=Cop, D=D, rho0=rho0, dt=dt, Nt=Nt, Ntau=Ntau, c2=c2, c3=c3,
         c4=c4, c32=c32, cordat=np.array(cordat))


@golden
def corr3p_1t():
    """correlation.correlation_3p_1t (pyqed/correlation.py:17-70) with dyn = oqs.liouvillian:
    returns None, writes cor.dat (t, <A B(t) C>) and dm.dat (t, ravel rho) in the CWD."""
    import tempfile
    import pyqed.oqs as oqs
    from pyqed.correlation import correlation_3p_1t
    rng = np.random.default_rng(17)
    N = 4
    H = _herm(rng, N, 1 / np.sqrt(N))
    C = _ginibre(rng, N, 0.2 / np.sqrt(N))
    A, B, Cop = (_ginibre(rng, N) for _ in range(3))
    psi = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    psi /= np.linalg.norm(psi)
    rho0 = np.outer(psi, psi.conj())
    tlist = np.linspace(0, 0.3, 16)
    with tempfile.TemporaryDirectory() as d:
        cwd = os.getcwd()
        os.chdir(d)
        try:
            ret = correlation_3p_1t(csr_matrix(H), csr_matrix(rho0), [csr_matrix(A), csr_matrix(B), csr_matrix(Cop)],
                                    [csr_matrix(C)], tlist, oqs.liouvillian)
            cordat, dmdat = open("cor.dat").read(), open("dm.dat").read()
        finally:
            os.chdir(cwd)
    save("corr3p_1t", H=H, C=C, A=A, B=B, Cop=Cop, rho0=rho0, tlist=tlist, returned_none=ret is None,
         cordat=np.array(cordat), dmdat=np.array(dmdat))


@golden
def lindblad_eig():
    """superoperator.Lindblad_solver eigen path (superoperator.py:455-772), N=3 ladder."""
    import pyqed.superoperator as so
    N = 3
    H = np.diag([0.0, 1.0, 1.6]).astype(complex)
    H[0, 1] = H[1, 0] = 0.1
    c1 = np.zeros((N, N), complex); c1[0, 1] = np.sqrt(0.1)
    c2 = np.zeros((N, N), complex); c2[1, 2] = np.sqrt(0.05)
    dip = np.zeros((N, N), complex); dip[0, 1] = dip[1, 0] = 1.0; dip[1, 2] = dip[2, 1] = 0.7
    rho0 = np.zeros((N, N), complex); rho0[0, 0] = 1
    sol = so.Lindblad_solver(H, [c1, c2])
    L = sol.liouvillian()
    w, vr, vl = sol.eigenstates()
    t = 0.3 * np.arange(40)
    tau = 0.25 * np.arange(11)
    freq = np.linspace(-3, 3, 33)
    out = dict(H=H, c1=c1, c2=c2, dip=dip, rho0=rho0, L=L.toarray(), eigvals=w, norm=sol.norm, t=t, tau=tau, w=freq)
    out["c2t"] = sol.correlation_2op_1t(rho0, [dip, dip], t)
    out["c2w"] = sol.correlation_2op_1w(rho0, [dip, dip], freq)
    out["c3t"] = sol.correlation_3op_1t(rho0, [dip, dip, dip], t)
    out["c3w"] = sol.correlation_3op_1w(rho0, [dip, dip, dip], freq)
    out["c32"] = sol.correlation_3op_2t(rho0, [dip, dip, dip], t[:9], tau)
    out["c42"] = sol.correlation_4op_2t(rho0, [dip, dip, dip, dip], t[:9], tau)
    save("lindblad_eig", **out)


@golden
def sesolver():
    """SESolver.run / Mol.run -> _quantum_dynamics (mol.py:1392-1459, 628-674, 1603-1691)."""
    from pyqed.mol import Mol, SESolver
    rng = np.random.default_rng(31)
    out = {}
    for tag, N, Nt, nout, dt in [("a", 8, 10, 2, 0.05), ("b", 37, 31, 4, 0.02)]:
        H = _herm(rng, N, 1 / np.sqrt(N))
        E = [_herm(rng, N) for _ in range(2)]
        psi0 = rng.standard_normal(N) + 1j * rng.standard_normal(N)
        psi0 /= np.linalg.norm(psi0)
        r = SESolver(H).run(psi0=psi0, dt=dt, Nt=Nt, e_ops=E, nout=nout)
        r2 = Mol(H).run(psi0=psi0, dt=dt, e_ops=E, nt=Nt, nout=nout)
        assert np.allclose(r.observables, r2.observables)
        out.update({f"{tag}_H": H, f"{tag}_E": np.array(E), f"{tag}_psi0": psi0, f"{tag}_Nt": Nt,
                    f"{tag}_nout": nout, f"{tag}_dt": dt, f"{tag}_obs": r.observables,
                    f"{tag}_psilist": np.array(r.psilist), f"{tag}_times": r.times})
    save("sesolver", **out)


@golden
def tdse_driven():
    """Laser-driven TDSE: SESolver.run / Mol.run with pulses -> driven_dynamics (mol.py:1392-1456,
    628-675, 1862-1958) and optics.Pulse.efield (optics.py:229-318)."""
    from pyqed.mol import Mol, SESolver
    from pyqed.optics import Pulse
    rng = np.random.default_rng(37)
    out = {}
    # a: single pulse, SESolver, 2D dipole, csr psi (use_sparse=True)
    N = 6
    H = np.diag(np.linspace(0.0, 1.5, N)).astype(complex) + 0.05 * _herm(rng, N)
    d = _herm(rng, N, 0.5)
    E = [_herm(rng, N) for _ in range(2)]
    psi0 = np.zeros(N, complex); psi0[0] = 1.0
    p = dict(omegac=0.8, tau=2.0, tc=3.0, amplitude=0.3)
    r = SESolver(H).run(psi0=psi0, dt=0.05, Nt=60, e_ops=[csr_matrix(e) for e in E], nout=3, edip=d,
                        pulse=Pulse(**p))
    out.update({"a_H": H, "a_d": d, "a_E": np.array(E), "a_psi0": psi0, "a_dt": 0.05, "a_Nt": 60, "a_nout": 3,
                "a_t0": 0.0, "a_pulse": np.array([p["omegac"], p["tau"], p["tc"], p["amplitude"]]),
                "a_obs": r.observables, "a_psit": r.psi,
                "a_psilist": np.array([np.asarray(x.toarray() if hasattr(x, "toarray") else x).reshape(N)
                                       for x in r.psilist])})
    # b: two pulses, Mol.run (self.edip list), t0 != 0, nout = 1
    N = 9
    H = np.diag(np.linspace(0.0, 2.0, N)).astype(complex) + 0.1 * _herm(rng, N)
    ds = [_herm(rng, N, 0.3), _herm(rng, N, 0.2)]
    E = [_herm(rng, N)]
    psi0 = rng.standard_normal(N) + 1j * rng.standard_normal(N); psi0 /= np.linalg.norm(psi0)
    ps = [dict(omegac=1.1, tau=1.5, tc=1.0, amplitude=0.2), dict(omegac=0.6, tau=3.0, tc=2.5, amplitude=0.1)]
    r = Mol(H, edip=ds).run(psi0=psi0, dt=0.04, e_ops=[csr_matrix(e) for e in E], nt=50, nout=1, t0=0.3, pulse=[Pulse(**q) for q in ps])
    out.update({"b_H": H, "b_d": np.array(ds), "b_E": np.array(E), "b_psi0": psi0, "b_dt": 0.04, "b_Nt": 50,
                "b_nout": 1, "b_t0": 0.3,
                "b_pulse": np.array([[q["omegac"], q["tau"], q["tc"], q["amplitude"]] for q in ps]),
                "b_obs": r.observables, "b_psit": r.psi,
                "b_psilist": np.array([np.asarray(x.toarray() if hasattr(x, "toarray") else x).reshape(N)
                                       for x in r.psilist])})
    save("tdse_driven", **out)


def vector_field(t, p):
    """Polarized test field E(t) (3-vector) of the tdse_driven3d fixture: a Gaussian carrier per component."""
    amp, om, tc, tau = p[:, 0], p[:, 1], p[:, 2], p[:, 3]
    return amp * np.cos(om * t) * np.exp(-((t - tc) / tau) ** 2)


@golden
def tdse_driven3d():
    """SESolver.run with a full [N, N, 3] dipole -> mol._driven_dynamics (mol.py:1441-1445, 1772-1859)."""
    from pyqed.mol import SESolver
    rng = np.random.default_rng(41)
    N = 5
    H = np.diag(np.linspace(0.0, 1.2, N)).astype(complex) + 0.05 * _herm(rng, N)
    edip = np.stack([_herm(rng, N, 0.4) for _ in range(3)], axis=2)
    E = [_herm(rng, N) for _ in range(2)]
    psi0 = np.zeros(N, complex); psi0[0] = 1.0
    fp = np.array([[0.3, 0.9, 1.0, 0.8], [0.2, 1.1, 1.5, 1.0], [0.1, 0.7, 0.5, 2.0]])

    class VPulse:
        def E(self, t):
            return vector_field(t, fp)

    r = SESolver(H).run(psi0=psi0, dt=0.04, Nt=60, e_ops=[csr_matrix(e) for e in E], nout=3, edip=edip,
                        pulse=VPulse())
    save("tdse_driven3d", H=H, edip=edip, E=np.array(E), psi0=psi0, dt=0.04, Nt=60, nout=3, field=fp,
         obs=r.observables, psit=r.psi,
         psilist=np.array([np.asarray(x.toarray()).reshape(N) for x in r.psilist]))


@golden
def photon_echo():
    """sos.photon_echo (signal/sos.py:962-1052) via Mol.photon_echo (mol.py:804-829)."""
    import tempfile
    from pyqed.mol import Mol
    import pyqed.signal.sos as sos
    out = {}
    H3 = np.diag([0.0, 1.0, 1.5])
    dip3 = np.zeros((3, 3)); dip3[0, 1] = dip3[1, 0] = 1.0; dip3[1, 2] = dip3[2, 1] = 1.0
    rng = np.random.default_rng(41)
    H4 = np.diag([0.0, 0.9, 1.1, 2.05])
    d4 = rng.standard_normal((4, 4)); d4 = d4 + d4.T
    cases = {"l3_t0": (H3, dip3, np.array([0, 0.1, 0.1]), 32, 0.0),
             "l3_t2": (H3, dip3, np.array([0, 0.1, 0.05]), 32, 1.5),
             "r4": (H4, d4, np.array([0.0, 0.05, 0.08, 0.1]), 48, 0.7)}
    for tag, (H, dip, gam, n, t2) in cases.items():
        mol = Mol(H, dip)
        mol.edip_rms = dip
        mol.gamma = gam
        pump = np.linspace(0.5, 2.0, n)
        probe = np.linspace(0.4, 2.2, n)
        with tempfile.TemporaryDirectory() as d:
            cwd = os.getcwd(); os.chdir(d)
            try:
                S = mol.photon_echo(pump=pump, probe=probe, t2=t2)
                saved = np.load("signal.npz")
                assert np.array_equal(saved["arr_2"], S)
            finally:
                os.chdir(cwd)
        out.update({f"{tag}_H": H, f"{tag}_dip": dip, f"{tag}_gamma": gam, f"{tag}_pump": pump,
                    f"{tag}_probe": probe, f"{tag}_t2": t2, f"{tag}_S": S})
    save("photon_echo", **out)


@golden
def fft_phys():
    """pyqed.fft fft / ifft / fft2 / dft2 (fft.py:11-160)."""
    import importlib
    pf = importlib.import_module("pyqed.fft")   # `pyqed.fft` the attribute is a function (phys *)
    x = np.linspace(-10, 10, 256)
    a = np.exp(-x ** 2 / 2) * (1 + 0.3j * x)
    out = dict(x=x, a=a)
    out["fft_g"], out["fft_w"] = pf.fft(a, x)
    out["ifft_g"], out["ifft_w"] = pf.ifft(a, x)
    x2 = np.linspace(-5, 7, 100)                       # non power of two
    b = np.exp(-(x2 - 1) ** 2) * np.exp(0.5j * x2)
    out["x2"], out["b"] = x2, b
    out["fft100_g"], out["fft100_w"] = pf.fft(b, x2)
    rng = np.random.default_rng(51)
    M = rng.standard_normal((32, 48)) + 1j * rng.standard_normal((32, 48))
    out["M"] = M
    out["fftax0_g"], out["fftax0_w"] = pf.fft(M, x=np.linspace(0, 3.1, 32), axis=0)
    out["ifftax0_g"], _ = pf.ifft(M, x=np.linspace(0, 3.1, 32), axis=0)
    fx, fy, g2 = pf.fft2(M[:, :32], dx=0.1, dy=0.2)
    out["fft2_fx"], out["fft2_fy"], out["fft2_g"] = fx, fy, g2
    xs, ys = np.linspace(0, 1, 9), np.linspace(-1, 1, 7)
    F = rng.standard_normal((7, 9)) + 0j
    kx, ky = np.linspace(-3, 3, 5), np.linspace(-2, 2, 4)
    out.update(xs=xs, ys=ys, F=F, kx=kx, ky=ky, dft2=pf.dft2(xs, ys, F, kx, ky))
    save("fft_phys", **out)


@golden
def fft_any():
    """pyqed.fft.fft / ifft at lengths the round-3 GPU path refused or ran as a direct DFT (fft.py:11-102), with the
    caller's kwargs forwarded to np.fft.fft (fft.py:49): norm, n; axis 0 of a 3-D array; odd / prime lengths."""
    import importlib
    pf = importlib.import_module("pyqed.fft")
    rng = np.random.default_rng(77)
    out = {}
    for n in (8, 2048, 4096, 5000, 7919, 12288, 1000):
        x = np.linspace(-7.0, 9.0, n)
        a = np.exp(-(x - 1) ** 2 / 3) * np.exp(0.7j * x) + 0.01 * rng.standard_normal(n)
        out[f"x{n}"], out[f"a{n}"] = x, a
        out[f"fft{n}_g"], out[f"fft{n}_w"] = pf.fft(a, x)
        out[f"ifft{n}_g"], _ = pf.ifft(a, x)
    out["fft5000_ortho_g"], _ = pf.fft(out["a5000"], out["x5000"], norm="ortho")
    out["fft2048_forward_g"], _ = pf.fft(out["a2048"], out["x2048"], norm="forward")
    out["fft7919_n_g"], _ = pf.fft(out["a7919"], out["x7919"], n=7919)
    out["fft1000_n1_g"], _ = pf.fft(out["a1000"], out["x1000"], n=1)
    try:
        pf.fft(out["a1000"], out["x1000"], n=900)
        out["n900_raises"] = np.array(False)
    except ValueError:
        out["n900_raises"] = np.array(True)
    T = rng.standard_normal((45, 6, 7)) + 1j * rng.standard_normal((45, 6, 7))
    xt = np.linspace(0.5, 3.0, 45)
    out["T"], out["xt"] = T, xt
    out["fftT0_g"], out["fftT0_w"] = pf.fft(T, xt, axis=0)
    out["fftT1_ortho_g"], _ = pf.fft(T, np.linspace(0, 1, 6), axis=1, norm="ortho")
    out["ifftT0_g"], _ = pf.ifft(T, xt, axis=0)
    out["ifftTm1_g"], _ = pf.ifft(T, np.linspace(-1, 1, 7), axis=-1)
    save("fft_any", **out)


# ----------------------------------------------------------------- Redfield / 2DES
# Spectral functions by name (tests/conftest.py SPECTRA holds the same definitions).
SPECTRA = {
    "flat005": lambda w: 0.05,
    "tanh": lambda w: 0.02 * (1.0 + np.tanh(2.0 * w)),
}


def _redfield_case(name, N, nk, Nt, dt, seed, spectrum):
    import pyqed.oqs as oqs
    rng = np.random.default_rng(seed)
    H = _herm(rng, N)
    a_ops = [_herm(rng, N, 0.5) for _ in range(nk)]
    E = np.array([_herm(rng, N) for _ in range(2)])
    psi = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    psi /= np.linalg.norm(psi)
    rho0 = np.outer(psi, psi.conj())
    sol = oqs.RedfieldSolver(H, c_ops=a_ops, spectra=[SPECTRA[spectrum]] * nk)
    R, evecs = sol.redfield_tensor()
    r = sol.evolve(rho0, dt=dt, Nt=Nt, e_ops=list(E))
    save(name, H=H, a_ops=np.array(a_ops), E=E, rho0=rho0, dt=dt, Nt=Nt, spectrum=spectrum,
         R=R.toarray(), evecs=evecs, observables=r.observables, rholist=np.array(r.rholist))


@golden
def redfield_n4():
    _redfield_case("redfield_n4", N=4, nk=1, Nt=10, dt=0.05, seed=21, spectrum="tanh")


@golden
def redfield_n6_k2():
    _redfield_case("redfield_n6_k2", N=6, nk=2, Nt=8, dt=0.02, seed=22, spectrum="flat005")


@golden
def redfield_eom():
    """RedfieldSolver.propagator(t, 'EOM') (oqs.py:160-200 -> phys.expm, phys.py:2049-2097) and
    gf(t, method='eseries') (oqs.py:136-158 -> getG, oqs.py:465-508) on an N = 4 system.  In the imported package
    the name `expm` that oqs.py binds is a later star-import's one-argument expm, so propagator('EOM') raises
    TypeError there; the fixture calls the function oqs.py means, pyqed.phys.expm(R, t), directly."""
    import contextlib
    import io
    import pyqed.oqs as oqs
    from pyqed.phys import expm as phys_expm
    rng = np.random.default_rng(31)
    N = 4
    H = _herm(rng, N)
    a_ops = [_herm(rng, N, 0.5)]
    sol = oqs.RedfieldSolver(H, c_ops=a_ops, spectra=[SPECTRA["tanh"]])
    R, evecs = sol.redfield_tensor()
    t = 0.05 * np.arange(12)
    with contextlib.redirect_stdout(io.StringIO()):
        U = np.dstack([u.toarray() for u in phys_expm(sol.R, t)])
    G = sol.gf(t, method="eseries")
    save("redfield_eom", H=H, a_ops=np.array(a_ops), spectrum="tanh", t=t, R=R.toarray(), U_eom=U, G_eseries=G)


def _three_level(E=(0.0, 1.0, 1.5)):
    N = 3
    H = np.diag(np.asarray(E, float))
    dip = np.zeros((N, N))
    dip[0, 1] = dip[1, 0] = 1.0
    dip[1, 2] = dip[2, 1] = 1.0
    a = np.diag([0.0, 1.0, 2.0])
    rho0 = np.zeros((N, N), dtype=complex)
    rho0[0, 0] = 1.0
    return H, dip, a, rho0


@golden
def corr4_3level():
    """correlation_4op_3t cubes (3-level ladder, Redfield flat 0.05) for three signatures,
    plus 2D slices S[:, j, :] of a 64-point cube."""
    import pyqed.oqs as oqs
    H, dip, a, rho0 = _three_level()
    out = dict(H=H, dip=dip, a_op=a, rho0=rho0, spectrum="flat005")
    tau16 = 0.5 * np.arange(16)
    for sig in ["lccc", "llll", "lrlr"]:
        sol = oqs.RedfieldSolver(H, c_ops=[a], spectra=[SPECTRA["flat005"]])
        sol.redfield_tensor()
        sol.propagator(tau16)
        out["cube_" + sig] = sol.correlation_4op_3t(rho0, [dip, dip, dip, dip], sig, tau16)
    out["tau16"] = tau16
    out["R"] = sol.R.toarray()
    tau64 = 0.5 * np.arange(64)
    sol = oqs.RedfieldSolver(H, c_ops=[a], spectra=[SPECTRA["flat005"]])
    sol.redfield_tensor()
    sol.propagator(tau64)
    cube = sol.correlation_4op_3t(rho0, [dip, dip, dip, dip], "lccc", tau64)
    out["tau64"] = tau64
    out["slice64_j0"] = cube[:, 0, :]
    out["slice64_j5"] = cube[:, 5, :]
    out["U64_k7"] = sol.U[:, :, 7]
    save("corr4_3level", **out)


@golden
def corr4_ensemble():
    """Static-disorder ensemble (3 members): 'lccc' slices at tau2 index 3, n_tau = 32."""
    import pyqed.oqs as oqs
    rng = np.random.default_rng(3)
    tau = 0.5 * np.arange(32)
    Es, slices = [], []
    for m in range(3):
        E = np.array([0.0, 1.0, 1.5]) + np.array([0.0, 0.05, 0.08]) * rng.standard_normal(3)
        H, dip, a, rho0 = _three_level(E)
        sol = oqs.RedfieldSolver(H, c_ops=[a], spectra=[SPECTRA["flat005"]])
        sol.redfield_tensor()
        sol.propagator(tau)
        cube = sol.correlation_4op_3t(rho0, [dip, dip, dip, dip], "lccc", tau)
        Es.append(E)
        slices.append(cube[:, 3, :])
    save("corr4_ensemble", E=np.array(Es), tau=tau, j=3, slices=np.array(slices),
         ens_sum=np.sum(slices, axis=0))


# ----------------------------------------------------------------- split-operator
def spo2_model(n, L=6.0, complex_coupling=False):
    """BASELINE config d2 model: surfaces 1/2((X+-1)^2+Y^2) (+0.1 offset), coupling 0.2*X."""
    x = np.linspace(-L, L, n)
    y = np.linspace(-L, L, n)
    X, Y = np.meshgrid(x, y, indexing="ij")
    v0 = 0.5 * ((X + 1) ** 2 + Y ** 2)
    v1 = 0.5 * ((X - 1) ** 2 + Y ** 2) + 0.1
    c = 0.2 * X + (0.1j * Y if complex_coupling else 0)
    psi0 = np.zeros((n, n, 2), dtype=complex)
    psi0[:, :, 0] = np.exp(-((X + 1.5) ** 2 + Y ** 2) / 2 + 0.5j * X) / np.sqrt(np.pi)
    return x, y, v0, v1, c, psi0


def _spo2_case(name, n, nt, nout, dt, complex_coupling=False, masses=(1.0, 1.0), keep_ops=True):
    from pyqed.wpd import SPO2
    x, y, v0, v1, c, psi0 = spo2_model(n, complex_coupling=complex_coupling)
    sol = SPO2(x, y, mass=list(masses), nstates=2)
    if complex_coupling:
        # set_DPES builds a real array (wpd.py:466) and drops Im; set_dpes keeps a complex
        # Hermitian potential -> exercises the complex branch of build (wpd.py:583-600)
        v = np.zeros((n, n, 2, 2), dtype=complex)
        v[:, :, 0, 0], v[:, :, 1, 1], v[:, :, 0, 1], v[:, :, 1, 0] = v0, v1, c, np.conj(c)
        sol.set_dpes(v)
    else:
        sol.set_DPES([v0, v1], [[[0, 1], c]])
    r = sol.run(psi0, dt=dt, nt=nt, nout=nout)
    out = dict(x=x, y=y, v0=v0, v1=v1, coupling=np.asarray(c), psi0=psi0, dt=dt, nt=nt, nout=nout,
               masses=np.array(masses), psilist=np.array(r.psilist), times=r.times,
               apes=sol.apes if sol.apes is not None else np.zeros(0))
    if keep_ops:
        out.update(exp_V_half=sol.exp_V_half, exp_K=sol.exp_K)
    save(name, **out)


@golden
def spo2_32():
    _spo2_case("spo2_32", n=32, nt=6, nout=2, dt=0.05)


@golden
def spo2_64_complex():
    _spo2_case("spo2_64_complex", n=64, nt=3, nout=1, dt=0.05, complex_coupling=True, masses=(1.0, 2.0),
               keep_ops=False)


@golden
def spo2nh_32():
    """SPO2NH (wpd.py:921-1077): complex potential (absorbing wall -i eta (x-3)^2 on both surfaces),
    Strang (return_states=True) and merged (return_states=False) runs."""
    from pyqed.wpd import SPO2NH
    n = 32
    x, y, v0, v1, c, psi0 = spo2_model(n)
    X, Y = np.meshgrid(x, y, indexing="ij")
    v = np.zeros((n, n, 2, 2), dtype=complex)
    absorb = -1j * 0.02 * np.clip(X - 3.0, 0, None) ** 2
    v[:, :, 0, 0], v[:, :, 1, 1] = v0 + absorb, v1 + absorb
    v[:, :, 0, 1] = v[:, :, 1, 0] = c
    out = dict(x=x, y=y, v=v, psi0=psi0, dt=0.1, nt=6, nout=2)
    for tag, rs in (("strang", True), ("merged", False)):
        sol = SPO2NH(x, y, mass=[1.0, 1.0], nstates=2)
        sol.set_dpes(v)
        r = sol.run(psi0, dt=0.1, nt=6, nout=2, return_states=rs)
        out[f"{tag}_psilist"] = np.array(r.psilist)
        out[f"{tag}_psi"] = r.psi
    out["exp_V_half"] = sol.exp_V_half
    out["exp_V"] = sol.exp_V
    save("spo2nh_32", **out)


@golden
def spo2_jacobi_32():
    """SPO2 coords='jacobi' (build wpd.py:540-553, _KEO_jacobi wpd.py:850-887), I(x) = 1.5 + 0.2 x^2."""
    from pyqed.wpd import SPO2
    n = 32
    x, y, v0, v1, c, psi0 = spo2_model(n)
    sol = SPO2(x, y, mass=[1.0, lambda r: 1.5 + 0.2 * r ** 2], nstates=2, coords='jacobi')
    sol.set_DPES([v0, v1], [[[0, 1], c]])
    r = sol.run(psi0, dt=0.05, nt=6, nout=3)
    save("spo2_jacobi_32", x=x, y=y, v0=v0, v1=v1, coupling=np.asarray(c), psi0=psi0, dt=0.05, nt=6, nout=3,
         inertia=np.array([1.5, 0.2]), psilist=np.array(r.psilist), exp_Kx=sol.exp_Kx, exp_Ky=sol.exp_Ky)


@golden
def spo3_16():
    """SPO3 (wpd.py:1105-1432) on a 16^3 x 2 grid, examples/spo.py model (64^3 x 2 there)."""
    from pyqed.wpd import SPO3
    n = 16
    x = np.linspace(-6, 6, n)
    X, Y, Z = np.meshgrid(x, x, x, indexing="ij")
    sol = SPO3(x, x, x, masses=[1.0, 1.0, 1.0], nstates=2)
    sol.set_DPES([0.5 * ((X + 1) ** 2 + Y ** 2 + Z ** 2), 0.5 * ((X - 1) ** 2 + Y ** 2 + Z ** 2)],
                 [[[0, 1], 0.2 * X]])
    psi0 = np.zeros((n, n, n, 2), dtype=complex)
    psi0[..., 1] = np.exp(-((X + 1) ** 2 + Y ** 2 + Z ** 2) / 2) / np.pi ** 0.75
    r = sol.run(psi0=psi0, dt=0.25, nt=4, nout=2)
    save("spo3_16", x=x, psi0_norm=np.vdot(psi0, psi0).real, dt=0.25, nt=4, nout=2,
         psilist=np.array(r.psilist), psi=r.psi)


def _spo1d_case(name, n, nt, nout, dt):
    from pyqed.wpd import SPO
    x = np.linspace(-8, 8, n)
    psi0 = (np.exp(-(x + 2) ** 2 / 2 + 1j * 0.5 * x) / np.pi ** 0.25).astype(complex)
    sol = SPO(x, mass=1.0)
    sol.set_potential(lambda x: x ** 2 / 2)
    r = sol.run(psi0, dt=dt, nt=nt, nout=nout)
    save(name, x=x, psi0=psi0, dt=dt, nt=nt, nout=nout, psilist=np.array(r.psilist).reshape(-1, n), psi=r.psi,
         times=r.times)


@golden
def spo1d_256():
    _spo1d_case("spo1d_256", n=256, nt=20, nout=1, dt=0.01)


@golden
def spo1d_256_nout3():
    _spo1d_case("spo1d_256_nout3", n=256, nt=20, nout=3, dt=0.01)


# ----------------------------------------------------------------- DEOM / HEOM
def _drude_bath(lam, gam, beta, npsd):
    import sympy as sp
    from pyqed.heom.deom import Bath
    w_sp = sp.symbols(r"\omega", real=True)
    spe = 2 * lam * gam * w_sp / (gam ** 2 + w_sp ** 2)
    # list form (the scalar form of Bath.__init__ fails at heom/deom.py:917: len() of a sympy expr)
    return Bath([spe], w_sp, [beta], [npsd], [0] * (1 + npsd))


@golden
def deom_bath():
    """Pade decomposition of a Drude bath (decompose_spectrum_pade, heom/deom.py:226-307)."""
    out = {}
    for lam, gam, tag in [(0.5, 1.0, "d4"), (1.0, 1.0, "ll"), (0.2, 2.0, "g2")]:
        for npsd in [1, 2, 3, 4]:
            b = _drude_bath(lam, gam, 1.0, npsd)
            for k in ["etal", "etar", "etaa", "expn"]:
                out[f"{tag}_n{npsd}_{k}"] = np.asarray(getattr(b, k), dtype=complex)
    from pyqed.heom.deom import pade_approximation_distribution
    for N in [1, 2, 3, 4, 6]:
        pole, resi = pade_approximation_distribution(N, 1, 1)
        out[f"pade_pole_{N}"] = np.asarray(pole)
        out[f"pade_resi_{N}"] = np.asarray(resi)
    save("deom_bath", **out)


@golden
def deom_bath_pade3():
    """Extended PSD (pade=3, heom/deom.py:163-206) poles / residues for Bose and Fermi, and Drude baths decomposed
    with it through decompose_spectrum_pade(..., pade=3) (heom/deom.py:226-307)."""
    import sympy as sp
    from pyqed.heom.deom import decompose_spectrum_pade, pade_approximation_distribution
    out = {}
    for bf in (1, 2):
        for N in range(1, 8):
            pole, resi = pade_approximation_distribution(N, bf, 3)
            out[f"bf{bf}_N{N}_pole"] = np.asarray(pole)
            out[f"bf{bf}_N{N}_resi"] = np.asarray(resi)
    w_sp = sp.symbols(r"\omega", real=True)
    for lam, gam, beta, tag in [(0.5, 1.0, 1.0, "d4"), (0.2, 2.0, 0.5, "g2")]:
        spe = 2 * lam * gam * w_sp / (gam ** 2 + w_sp ** 2)
        for npsd in (2, 4):
            etal, etar, etaa, expn = decompose_spectrum_pade(spe, w_sp, beta, npsd, pade=3)
            for k, v in zip(("etal", "etar", "etaa", "expn"), (etal, etar, etaa, expn)):
                out[f"{tag}_n{npsd}_{k}"] = np.asarray(v, dtype=complex)
            out[f"{tag}_n{npsd}_params"] = np.array([lam, gam, beta])
    save("deom_bath_pade3", **out)


@golden
def deom_keys():
    """Graded ADO index (init_/gen_keys, heom/deom.py:1048-1064, 555-638)."""
    from pyqed.heom.deom import gen_keys
    out = {}
    for L, K in [(3, 2), (10, 3), (4, 3), (12, 5)]:
        combmax = K + L + 1
        comb = np.zeros((combmax, combmax), dtype=np.int64)
        comb[0, 0] = 1
        for i in range(1, combmax):
            for j in range(1, combmax):
                comb[i, j] = comb[i - 1, j] + comb[i - 1, j - 1]
            comb[i, 0] = 1
        nmax = comb[L + K, L]
        keys = np.zeros((nmax, K), dtype=np.int64)
        gen_keys(keys, L, K, comb)
        out[f"keys_L{L}_K{K}"] = keys
    save("deom_keys", **out)


def _deom_case(lmax, npsd, nt, dt, pulses=False, p1=True, lam=0.5, gam=1.0, beta=1.0):
    from pyqed.heom.deom import DEOMSolver
    s0 = np.eye(2, dtype=complex)
    sx = np.array([[0, 1], [1, 0]], dtype=complex)
    sz = np.array([[1, 0], [0, -1]], dtype=complex)
    H = sz + sx
    bath = _drude_bath(lam, gam, beta, npsd)
    rho0 = np.zeros((2, 2), dtype=complex)
    rho0[0, 0] = 1
    if pulses:
        fs, fc = (lambda t: 0.3 * np.sin(2 * t)), (lambda t: 0.1 * np.cos(t))
        sdip, cdip = sx.copy(), np.array([sz])
    else:
        fs, fc = (lambda t: 0), (lambda t: 0)
        sdip, cdip = np.zeros((2, 2), complex), np.zeros((1, 2, 2), complex)
    solver = DEOMSolver(H, sdip, bath, np.array([sx]), cdip, fs, fc, lmax)
    P1 = np.array([[1, 0], [0, 0]], dtype=complex)
    t_save, ddos_save = solver.run(rho0.copy(), dt, nt, P1 if p1 else None)
    out = dict(H=H, Q=np.array([sx]), sdip=sdip, cdip=cdip, lmax=lmax, npsd=npsd, dt=dt, nt=nt, lam=lam,
               gam=gam, beta=beta, pulses=pulses, t_save=t_save, nmax=solver.nmax,
               etal=bath.etal, etar=bath.etar, etaa=bath.etaa, expn=bath.expn)
    if p1:
        out["trace_p1"] = np.asarray(ddos_save)
    else:
        out["rho_sys"] = np.array([np.asarray(x) for x in ddos_save])
    out["ado_final"] = np.array([np.asarray(x.toarray() if hasattr(x, "toarray") else x) for x in solver.ddos])
    return out


@golden
def deom_corr4():
    """DEOMSolver.correlation_4op_3t (heom/deom.py:1127-1209): dense ADO Liouvillian (generate_propgator,
    :769-893), eig + pinv, frequency-domain (w_x, w_y) signal; full and eigenvalue-cut variants."""
    import contextlib
    import io
    from pyqed.heom.deom import DEOMSolver
    s0 = np.eye(2, dtype=complex)
    sx = np.array([[0, 1], [1, 0]], dtype=complex)
    sz = np.array([[1, 0], [0, -1]], dtype=complex)
    H = sz + sx
    lmax, npsd = 4, 2
    bath = _drude_bath(0.5, 1.0, 1.0, npsd)
    solver = DEOMSolver(H, np.zeros((2, 2), complex), bath, np.array([sx]), np.zeros((1, 2, 2), complex),
                        lambda t: 0, lambda t: 0, lmax)
    rho0 = np.zeros((2, 2), dtype=complex)
    rho0[0, 0] = 1
    wx = np.linspace(-4, 4, 24)
    wy = np.linspace(-3, 5, 20)
    T = 0.5
    out = dict(H=H, Q=np.array([sx]), lmax=lmax, npsd=npsd, rho0=rho0, wx=wx, wy=wy, T=T,
               etal=bath.etal, etar=bath.etar, etaa=bath.etaa, expn=bath.expn)
    with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
        for lcr in ["llll", "lrlr", "lccc"]:
            out["cw_" + lcr] = solver.correlation_4op_3t(sx, sx, sx, sx, rho0, T, wx, wy, lcr=lcr)
        out["cw_cut_llll"] = solver.correlation_4op_3t(sz, sx, sx, sz, rho0, T, wx, wy, if_full=False,
                                                        cut_off_min=0.5, cut_off_max=1.1, lcr="llll")
    out["propagator"] = solver.propgator
    out["nmax"] = solver.nmax
    save("deom_corr4", **out)


@golden
def heom_chain():
    """Single-exponential HEOM chains: HEOM/heom.py _heom (RK4, :275-347) and oqs._heom
    (in-place explicit sweep, oqs.py:1808-1875), examples/heom.py:79-97 model."""
    import pyqed.HEOM.heom as hh
    import pyqed.oqs as oqs
    sx = np.array([[0, 1], [1, 0]], complex)
    sz = np.array([[1, 0], [0, -1]], complex)
    H = -1 / 2.0 * sx - 1.0 / 2.0 * sz
    rho0 = np.zeros((2, 2), complex)
    rho0[1, 1] = 1
    out = dict(H=H, Q=sz, rho0=rho0)
    cases = {"ex": dict(temperature=600, cutoff=5, reorganization=0.2, nado=5, dt=0.02, nt=100),
             "mild": dict(temperature=1.0, cutoff=0.5, reorganization=0.2, nado=6, dt=0.02, nt=80)}
    for tag, c in cases.items():
        for mod, name in [(hh, "rk4"), (oqs, "euler")]:
            sol = mod.HEOMSolver(H, c_ops=[sz], e_ops=[sz, sx])
            obs = sol.run(rho0=rho0.copy(), dt=c["dt"], nt=c["nt"], temperature=c["temperature"],
                          cutoff=c["cutoff"], reorganization=c["reorganization"], nado=c["nado"])
            out[f"{tag}_{name}"] = np.asarray(obs)
        for k, v in c.items():
            out[f"{tag}_{k}"] = v
    save("heom_chain", **out)


@golden
def deom_run_small():
    save("deom_run_small", **_deom_case(lmax=4, npsd=2, nt=20, dt=0.01))


@golden
def deom_run_pulsed():
    save("deom_run_pulsed", **_deom_case(lmax=3, npsd=1, nt=15, dt=0.02, pulses=True, p1=False))


@golden
def deom_run_bench():
    """BASELINE config d4 (L=12, npsd=4 -> K=5, 6188 ADOs), 3 steps (reference ~0.3 steps/s)."""
    out = _deom_case(lmax=12, npsd=4, nt=3, dt=0.01)
    out.pop("ado_final")
    save("deom_run_bench", **out)


# ----------------------------------------------------------------- BASELINE-size pins
@golden
def lindblad_n128_long():
    """Config d1 size, 60 steps (the bench runs many steps; the 3-step lindblad_n128 pins only the start)."""
    _lindblad_case("lindblad_n128_long", N=128, nc=1, ne=2, Nt=60, dt=5e-3, seed=15, keep_all=False)


@golden
def redfield_n128():
    """Config d1 Redfield half at its benchmarked size: N = 128, one Hermitian a_op, flat spectrum 0.05
    (oqs.py:519-570 redfield_tensor, then RedfieldSolver.evolve -> _redfield, oqs.py:57-81, 364-459).  The csr R
    has N^4 = 2.7e8 nonzeros; a few of its rows are kept (R[rows, :]) to pin the tensor itself."""
    import pyqed.oqs as oqs
    N, Nt, dt = 128, 6, 0.02
    rng = np.random.default_rng(5)
    a = rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N))
    H = (a + a.conj().T) / 2 / np.sqrt(N)
    x = rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N))
    a_op = 0.2 * (x + x.conj().T) / 2 / np.sqrt(N)
    E = np.array([_herm(rng, N, 1 / np.sqrt(N)), np.diag(np.arange(N) / N).astype(complex)])
    psi = rng.standard_normal(N) + 1j * rng.standard_normal(N)
    psi /= np.linalg.norm(psi)
    rho0 = np.outer(psi, psi.conj())
    sol = oqs.RedfieldSolver(H, c_ops=[a_op], spectra=[SPECTRA["flat005"]])
    R, evecs = sol.redfield_tensor()
    rows = np.array([0, 1, 129, 8191, 16383])
    R_rows = R[rows, :].toarray()
    r = sol.evolve(rho0, dt=dt, Nt=Nt, e_ops=list(E))
    save("redfield_n128", H=H, a_op=a_op, E=E, rho0=rho0, dt=dt, Nt=Nt, spectrum="flat005", evecs=evecs,
         R_rows=R_rows, R_row_index=rows, R_nnz=R.nnz, observables=r.observables, rho_final=r.rholist[-1])


@golden
def corr4_2des_256():
    """Config d5 at its benchmarked grid: correlation_4op_3t(..., 'lccc', tau = 0.5 arange(256)) (oqs.py:268-357)
    on the 3-level ladder (Redfield a_op diag(0,1,2), flat 0.05); (t3, t1) slices at t2 index 0 and 37, for the
    unperturbed ladder and for members 0 and 1 of bench.py's static-disorder ensemble (seed 3)."""
    import pyqed.oqs as oqs
    tau = 0.5 * np.arange(256)
    rng = np.random.default_rng(3)
    dE = np.array([0.0, 0.05, 0.08]) * rng.standard_normal((2, 3))
    Es = [np.array([0.0, 1.0, 1.5])] + [np.array([0.0, 1.0, 1.5]) + dE[m] for m in range(2)]
    out = dict(tau=tau, E=np.array(Es), j=np.array([0, 37]))
    for m, E in enumerate(Es):
        H, dip, a, rho0 = _three_level(E)
        sol = oqs.RedfieldSolver(H, c_ops=[a], spectra=[SPECTRA["flat005"]])
        sol.redfield_tensor()
        sol.propagator(tau)
        cube = sol.correlation_4op_3t(rho0, [dip, dip, dip, dip], "lccc", tau)
        out[f"m{m}_j0"] = cube[:, 0, :]
        out[f"m{m}_j37"] = cube[:, 37, :]
        del cube
    save("corr4_2des_256", **out)


@golden
def spo2_256():
    """Config d2 at its benchmarked size: SPO2.run (wpd.py:692-758) on 256 x 256 x 2 with the bench potential,
    dt = 0.05, 20 Strang steps (return_states=True); the final state and the populations along the way."""
    from pyqed.wpd import SPO2
    n, nt, nout, dt = 256, 20, 5, 0.05
    x, y, v0, v1, c, psi0 = spo2_model(n)
    sol = SPO2(x, y, mass=[1.0, 1.0], nstates=2)
    sol.set_DPES([v0, v1], [[[0, 1], c]])
    r = sol.run(psi0, dt=dt, nt=nt, nout=nout)
    dx = x[1] - x[0]
    pops = np.array([[np.vdot(p[:, :, k], p[:, :, k]).real * dx * dx for k in range(2)] for p in r.psilist])
    save("spo2_256", dt=dt, nt=nt, nout=nout, n=n, psi_final=r.psilist[-1], populations=pops,
         n_psilist=len(r.psilist), times=r.times, exp_K_row7=sol.exp_K[7], exp_V_half_row100=sol.exp_V_half[100])


def spo2_model_rect(nx, ny, ns=2, L=6.0):
    """spo2_model on an nx x ny grid with ns surfaces: 1/2((X + 1 - a)^2 + Y^2) + 0.05 a, couplings 0.2 X / (1 + |a-b|)
    between neighbours a, a + 1 (ns > 2 exercises the host eigh build, wpd.py:583-623)."""
    x = np.linspace(-L, L, nx)
    y = np.linspace(-L * 0.9, L * 0.9, ny)
    X, Y = np.meshgrid(x, y, indexing="ij")
    surfaces = [0.5 * ((X + 1 - a) ** 2 + Y ** 2) + 0.05 * a for a in range(ns)]
    couplings = [[[a, a + 1], 0.2 * X + 0.05 * Y] for a in range(ns - 1)]
    psi0 = np.zeros((nx, ny, ns), dtype=complex)
    psi0[:, :, 0] = np.exp(-((X + 1.5) ** 2 + Y ** 2) / 2 + 0.5j * X) / np.sqrt(np.pi)
    return x, y, surfaces, couplings, psi0


def _spo2_rect_case(name, nx, ny, ns, nt, nout, dt, full=True):
    """SPO2.run (wpd.py:692-758, return_states=True) on a non-power-of-two grid: the reference transforms any
    length with scipy.fftpack (wpd.py:837-848).  full=False keeps a strided sample of each state (large grids)."""
    from pyqed.wpd import SPO2
    x, y, surfaces, couplings, psi0 = spo2_model_rect(nx, ny, ns)
    sol = SPO2(x, y, mass=[1.0, 1.3], nstates=ns)
    sol.set_DPES(surfaces, couplings)
    r = sol.run(psi0, dt=dt, nt=nt, nout=nout)
    dx, dy = x[1] - x[0], y[1] - y[0]
    pops = np.array([[np.vdot(p[:, :, k], p[:, :, k]).real * dx * dy for k in range(ns)] for p in r.psilist])
    out = dict(nx=nx, ny=ny, ns=ns, dt=dt, nt=nt, nout=nout, populations=pops, n_psilist=len(r.psilist),
               times=r.times)
    if full:
        out["psilist"] = np.array(r.psilist)
    else:
        out["psi_final_sample"] = r.psilist[-1][::16, ::16]
        out["psi_final_row"] = r.psilist[-1][nx // 2]
        out["psi_final_col"] = r.psilist[-1][:, ny // 3]
    save(name, **out)


@golden
def spo2_20x20():
    _spo2_rect_case("spo2_20x20", 20, 20, 2, nt=6, nout=2, dt=0.05)


@golden
def spo2_96x80():
    _spo2_rect_case("spo2_96x80", 96, 80, 2, nt=4, nout=2, dt=0.05)


@golden
def spo2_67x45_ns3():
    """67 is a prime above the direct-radix limit (Bluestein axis); three surfaces."""
    _spo2_rect_case("spo2_67x45_ns3", 67, 45, 3, nt=4, nout=2, dt=0.05)


@golden
def spo2_12x10_ns9():
    """Nine surfaces (above round 2's ns <= 8 cap)."""
    _spo2_rect_case("spo2_12x10_ns9", 12, 10, 9, nt=3, nout=1, dt=0.05)


@golden
def spo2_1024():
    """1024 x 1024 x 2 (round 2 refused ns * n / 4 > 256): 3 Strang steps; strided sample + one row / column."""
    _spo2_rect_case("spo2_1024", 1024, 1024, 2, nt=3, nout=1, dt=0.05, full=False)


@golden
def spo3_24x20x18():
    """SPO3 (wpd.py:1105-1432, numpy fftn) on a 24 x 20 x 18 x 2 grid."""
    from pyqed.wpd import SPO3
    x, y, z = np.linspace(-6, 6, 24), np.linspace(-5, 5, 20), np.linspace(-5.5, 5.5, 18)
    X, Y, Z = np.meshgrid(x, y, z, indexing="ij")
    sol = SPO3(x, y, z, masses=[1.0, 1.2, 0.9], nstates=2)
    sol.set_DPES([0.5 * ((X + 1) ** 2 + Y ** 2 + Z ** 2), 0.5 * ((X - 1) ** 2 + Y ** 2 + Z ** 2)],
                 [[[0, 1], 0.2 * X]])
    psi0 = np.zeros((24, 20, 18, 2), dtype=complex)
    psi0[..., 1] = np.exp(-((X + 1) ** 2 + Y ** 2 + Z ** 2) / 2 + 0.3j * Y) / np.pi ** 0.75
    r = sol.run(psi0=psi0, dt=0.2, nt=4, nout=2)
    save("spo3_24x20x18", dt=0.2, nt=4, nout=2, psilist=np.array(r.psilist), psi=r.psi)


@golden
def spo1d_any():
    """SPO.run (wpd.py:225-273) on 50, 97 (prime: Bluestein), 200, 2053 (prime, M = 4320) and 6000 (beyond the
    LDS line: direct DFT) points."""
    from pyqed.wpd import SPO
    out = {}
    for n, nt, nout in ((50, 12, 3), (97, 7, 2), (200, 10, 1), (2053, 4, 1), (6000, 3, 1)):
        x = np.linspace(-8, 8, n)
        psi0 = (np.exp(-(x + 2) ** 2 / 2 + 1j * 0.5 * x) / np.pi ** 0.25).astype(complex)
        sol = SPO(x, mass=1.0)
        sol.set_potential(lambda x: x ** 2 / 2)
        r = sol.run(psi0, dt=0.01, nt=nt, nout=nout)
        out[f"n{n}_nt"] = nt
        out[f"n{n}_nout"] = nout
        out[f"n{n}_psilist"] = np.array(r.psilist).reshape(-1, n)
        out[f"n{n}_psi"] = r.psi
    out["sizes"] = np.array([50, 97, 200, 2053, 6000])
    save("spo1d_any", **out)


@golden
def deom_run_bench_long():
    """Config d4 (L = 12, npsd = 4 -> K = 5, 6188 ADOs) for 25 steps at the bench's dt = 0.002 (DEOMSolver.run,
    heom/deom.py:1072-1114): Tr(p1 rho_0) along the way and the final ADO set."""
    save("deom_run_bench_long", **_deom_case(lmax=12, npsd=4, nt=25, dt=0.002))


if __name__ == "__main__":
    names = sys.argv[1:] or list(GENERATORS)
    for n in names:
        GENERATORS[n]()
