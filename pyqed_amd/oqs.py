"""Open-quantum-system solvers on MI355X (drop-in for pyqed/oqs.py).

Class surface mirrors the reference:
  LindbladSolver(H, c_ops, e_ops).run(rho0, dt, Nt, t0, e_ops, return_result)
      -> Result  (pyqed/oqs.py:1114-1187, loop _lindblad oqs.py:1596-1696)

All propagation runs in libqdyn (HIP).  Host code only converts operators and
packages results.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import _lib
from ._util import default_device, issparse, stack_ops, to_device, to_numpy
from .mol import Result

try:
    from scipy.sparse import csr_matrix
except Exception:  # pragma: no cover
    csr_matrix = None


# --------------------------------------------------------------------------- functional
# Below this many matrices the general kernel's split path (a workgroup per output block and phase)
# outruns the persistent Hermitian kernel (one workgroup per matrix): tools/glf_split_bench.py.
HERM_MIN_BATCH = 192        # Redfield (glf_rk4): persistent Hermitian kernel from this batch size
HERM_SPLIT_MIN_BATCH = 16   # Lindblad: Hermitian kernels from this batch size (qd_lindblad_rk4_herm runs its
                            # pair-block split path below 208 matrices and the persistent kernel from there)
HERM_NP64_MIN_BATCH = 160   # 33 <= N <= 64 (padded to 64): the general split-K path up to here
                            # (profiles/r03/lindblad/hsplit_np64_sweep.txt: B = 64 702k general vs 483k persistent
                            # Hermitian DM-steps/s; B = 192 1.18M vs 1.40M)


_HERM_CHECKED = {}   # id(H) -> (weakref to H, H._version, H.data_ptr(), result)


def _is_hermitian_cached(H: torch.Tensor) -> bool:
    """H == H^+ bit for bit.  The check is a device reduction plus a host synchronisation, so a True result is kept
    per tensor object, version and storage address (a weak reference guards against a new tensor at a recycled id; an
    in-place torch update bumps _version; a re-pointed .data changes data_ptr): repeated calls on the same
    Hamiltonian skip it.  Writes torch cannot see -- raw device-pointer writes through ctypes / DLPack into H's
    storage -- are not detected: a caller that mutates H that way passes hermitian= explicitly."""
    import weakref
    key = id(H)
    hit = _HERM_CHECKED.get(key)
    if hit is not None and hit[0]() is H and hit[1] == H._version and hit[2] == H.data_ptr():
        return True
    res = bool(torch.equal(H, H.transpose(-1, -2).conj()))
    if len(_HERM_CHECKED) > 64:
        _HERM_CHECKED.clear()
    if res:   # a False result is cheap to recompute and must not stick (the Hermitian kernel is the risky pick)
        _HERM_CHECKED[key] = (weakref.ref(H), H._version, H.data_ptr(), res)
    else:
        _HERM_CHECKED.pop(key, None)
    return res


def lindblad_rk4(H: torch.Tensor, c_ops: torch.Tensor | None, rho: torch.Tensor, dt: float, nsteps: int,
                 e_ops: torch.Tensor | None = None, save_every: int = 0, stream=None,
                 hermitian: bool | None = None):
    """Propagate a batch of density matrices in place with RK4 on the GPU.

    H [N,N], c_ops [nc,N,N] or None, rho [B,N,N] (or [N,N]), e_ops [ne,N,N] or None
    (all complex128 on one cuda device).  Returns (obs [B,nsteps+1,ne] | None,
    snap [B,nsteps//save_every,N,N] | None).  Reference RHS: oqs.py:697-714.

    hermitian: use the Hermitian-state kernel (qd_lindblad_rk4_herm: L[rho] = X + X^+,
    1 + 2nc complex GEMMs per RHS instead of 2 + 2nc, one persistent workgroup per matrix).
    None = auto: on when H and every rho in the batch equal their conjugate transposes bit for bit,
    N <= 128 and B >= HERM_SPLIT_MIN_BATCH, or one or two matrices at 64 < N <= 128 with 1 or 2 collapse operators (the
    Hermitian single-trajectory launch, glf_single_herm_kernel).  From 208 matrices the library runs the persistent
    Hermitian kernel (one workgroup per matrix); below that its pair-block split path
    (one workgroup per upper block pair, 2/3 of the general split path's GEMM work); smaller batches run
    the general kernel's split path, which spreads each matrix over many workgroups (qd_lindblad_rk4:
    8.3k instead of 1.3k steps/s for one N = 128 trajectory).  The Lindblad generator preserves
    Hermiticity, and the Hermitian kernels keep it exact at every stage.
    """
    squeeze = rho.dim() == 2
    if squeeze:
        rho = rho.unsqueeze(0)
    if rho.dim() != 3 or rho.shape[-1] != rho.shape[-2]:
        raise ValueError(f"rho must be [B,N,N] or [N,N], got {tuple(rho.shape)}")
    B, N = rho.shape[0], rho.shape[-1]
    dev = rho.device
    _lib.ensure_device(dev)
    for name, t in (("H", H), ("rho", rho), ("c_ops", c_ops), ("e_ops", e_ops)):
        if t is not None and (t.dtype != torch.complex128 or t.device != dev or not t.is_contiguous()):
            raise ValueError(f"{name} must be a contiguous complex128 tensor on {dev}")
    if tuple(H.shape) != (N, N):
        raise ValueError(f"H has shape {tuple(H.shape)}, expected {(N, N)}")
    for name, t in (("c_ops", c_ops), ("e_ops", e_ops)):
        if t is not None and (t.dim() != 3 or tuple(t.shape[1:]) != (N, N)):
            raise ValueError(f"{name} must be [k,{N},{N}], got {tuple(t.shape)}")
    nc = 0 if c_ops is None else c_ops.shape[0]
    ne = 0 if e_ops is None else e_ops.shape[0]
    obs = torch.empty((B, nsteps + 1, ne), dtype=torch.complex128, device=dev) if ne else None
    nsave = nsteps // save_every if save_every > 0 else 0
    snap = torch.empty((B, nsave, N, N), dtype=torch.complex128, device=dev) if nsave else None
    st = stream if stream is not None else _lib.stream_ptr(dev)
    # X + X^+ equals the reference's -i[H, rho] + D[rho] only for Hermitian H and rho (oqs.py:697-714 uses
    # rho H, not rho H^+), so the Hermitian kernel is gated on both, bit for bit.
    h_herm = _is_hermitian_cached(H)
    if hermitian is None:
        min_b = HERM_NP64_MIN_BATCH if 32 < N <= 64 else HERM_SPLIT_MIN_BATCH
        # one or two trajectories at N_p = 128 with 1 or 2 collapse operators: the Hermitian single launch
        single_h = 64 < N <= 128 and B <= 2 and 1 <= nc <= 2
        hermitian = (N <= 128 and (B >= min_b or single_h) and h_herm
                     and bool(torch.equal(rho, rho.transpose(-1, -2).conj())))
    elif hermitian and not h_herm:
        raise ValueError("hermitian=True needs a Hermitian H (the X + X^+ form drops the anti-Hermitian part of H)")
    fn = "qd_lindblad_rk4_herm" if hermitian else "qd_lindblad_rk4"
    with torch.cuda.device(dev):
        rc = getattr(_lib.load(), fn)(_lib.ptr(H), _lib.ptr(c_ops), nc, _lib.ptr(rho), B, N, float(dt),
                                      int(nsteps), _lib.ptr(e_ops), ne, _lib.ptr(obs), _lib.ptr(snap),
                                      int(save_every if nsave else 0), st)
    _lib.check(rc, fn)
    return obs, snap


# --------------------------------------------------------------------------- solvers
class LindbladSolver:
    """Drop-in for pyqed.oqs.LindbladSolver (oqs.py:1114)."""

    def __init__(self, H=None, c_ops=None, e_ops=None):
        self.c_ops = c_ops
        self.e_ops = e_ops
        self.H = H
        return

    def set_c_ops(self, c_ops):
        self.c_ops = c_ops

    def set_e_ops(self, e_ops):
        self.e_ops = e_ops

    def setH(self, H):
        self.H = H

    def configure(self, c_ops, e_ops):
        self.c_ops = c_ops
        self.e_ops = e_ops

    def liouvillian(self):
        from . import superoperator as superop
        return superop.liouvillian(self.H, self.c_ops)

    def run(self, rho0, dt, Nt, t0=0., e_ops=None, return_result=True, return_states=True):
        """Propagate rho0 for Nt RK4 steps (oqs.py:1149-1187).

        Returns a Result with observables (Nt+1, n_e) including t0 and rholist of Nt
        csr matrices excluding rho0, as oqs._lindblad (oqs.py:1676-1696).
        `return_states=False` (extension) skips the per-step snapshots.
        """
        if isinstance(self.H, list):
            return _lindblad_driven(self.H, rho0=rho0, c_ops=self.c_ops, e_ops=e_ops, Nt=Nt, dt=dt, t0=t0,
                                    return_states=return_states)
        return _lindblad(self.H, rho0, c_ops=self.c_ops, e_ops=e_ops, Nt=Nt, dt=dt,
                         return_states=return_states)

    # ---- quantum-regression correlation functions (oqs.py:1193-1329)
    def correlation_2op_1t(self, rho0, a_op, b_op, dt, Nt, output='cor.dat'):
        """<A(t)B> (oqs.py:1193-1222 -> _correlation_2p_1t oqs.py:717-791): rho <- B rho0,
        Nt RK4 steps, cor[k] = Tr(A rho_k) AFTER each step (t0 excluded); writes `output`."""
        return _correlation_2p_1t(self.H, rho0, [a_op, b_op], self.c_ops, dt, Nt, output=output)

    def correlation_3op_1t(self, rho0, oplist, dt=0.005, Nt=1):
        """<A B(t) C> (oqs.py:1224-1243): Tr(B rho(t)) from rho(0) = C rho0 A, Nt+1 values incl. t0."""
        a_op, b_op, c_op = oplist
        r0 = _dense(c_op) @ _dense(rho0) @ _dense(a_op)
        return _lindblad(self.H, r0, c_ops=self.c_ops, e_ops=[b_op], dt=dt, Nt=Nt,
                         return_states=False).observables[:, 0]

    def correlation_3op_2t(self, rho0, ops, dt, Nt, Ntau):
        """<A(t) B(t+tau) C(t)> (oqs.py:1264-1296).  All Nt restarts C rho(t_k) A are propagated
        together as ONE batch on the GPU.  The reference fills an (Nt, Ntau) array with Ntau+1
        observables and raises; this returns corr[t_k, tau_j] for tau_j = j*dt, j < Ntau."""
        a_op, b_op, c_op = (_dense(x) for x in ops)
        dev = default_device()
        H = _dense(self.H)
        N = H.shape[0]
        Hd = torch.from_numpy(H).to(dev)
        Cd = stack_ops(self.c_ops or [], N, dev)
        rho = torch.from_numpy(_dense(rho0).reshape(1, N, N).copy()).to(dev)
        _, snap = lindblad_rk4(Hd, Cd, rho, dt, Nt, None, save_every=1)   # rho_t, t = dt..Nt dt
        at = torch.from_numpy(a_op).to(dev)
        ct = torch.from_numpy(c_op).to(dev)
        r = snap[0].contiguous()                                           # [Nt, N, N]
        sandwich(ct, at, r)                                                # C rho(t_k) A, batched

        Ed = torch.from_numpy(b_op.reshape(1, N, N).copy()).to(dev)
        obs, _ = lindblad_rk4(Hd, Cd, r, dt, Ntau, Ed)
        return obs[:, :Ntau, 0].cpu().numpy()

    def correlation_4op_1t(self, rho0, ops, dt, nt):
        """<A B(t) C(t) D> (oqs.py:1298-1313, the definition that wins): 3op_1t with [a, b@c, d]."""
        if len(ops) != 4:
            raise ValueError('Number of operators is not 4.')
        a, b, c, d = ops
        return self.correlation_3op_1t(rho0, [a, _dense(b) @ _dense(c), d], dt, nt)

    def correlation_4op_2t(self, rho0, ops, dt, nt, ntau):
        """<A(t) B(t+tau) C(t+tau) D(t)> (oqs.py:1315-1329): 3op_2t with [a, b@c, d]."""
        if len(ops) != 4:
            raise ValueError('Number of operators is not 4.')
        a, b, c, d = ops
        return self.correlation_3op_2t(rho0, [a, _dense(b) @ _dense(c), d], dt, nt, ntau)


def _lindblad_driven(H, rho0, c_ops=None, e_ops=None, Nt=1, dt=0.005, t0=0., return_result=True,
                     return_states=True):
    """oqs.py:1699-1806: H = [H0, [H1, f1], ...], H(t) = H0 - sum f_i(t) H_i evaluated once per step at
    t_k = t0 + (k+1) dt.  observables (Nt, n_e) EXCLUDE t0; rholist has Nt csr matrices.
    (With the csr H0 the reference requires, `Ht += ...` rebinds instead of mutating H0, so no
    drive accumulates; a dense H0 fails in the reference's RHS.)"""
    if c_ops is None:
        c_ops = []
    if e_ops is None:
        e_ops = []
    dev = default_device()
    H0 = _dense(H[0])
    N = H0.shape[0]
    drives = H[1:]
    nd = len(drives)
    Hd = torch.from_numpy(np.ascontiguousarray(np.array([_dense(h[0]) for h in drives]).reshape(nd, N, N))).to(dev)
    f = np.zeros((Nt, nd), dtype=complex)
    t = t0
    for k in range(Nt):
        t += dt
        f[k] = [h[1](t) for h in drives]
    f = np.ascontiguousarray(f)
    Cd = stack_ops(c_ops, N, dev)
    Ed = stack_ops(e_ops, N, dev)
    rho = to_device(rho0, dev).reshape(1, N, N).clone()
    ne = len(e_ops)
    obs = torch.empty((1, Nt + 1, ne), dtype=torch.complex128, device=dev) if ne else None
    snap = torch.empty((1, Nt, N, N), dtype=torch.complex128, device=dev) if (return_states and Nt) else None
    H0d = torch.from_numpy(H0).to(dev)
    _lib.ensure_device(dev)
    with torch.cuda.device(dev):
        rc = _lib.load().qd_lindblad_driven_rk4(H0d.data_ptr(), Hd.data_ptr(), nd, f.ctypes.data, _lib.ptr(Cd),
                                                0 if Cd is None else Cd.shape[0], rho.data_ptr(), 1, N, float(dt),
                                                int(Nt), _lib.ptr(Ed), ne, _lib.ptr(obs), _lib.ptr(snap),
                                                1 if snap is not None else 0, _lib.stream_ptr(dev))
    _lib.check(rc, "qd_lindblad_driven_rk4")
    result = Result(dt=dt, Nt=Nt, rho0=rho0)
    result.observables = obs[0, 1:].cpu().numpy() if obs is not None else np.zeros((Nt, 0), complex)
    if snap is not None:
        host = snap[0].cpu().numpy()
        result.rholist = [csr_matrix(host[k]) for k in range(Nt)]
    else:
        result.rholist = []
    result.rho = rho[0].cpu().numpy()
    return result


def _dense(a):
    return np.ascontiguousarray(to_numpy(a, np.complex128))


def _correlation_2p_1t(H, rho0, ops, c_ops, dt, Nt, method='lindblad', output='cor.dat'):
    """oqs.py:717-791 on the GPU."""
    if method != 'lindblad':
        raise NotImplementedError(f'The method {method} has not been implemented yet! Please try lindblad.')
    A, B = ops
    r0 = _dense(B) @ _dense(rho0)
    res = _lindblad(H, r0, c_ops=c_ops or [], e_ops=[A], Nt=Nt, dt=dt, return_states=False)
    cor = res.observables[1:, 0].copy()
    if output is not None:
        with open(output, 'w') as f:
            t = 0.0
            for k in range(Nt):
                t += dt
                f.write('{} {} \n'.format(t, cor[k]))
    return cor


def _lindblad(H, rho0, c_ops, e_ops=None, Nt=1, t0=0, dt=0.005, return_result=True, return_states=True):
    """GPU restatement of oqs._lindblad (oqs.py:1596-1696)."""
    if e_ops is None:
        e_ops = []
    if c_ops is None:
        c_ops = []
    dev = default_device()
    Hn = to_numpy(H, np.complex128)
    N = Hn.shape[0]
    Hd = torch.from_numpy(np.ascontiguousarray(Hn)).to(dev)
    Cd = stack_ops(c_ops, N, dev)
    Ed = stack_ops(e_ops, N, dev)
    rho = to_device(rho0, dev).reshape(1, N, N).clone()
    obs, snap = lindblad_rk4(Hd, Cd, rho, dt, Nt, Ed, save_every=1 if return_states else 0)
    torch.cuda.synchronize(dev)

    result = Result(dt=dt, Nt=Nt, rho0=rho0)
    if obs is not None:
        result.observables = obs[0].cpu().numpy()
    else:
        result.observables = np.zeros((Nt + 1, 0), dtype=complex)
    if return_states and snap is not None:
        host = snap[0].cpu().numpy()
        result.rholist = [csr_matrix(host[k]) for k in range(Nt)]
    else:
        result.rholist = []
    result.rho = rho[0].cpu().numpy()
    return result


# --------------------------------------------------------------------------- GLF
def glf_rk4(P, Q, L, R, rho, dt, nsteps, e_ops=None, save_every=0, stream=None, hermitian=False):
    """d rho/dt = P rho + rho Q + sum_c L_c rho R_c, batched RK4 on the GPU (qd_glf_rk4).

    P, Q [N,N]; L, R [npairs,N,N] or None; rho [B,N,N] in place; e_ops [ne,N,N] or None.
    hermitian=True: the Hermitian-state form d rho/dt = X + X^+, X = P rho + sum_c L_c rho R_c
    (qd_glf_rk4_herm; Q is unused and R holds the W_c): rho must be exactly Hermitian, N <= 128."""
    B, N = rho.shape[0], rho.shape[-1]
    dev = rho.device
    _lib.ensure_device(dev)
    for name, t in (("P", P), ("Q", Q), ("rho", rho), ("L", L), ("R", R), ("e_ops", e_ops)):
        if t is not None and (t.dtype != torch.complex128 or t.device != dev or not t.is_contiguous()):
            raise ValueError(f"{name} must be a contiguous complex128 tensor on {dev}")
    if rho.dim() != 3 or rho.shape[1] != N:
        raise ValueError(f"rho must be [B,N,N], got {tuple(rho.shape)}")
    npairs = 0 if L is None else L.shape[0]
    ne = 0 if e_ops is None else e_ops.shape[0]
    obs = torch.empty((B, nsteps + 1, ne), dtype=torch.complex128, device=dev) if ne else None
    nsave = nsteps // save_every if save_every > 0 else 0
    snap = torch.empty((B, nsave, N, N), dtype=torch.complex128, device=dev) if nsave else None
    st = stream if stream is not None else _lib.stream_ptr(dev)
    with torch.cuda.device(dev):
        if hermitian:
            rc = _lib.load().qd_glf_rk4_herm(_lib.ptr(P), _lib.ptr(L), _lib.ptr(R), npairs, _lib.ptr(rho), B, N,
                                             float(dt), int(nsteps), _lib.ptr(e_ops), ne, _lib.ptr(obs),
                                             _lib.ptr(snap), int(save_every if nsave else 0), st)
        else:
            rc = _lib.load().qd_glf_rk4(_lib.ptr(P), _lib.ptr(Q), _lib.ptr(L), _lib.ptr(R), npairs, _lib.ptr(rho), B,
                                        N, float(dt), int(nsteps), _lib.ptr(e_ops), ne, _lib.ptr(obs), _lib.ptr(snap),
                                        int(save_every if nsave else 0), st)
    _lib.check(rc, "qd_glf_rk4_herm" if hermitian else "qd_glf_rk4")
    return obs, snap


def superop_rk4(L: torch.Tensor, v: torch.Tensor, dt, nsteps, W: torch.Tensor | None = None, save_every=0):
    """d v/dt = L v, batched RK4 with a dense superoperator (qd_superop_rk4).  L [N2,N2], v [B,N2] in place,
    W [ne,N2] observable weights.  Returns (obs [B,nsteps+1,ne] | None, snap [B,nsave,N2] | None)."""
    dev = v.device
    _lib.ensure_device(dev)
    for name, t in (("L", L), ("v", v), ("W", W)):
        if t is not None and (t.dtype != torch.complex128 or t.device != dev or not t.is_contiguous()):
            raise ValueError(f"{name} must be a contiguous complex128 tensor on {dev}")
    B, N2 = v.shape
    if tuple(L.shape) != (N2, N2) or (W is not None and (W.dim() != 2 or W.shape[1] != N2)):
        raise ValueError(f"superop_rk4: L {tuple(L.shape)} / W shapes do not match v {tuple(v.shape)}")
    ne = 0 if W is None else W.shape[0]
    obs = torch.empty((B, nsteps + 1, ne), dtype=torch.complex128, device=dev) if ne else None
    nsave = nsteps // save_every if save_every > 0 else 0
    snap = torch.empty((B, nsave, N2), dtype=torch.complex128, device=dev) if nsave else None
    with torch.cuda.device(dev):
        rc = _lib.load().qd_superop_rk4(_lib.ptr(L), _lib.ptr(v), B, N2, float(dt), int(nsteps), _lib.ptr(W), ne,
                                        _lib.ptr(obs), _lib.ptr(snap), int(save_every if nsave else 0),
                                        _lib.stream_ptr(dev))
    _lib.check(rc, "qd_superop_rk4")
    return obs, snap


def lindblad_superop(H: torch.Tensor, c_ops: torch.Tensor | None) -> torch.Tensor:
    """Dense Lindblad superoperator [N^2, N^2] built on the device (qd_superop_lindblad): the matrix of
    oqs.liouvillian (oqs.py:697-714) on row-major vec(rho), i.e. superoperator.liouvillian (superoperator.py:29-58)
    without the host kron assembly (N = 128: 4 GiB)."""
    dev = H.device
    _lib.ensure_device(dev)
    N = H.shape[0]
    nc = 0 if c_ops is None else c_ops.shape[0]
    out = torch.empty((N * N, N * N), dtype=torch.complex128, device=dev)
    with torch.cuda.device(dev):
        rc = _lib.load().qd_superop_lindblad(_lib.ptr(H), _lib.ptr(c_ops), nc, N, out.data_ptr(), _lib.stream_ptr(dev))
    _lib.check(rc, "qd_superop_lindblad")
    return out


def glf_superop(P: torch.Tensor, Q: torch.Tensor, L: torch.Tensor | None, R: torch.Tensor | None) -> torch.Tensor:
    """Dense superoperator of d rho/dt = P rho + rho Q + sum_c L_c rho R_c on row-major vec(rho)
    (qd_superop_from_glf), e.g. RedfieldSolver.glf_terms() -> the reference's R (oqs.py:563-570)."""
    dev = P.device
    _lib.ensure_device(dev)
    N = P.shape[0]
    nc = 0 if L is None else L.shape[0]
    out = torch.empty((N * N, N * N), dtype=torch.complex128, device=dev)
    with torch.cuda.device(dev):
        rc = _lib.load().qd_superop_from_glf(_lib.ptr(P), _lib.ptr(Q), _lib.ptr(L), _lib.ptr(R), nc, N, out.data_ptr(),
                                             _lib.stream_ptr(dev))
    _lib.check(rc, "qd_superop_from_glf")
    return out


def _redfield(R, rho0, evecs=None, Nt=1, dt=0.005, t0=0, e_ops=[], return_result=True):
    """oqs.py:364-459 with an explicit (dense or csr) R: RK4 on vec(rho~) on the GPU, observables
    (Nt, n_e) EXCLUDING t0, rholist back-transformed with dag(evecs)."""
    N = np.asarray(rho0.toarray() if hasattr(rho0, "toarray") else rho0).shape[0]
    dev = default_device()
    if e_ops is None:
        e_ops = []
    Rd = torch.from_numpy(np.ascontiguousarray(_dense(R))).to(dev)
    rho = to_device(rho0, dev).reshape(1, N, N).clone()
    Ed = stack_ops(e_ops, N, dev)
    if evecs is not None:
        ev = torch.from_numpy(np.ascontiguousarray(np.asarray(evecs, dtype=complex))).to(dev)
        basis_transform(ev, rho, inverse=False)
        if Ed is not None:
            basis_transform(ev, Ed, inverse=False)
    W = Ed.transpose(1, 2).reshape(len(e_ops), N * N).contiguous() if Ed is not None else None  # vec(E^T)
    v = rho.reshape(1, N * N).contiguous()
    if return_result == False:  # noqa: E712  (same truthiness as oqs.py:406)
        # oqs.py:406-431: 'obs.dat' gets one line per step, "t" after the increment followed by the
        # observables of the state BEFORE the step, and the final vec(rho) (eigenbasis) is returned.  The
        # reference evaluates obs_dm(vec(rho), e) = e.dot(vec).diagonal(), which fails for any e_op (an
        # N x N operator against an N^2 vector); that failure is reproduced, so only empty e_ops run.
        if len(e_ops):
            raise ValueError(f"shapes ({N},{N}) and ({N * N},) not aligned: {N} (dim 1) != {N * N} (dim 0)")
        superop_rk4(Rd, v, dt, Nt, None, save_every=0)
        t = t0
        with open('obs.dat', 'w') as f_obs:
            for _ in range(Nt):
                t += dt
                f_obs.write('{} \n'.format(t))
        return v[0].cpu().numpy()
    rho0_eb = rho[0].cpu().numpy()
    obs, snap = superop_rk4(Rd, v, dt, Nt, W, save_every=1)
    result = Result(dt=dt, Nt=Nt, rho0=rho0_eb)
    result.observables = obs[0, 1:].cpu().numpy() if obs is not None else np.zeros((Nt, 0), complex)
    if snap is not None:
        back = snap[0].reshape(Nt, N, N).contiguous()
        if evecs is not None:
            basis_transform(ev, back, inverse=True)
        host = back.cpu().numpy()
        result.rholist = [host[k] for k in range(Nt)]
    else:
        result.rholist = []
    return result


def rhs(psi, H):
    """oqs.py:462-463 (host helper of the reference's RK4 RHS)."""
    return H.dot(psi)


def basis_transform(V: torch.Tensor, A: torch.Tensor, inverse=False):
    """In place: A <- V^+ A V (inverse=False, phys.transform) or V A V^+ (inverse=True). A [B,N,N]."""
    dev = A.device
    _lib.ensure_device(dev)
    B, N = A.shape[0], A.shape[-1]
    with torch.cuda.device(dev):
        rc = _lib.load().qd_basis_transform(_lib.ptr(V), _lib.ptr(A), B, N, int(bool(inverse)), _lib.stream_ptr(dev))
    _lib.check(rc, "qd_basis_transform")
    return A


def sandwich(L: torch.Tensor, R: torch.Tensor, A: torch.Tensor):
    """In place A[b] <- L A[b] R on the GPU (qd_sandwich).  A [B,N,N]."""
    dev = A.device
    _lib.ensure_device(dev)
    B, N = A.shape[0], A.shape[-1]
    with torch.cuda.device(dev):
        rc = _lib.load().qd_sandwich(_lib.ptr(L), _lib.ptr(R), _lib.ptr(A), B, N, _lib.stream_ptr(dev))
    _lib.check(rc, "qd_sandwich")
    return A


def _isherm(a):
    return np.allclose(a, a.conj().T)


class RedfieldSolver:
    """Drop-in for pyqed.oqs.RedfieldSolver (oqs.py:30-357).

    redfield_tensor() returns the reference's csr R (built on the host, as the
    reference does); evolve() propagates in the H eigenbasis on the GPU with the
    commutator ("GLF") form of the same generator instead of R.vec(rho)."""

    def __init__(self, H, c_ops=None, spectra=None, e_ops=None):
        self.H = H
        self.c_ops = c_ops
        self.R = None
        self.spectra = spectra
        self.evecs = None
        self.dim = H.shape[0]
        self.U = None
        self.G = None
        self.e_ops = e_ops
        self._glf = None
        self._sos = None

    def idm(self, sp=True):
        from scipy.sparse import identity
        from .superoperator import dm2vec
        if sp:
            return dm2vec(identity(self.dim))
        return dm2vec(identity(self.dim).toarray())

    def configure(self, H, c_ops, e_ops):
        self.c_ops = c_ops
        self.e_ops = e_ops
        self.H = H

    # ---- setup (host): eigenbasis, spectra, Lambda operators (oqs.py:519-560)
    def _prepare(self):
        if self._glf is not None:
            return self._glf
        if self.spectra is None:
            raise TypeError('Specify the bath spectral function.')
        a_ops = self.c_ops or []
        for a in a_ops:
            if not _isherm(to_numpy(a)):
                raise TypeError("Operators in a_ops must be Hermitian.")
        from scipy.linalg import eigh
        evals, evecs = eigh(to_numpy(self.H))
        W = np.real(evals[:, None] - evals[None, :])
        N = len(evals)
        A, Lam = [], []
        for k, a in enumerate(a_ops):
            c = np.zeros((N, N))
            for n in range(N):
                for m in range(N):
                    c[n, m] = self.spectra[k](-W[n, m])
            Ak = evecs.conj().T @ to_numpy(a, np.complex128) @ evecs
            A.append(Ak)
            Lam.append(c * Ak)
        self._glf = (evals, evecs, A, Lam)
        self.evecs = evecs
        return self._glf

    def redfield_tensor(self, secular=False):
        """(R csr (N^2, N^2) with -i included, evecs) as oqs.py:519-570."""
        from scipy.sparse import csr_matrix as _csr
        from .superoperator import left, op2sop, right
        evals, evecs, A, Lam = self._prepare()
        R = 0
        for a, l in zip(A, Lam):
            R = R + op2sop(a).dot(left(l) - right(l.conj().T))
        R = _csr(-1j * op2sop(np.diag(evals)) - R)
        self.R = R
        self.evecs = evecs
        return R, evecs

    def glf_terms(self):
        """(P, Q, L[], R[]) of d rho~/dt = P rho~ + rho~ Q + sum L rho~ R in the eigenbasis."""
        evals, evecs, A, Lam = self._prepare()
        E = np.diag(evals).astype(complex)
        P = -1j * E
        Q = 1j * E
        Ls, Rs = [], []
        for a, l in zip(A, Lam):
            ld = l.conj().T
            P = P - a @ l
            Q = Q - ld @ a
            Ls += [a, l]
            Rs += [ld, a]
        return P, Q, Ls, Rs

    def glf_terms_herm(self):
        """(P, L[], W[]) of the Hermitian-state form d rho~/dt = X + X^+, X = P rho~ + sum_k A_k rho~ Lam_k^+
        (the pair (Lam_k, A_k) of glf_terms is the conjugate transpose of (A_k, Lam_k^+) acting on a
        Hermitian rho~, and Q = P^+)."""
        evals, evecs, A, Lam = self._prepare()
        P = -1j * np.diag(evals).astype(complex)
        Ls, Ws = [], []
        for a, l in zip(A, Lam):
            P = P - a @ l
            Ls.append(a)
            Ws.append(l.conj().T)
        return P, Ls, Ws

    def evolve(self, rho0, dt, Nt, evecs=None, e_ops=[], store_states=False, t0=0, nout=1):
        """oqs.py:57-81 -> _redfield (oqs.py:364-459): observables (Nt, n_e) EXCLUDING t0,
        rholist (Nt) back-transformed to the original basis.  With an R set by the caller (no
        spectra), the dense-superoperator kernel propagates R.vec(rho) as the reference does."""
        if self.spectra is None and self.R is not None:
            return _redfield(self.R, rho0, evecs=self.evecs, Nt=Nt, dt=dt, t0=t0, e_ops=e_ops)
        self._prepare()
        dev = default_device()
        P, Q, Ls, Rs = self.glf_terms()
        N = self.dim
        evecs_t = torch.from_numpy(np.ascontiguousarray(self.evecs.astype(complex))).to(dev)
        rho = to_device(rho0, dev).reshape(1, N, N).clone()
        basis_transform(evecs_t, rho, inverse=False)
        e_ops = e_ops or []
        Ed = stack_ops(e_ops, N, dev)
        if Ed is not None:
            basis_transform(evecs_t, Ed, inverse=False)
        rho0_eb = rho[0].cpu().numpy()
        r0 = to_numpy(rho0, np.complex128)
        # one trajectory (B = 1 < HERM_MIN_BATCH): the general GLF kernel's split path outruns the persistent
        # Hermitian-state kernel, which serves batches of Hermitian states (glf_rk4(..., hermitian=True))
        B = 1
        herm = N <= 128 and B >= HERM_MIN_BATCH and np.array_equal(r0, r0.conj().T)
        if herm:
            # Hermitian input: symmetrise the transformed state (rounding of V^+ rho V only) and propagate
            # with the Hermitian-state kernel (1 + 2 n_a GEMMs per RHS instead of 2 + 4 n_a)
            rho = (0.5 * (rho + rho.transpose(-1, -2).conj())).contiguous()
            P, Ls, Rs = self.glf_terms_herm()
        Pd, Qd = (torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in (P, Q))
        Ld = stack_ops(Ls, N, dev)
        Rd = stack_ops(Rs, N, dev)
        obs, snap = glf_rk4(Pd, Qd, Ld, Rd, rho, dt, Nt, Ed, save_every=1, hermitian=herm)
        result = Result(dt=dt, Nt=Nt, rho0=rho0_eb)
        result.observables = obs[0, 1:].cpu().numpy() if obs is not None else np.zeros((Nt, 0), complex)
        if snap is not None:
            back = snap[0].contiguous()
            basis_transform(evecs_t, back, inverse=True)
            host = back.cpu().numpy()
            result.rholist = [host[k] for k in range(Nt)]
        else:
            result.rholist = []
        torch.cuda.synchronize(dev)
        return result

    # ---- Liouville-space Green's functions
    def _propagator_eom(self, R, t):
        """phys.expm(R, t, 'EOM') (phys.py:2049-2097): U_0 = I, U_{k+1} = rk4(U_k, ldo, dt, R) with ldo(b, A) = A.b
        and dt = t[1] - t[0], i.e. d U/dt = R U.  On the GPU each column of U is one vector of the batched dense
        superoperator RK4 (qd_superop_rk4: MFMA GEMM stages once the batch fills 64-wide blocks), every step saved.
        Returns U (nL, nL, len(t)) with U[:, :, k] = U_k, as np.dstack of the reference's list."""
        from scipy.sparse import issparse
        t = np.asarray(t, dtype=float)
        Nt = len(t)
        Rd = R.toarray() if issparse(R) else np.asarray(R)
        nL = Rd.shape[0]
        U = np.empty((nL, nL, Nt), dtype=complex)
        U[:, :, 0] = np.eye(nL)
        if Nt > 1:
            dev = default_device()
            L = torch.from_numpy(np.ascontiguousarray(Rd.astype(complex))).to(dev)
            v = torch.eye(nL, dtype=torch.complex128, device=dev)       # row b = column b of U
            _, snap = superop_rk4(L, v, float(t[1] - t[0]), Nt - 1, save_every=1)
            U[:, :, 1:] = snap.permute(2, 0, 1).cpu().numpy()          # snap[b, k, a] = U_{k+1}[a, b]
        return U

    def propagator(self, t, method='SOS'):
        """oqs.py:160-214: U (nL, nL, nt); G = -1j U.  'SOS' / 'eseries': eigen form on the GPU; 'EOM': the
        reference's RK4 propagation of the identity (phys.expm) on the dense-superoperator RK4 kernel."""
        if self.R is None:
            raise TypeError('Redfield tensor is not computed. Please call redfield_tensor()')
        if method == 'EOM':
            self.U = self._propagator_eom(self.R, t)
        elif method in ['eseries', 'SOS']:
            from .response import sos_eig, sos_propagator
            lam, U1, U2 = sos_eig(self.R)
            t = np.asarray(t, dtype=float)
            self._sos = (lam, U1, U2, t)
            self.U = sos_propagator(lam, U1, U2, t).cpu().numpy()
        else:
            # the reference falls through to `self.G = -1j * self.U` with U unset
            raise NotImplementedError(f"propagator method {method!r}: choose 'SOS', 'eseries' or 'EOM'")
        self.G = -1j * self.U
        return self.U

    def gf(self, t, w=None, secular=False, k=1, domain='time', method='EOM'):
        """Liouville-space Green's function with Redfield dissipation (oqs.py:136-158).
        'EOM': -1j * expm(R, t), i.e. -1j U_k for every t_k as an (nL, nL, nt) array (the reference multiplies the
        expm list by -1j, which raises; the array is its evident meaning).  'eseries' / 'diag' / 'diagonalization':
        getG(1j R, t) (oqs.py:465-508), G(t) = -1j exp(R t) in the eigen form, evaluated on the GPU.  As in the
        reference, `w`, `k` and `domain` are accepted and unused (gf calls getG(1j R, t) with getG's default
        domain='time')."""
        if self.R is None:
            self.redfield_tensor(secular=secular)
        if method == 'EOM':
            return -1j * self._propagator_eom(self.R, t)
        if method in ['eseries', 'diag', 'diagonalization']:
            from .response import sos_eig, sos_propagator
            lam, U1, U2 = sos_eig(self.R)
            return -1j * sos_propagator(lam, U1, U2, np.asarray(t, dtype=float)).cpu().numpy()
        return None

    def correlation_4op_3t(self, rho0, oplist, signature, tau):
        """<<I|A G(tau3) B G(tau2) C G(tau1) D|rho0>> cube [i=tau3, j=tau2, k=tau1] (oqs.py:268-357)."""
        if len(oplist) != 4:
            raise ValueError('Number of operators is not 4.')
        if self.G is None:
            self.propagator(tau)
        from .response import eigen_factors, response_cube
        lam, U1, U2, tG = self._sos
        alpha, B, C, beta = eigen_factors(lam, U1, U2, oplist, signature, rho0)
        return response_cube(lam, alpha, B, C, beta, tG, tG, tG).cpu().numpy()


class HEOMSolver:
    """Drop-in for pyqed.oqs.HEOMSolver (oqs.py:1332-1403): single-exponential chain with the
    reference's explicit in-place sweep (oqs._heom, oqs.py:1808-1875) on the GPU."""

    def __init__(self, H=None, c_ops=None, e_ops=None):
        self.c_ops = c_ops
        self.e_ops = e_ops
        self.H = H

    def set_c_ops(self, c_ops):
        self.c_ops = c_ops

    def set_e_ops(self, e_ops):
        self.e_ops = e_ops

    def setH(self, H):
        self.H = H

    def configure(self, c_ops, e_ops):
        self.c_ops = c_ops
        self.e_ops = e_ops

    def run(self, rho0, dt, nt, temperature, cutoff, reorganization, nado):
        return _heom(self.H, rho0, self.c_ops, self.e_ops, temperature, cutoff, reorganization, nado, dt, nt)

    def correlation_2op_1t(self, rho0, a_op, b_op, dt, Nt, output='cor.dat'):
        """oqs.py:1374-1403: as the reference, computed with the Lindblad RHS."""
        return _correlation_2p_1t(self.H, rho0, [a_op, b_op], self.c_ops, dt, Nt, output=output)


def _heom(H, rho0, c_ops, e_ops, temperature, cutoff, reorganization, nado, dt, nt, fname=None,
          return_result=True):
    """oqs.py:1808-1875: observables (len(e_ops), nt) after every sweep step."""
    gamma, T, reorg = cutoff, temperature, reorganization
    D0 = reorg * gamma * (1.0 / np.tanh(gamma / (2. * T)) - 1j)
    dev = default_device()
    _lib.ensure_device(dev)
    Hn = _dense(H)
    ns = Hn.shape[0]
    e_ops = list(e_ops or [])
    ados = torch.zeros((1, nado, ns, ns), dtype=torch.complex128, device=dev)
    ados[0, 0] = torch.from_numpy(_dense(rho0)).to(dev)
    Hd = torch.from_numpy(Hn).to(dev)
    Qd = torch.from_numpy(_dense(c_ops[0])).to(dev)
    ne = len(e_ops)
    Ed = stack_ops(e_ops, ns, dev)
    obs = torch.empty((1, nt + 1, ne), dtype=torch.complex128, device=dev) if ne else None
    with torch.cuda.device(dev):
        rc = _lib.load().qd_heom_chain_euler(ados.data_ptr(), 1, int(nado), ns, Hd.data_ptr(), Qd.data_ptr(),
                                             float(gamma), float(D0.real), float(D0.imag), float(dt), int(nt),
                                             None, _lib.ptr(Ed), ne, _lib.ptr(obs), _lib.stream_ptr(dev))
    _lib.check(rc, "qd_heom_chain_euler")
    if not ne:
        return np.zeros((0, nt), dtype=complex)
    return obs[0, 1:].T.cpu().numpy()
