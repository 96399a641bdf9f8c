"""Tier-banded sharding of ONE ADO hierarchy over ranks (BASELINE configs[3]).

DEOMSolver.run (pyqed/heom/deom.py:1072-1114) propagates every ADO of the graded hierarchy with RK4 whose
right-hand side (rem_cal / generate_dot_element, :641-673) couples ADO n only to n -/+ e_k, i.e. to tiers
l -/+ 1.  The keys are tier-ordered (hash(key) == index, §8(a16)), so contiguous index ranges are unions of whole
or partial tiers and a band's outside neighbours sit in a narrow window around it:

  * partition: contiguous, ADO-count-balanced bands [lo_r, hi_r) (``shard_range``), one per rank;
  * halo: the sorted global indices a band's stencil reads outside its range, grouped by owning rank; local row
    order is [owned rows | halo rows], and the band's minus / plus tables are remapped to local rows;
  * per RK4 stage: every band runs ``qd_deom_stage`` on its rows (same HIP kernels as qd_deom_rk4: the group
    kernel for ns <= 8, MFMA 16 x 16 tiles for 9 <= ns <= 16), then exchanges the rows it just wrote that other
    bands read (point-to-point send / recv with each peer that needs them: ``torch.distributed`` P2P, i.e. RCCL
    over xGMI with backend "nccl"), packing them with ``qd_gather_rows``;
  * rank 0 owns ADO 0 and records rho_0 / Tr(p1 rho_0) after every step.

There is no data-path collective besides those halo exchanges; the arithmetic per ADO is identical to the
single-process run, so the result equals it to rounding (bit-exact in practice: same kernels, same operand order).
``LoopbackExchange`` runs several bands in one process (one device) with the same plans and device-side copies
in place of the send / recv pairs; tests use it to check the banded path on one GPU, and the gloo tests drive
``TorchExchange`` with a host stage function on CPU.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib
from .distributed import shard_range, world

_STAGE_TIME = (0, 1, 1, 2)     # index into the (t, t + dt/2, t + dt) pulse values of a step (deom.py:725-766)


@dataclass
class BandPlan:
    """One band of the partition: owned global range, halo rows and the exchange lists."""
    rank: int
    lo: int
    hi: int
    halo: np.ndarray                              # global indices of the halo rows, ascending
    recv: dict = field(default_factory=dict)      # peer -> (first halo row, count)
    send: dict = field(default_factory=dict)      # peer -> local owned rows that peer reads, in its halo order
    minus: np.ndarray = None                      # [n_own, K] local rows (-1 absent)
    plus: np.ndarray = None

    @property
    def n_own(self):
        return self.hi - self.lo

    @property
    def n_loc(self):
        return self.n_own + len(self.halo)


def make_plans(minus: np.ndarray, plus: np.ndarray, nbands: int) -> list[BandPlan]:
    """Partition the nmax ADOs into `nbands` contiguous ADO-count-balanced bands and build every band's halo,
    local tables and send / receive lists (deterministic: every rank computes the same plans)."""
    nmax, K = minus.shape
    if nbands < 1 or nbands > nmax:
        raise ValueError(f"cannot split {nmax} ADOs into {nbands} bands")
    ranges = [shard_range(nmax, r, nbands) for r in range(nbands)]
    starts = np.array([lo for lo, _ in ranges])
    plans = []
    for r, (lo, hi) in enumerate(ranges):
        nb = np.concatenate([minus[lo:hi].ravel(), plus[lo:hi].ravel()])
        nb = np.unique(nb[nb >= 0])
        halo = nb[(nb < lo) | (nb >= hi)]
        g2l = {int(g): hi - lo + i for i, g in enumerate(halo)}

        def remap(tab):
            out = np.full((hi - lo, K), -1, dtype=np.int32)
            t = tab[lo:hi]
            inside = (t >= lo) & (t < hi)
            out[inside] = (t[inside] - lo).astype(np.int32)
            outside = (t >= 0) & ~inside
            out[outside] = [g2l[int(g)] for g in t[outside]]
            return out

        owner = np.searchsorted(starts, halo, side="right") - 1
        recv = {}
        for q in np.unique(owner):
            sel = np.nonzero(owner == q)[0]
            recv[int(q)] = (int(sel[0]), int(len(sel)))
        plans.append(BandPlan(rank=r, lo=lo, hi=hi, halo=halo, recv=recv, minus=remap(minus), plus=remap(plus)))
    for r, p in enumerate(plans):
        for q, pq in enumerate(plans):
            if q != r and r in pq.recv:
                s, c = pq.recv[r]
                p.send[q] = (pq.halo[s:s + c] - p.lo).astype(np.int32)
    return plans


class DeomBand:
    """State and tables of one band on one device; ``stage`` runs qd_deom_stage (or a host stage function)."""

    def __init__(self, plan: BandPlan, coef, damp, mode, H, Q, Hdip, Qdip, ns, nt, device, stage_fn=None):
        self.plan, self.ns, self.nt, self.dev = plan, ns, nt, torch.device(device)
        c128 = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=complex))).to(self.dev)
        i32 = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.int32))).to(self.dev)
        lo, hi = plan.lo, plan.hi
        self.minus, self.plus = i32(plan.minus), i32(plan.plus)
        self.coef, self.damp, self.mode = c128(coef[lo:hi]), c128(damp[lo:hi]), i32(mode)
        self.H, self.Q = c128(H), c128(np.asarray(Q).reshape(-1, ns, ns))
        self.nmod = self.Q.shape[0]
        self.Hdip = c128(Hdip) if Hdip is not None else None
        self.Qdip = c128(Qdip) if Qdip is not None else None
        z = lambda n: torch.zeros((n, ns, ns), dtype=torch.complex128, device=self.dev)
        self.bufs = {"rho": z(plan.n_loc), "x0": z(plan.n_loc), "x1": z(plan.n_loc)}
        # RK4 accumulator only for driven stages; undriven bands run the accumulator-free Horner form (qd_deom_stage
        # with acc = NULL, as qd_deom_rk4 does)
        self.acc = z(plan.n_own) if (Hdip is not None or Qdip is not None) else None
        self.snap = z(nt + 1) if lo == 0 else None
        for q, v in plan.send.items():   # packed rows are this band's own rows (qd_gather_rows also bounds-checks)
            if len(v) and (int(np.min(v)) < 0 or int(np.max(v)) >= plan.n_own):
                raise ValueError(f"band {plan.rank}: send rows for band {q} outside [0, {plan.n_own})")
        self.send_idx = {q: i32(v) for q, v in plan.send.items()}
        self.send_buf = {q: z(len(v)) for q, v in plan.send.items()}
        self.stage_fn = stage_fn
        self.K = plan.minus.shape[1]

    def stage(self, stage, step, dt, fs, fc):
        """RK4 stage `stage` of step `step`; returns the name of the buffer whose owned rows it wrote."""
        xin = self.bufs["rho"] if stage == 0 else self.bufs["x0" if stage in (1, 3) else "x1"]
        out = "rho" if stage == 3 else ("x0" if stage in (0, 2) else "x1")
        xout = self.bufs[out]
        snap = self.snap if (stage == 3 and self.snap is not None) else None
        if self.stage_fn is not None:
            self.stage_fn(self, stage, step, dt, fs, fc, xin, xout)
            if snap is not None:
                snap[step + 1] = self.bufs["rho"][0]
            return out
        p = self.plan
        with torch.cuda.device(self.dev):
            rc = _lib.load().qd_deom_stage(
                self.bufs["rho"].data_ptr(), xin.data_ptr(), xout.data_ptr(), _lib.ptr(self.acc), p.n_own, self.K,
                self.ns, self.minus.data_ptr(), self.plus.data_ptr(), self.coef.data_ptr(), self.damp.data_ptr(),
                self.mode.data_ptr(), self.nmod, self.H.data_ptr(), _lib.ptr(self.Hdip), self.Q.data_ptr(),
                _lib.ptr(self.Qdip), float(fs.real), float(fs.imag), float(fc.real), float(fc.imag), int(stage),
                float(dt), _lib.ptr(snap), int(step), int(self.nt), _lib.stream_ptr(self.dev))
        _lib.check(rc, "qd_deom_stage")
        return out

    def pack(self, name, q):
        """Owned rows of buffer `name` that band q reads, packed in q's halo order."""
        src, dst, idx = self.bufs[name], self.send_buf[q], self.send_idx[q]
        if self.dev.type != "cuda":
            torch.index_select(src, 0, idx.long(), out=dst)
            return dst
        with torch.cuda.device(self.dev):
            rc = _lib.load().qd_gather_rows(src.data_ptr(), src.shape[0], idx.data_ptr(), len(idx), self.ns * self.ns,
                                            dst.data_ptr(), 0, _lib.stream_ptr(self.dev))
        _lib.check(rc, "qd_gather_rows")
        return dst

    def halo_view(self, name, q):
        s, c = self.plan.recv[q]
        n0 = self.plan.n_own + s
        return self.bufs[name][n0:n0 + c]


class TorchExchange:
    """Halo exchange between ranks with torch.distributed point-to-point ops (one band per rank): batched isend of
    the packed rows each peer reads, irecv straight into this band's halo rows (RCCL over xGMI with "nccl")."""

    def __init__(self, group=None):
        self.group = group

    def _peer(self, q):
        """Band q is group rank q; P2POp takes global ranks."""
        import torch.distributed as dist
        return q if self.group is None else dist.get_global_rank(self.group, q)

    def __call__(self, bands, name):
        import torch.distributed as dist
        (b,) = bands
        ops = []
        for q in sorted(b.plan.send):
            ops.append(dist.P2POp(dist.isend, b.pack(name, q), self._peer(q), group=self.group))
        for q in sorted(b.plan.recv):
            ops.append(dist.P2POp(dist.irecv, b.halo_view(name, q), self._peer(q), group=self.group))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()


class CollectiveExchange:
    """Halo exchange as ONE all-gather per stage (one band per rank): every rank packs the union of its owned rows
    any peer reads (its export set, padded to the largest export of all bands), all ranks all-gather those, and each
    rank copies its halo rows out of the gathered block with one precomputed index (torch index_select).  More bytes
    than the point-to-point exchange (every rank receives every export set), but a single standard collective per
    stage (RCCL all-gather over xGMI with "nccl"), no send / recv pairing to get wrong; the bench's multi-GPU leg
    uses it."""

    def __init__(self, plans, rank, ns, device, group=None):
        self.group, self.rank, self.ns = group, rank, ns
        self.dev = torch.device(device)
        exp = []
        for p in plans:
            rows = np.unique(np.concatenate(list(p.send.values()))) if p.send else np.zeros(0, np.int32)
            exp.append(rows.astype(np.int32))
        self.E = max(1, max(len(e) for e in exp))
        self.world = len(plans)
        me = plans[rank]
        idx = []
        for q in sorted(me.recv):
            pos = np.searchsorted(exp[q], plans[q].send[rank])
            idx.append(q * self.E + pos)
        # the packed export rows are this band's own rows, checked once here (the device gather runs unchecked)
        if len(exp[rank]) and (int(exp[rank].min()) < 0 or int(exp[rank].max()) >= me.n_own):
            raise ValueError(f"band {rank}: export rows outside [0, {me.n_own})")
        self.n_halo = len(me.halo)
        self.halo_idx = torch.from_numpy(np.concatenate(idx).astype(np.int64) if idx else np.zeros(0, np.int64)).to(
            self.dev)
        self.export = torch.from_numpy(exp[rank]).to(self.dev)
        z = lambda n: torch.zeros((n, ns, ns), dtype=torch.complex128, device=self.dev)
        self.sendbuf, self.recvbuf = z(self.E), z(self.world * self.E)
        self.bytes_per_exchange = self.world * self.E * ns * ns * 16

    def __call__(self, bands, name):
        import torch.distributed as dist
        (b,) = bands
        src = b.bufs[name]
        n = len(self.export)
        if n:
            if self.dev.type == "cuda":
                with torch.cuda.device(self.dev):
                    rc = _lib.load().qd_gather_rows(src.data_ptr(), src.shape[0], self.export.data_ptr(), n,
                                                    self.ns * self.ns, self.sendbuf.data_ptr(), 0,
                                                    _lib.stream_ptr(self.dev))
                _lib.check(rc, "qd_gather_rows")
            else:
                torch.index_select(src, 0, self.export.long(), out=self.sendbuf[:n])
        if dist.get_backend(self.group) == "nccl":
            dist.all_gather_into_tensor(self.recvbuf, self.sendbuf, group=self.group)
        elif self.dev.type == "cuda":   # gloo with device bands (tests: ranks sharing one GPU): stage through host
            host = self.sendbuf.cpu()
            parts = [torch.empty_like(host) for _ in range(self.world)]
            dist.all_gather(parts, host, group=self.group)
            self.recvbuf.copy_(torch.cat(parts).to(self.dev))
        else:
            dist.all_gather(list(self.recvbuf.chunk(self.world)), self.sendbuf, group=self.group)
        if self.n_halo:
            n0 = b.plan.n_own
            src[n0:n0 + self.n_halo] = torch.index_select(self.recvbuf, 0, self.halo_idx)


class LoopbackExchange:
    """All bands in one process: each band's halo rows are copied from the owners' packed rows (same plans)."""

    def __call__(self, bands, name):
        by_rank = {b.plan.rank: b for b in bands}
        for b in bands:
            for q in b.plan.recv:
                b.halo_view(name, q).copy_(by_rank[q].pack(name, b.plan.rank))


def run_bands(bands, exchange, rho0, dt, nt, fs=None, fc=None):
    """Drive the bands through nt RK4 steps (the loop of DEOMSolver.run, deom.py:1107-1113).  fs / fc: host pulse
    values [nt][3] at (t, t + dt/2, t + dt) or None.  The band owning ADO 0 gets rho0 and records rho_0 per step."""
    for b in bands:
        for t in b.bufs.values():
            t.zero_()
        if b.plan.lo == 0:
            b.bufs["rho"][0] = torch.from_numpy(np.asarray(rho0, dtype=complex)).to(b.dev)
            b.snap[0] = b.bufs["rho"][0]
    exchange(bands, "rho")
    zero = complex(0.0)
    for s in range(nt):
        for stage in range(4):
            ti = _STAGE_TIME[stage]
            vs = complex(fs[s][ti]) if fs is not None else zero
            vc = complex(fc[s][ti]) if fc is not None else zero
            name = None
            for b in bands:
                name = b.stage(stage, s, dt, vs, vc)
            exchange(bands, name)


class ShardedDEOM:
    """DEOMSolver.run with the hierarchy split into tier bands over the ranks of the default process group (or an
    in-process set of `nbands` bands on one device when no group is initialised / loopback=True).

    run(rho0, dt, nt, p1) returns (t_save, Tr(p1 rho_0) [nt+1] or rho_0 stack [nt+1, ns, ns]) on the rank owning
    ADO 0 (rank 0) and (t_save, None) elsewhere; gather_ados() assembles the final hierarchy on rank 0."""

    def __init__(self, solver, nbands=None, loopback=None, device=None, group=None, stage_fn=None,
                 exchange="p2p"):
        from .deom import ado_coefficients
        solver.check_()
        solver.init_()
        self.solver = solver
        rank, ws = world()
        if group is not None:  # bands are numbered by the rank within `group`
            import torch.distributed as dist
            rank, ws = dist.get_rank(group), dist.get_world_size(group)
        self.loopback = (ws == 1) if loopback is None else loopback
        self.rank = 0 if self.loopback else rank
        self.nbands = (nbands or 2) if self.loopback else ws
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if stage_fn is None else torch.device("cpu")
        self.device = torch.device(device)
        b = solver.bath
        self.coef, self.damp = ado_coefficients(solver.keys, np.asarray(b.etal), np.asarray(b.etar),
                                                np.asarray(b.etaa), np.asarray(b.expn), solver.lmax)
        self.plans = make_plans(solver._minus, solver._plus, self.nbands)
        self.group, self.stage_fn = group, stage_fn
        if exchange not in ("p2p", "allgather"):
            raise ValueError(f"exchange must be 'p2p' or 'allgather', got {exchange!r}")
        self.exchange_kind = exchange
        self.bands = None
        self.exchange = None

    def setup(self, dt, nt):
        """Bands (tables and state on the device) and the exchange for an nt-step run; returns the pulse tables."""
        s = self.solver
        ns = s.nsys
        Q = np.asarray(s.coupling, dtype=complex).reshape(-1, ns, ns)
        Hdip, fs = s._dip_values(s.system_dipole, s.pulse_system_func, nt, dt, (ns, ns))
        Qdip, fc = s._dip_values(s.coupling_dipole, s.pulse_coupling_func, nt, dt, Q.shape)
        mine = self.plans if self.loopback else [self.plans[self.rank]]
        self.bands = [DeomBand(p, self.coef, self.damp, np.asarray(s.bath.mode), s.system, Q, Hdip, Qdip, ns, nt,
                               self.device, self.stage_fn) for p in mine]
        if self.loopback:
            exch = LoopbackExchange()
        elif self.exchange_kind == "allgather":
            exch = CollectiveExchange(self.plans, self.rank, ns, self.device, self.group)
        else:
            exch = TorchExchange(self.group)
        self.exchange = exch
        return fs, fc

    def run(self, rho0, dt, nt, p1=None):
        s = self.solver
        ns = s.nsys
        fs, fc = self.setup(dt, nt)
        run_bands(self.bands, self.exchange, rho0, dt, nt, fs, fc)
        t_save = np.arange(nt + 1) * dt
        root = [b for b in self.bands if b.plan.lo == 0]
        if not root:
            return t_save, None
        snap = root[0].snap
        if p1 is None:
            return t_save, snap.cpu().numpy()
        E = torch.from_numpy(np.asarray(p1, dtype=complex).reshape(1, ns, ns)).to(self.device)
        if self.device.type != "cuda":
            return t_save, torch.einsum("ij,sji->s", E[0], snap).cpu().numpy()
        tr = torch.empty((nt + 1, 1), dtype=torch.complex128, device=self.device)
        with torch.cuda.device(self.device):
            rc = _lib.load().qd_deom_trace(snap.data_ptr(), E.data_ptr(), 1, nt + 1, ns, tr.data_ptr(),
                                           _lib.stream_ptr(self.device))
        _lib.check(rc, "qd_deom_trace")
        return t_save, tr[:, 0].cpu().numpy()

    def gather_ados(self):
        """The final hierarchy [nmax, ns, ns] (host numpy) on rank 0 (None elsewhere)."""
        own = [(b.plan.lo, b.bufs["rho"][:b.plan.n_own].cpu().numpy()) for b in self.bands]
        if not self.loopback and self.nbands > 1:
            import torch.distributed as dist
            got = [None] * self.nbands if self.rank == 0 else None
            dst = 0 if self.group is None else dist.get_global_rank(self.group, 0)
            dist.gather_object(own, got, dst=dst, group=self.group)
            if self.rank != 0:
                return None
            own = [x for part in got for x in part]
        out = np.zeros((self.solver.nmax, self.solver.nsys, self.solver.nsys), dtype=complex)
        for lo, rows in own:
            out[lo:lo + len(rows)] = rows
        return out
