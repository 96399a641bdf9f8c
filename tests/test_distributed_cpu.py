"""Multi-process path on CPU with gloo (world_size 2): sharding + the single reduce reproduce the
single-process result.  The per-rank compute is the oracle's closed-form 2DES slice (CPU)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(M=37, n=24):
    rng = np.random.default_rng(5)
    lam = -0.1 * rng.random((M, 9)) + 1j * rng.standard_normal((M, 9))
    alpha = rng.standard_normal((M, 9)) + 1j * rng.standard_normal((M, 9))
    beta = rng.standard_normal((M, 9)) + 1j * rng.standard_normal((M, 9))
    Mt = rng.standard_normal((M, 9, 9)) + 1j * rng.standard_normal((M, 9, 9))
    t = 0.5 * np.arange(n)
    return lam, alpha, Mt, beta, t


def _slice_sum(lam, alpha, Mt, beta, t, lo, hi):
    out = np.zeros((len(t), len(t)), complex)
    for m in range(lo, hi):
        X = alpha[m][None, :] * np.exp(np.outer(t, lam[m]))
        Y = beta[m][None, :] * np.exp(np.outer(t, lam[m]))
        out += (-1j) ** 3 * X @ Mt[m] @ Y.T
    return out


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pyqed_amd.distributed import sharded_sum, world as w
    assert w() == (rank, world)
    lam, alpha, Mt, beta, t = _inputs()

    def local(lo, hi):
        return torch.from_numpy(_slice_sum(lam, alpha, Mt, beta, t, lo, hi))

    out = sharded_sum(local, len(lam), dst=0)
    allr = sharded_sum(local, len(lam), dst=None)
    if rank == 0:
        q.put((out.numpy(), allr.numpy()))
    else:
        q.put((None, allr.numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_2des_reduce_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    lam, alpha, Mt, beta, t = _inputs()
    full = _slice_sum(lam, alpha, Mt, beta, t, 0, len(lam))
    reduced = [r[0] for r in res if r[0] is not None]
    assert len(reduced) == 1
    assert np.allclose(reduced[0], full, rtol=1e-12, atol=1e-12 * np.abs(full).max())
    for _, a in res:
        assert np.allclose(a, full, rtol=1e-12, atol=1e-12 * np.abs(full).max())


def _worker_buckets(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pyqed_amd.distributed import sharded_sum_buckets
    lam, alpha, Mt, beta, t = _inputs()
    n2 = 5
    out = torch.zeros((n2, len(t), len(t)), dtype=torch.complex128)
    calls = []

    def local(lo, hi, b):
        calls.append((lo, hi, b.start, b.stop))
        for j in range(b.start, b.stop):   # waiting time j scales member m's slice by (j + 1 + m % 3)
            acc = np.zeros((len(t), len(t)), complex)
            for m in range(lo, hi):
                acc += (j + 1 + m % 3) * _slice_sum(lam, alpha, Mt, beta, t, m, m + 1)
            out[j] = torch.from_numpy(acc)

    sharded_sum_buckets(local, len(lam), out, [slice(0, 2), slice(2, 4), slice(4, 5)], dst=0)
    q.put((rank, out.numpy() if rank == 0 else None, calls))
    dist.barrier()
    dist.destroy_process_group()


def test_bucketed_overlapped_reduce_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_buckets, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    lam, alpha, Mt, beta, t = _inputs()
    M = len(lam)
    full = np.array([sum((j + 1 + m % 3) * _slice_sum(lam, alpha, Mt, beta, t, m, m + 1) for m in range(M))
                     for j in range(5)])
    got = res[0][1]
    assert np.allclose(got, full, rtol=1e-12, atol=1e-12 * np.abs(full).max())
    # each rank computed its own member shard for every bucket, in order
    assert [c[:2] for c in res[0][2]] == [(0, M // 2)] * 3
    assert [c[:2] for c in res[1][2]] == [(M // 2, M)] * 3
    assert [c[2:] for c in res[1][2]] == [(0, 2), (2, 4), (4, 5)]


def test_shard_range_partition():
    from pyqed_amd.distributed import shard_range
    for n in [0, 1, 7, 4096, 4097]:
        for ws in [1, 2, 3, 8]:
            parts = [shard_range(n, r, ws) for r in range(ws)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(ws - 1))
            sizes = [h - l for l, h in parts]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(4, 2, 2)


@pytest.mark.gpu
def test_native_rccl_reduce_single_rank():
    """The C-ABI's own RCCL path (qd_comm_* / qd_reduce_sum) on a one-rank communicator: the reduce of one
    contribution is the identity, errors come back as return codes."""
    import ctypes
    from pyqed_amd import _lib
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    uid = ctypes.create_string_buffer(128)
    _lib.check(lib.qd_comm_unique_id(uid), "qd_comm_unique_id")
    _lib.check(lib.qd_comm_init(1, 0, uid), "qd_comm_init")
    try:
        x = torch.randn(1000, dtype=torch.complex128, device=dev)
        ref = x.clone()
        _lib.check(lib.qd_reduce_sum(x.data_ptr(), x.numel(), 0, _lib.stream_ptr(dev)), "qd_reduce_sum")
        torch.cuda.synchronize(dev)
        assert torch.equal(x, ref)
        assert lib.qd_reduce_sum(x.data_ptr(), x.numel(), 1, _lib.stream_ptr(dev)) != 0   # bad root
        assert lib.qd_comm_init(1, 0, uid) != 0                                            # double init
    finally:
        _lib.check(lib.qd_comm_destroy(), "qd_comm_destroy")


def _worker_pipeline(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pyqed_amd.distributed import ReducePipeline, shard_range
    lam, alpha, Mt, beta, t = _inputs()
    lo, hi = shard_range(len(lam), rank, world)
    part = _slice_sum(lam, alpha, Mt, beta, t, lo, hi)
    pipe = ReducePipeline((len(t), len(t)), torch.complex128, "cpu", depth=2, dst=0)
    got = {}
    ngrid = 5
    for g in range(ngrid):
        buf = pipe.next_buffer()
        if g >= 2 and rank == 0:       # this buffer last held grid g-2, whose reduce has now completed
            got[g - 2] = buf.numpy().copy()
        buf.copy_(torch.from_numpy((g + 1) * part))
        pipe.submit(buf)
    pipe.finish()
    if rank == 0:
        for g in (ngrid - 2, ngrid - 1):
            got[g] = pipe.bufs[g % 2].numpy().copy()
    q.put((rank, got))
    dist.barrier()
    dist.destroy_process_group()


def test_reduce_pipeline_gloo():
    """ReducePipeline (a sequence of grids, each reduce overlapping the next grid's compute, 2 rotating buffers):
    rank 0 ends up with the exact cross-rank sum of every grid in the sequence."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_pipeline, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    lam, alpha, Mt, beta, t = _inputs()
    full = _slice_sum(lam, alpha, Mt, beta, t, 0, len(lam))
    got = res[0][1]
    assert sorted(got) == list(range(5))
    for g in range(5):
        assert np.allclose(got[g], (g + 1) * full, rtol=1e-12, atol=1e-12 * np.abs(full).max()), g


# ---------------------------------------------------------------- tier-banded DEOM
def _deom_model(ns=3, npsd=2, L=4, pulsed=True):
    import sympy as sp
    from pyqed_amd.deom import Bath, DEOMSolver
    rng = np.random.default_rng(17)
    A = rng.standard_normal((ns, ns)) + 1j * rng.standard_normal((ns, ns))
    H = (A + A.conj().T) / 2
    Qm = np.diag(np.linspace(-1, 1, ns)).astype(complex)
    w = sp.symbols(r"\omega", real=True)
    bath = Bath([2 * 0.5 * 1.0 * w / (1.0 + w ** 2)], w, [1.0], [npsd], [0] * (1 + npsd))
    sdip = np.roll(np.eye(ns), 1, axis=1).astype(complex)
    sdip = sdip + sdip.T
    fs = (lambda t: 0.3 * np.sin(2 * t)) if pulsed else None
    fc = (lambda t: 0.1 * np.cos(t)) if pulsed else None
    cdip = np.array([0.5 * Qm]) if pulsed else None
    sol = DEOMSolver(H, sdip if pulsed else None, bath, np.array([Qm]), cdip, fs, fc, L)
    rho0 = np.zeros((ns, ns), complex)
    rho0[0, 0] = 1
    return sol, bath, H, Qm, sdip, cdip, fs, fc, rho0


def _host_stage(band, stage, step, dt, fs, fc, xin, xout):
    """Host (numpy) restatement of qd_deom_stage's arithmetic for a band: oracle.deom.band_rhs + the kernel's RK4
    bookkeeping (deom.py:725-766 order)."""
    from oracle import deom as od
    ns = band.ns
    p = band.plan
    H = band.H.numpy() + (band.Hdip.numpy() * fs if band.Hdip is not None else 0)
    Q = band.Q.numpy() + (band.Qdip.numpy() * fc if band.Qdip is not None else 0)
    d = od.band_rhs(xin.numpy(), p.n_own, p.minus, p.plus, band.coef.numpy(), band.damp.numpy(), band.mode.numpy(),
                    H, Q)
    r0 = band.bufs["rho"][:p.n_own].numpy()
    if band.acc is None:   # undriven band: the kernel's Horner-form stages (deom_rk4_next)
        v = torch.from_numpy(r0 + d * (dt / (4 - stage)))
        if stage < 3:
            xout[:p.n_own] = v
        else:
            band.bufs["rho"][:p.n_own] = v
        return
    acc = band.acc.numpy()
    if stage == 0:
        acc[...] = d
        xout[:p.n_own] = torch.from_numpy(r0 + d * (dt / 2))
    elif stage == 1:
        acc += d * 2.0
        xout[:p.n_own] = torch.from_numpy(r0 + d * (dt / 2))
    elif stage == 2:
        acc += d * 2.0
        xout[:p.n_own] = torch.from_numpy(r0 + d * dt)
    else:
        band.bufs["rho"][:p.n_own] = torch.from_numpy(r0 + (acc + d) * dt / 6.0)


def _worker_deom_bands(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pyqed_amd.deom_shard import ShardedDEOM
    sol, *_, rho0 = _deom_model()
    sh = ShardedDEOM(sol, stage_fn=_host_stage, device="cpu")
    P1 = np.diag([1.0, 0, 0]).astype(complex)
    t, tr = sh.run(rho0, 0.01, 6, P1)
    ados = sh.gather_ados()
    q.put((rank, tr, ados, [(p.lo, p.hi, len(p.halo), sorted(p.recv), sorted(p.send)) for p in sh.plans]))
    dist.barrier()
    dist.destroy_process_group()


def test_deom_tier_bands_gloo():
    """One hierarchy (ns = 3, K = 3, L = 4: 35 ADOs, driven H(t), Q(t)) split into 2 tier bands over 2 gloo ranks,
    halo rows exchanged by send / recv after every RK4 stage (TorchExchange): Tr(p1 rho_0) on rank 0 and the
    gathered final hierarchy equal the single-process oracle run (oracle.deom.run restates DEOMSolver.run,
    heom/deom.py:1072-1114)."""
    from oracle import deom as od
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_deom_bands, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sol, bath, H, Qm, sdip, cdip, fs, fc, rho0 = _deom_model()
    P1 = np.diag([1.0, 0, 0]).astype(complex)
    _, tr_ref, ados_ref = od.run(H, sdip, fs, np.array([Qm]), cdip, fc, (bath.etal, bath.etar, bath.etaa, bath.expn),
                                 4, rho0, 0.01, 6, P1)
    assert res[1][1] is None and res[1][2] is None
    assert np.allclose(res[0][1], tr_ref, rtol=1e-12, atol=1e-13)
    assert np.allclose(res[0][2], ados_ref, rtol=1e-11, atol=1e-13)
    plans = res[0][3]
    assert plans[0][:2] == (0, 17) and plans[1][:2] == (17, 35)
    assert plans[0][3] == [1] and plans[1][3] == [0]          # each band reads halo rows from the other


def test_deom_band_plans_properties():
    """make_plans on the bench hierarchy (L = 12, K = 5, 6188 ADOs) over 8 bands: the bands tile [0, nmax), every
    stencil neighbour of an owned ADO is either owned or in the halo, local tables point at the right global rows,
    and the send lists are the receivers' halo rows."""
    from pyqed_amd.deom import ado_tables
    from pyqed_amd.deom_shard import make_plans
    keys, minus, plus, _ = ado_tables(12, 5)
    plans = make_plans(minus, plus, 8)
    assert plans[0].lo == 0 and plans[-1].hi == len(keys)
    assert all(a.hi == b.lo for a, b in zip(plans, plans[1:]))
    for p in plans:
        glob = np.concatenate([np.arange(p.lo, p.hi), p.halo])
        for tab, loc in ((minus, p.minus), (plus, p.plus)):
            t = tab[p.lo:p.hi]
            assert np.array_equal(loc < 0, t < 0)
            assert np.array_equal(glob[loc[loc >= 0]], t[t >= 0])
        for q, (s, c) in p.recv.items():
            assert np.array_equal(plans[q].send[p.rank] + plans[q].lo, p.halo[s:s + c])


def _worker_deom_bands_subgroup(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sub = dist.new_group([1, 2])       # every rank must take part in new_group
    if rank in (1, 2):
        from pyqed_amd.deom_shard import ShardedDEOM
        sol, *_, rho0 = _deom_model()
        sh = ShardedDEOM(sol, stage_fn=_host_stage, device="cpu", group=sub)
        P1 = np.diag([1.0, 0, 0]).astype(complex)
        t, tr = sh.run(rho0, 0.01, 6, P1)
        ados = sh.gather_ados()
        q.put((rank, tr, ados))
    else:
        q.put((rank, None, None))
    dist.barrier()
    dist.destroy_process_group()


def test_deom_tier_bands_subgroup_gloo():
    """ShardedDEOM on a process SUBgroup (global ranks 1, 2 of 3).  Bands are numbered by the rank within
    the group and peers are mapped to global ranks for the P2P ops and the final gather, so group rank 0 (global
    rank 1) returns the oracle's Tr(p1 rho_0) and final hierarchy."""
    from oracle import deom as od
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_deom_bands_subgroup, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sol, bath, H, Qm, sdip, cdip, fs, fc, rho0 = _deom_model()
    P1 = np.diag([1.0, 0, 0]).astype(complex)
    _, tr_ref, ados_ref = od.run(H, sdip, fs, np.array([Qm]), cdip, fc, (bath.etal, bath.etar, bath.etaa, bath.expn),
                                 4, rho0, 0.01, 6, P1)
    assert res[0][1] is None and res[2][1] is None and res[2][2] is None
    assert np.allclose(res[1][1], tr_ref, rtol=1e-12, atol=1e-13)
    assert np.allclose(res[1][2], ados_ref, rtol=1e-11, atol=1e-13)


def _worker_deom_bands_allgather(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pyqed_amd.deom_shard import ShardedDEOM
    sol, *_, rho0 = _deom_model()
    sh = ShardedDEOM(sol, stage_fn=_host_stage, device="cpu", exchange="allgather")
    P1 = np.diag([1.0, 0, 0]).astype(complex)
    t, tr = sh.run(rho0, 0.01, 6, P1)
    ados = sh.gather_ados()
    q.put((rank, tr, ados, sh.exchange.E, sh.exchange.n_halo))
    dist.barrier()
    dist.destroy_process_group()


def test_deom_tier_bands_allgather_gloo():
    """The bench's multi-GPU DEOM exchange (CollectiveExchange: one all-gather of every band's export rows per stage,
    halo rows picked by a precomputed index) over 3 gloo ranks equals the single-process oracle run."""
    from oracle import deom as od
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_deom_bands_allgather, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sol, bath, H, Qm, sdip, cdip, fs, fc, rho0 = _deom_model()
    P1 = np.diag([1.0, 0, 0]).astype(complex)
    _, tr_ref, ados_ref = od.run(H, sdip, fs, np.array([Qm]), cdip, fc, (bath.etal, bath.etar, bath.etaa, bath.expn),
                                 4, rho0, 0.01, 6, P1)
    assert np.allclose(res[0][1], tr_ref, rtol=1e-12, atol=1e-13)
    assert np.allclose(res[0][2], ados_ref, rtol=1e-11, atol=1e-13)
    assert all(r[4] > 0 for r in res)          # every band has halo rows


# ---------------------------------------------------------------- bench warm-up under collectives
def _worker_ramp(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    import time
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    calls = [0]
    x = torch.ones(4)

    def fn():                           # a leg call that issues a collective, slower on rank 1
        time.sleep(0.002 * (1 + 2 * rank))
        dist.all_reduce(x)
        calls[0] += 1

    bench.ramp_warmup(fn, "cpu", min_ms=40.0, agree=True)
    q.put((rank, calls[0]))
    dist.barrier()
    dist.destroy_process_group()


def test_ramp_warmup_agrees_on_call_count_gloo():
    """bench.ramp_warmup(agree=True) (the 2DES legs, whose calls issue the reduce at world > 1): ranks whose calls take
    different times still make the same number of calls, so no collective is left unmatched."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_ramp, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][1] == res[1][1] >= 3, res
