"""The tier-banded DEOM path with the HIP stage kernels in SEPARATE processes (qd_deom_stage had
run only in single-process loopback): two ranks on the one GPU of the box, gloo process group, every band stage on
qd_deom_stage, the halo all-gathered through host memory (CollectiveExchange's gloo fallback).  Rank 0's
Tr(p1 rho_0) and the gathered final hierarchy must equal the single-process qd_deom_rk4 run of the same hierarchy."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import relerr

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(ns=3, L=5):
    import sympy as sp
    from pyqed_amd.deom import Bath, DEOMSolver
    rng = np.random.default_rng(ns)
    a = rng.standard_normal((ns, ns)) + 1j * rng.standard_normal((ns, ns))
    H = (a + a.conj().T) / 2
    Qm = np.diag(np.linspace(-1, 1, ns)).astype(complex)
    w = sp.symbols(r"\omega", real=True)
    bath = Bath([2 * 0.5 * 1.0 * w / (1.0 + w ** 2)], w, [1.0], [3], [0] * 4)
    sdip = (np.roll(np.eye(ns), 1, axis=1) + np.roll(np.eye(ns), -1, axis=1)).astype(complex)
    sol = DEOMSolver(H, sdip, bath, np.array([Qm]), np.array([0.5 * Qm]), lambda t: 0.3 * np.sin(2 * t),
                     lambda t: 0.1 * np.cos(t), L)
    rho0 = np.zeros((ns, ns), complex)
    rho0[0, 0] = 1
    return sol, rho0


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from pyqed_amd.deom_shard import ShardedDEOM
        sol, rho0 = _model()
        sh = ShardedDEOM(sol, device=torch.device("cuda", 0), exchange="allgather")
        P1 = np.diag(np.linspace(1, 0, rho0.shape[0])).astype(complex)
        t, tr = sh.run(rho0, 0.01, 8, P1)
        ados = sh.gather_ados()
        q.put((rank, tr, ados, [len(p.halo) for p in sh.plans]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_deom_bands_two_processes_hip_stages_match_single():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sol, rho0 = _model()
    P1 = np.diag(np.linspace(1, 0, rho0.shape[0])).astype(complex)
    t, tr_ref = sol.run(rho0.copy(), 0.01, 8, P1)
    assert res[1][1] is None and res[1][2] is None
    assert all(h > 0 for h in res[0][3])
    assert relerr(np.asarray(res[0][1]), np.asarray(tr_ref)) < 1e-12
    assert relerr(res[0][2], sol.ddos) < 1e-12
