#!/usr/bin/env python3
"""bench.py — headline benchmark of pyqed_amd on MI355X.

Workload (BASELINE.json configs[1]): Lindblad propagation, N = 128 Hilbert
space, one dense collapse operator, RK4, fp64 (complex128), dt = 1e-3.
One "step" = one RK4 step of every density matrix in the per-GPU batch
(B independent density matrices).  value = density-
matrix steps/s over all ranks (weak scaling: each rank owns its own batch;
no data-path collective).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
    torchrun --nproc-per-node N bench.py --gpus N ...

Rank 0 prints ONE JSON line.  The CPU baseline (rank 0, N=1 only) is the
oracle's reference-faithful scipy.sparse csr restatement of oqs._lindblad,
timed on a bounded sample on this host.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HEADLINE_REPS = 5   # timed regions of the headline leg; the line reports their median
FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X dense FP64 matrix peak (spec)
HBM_PEAK_GBS = 8000.0


def measured_traffic(kernel: str, units: float):
    """HBM bytes per launch from the committed PMC measurement (profiles/pmc_traffic.json), or None."""
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))[kernel]
    except Exception:
        return None
    return (d["read_bytes_per_unit"] + d["write_bytes_per_unit"]) * units


def ramp_warmup(fn, dev, min_ms=60.0, max_calls=10000, agree=False):
    """Untimed calls of a leg's own work for >= min_ms of steady calls.  A leg whose inputs were just built on the host
    starts on an idle GPU, whose clocks take tens of ms to come up (profiles/r04/lindblad/launch_overhead.txt: a
    20-step Lindblad launch after 20 ms idle runs 0.825 ms per step against 0.726 behind other work;
    tools/ramp_probe*.py: a 2DES grid needs ~25 ms of sustained load); the timed region then measures the leg at the
    clocks a running job has, not the ramp.  The number of calls is fixed from the second call's time, so that with
    agree=True (legs whose calls issue collectives, world > 1) every rank makes the same number of calls: the ranks
    take the largest count (one all-reduce before the loop)."""
    import torch
    dev = torch.device(dev)
    sync = (lambda: torch.cuda.synchronize(dev)) if dev.type == "cuda" else (lambda: None)
    fn()                                  # first call: one-time setup (code objects, pool growth, cached operands)
    sync()
    t0 = time.perf_counter()              # the budget counts steady calls only
    fn()
    sync()
    one = max(time.perf_counter() - t0, 1e-6)
    n = int(min(max_calls, max(0, np.ceil(min_ms / 1e3 / one) - 1)))
    if agree:
        import torch.distributed as dist
        c = torch.tensor([n], dtype=torch.int64, device=dev)
        dist.all_reduce(c, op=dist.ReduceOp.MAX)
        n = int(c.item())
    per_sync = max(1, int(0.005 / one))   # short calls are queued back to back, ~5 ms of work per synchronisation
    done = 0
    while done < n:
        for _ in range(min(per_sync, n - done)):
            fn()
        done += min(per_sync, n - done)
        sync()


def synthetic_lindblad(N, seed_h=0, seed_c=1, nc=1, gamma=0.1):
    """Seeded BASELINE config d1 inputs: GUE H/sqrt(N), dense Ginibre c_op * 0.1/sqrt(N) (the
    same draws as the tests' oracle.lindblad.synthetic_lindblad; kept here so the timed legs import no oracle)."""
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
    """B seeded random pure-state density matrices [B, N, N]."""
    rng = np.random.default_rng(seed)
    psi = rng.standard_normal((B, N)) + 1j * rng.standard_normal((B, N))
    psi /= np.linalg.norm(psi, axis=1, keepdims=True)
    return np.einsum("bi,bj->bij", psi, psi.conj())


def lindblad_flops_per_step(N: int, nc: int, hermitian: bool = False) -> float:
    # 4 RK4 stages x (complex N^3 GEMMs per RHS) x 8 real flop per complex MAC.
    # general GLF kernel: (-iK)r, r(iK^+), C r, (C r)C^+      -> 2 + 2*nc GEMMs
    # Hermitian kernel:   X = (-iK)r + 1/2 (C r)C^+, L = X + X^+ -> 1 + 2*nc GEMMs
    return 4.0 * ((1 if hermitian else 2) + 2 * nc) * 8.0 * N ** 3


def lindblad_executed_flops_per_step(N: int, nc: int, hermitian: bool = False) -> float:
    # What the MFMA units execute: the Hermitian kernel at 128-blocks (N_p = 128) skips the Hermitian part's
    # redundant 16 x 16 tiles below the diagonal (glf.hip / cgemm_block.hpp cg_herm_x_gemm: 28 of the 64 tiles of
    # each (C r)C^+ GEMM, so 36/64 of it runs).
    if hermitian and N == 128:
        return 4.0 * (1 + nc + (36.0 / 64.0) * nc) * 8.0 * N ** 3
    return lindblad_flops_per_step(N, nc, hermitian)


def cpu_baseline(N, nc, dt, budget_s=10.0):
    """Reference-faithful csr restatement (oracle.lindblad.lindblad_csr), bounded sample."""
    from oracle import lindblad as olb
    H, cs = olb.synthetic_lindblad(N, nc=nc)
    rho0 = olb.random_pure_states(1, N)[0]
    olb.lindblad_csr(H, rho0, cs, [], 1, dt)  # warm-up
    steps, t0 = 0, time.perf_counter()
    chunk = 2
    while True:
        olb.lindblad_csr(H, rho0, cs, [], chunk, dt)
        steps += chunk
        el = time.perf_counter() - t0
        if el >= budget_s or steps >= 400:
            break
    csr_rate = steps / el
    # dense NumPy variant of the same arithmetic (informational)
    t0 = time.perf_counter()
    nd = 0
    while time.perf_counter() - t0 < min(3.0, budget_s / 3):
        olb.lindblad_batch(H, cs, rho0[None], dt, 5)
        nd += 5
    dense_rate = nd / (time.perf_counter() - t0)
    threads = os.environ.get("OMP_NUM_THREADS") or os.environ.get("OPENBLAS_NUM_THREADS") or str(os.cpu_count())
    return {
        "value": round(csr_rate, 4),
        "unit": "density-matrix steps/s",
        "cores": 1,
        "kind": "port",
        "sample": f"1 density matrix, N={N}, {steps} RK4 steps of the csr restatement of oqs._lindblad "
                  f"(scipy.sparse csr x csr, single-threaded) in {el:.1f}s",
        "dense_numpy_steps_per_s": round(dense_rate, 2),
        "dense_numpy_threads": threads,
    }


def redfield_inputs(N, seed=5):
    """Redfield N = 128 (BASELINE.json configs[1]): GUE H / sqrt(N), one Hermitian a_op
    (0.2 (A + A^+)/2 / sqrt(N)), flat spectrum S = 0.05.  Returns the solver (host setup done)."""
    from pyqed_amd import RedfieldSolver
    rng = np.random.default_rng(seed)
    a = rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N))
    H = (a + a.conj().T) / 2 / np.sqrt(N)
    x = rng.standard_normal((N, N)) + 1j * rng.standard_normal((N, N))
    a_op = 0.2 * (x + x.conj().T) / 2 / np.sqrt(N)
    sol = RedfieldSolver(H, c_ops=[a_op], spectra=[lambda w: 0.05 + 0.0 * w])
    sol.redfield_tensor()
    return sol


def bench_redfield(dev, steps, B, N=128, dt=1e-3, warmup=3):
    """Redfield propagation in the H eigenbasis (RedfieldSolver.evolve's kernel, Hermitian-state GLF form:
    X = P rho + A rho Lam^+, d rho/dt = X + X^+), B independent density matrices."""
    import torch
    from pyqed_amd.oqs import glf_rk4
    sol = redfield_inputs(N)
    P, Ls, Ws = sol.glf_terms_herm()
    t = lambda x: torch.from_numpy(np.ascontiguousarray(np.asarray(x, complex))).to(dev)
    Pd, Ld, Wd = t(P), t(Ls), t(Ws)
    rho = t(random_pure_states(B, N, seed=7))
    ramp_warmup(lambda: glf_rk4(Pd, None, Ld, Wd, rho, dt, warmup, hermitian=True), dev)
    stream = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    glf_rk4(Pd, None, Ld, Wd, rho, dt, steps, hermitian=True)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    kern = e0.elapsed_time(e1) / 1e3
    flops = lindblad_flops_per_step(N, len(Ls), hermitian=True) * B * steps
    tr = torch.diagonal(rho, dim1=1, dim2=2).sum(-1)
    return {
        "value": round(B * steps / wall, 1), "unit": "density-matrix steps/s",
        "config": {"workload": "redfield_n128_rk4_fp64 (BASELINE.json configs[1], Redfield half)", "N": N,
                   "n_a_ops": len(Ls), "batch": B, "dt": dt, "kernel": "qd_glf_rk4_herm"},
        "roofline": {"bound": "mfma", "kernel": "lindblad_rk4_kernel<128,herm> (GLF operands)",
                     "achieved": round(flops / kern / 1e12, 3), "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(flops / kern / 1e12 / FP64_MFMA_PEAK_TFLOPS, 4),
                     "flop_per_dm_step": lindblad_flops_per_step(N, len(Ls), hermitian=True), "traffic": None},
        "trace_err": float((tr - 1).abs().max().item()),
    }, sol


def cpu_baseline_redfield(sol, dt=1e-3, budget_s=5.0):
    """NumPy port of the same RHS (dense GLF form, BLAS threads as set), one density matrix."""
    from oracle import lindblad as olb
    P, Q, Ls, Rs = sol.glf_terms()
    N = P.shape[0]
    rho = olb.random_pure_states(1, N, seed=7)[0]

    def rhs(r):
        out = P @ r + r @ Q
        for L, R in zip(Ls, Rs):
            out = out + L @ r @ R
        return out

    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        rho = olb.rk4(rho, rhs, dt)
        steps += 1
    el = time.perf_counter() - t0
    threads = os.environ.get("OMP_NUM_THREADS") or os.environ.get("OPENBLAS_NUM_THREADS") or str(os.cpu_count())
    return {"value": round(steps / el, 3), "unit": "density-matrix steps/s", "cores": int(threads) if threads.isdigit()
            else threads, "kind": "port",
            "sample": f"1 density matrix, N={N}, {steps} RK4 steps of the dense NumPy GLF form of R vec(rho) "
                      f"(oqs.py:519-570 in the eigenbasis) in {el:.1f}s; the reference's csr R (N^4 = 2.7e8 "
                      f"nonzeros) runs ~0.42 steps/s here (SURVEY.md §8(a5))"}


def bench_superop(dev, steps=10, N=128, dt=1e-3, batch=64, gemm_steps=2):
    """Dense L vec(rho) RK4 (BASELINE.json configs[1] "dense L.vec(rho) RK4", SURVEY §8(d) d1 GEMV alternative):
    the N = 128 Lindblad superoperator (16384^2 c128 = 4 GiB) built on the device, then (a) one density matrix on the
    HBM-streaming GEMV (16 N^4 B of L per stage) and (b) a batch on the MFMA GEMM stages."""
    import torch
    from pyqed_amd.oqs import lindblad_superop, superop_rk4
    H, cs = synthetic_lindblad(N, nc=1)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
    L = lindblad_superop(t(H), t(np.array(cs)))
    N2 = N * N
    stream = torch.cuda.current_stream(dev)

    def timed(v, k):
        ramp_warmup(lambda: superop_rk4(L, v, dt, 1), dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        superop_rk4(L, v, dt, k)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        return time.perf_counter() - t0, e0.elapsed_time(e1) / 1e3

    v1 = t(random_pure_states(1, N, seed=3).reshape(1, N2))
    wall, ev = timed(v1, steps)
    bytes_per_step = 4 * 16.0 * N2 * N2
    tr1 = abs(complex(torch.diagonal(v1.reshape(N, N)).sum().item()) - 1)
    vb = t(random_pure_states(batch, N, seed=4).reshape(batch, N2))
    wall_b, ev_b = timed(vb, gemm_steps)
    Bp = 64 if batch <= 64 else (batch + 127) // 128 * 128
    flop_b = 4 * 8.0 * N2 * N2 * Bp
    del L
    torch.cuda.empty_cache()
    return {
        "value": round(steps / wall, 2), "unit": "density-matrix steps/s (one rho, dense L vec(rho))",
        "config": {"workload": "lindblad_n128_dense_superop_rk4_fp64 (BASELINE.json configs[1], dense L.vec(rho))",
                   "N": N, "N2": N2, "L_bytes": 16 * N2 * N2, "dt": dt, "steps": steps,
                   "kernel": "superop_rows_kernel<1,4,4> (VALU GEMV, L streamed nontemporal)"},
        "us_per_step": round(ev / steps * 1e6, 1),
        "roofline": {"bound": "hbm", "kernel": "superop_rows_kernel<1,4,4>",
                     "achieved": round(bytes_per_step * steps / ev / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(bytes_per_step * steps / ev / 1e9 / HBM_PEAK_GBS, 4),
                     "bytes_per_step": bytes_per_step,
                     "traffic": measured_traffic("superop_rows_kernel<1,4,4>", 1) if N == 128 else None,
                     "traffic_unit": "HBM bytes per RK4 step (PMC FETCH_SIZE+WRITE_SIZE, calibrated; "
                                     "profiles/pmc_traffic.json)"},
        "trace_err": tr1,
        "batched": {"batch": batch, "steps": gemm_steps, "dm_steps_per_s": round(batch * gemm_steps / wall_b, 1),
                    "ms_per_step": round(ev_b / gemm_steps * 1e3, 3),
                    "roofline": {"bound": "mfma", "kernel": "ens_gemm_kernel<64> (L x X[N2][64] split-K)",
                                 "achieved": round(flop_b * gemm_steps / ev_b / 1e12, 3),
                                 "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                                 "frac": round(flop_b * gemm_steps / ev_b / 1e12 / FP64_MFMA_PEAK_TFLOPS, 4),
                                 "flop_per_step": flop_b,
                                 "note": "executed flops (batch padded to the 64-wide block); L read once per stage"}},
    }, (H, cs)


def cpu_baseline_superop(H, cs, dt=1e-3, budget_s=6.0):
    """NumPy dense GEMV form of _redfield's rhs = R.dot(rho) (oqs.py:462-463) with the N = 128 dense L (built here
    by the host kron restatement of superoperator.liouvillian), one density matrix, BLAS threads as set."""
    from oracle import lindblad as olb
    N = H.shape[0]
    I = np.eye(N)
    L = -1j * (np.kron(H, I) - np.kron(I, H.T))
    for c in cs:
        cdc = c.conj().T @ c
        L += np.kron(c, c.conj()) - 0.5 * (np.kron(cdc, I) + np.kron(I, cdc.T))
    v = olb.random_pure_states(1, N, seed=3).reshape(N * N)
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        v = olb.rk4(v, lambda x: L @ x, dt)
        steps += 1
    el = time.perf_counter() - t0
    del L
    threads = os.environ.get("OMP_NUM_THREADS") or os.environ.get("OPENBLAS_NUM_THREADS") or str(os.cpu_count())
    return {"value": round(steps / el, 3), "unit": "density-matrix steps/s", "kind": "port",
            "cores": int(threads) if threads.isdigit() else threads,
            "sample": f"{steps} RK4 steps of a dense NumPy L @ vec(rho) (N = 128, L 4 GiB) in {el:.1f}s"}


def twodes_inputs(M, seed=3):
    """BASELINE config d5: 3-level ladder E=[0,1,1.5] + static disorder (seed 3), Redfield with
    a_op = diag(0,1,2), flat spectrum 0.05, signature 'lccc', t2 = 0, t1 = t3 = 0.5*arange(256)."""
    from pyqed_amd.response import ensemble_factors, redfield_superop_batch
    from pyqed_amd.superoperator import operator_to_superoperator
    rng = np.random.default_rng(seed)
    E = np.array([0.0, 1.0, 1.5]) + np.array([0.0, 0.05, 0.08]) * rng.standard_normal((M, 3))
    dip = np.zeros((3, 3)); dip[0, 1] = dip[1, 0] = dip[1, 2] = dip[2, 1] = 1.0
    a = np.diag([0.0, 1.0, 2.0])
    rho0 = np.zeros((3, 3), complex); rho0[0, 0] = 1
    R = redfield_superop_batch(E, a, np.full((M, 3, 3), 0.05))
    lam, U1 = np.linalg.eig(R)
    U2 = np.linalg.inv(U1)
    ops = [operator_to_superoperator(dip, s).toarray() for s in "lccc"]
    alpha, Mt, beta = ensemble_factors(lam, U1, U2, ops, rho0.flatten(), 0.0)
    return lam, alpha, Mt, beta


def bench_2des(dev, world, rank, M_total, reps, n=256):
    """Ensemble 2DES (t3, t1) grid at fixed t2: members sharded over ranks, one RCCL reduce."""
    import torch
    import torch.distributed as dist
    from pyqed_amd.distributed import shard_range, sharded_sum
    from pyqed_amd.response import response2d_ensemble
    lo, hi = shard_range(M_total, rank, world)
    lam, alpha, Mt, beta = twodes_inputs(M_total)
    sl = slice(lo, hi)
    to = lambda x: torch.from_numpy(np.ascontiguousarray(x[sl])).to(dev)
    lam_t, alpha_t, Mt_t, beta_t = to(lam), to(alpha), to(Mt), to(beta)
    t = 0.5 * np.arange(n)  # uniform host grid -> exponential-table operand build (no device time arrays)
    out = torch.empty((n, n), dtype=torch.complex128, device=dev)

    from pyqed_amd.distributed import ReducePipeline
    # a sequence of `reps` grids; each grid's RCCL reduce(sum) to rank 0 runs asynchronously behind the next
    # grid's compute (two output buffers), and every reduce has completed before the timed region ends
    pipe = ReducePipeline((n, n), torch.complex128, dev, depth=2, dst=0)

    def once():
        buf = pipe.next_buffer()
        # this rank's members are already resident on its GPU (inputs in HBM before timing)
        response2d_ensemble(lam_t, alpha_t, Mt_t, beta_t, t, t, out=buf, accumulate=False)
        pipe.submit(buf)
        return buf

    def warm():
        once()
        pipe.finish()

    ramp_warmup(warm, dev, agree=world > 1)   # its calls issue the RCCL reduce at world > 1
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    stream = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    evs, host_ms = [], []
    for _ in range(reps):
        h0 = time.perf_counter()
        out = once()
        host_ms.append((time.perf_counter() - h0) * 1e3)
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(stream)
        evs.append(ev)
    pipe.finish()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    grid_ms = [round(e0.elapsed_time(evs[0]), 4)] + [round(evs[k - 1].elapsed_time(evs[k]), 4) for k in range(1, reps)]
    if world > 1:
        dist.barrier()
    tt = torch.tensor([wall], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    wall = float(tt.item())
    # executed GEMM K: members x the smaller pruned eigen-index set (exact structural zeros dropped,
    # pyqed_amd.response._prune_fixed_t2), padded to the 16-wide K-tile
    from pyqed_amd.response import _prune_fixed_t2
    nk = _prune_fixed_t2(lam_t, alpha_t, Mt_t, beta_t)[1].shape[1]
    K = (hi - lo) * nk
    Kp = (K + 15) // 16 * 16
    gemm_flop = 8.0 * n * n * Kp
    res = {
        "value": round(n * n * M_total * reps / wall, 1),
        "unit": "grid-points/s ((t3,t1) points x ensemble members)",
        "config": {"workload": "2des_3level_256x256_redfield_ensemble (BASELINE.json configs[4])",
                   "grid": [n, n], "ensemble_members": M_total, "members_per_rank": hi - lo, "t2": 0.0,
                   "signature": "lccc", "scaling": "strong",
                   "collective": "RCCL reduce(sum) of each 1 MiB grid to rank 0, pipelined behind the next grid's "
                                 "compute (2 output buffers)" if world > 1 else "none"},
        "ms_per_grid": round(wall / reps * 1e3, 4),
        "roofline": {"bound": "mfma", "kernel": "ens_gemm_kernel<128,xtab>" if Kp >= 32768 else "ens_gemm_kernel<64>",
                     "achieved": round(gemm_flop / (e0.elapsed_time(e1) / reps / 1e3) / 1e12, 3),
                     "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(gemm_flop / (e0.elapsed_time(e1) / reps / 1e3) / 1e12 / FP64_MFMA_PEAK_TFLOPS, 4),
                     "flop_per_grid": gemm_flop,
                     "traffic": measured_traffic("ens_gemm_kernel_xtab", 1) if (M_total, n, world) == (65536, 256, 1)
                     else None,
                     "traffic_unit": "HBM bytes per ens_gemm_kernel launch (PMC FETCH_SIZE+WRITE_SIZE, calibrated; "
                                     "profiles/pmc_traffic.json)",
                     "note": "8 n3 n1 K flop per grid (K = members x pruned index set) / event time of the whole grid "
                             "(operand tables, Z build, GEMM, slab reduction): a lower bound on the GEMM's own rate"},
        "gemm_flop_per_grid_per_rank": gemm_flop,
        "grid_event_ms": grid_ms, "host_issue_ms": [round(x, 3) for x in host_ms],
        "gemm_k_per_member": nk,
        "event_ms_per_grid": round(e0.elapsed_time(e1) / reps, 4),
    }
    return res, out, (lam, alpha, Mt, beta)


def bench_2des_t2scan(dev, world, rank, M_total, n2, reps, n=256):
    """2DES waiting-time scan: n2 (t3, t1) grids at t2 = 2.5*j of the M_total-member ensemble.  Members
    shard over ranks; each rank runs ONE qd_response2d_t2scan launch sequence per rep (t3 operand built
    once, every t2 in one split-K MFMA GEMM), then ONE RCCL reduce(sum) of the [n2, n, n] stack."""
    import torch
    import torch.distributed as dist
    from pyqed_amd.distributed import shard_range
    from pyqed_amd.response import ensemble_factors_bc, redfield_superop_batch
    from pyqed_amd.superoperator import operator_to_superoperator
    lo, hi = shard_range(M_total, rank, world)
    rng = np.random.default_rng(3)
    E = np.array([0.0, 1.0, 1.5]) + np.array([0.0, 0.05, 0.08]) * rng.standard_normal((M_total, 3))
    E = E[lo:hi]
    dip = np.zeros((3, 3)); dip[0, 1] = dip[1, 0] = dip[1, 2] = dip[2, 1] = 1.0
    R = redfield_superop_batch(E, np.diag([0.0, 1.0, 2.0]), np.full((len(E), 3, 3), 0.05))
    lam, U1 = np.linalg.eig(R)
    U2 = np.linalg.inv(U1)
    rho0v = np.zeros(9, complex); rho0v[0] = 1
    ops = [operator_to_superoperator(dip, s).toarray() for s in "lccc"]
    alpha, B, C, beta = ensemble_factors_bc(lam, U1, U2, ops, rho0v)
    to = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
    lam_t, alpha_t, B_t, C_t, beta_t = to(lam), to(alpha), to(B), to(C), to(beta)
    t = 0.5 * np.arange(n)
    t2 = to(2.5 * np.arange(n2))
    out = torch.empty((n2, n, n), dtype=torch.complex128, device=dev)
    from pyqed_amd.response import T2Scan

    from pyqed_amd.distributed import sharded_sum_buckets
    bucket = max(1, min(n2, 4))           # 4 waiting times = 4 MiB per RCCL reduce
    buckets = [slice(b, min(n2, b + bucket)) for b in range(0, n2, bucket)]

    scan = [None]

    def local(lo_, hi_, b):               # this rank's members are resident; t2 bucket b of the scan
        scan[0].apply(t2[b], out=out[b])

    def once():
        # P = X B and Q = C Y on the (t3, t1) grids, once per scan; then the buckets of waiting times
        scan[0] = T2Scan(lam_t, alpha_t, B_t, C_t, beta_t, t, t)
        sharded_sum_buckets(local, M_total, out, buckets, dst=0)

    ramp_warmup(once, dev, agree=world > 1)   # its calls issue the bucket reduces at world > 1
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    stream = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(reps):
        once()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    tt = torch.tensor([wall], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    wall = float(tt.item())
    # the roofline comes from THIS timed region: HIP events on the launch stream around the same `reps` scans
    # (operand build + bucket applies, and the bucket reduces at world > 1), so frac follows ms_per_scan
    # (a separately timed loop gave a different frac)
    ev_scan = e0.elapsed_time(e1) / 1e3 / reps
    # compute-only time of this rank's launch sequence (no collective), for the scaling breakdown
    torch.cuda.synchronize(dev)
    c0 = time.perf_counter()
    for _ in range(reps):
        scan[0] = T2Scan(lam_t, alpha_t, B_t, C_t, beta_t, t, t)
        for b in buckets:
            local(lo, hi, b)
    torch.cuda.synchronize(dev)
    comp = (time.perf_counter() - c0) / reps
    nr = scan[0].nL                         # executed K per member: the pruned waiting-time index set
    Kp = ((hi - lo) * nr + 15) // 16 * 16
    gemm_flop = 8.0 * n * n * n2 * Kp
    return {
        "value": round(n * n * n2 * M_total * reps / wall, 1),
        "unit": "grid-points/s ((t3,t1,t2) points x ensemble members)",
        "config": {"workload": "2des_3level_256x256_redfield_ensemble_t2scan (BASELINE.json configs[4] x waiting times)",
                   "grid": [n, n], "n_t2": n2, "ensemble_members": M_total, "members_per_rank": hi - lo,
                   "signature": "lccc", "scaling": "strong",
                   "collective": f"RCCL reduce(sum) of the [{n2},{n},{n}] c128 stack in {len(buckets)} buckets of "
                   f"{bucket} waiting times, each overlapped with the next bucket's GEMM" if world > 1 else "none"},
        "ms_per_scan": round(wall / reps * 1e3, 4),
        "compute_ms_per_scan": round(comp * 1e3, 4),
        "gemm_tflops": round(gemm_flop / comp / 1e12, 2),
        "index_set_sizes_p_r_q": list(scan[0].index_sizes),
        "roofline": {"bound": "mfma", "kernel": "ens_t2_gemm_kernel", "achieved": round(gemm_flop / ev_scan / 1e12, 3),
                     "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(gemm_flop / ev_scan / 1e12 / FP64_MFMA_PEAK_TFLOPS, 4),
                     "ms_per_scan_events": round(ev_scan * 1e3, 4),
                     "flop_per_scan": gemm_flop,
                     "traffic": measured_traffic("ens_t2_gemm_kernel_pruned", 1) if (M_total, n, world) == (65536, 256, 1) else None,
                     "traffic_unit": "HBM bytes per ens_t2_gemm_kernel launch (4 waiting times; PMC FETCH_SIZE+WRITE_SIZE, "
                                     "calibrated; profiles/pmc_traffic.json)",
                     "note": "8 n3 n1 n2 K flop per scan (K = members x nL) / the timed region's HIP-event time per "
                             "scan (operand build, E tables, GEMM, slab reduction, and the reduces at world > 1): a "
                             "lower bound on the GEMM kernel's own rate"},
    }


def _blas_one_thread():
    """Context pinning BLAS to one thread (threadpoolctl), or a no-op without it."""
    import contextlib
    try:
        from threadpoolctl import threadpool_limits
        return threadpool_limits(1)
    except ImportError:
        return contextlib.nullcontext()


def cpu_baseline_2des(lam, alpha, Mt, beta, n=256, budget_s=5.0):
    """Closed-form slice per member with NumPy (oracle formula of correlation_4op_3t[:, j, :])."""
    t = 0.5 * np.arange(n)
    with _blas_one_thread():
        t0 = time.perf_counter()
        m = 0
        while time.perf_counter() - t0 < budget_s and m < len(lam):
            X = alpha[m][None, :] * np.exp(np.outer(t, lam[m]))
            Y = beta[m][None, :] * np.exp(np.outer(t, lam[m]))
            _ = (-1j) ** 3 * X @ Mt[m] @ Y.T
            m += 1
        el = time.perf_counter() - t0
    res = {"value": round(n * n * m / el, 1), "unit": "grid-points/s", "cores": 1, "kind": "port",
           "sample": f"{m} ensemble members x {n}x{n} grid, NumPy eigen-form slice in {el:.2f}s",
           "note": "1 core by choice (one member per slice, BLAS pinned to one thread); `multicore` times the "
                   "vectorised slices over the process's CPU share"}
    res["multicore"] = cpu_baseline_2des_multicore(lam, alpha, Mt, beta, n, budget_s)
    return res


def cpu_baseline_2des_multicore(lam, alpha, Mt, beta, n=256, budget_s=5.0, chunk=64):
    """The same eigen-form slices vectorised over chunks of `chunk` members (batched exp and matmul, which release the
    GIL) and dealt over a thread pool of the process's CPU share (OMP_NUM_THREADS: 16 on the GPU box), BLAS one thread
    per worker; a chunk's summed signal is one GEMM over K = chunk x nL (the GPU's formulation)."""
    from concurrent.futures import ThreadPoolExecutor
    env = os.environ.get("OMP_NUM_THREADS", "")
    cores = int(env) if env.isdigit() else min(16, os.cpu_count() or 1)
    t = 0.5 * np.arange(n)
    stop = time.perf_counter() + budget_s
    nch = (len(lam) + chunk - 1) // chunk

    def work(w):
        done = 0
        for c in range(w, nch, cores):
            if time.perf_counter() > stop:
                break
            sl = slice(c * chunk, min(len(lam), (c + 1) * chunk))
            E = np.exp(t[None, :, None] * lam[sl][:, None, :])                  # [c, n, nL]
            X = alpha[sl][:, None, :] * E
            Y = beta[sl][:, None, :] * E
            A = (X @ Mt[sl]).transpose(1, 0, 2).reshape(n, -1)                   # [n, c nL]: one GEMM per chunk
            _ = (-1j) ** 3 * (A @ Y.transpose(0, 2, 1).reshape(-1, n))
            done += sl.stop - sl.start
        return done

    with _blas_one_thread():
        t0 = time.perf_counter()
        with ThreadPoolExecutor(cores) as ex:
            m = sum(ex.map(work, range(cores)))
        el = time.perf_counter() - t0
    return {"value": round(n * n * m / el, 1), "unit": "grid-points/s", "cores": cores, "kind": "port",
            "sample": f"{m} ensemble members x {n}x{n} grid, chunks of {chunk} over {cores} threads in {el:.2f}s"}


def bench_spo2(dev, steps, n=256, dt=0.05):
    """BASELINE config d2: 2D vibronic SPO, 256x256 grid x 2 diabatic states, Strang steps."""
    import torch
    from pyqed_amd import _lib
    from pyqed_amd.wpd import SPO2
    x = np.linspace(-6, 6, n)
    X, Y = np.meshgrid(x, x, indexing="ij")
    sol = SPO2(x, x, mass=[1.0, 1.0], nstates=2)
    sol.set_DPES([0.5 * ((X + 1) ** 2 + Y ** 2), 0.5 * ((X - 1) ** 2 + Y ** 2) + 0.1], [[[0, 1], 0.2 * X]])
    sol.build(dt)
    psi0 = np.zeros((n, n, 2), complex)
    psi0[:, :, 0] = np.exp(-((X + 1.5) ** 2 + Y ** 2) / 2 + 0.5j * X) / np.sqrt(np.pi)
    psi = torch.from_numpy(psi0).to(dev)
    eVh = torch.from_numpy(sol.exp_V_half).to(dev)
    eK = torch.from_numpy(sol.exp_K).to(dev)
    lib = _lib.load()
    st = _lib.stream_ptr(dev)

    def run(k):
        _lib.check(lib.qd_spo2_run(psi.data_ptr(), eVh.data_ptr(), eK.data_ptr(), n, n, 2, k, k, None, st),
                   "qd_spo2_run")

    ramp_warmup(lambda: run(10), dev)
    stream = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    run(steps)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    ev = e0.elapsed_time(e1) / 1e3
    bytes_per_step = (4 * n * n * 2 + n * n * 4 + n * n) * 16  # psi r/w x2 kernels, exp_V_half, exp_K
    norm = float((psi.abs() ** 2).sum().item() / (np.abs(psi0) ** 2).sum())
    # drop-in end to end: SPO2.run (device build of the point propagators + upload + steps + download)
    sol.build(dt)
    torch.cuda.synchronize(dev)
    tb = time.perf_counter()
    sol.build(dt)
    torch.cuda.synchronize(dev)
    build_ms = (time.perf_counter() - tb) * 1e3
    tr = time.perf_counter()
    r = sol.run(psi0, dt=dt, nt=steps, nout=steps)
    run_wall = time.perf_counter() - tr
    # batched throughput: Bw independent wavepackets on the same potential (qd_spo2_run_batch, one launch per
    # pass for the whole batch); algorithmic bytes per step = Bw x psi read + write in both passes + the shared
    # exp_V_half / exp_K once
    Bw, bsteps = 64, max(10, steps // 10)
    psib = psi.unsqueeze(0).repeat(Bw, 1, 1, 1).contiguous()

    def runb(k):
        _lib.check(lib.qd_spo2_run_batch(psib.data_ptr(), Bw, eVh.data_ptr(), eK.data_ptr(), n, n, 2, k, k, None, st),
                   "qd_spo2_run_batch")

    ramp_warmup(lambda: runb(2), dev)
    b0, b1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    b0.record(stream)
    runb(bsteps)
    b1.record(stream)
    torch.cuda.synchronize(dev)
    bev = b0.elapsed_time(b1) / 1e3
    bbytes = (4 * n * n * 2 * Bw + n * n * 4 + n * n) * 16
    batched = {"wavepackets": Bw, "steps": bsteps, "wavepacket_steps_per_s": round(Bw * bsteps / bev, 1),
               "roofline": {"bound": "hbm", "achieved": round(bbytes * bsteps / bev / 1e9, 1), "peak": HBM_PEAK_GBS,
                            "unit": "GB/s", "frac": round(bbytes * bsteps / bev / 1e9 / HBM_PEAK_GBS, 4),
                            "bytes_per_step": bbytes,
                            "traffic": (measured_traffic("spo2_row_wave_kernel<4>_64wp", Bw)
                                        + measured_traffic("spo2_col_tile8_kernel<8>_64wp", Bw))
                            if (n, Bw) == (256, 64) and measured_traffic("spo2_row_wave_kernel<4>_64wp", 1) else None,
                            "traffic_unit": "HBM bytes per batched Strang step (row + column pass; PMC FETCH_SIZE+"
                                            "WRITE_SIZE, calibrated; profiles/pmc_traffic.json)",
                            "note": "wave-per-member row pass (lane-local 2x2 point operators) + 8-column tile "
                                    "column pass; working set 134 MiB"}}
    return {
        "value": round(steps / wall, 1), "unit": "SPO steps/s",
        "batched": batched,
        "config": {"workload": "spo2_256x256x2 (BASELINE.json configs[2])", "grid": [n, n], "nstates": 2,
                   "dt": dt},
        "roofline": {"bound": "hbm", "achieved": round(bytes_per_step * steps / ev / 1e9, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(bytes_per_step * steps / ev / 1e9 / HBM_PEAK_GBS, 4),
                     "bytes_per_step": bytes_per_step,
                     "traffic": (measured_traffic("spo2_row_q16_kernel<2>", 1) + measured_traffic("spo2_col_q16_kernel<2>", 1))
                     if n == 256 else None,
                     "traffic_unit": "HBM bytes per Strang step (row + column pass; PMC FETCH_SIZE+WRITE_SIZE, calibrated; "
                                     "profiles/pmc_traffic.json)",
                     "note": "working set (7 MiB) is MALL-resident; two dependent passes per step bound it (latency)"},
        "us_per_step": round(wall / steps * 1e6, 2), "norm_ratio": norm,
        "build_ms": round(build_ms, 3),
        "run_wall_s": round(run_wall, 4),
        "run_note": f"SPO2.run(nt={steps}) end to end incl. build, transfers and the 2 returned states",
    }


def bench_spo3(dev, steps=200, n=64, dt=0.05):
    """SPO3 at the examples/spo.py grid, 64^3 x 2 diabatic states (wpd.SPO3.run, wpd.py:1105-1432): one wavepacket,
    device-resident, HIP events over `steps` Strang steps on the path SPO3.run takes (qd_spo3_run_axes: the separable
    kinetic step as three register-FFT passes of F^-1 diag(e_a / n) F, the z pass with the point propagators), the
    four-pass path of the 3-D exp_K (qd_spo3_run) timed beside it, plus SPO3.run end to end."""
    import torch
    from pyqed_amd import _lib
    from pyqed_amd.wpd import SPO3, axis_propagator
    x = np.linspace(-6, 6, n)
    X, Y, Z = np.meshgrid(x, x, x, indexing="ij")
    sol = SPO3(x, x, x, masses=[1.0, 1.0, 1.0], nstates=2)
    sol.set_DPES([0.5 * ((X + 1) ** 2 + Y ** 2 + Z ** 2), 0.5 * ((X - 1) ** 2 + Y ** 2 + Z ** 2)], [[[0, 1], 0.2 * X]])
    sol.build(dt)
    assert sol._use_axes()
    psi0 = np.zeros((n, n, n, 2), complex)
    psi0[..., 1] = np.exp(-((X + 1) ** 2 + Y ** 2 + Z ** 2) / 2) / np.pi ** 0.75
    psi = torch.from_numpy(psi0).to(dev)
    eVh = torch.from_numpy(sol.exp_V_half).to(dev)
    eK = torch.from_numpy(sol.exp_K).to(dev)
    m = [torch.from_numpy(axis_propagator(k, ma, dt)).to(dev) for k, ma in zip((sol.kx, sol.ky, sol.kz), sol.masses)]
    lib = _lib.load()
    st = _lib.stream_ptr(dev)

    def run_sep(k):
        _lib.check(lib.qd_spo3_run_axes(psi.data_ptr(), eVh.data_ptr(), *(v.data_ptr() for v in m), n, n, n, 2, k, k,
                                        None, st), "qd_spo3_run_axes")

    def run_4pass(k):
        _lib.check(lib.qd_spo3_run(psi.data_ptr(), eVh.data_ptr(), eK.data_ptr(), n, n, n, 2, k, k, None, st),
                   "qd_spo3_run")

    def timed(run):
        ramp_warmup(lambda: run(5), dev)
        stream = torch.cuda.current_stream(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        run(steps)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / 1e3

    ev4 = timed(run_4pass)
    ev = timed(run_sep)
    norm = float((psi.abs() ** 2).sum().item() / (np.abs(psi0) ** 2).sum())
    # bytes per step of the three passes: psi (n^3 x 2 c128) read + written by each, exp_V_half (n^3 x 4) read by
    # the z pass (the 3 x 64 axis factors are negligible); the four-pass path: four psi round trips, exp_V_half, exp_K
    bytes_per_step = (3 * 2 * n ** 3 * 2 + n ** 3 * 4) * 16
    bytes_4pass = (4 * 2 * n ** 3 * 2 + n ** 3 * 4 + n ** 3) * 16
    tr = time.perf_counter()
    sol.run(psi0, dt=dt, nt=100, nout=100)
    run_wall = time.perf_counter() - tr
    ach = bytes_per_step / (ev / steps) / 1e9
    ach4 = bytes_4pass / (ev4 / steps) / 1e9
    return {
        "value": round(steps / ev, 1), "unit": "SPO steps/s", "us_per_step": round(ev / steps * 1e6, 2),
        "path": "spo3_sep64 (qd_spo3_run_axes)",
        "config": {"workload": "spo3_64x64x64x2 (examples/spo.py grid; SURVEY §8(f) SPO3 64^3)", "grid": [n, n, n],
                   "nstates": 2, "dt": dt, "steps": steps},
        "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(ach / HBM_PEAK_GBS, 4), "bytes_per_step": bytes_per_step,
                     "note": "three passes over an 8 MiB state that stays in the Infinity Cache: dependent-pass "
                             "latency, not bytes, bounds one wavepacket (the pass count, not the bytes per pass, is "
                             "what the separable form cut)"},
        "four_pass_path": {"kernel_path": "spo3_pow2 (qd_spo3_run, 3-D exp_K)", "us_per_step": round(ev4 / steps * 1e6, 2),
                           "value": round(steps / ev4, 1), "bytes_per_step": bytes_4pass,
                           "frac": round(ach4 / HBM_PEAK_GBS, 4)},
        "norm_ratio": norm, "run_100_steps_wall_s": round(run_wall, 4),
        "any_grid_60": _spo3_axes_leg(dev, steps, 60, dt, ev / steps),
    }


def _spo3_axes_leg(dev, steps, n, dt, us64_s):
    """SPO3 on a grid that is not a power of two (n^3 x 2, same model): the path SPO3.run takes there, the kinetic
    step as three per-axis mode products on the MFMAs (qd_spo3_run_axes), HIP events over `steps` Strang steps; the
    cost per point against the 64^3 line."""
    import torch
    from pyqed_amd import _lib
    from pyqed_amd.wpd import SPO3, axis_propagator
    x = np.linspace(-6, 6, n)
    X, Y, Z = np.meshgrid(x, x, x, indexing="ij")
    sol = SPO3(x, x, x, masses=[1.0, 1.0, 1.0], nstates=2)
    sol.set_DPES([0.5 * ((X + 1) ** 2 + Y ** 2 + Z ** 2), 0.5 * ((X - 1) ** 2 + Y ** 2 + Z ** 2)], [[[0, 1], 0.2 * X]])
    sol.build(dt)
    assert sol._use_axes()
    psi0 = np.zeros((n, n, n, 2), complex)
    psi0[..., 1] = np.exp(-((X + 1) ** 2 + Y ** 2 + Z ** 2) / 2) / np.pi ** 0.75
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    psi, eVh = t(psi0), t(sol.exp_V_half)
    m = [t(axis_propagator(k, ma, dt)) for k, ma in zip((sol.kx, sol.ky, sol.kz), sol.masses)]
    lib = _lib.load()
    st = _lib.stream_ptr(dev)

    def run(k):
        _lib.check(lib.qd_spo3_run_axes(psi.data_ptr(), eVh.data_ptr(), *(v.data_ptr() for v in m), n, n, n, 2, k, k,
                                        None, st), "qd_spo3_run_axes")

    ramp_warmup(lambda: run(5), dev)
    stream = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    run(steps)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    sec = e0.elapsed_time(e1) / 1e3 / steps
    return {"grid": [n, n, n], "nstates": 2, "path": "spo3_axes", "us_per_step": round(sec * 1e6, 2),
            "per_point_vs_64cubed": round(sec / n ** 3 / (us64_s / 64 ** 3), 3),
            "norm_ratio": float((psi.abs() ** 2).sum().item() / (np.abs(psi0) ** 2).sum())}


def cpu_baseline_spo3(n=64, dt=0.05, budget_s=5.0):
    from oracle import spo as ospo
    x = np.linspace(-6, 6, n)
    X, Y, Z = np.meshgrid(x, x, x, indexing="ij")
    v = np.zeros((n, n, n, 2, 2))
    v[..., 0, 0] = 0.5 * ((X + 1) ** 2 + Y ** 2 + Z ** 2)
    v[..., 1, 1] = 0.5 * ((X - 1) ** 2 + Y ** 2 + Z ** 2)
    v[..., 0, 1] = v[..., 1, 0] = 0.2 * X
    w, u = np.linalg.eigh(v)
    eVh = (u * np.exp(-1j * w * dt / 2)[..., None, :]) @ np.conj(np.swapaxes(u, -1, -2))
    kx = 2 * np.pi * np.fft.fftfreq(n, x[1] - x[0])
    KX, KY, KZ = np.meshgrid(kx, kx, kx, indexing="ij")
    eK = np.exp(-1j * (KX ** 2 + KY ** 2 + KZ ** 2) / 2 * dt)
    psi = np.zeros((n, n, n, 2), complex)
    psi[..., 1] = np.exp(-((X + 1) ** 2 + Y ** 2 + Z ** 2) / 2)
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < budget_s:
        psi = ospo.spo3_run(eVh, eK, psi, 2, 2)[-1]
        k += 2
    el = time.perf_counter() - t0
    return {"value": round(k / el, 2), "unit": "SPO steps/s", "cores": 1, "kind": "port",
            "sample": f"{k} Strang steps of the numpy.fft restatement of SPO3.run at {n}^3 x 2 in {el:.1f}s"}


def cpu_baseline_spo2(n=256, dt=0.05, budget_s=5.0):
    from oracle import spo as ospo
    x = np.linspace(-6, 6, n)
    X, Y = np.meshgrid(x, x, indexing="ij")
    v = np.zeros((n, n, 2, 2))
    v[:, :, 0, 0] = 0.5 * ((X + 1) ** 2 + Y ** 2)
    v[:, :, 1, 1] = 0.5 * ((X - 1) ** 2 + Y ** 2) + 0.1
    v[:, :, 0, 1] = v[:, :, 1, 0] = 0.2 * X
    w, u = np.linalg.eigh(v)
    eVh = (u * np.exp(-1j * w * dt / 2)[..., None, :]) @ np.conj(np.swapaxes(u, -1, -2))
    kx = 2 * np.pi * np.fft.fftfreq(n, x[1] - x[0])
    KX, KY = np.meshgrid(kx, kx, indexing="ij")
    eK = np.exp(-1j * (KX ** 2 + KY ** 2) / 2 * dt)
    psi = np.zeros((n, n, 2), complex)
    psi[:, :, 0] = np.exp(-((X + 1.5) ** 2 + Y ** 2) / 2)
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < budget_s:
        psi = ospo.spo2_run(eVh, eK, psi, 5, 5)[-1]
        k += 5
    el = time.perf_counter() - t0
    return {"value": round(k / el, 2), "unit": "SPO steps/s", "cores": 1, "kind": "port",
            "sample": f"{k} Strang steps of the scipy.fftpack restatement of SPO2.run at {n}x{n}x2 in {el:.1f}s"}


def _deom_event_rate(dev, sol, bath, H, Q, B, steps, dt=0.002, banded=True):
    """RK4 steps/s of B independent hierarchies of `sol` (device-resident state; HIP events on the launch stream
    around `steps` steps).  B = 1 runs what DEOMSolver.run runs: the persistent tier-banded launch
    (qd_deom_rk4_banded) where the hierarchy qualifies, else (or banded=False) 4 stage launches per step; B >= 16
    runs the ADO-major layout."""
    import torch
    from pyqed_amd import _lib
    from pyqed_amd.deom import ado_coefficients
    ns, K, nmax = H.shape[0], sol.nind, sol.nmax
    coef, damp = ado_coefficients(sol.keys, np.asarray(bath.etal), np.asarray(bath.etar), np.asarray(bath.etaa),
                                  np.asarray(bath.expn), sol.lmax)
    c128 = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=complex))).to(dev)
    i32 = lambda a: torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.int32))).to(dev)
    tabs = (i32(sol._minus), i32(sol._plus), c128(coef), c128(damp), i32(bath.mode))
    Hd, Qd = c128(H), c128(Q)
    lib = _lib.load()
    st = _lib.stream_ptr(dev)
    ado_major = B >= 16
    fn = lib.qd_deom_rk4_ado_major if ado_major else lib.qd_deom_rk4
    ados = torch.zeros((nmax, B, ns, ns) if ado_major else (B, nmax, ns, ns), dtype=torch.complex128, device=dev)
    (ados[0] if ado_major else ados[:, 0])[..., 0, 0] = 1
    rho_sys = torch.empty((B, steps + 1, ns, ns), dtype=torch.complex128, device=dev)

    bands = sol.band_tables(dev) if (B == 1 and banded) else None
    status = torch.zeros(1, dtype=torch.int32, device=dev)

    def run(n):
        if bands is not None:
            rc = lib.qd_deom_rk4_banded(ados.data_ptr(), nmax, K, ns, *bands.args(), *(t.data_ptr() for t in tabs[2:]),
                                        Qd.shape[0], Hd.data_ptr(), None, Qd.data_ptr(), None, None, None, dt, n,
                                        rho_sys.data_ptr(), None, 0, None, status.data_ptr(), st)
            _lib.check(rc, "qd_deom_rk4_banded")
            return
        rc = fn(ados.data_ptr(), B, nmax, K, ns, *(t.data_ptr() for t in tabs), Qd.shape[0], Hd.data_ptr(), None,
                Qd.data_ptr(), None, None, None, dt, n, rho_sys.data_ptr(), None, 0, None, st)
        _lib.check(rc, "qd_deom_rk4")

    ramp_warmup(lambda: run(5), dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    run(steps)
    e1.record()
    torch.cuda.synchronize(dev)
    assert int(status.item()) == 0, "qd_deom_rk4_banded: a band hand-off timed out"
    tr = torch.diagonal(rho_sys[:, -1], dim1=-2, dim2=-1).sum(-1)
    assert float((tr - 1).abs().max()) < 1e-10
    return steps / (e0.elapsed_time(e1) / 1e3)


def bench_deom(dev, steps, batch):
    """BASELINE config d4: spin-boson H = sz + sx, Q = sx, Drude lambda=0.5 gamma=1 beta=1, Pade npsd=4
    (K=5), L=12 -> 6188 ADOs.  dt=0.002 (RK4 stability: dt*L*max Re expn < 2.8; the SURVEY value 0.01
    diverges).  One hierarchy and a batch of independent hierarchies (ADO-major layout), state resident on the
    device, `steps` RK4 steps timed by HIP events on the launch stream; DEOMSolver.run end to end is timed too;
    the "~10k ADO" stretch hierarchy of SURVEY §8(d) d4 (npsd=5, K=6: 18,564 ADOs) as one more line."""
    import sympy as sp
    import torch
    from pyqed_amd.deom import Bath, DEOMSolver
    w = sp.symbols(r"\omega", real=True)
    sx = np.array([[0, 1], [1, 0]], complex)
    sz = np.diag([1.0, -1.0]).astype(complex)
    rho0 = np.zeros((2, 2), complex)
    rho0[0, 0] = 1
    bath = Bath([2 * 0.5 * 1.0 * w / (1.0 + w ** 2)], w, [1.0], [4], [0] * 5)
    sol = DEOMSolver(sz + sx, None, bath, np.array([sx]), None, None, None, 12)
    sol.run_batch(rho0[None], 0.01, 5)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    sol.run(rho0.copy(), 0.002, steps)
    wall_run = time.perf_counter() - t0
    nmax = sol.nmax
    rate = {B: _deom_event_rate(dev, sol, bath, sz + sx, sx[None], B, steps) for B in (1, batch)}
    bath5 = Bath([2 * 0.5 * 1.0 * w / (1.0 + w ** 2)], w, [1.0], [5], [0] * 6)
    sol5 = DEOMSolver(sz + sx, None, bath5, np.array([sx]), None, None, None, 12)
    sol5.check_()
    sol5.init_()
    rate5 = _deom_event_rate(dev, sol5, bath5, sz + sx, sx[None], 1, steps, dt=0.001)
    rate_stage = _deom_event_rate(dev, sol, bath, sz + sx, sx[None], 1, steps, banded=False)
    rate5_stage = _deom_event_rate(dev, sol5, bath5, sz + sx, sx[None], 1, steps, dt=0.001, banded=False)
    bt, bt5 = sol.band_tables(dev), sol5.band_tables(dev)
    single = rate[1]
    # per RK4 step ~4.75 MB of ADO traffic per hierarchy = 768 B per ADO-step (the survey's figure,
    # kept as the denominator; the Horner-form stages move 11 rows of 64 B = 704 B per ADO-step)
    bytes_per_step = 4.75e6
    bytes_per_ado_step = 768.0
    ado_b = rate[batch] * nmax * batch
    return {
        "value": round(single, 1), "unit": "RK4 steps/s (one hierarchy)",
        "ado_steps_per_s_single": round(single * nmax, 1),
        "kernel": (f"deom_band_kernel (one persistent launch, {bt.nbands} tier bands)" if bt is not None else
                   "stage launches"),
        "steps_per_s_stage_launches": round(rate_stage, 1),
        "run_steps_per_s_end_to_end": round(steps / wall_run, 1),
        "batched": {"hierarchies": batch, "ado_steps_per_s": round(ado_b, 1), "steps_per_s": round(rate[batch], 1),
                    "layout": "ADO-major [nmax][B][2][2], hierarchies dealt to the 8 XCD block classes",
                    "roofline": {"bound": "hbm", "kernel": "deom_stage_pipe_kernel<5>",
                                 "achieved": round(ado_b * bytes_per_ado_step / 1e9, 1), "peak": HBM_PEAK_GBS,
                                 "unit": "GB/s", "frac": round(ado_b * bytes_per_ado_step / 1e9 / HBM_PEAK_GBS, 4),
                                 "bytes_per_ado_step": bytes_per_ado_step,
                                 "traffic": measured_traffic("deom_stage_pipe_kernel<5>_64h", nmax * batch / 4)
                                 if batch == 64 else None,
                                 "traffic_unit": "HBM bytes per stage launch (PMC FETCH_SIZE+WRITE_SIZE, calibrated; "
                                                 "profiles/pmc_traffic.json)"}},
        "stretch_npsd5": {"nmax": sol5.nmax, "K": sol5.nind, "L": 12, "dt": 0.001, "steps_per_s": round(rate5, 1),
                          "bands": bt5.nbands if bt5 is not None else None,
                          "steps_per_s_stage_launches": round(rate5_stage, 1),
                          "ado_steps_per_s": round(rate5 * sol5.nmax, 1)},
        "roofline": {"bound": "hbm", "achieved": round(bytes_per_step * single / 1e9, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(bytes_per_step * single / 1e9 / HBM_PEAK_GBS, 4),
                     "bytes_per_step": bytes_per_step,
                     "kernel": "deom_band_kernel<4,5,true,256,true>" if bt is not None else "deom_stage_grp_kernel",
                     "traffic": measured_traffic("deom_band_kernel<4,5,true,256,true>", 1) if bt is not None else None,
                     "traffic_unit": "HBM / fabric bytes per RK4 step (PMC FETCH_SIZE+WRITE_SIZE, calibrated; "
                                     "profiles/pmc_traffic.json): the halo rows every band gathers per stage",
                     "note": "latency-bound: 4 dependent RK4 stages per step on a 396 KB state; the banded launch "
                             "hands each stage's rows between the bands inside one launch (per-stage hand-off "
                             "latency, no kernel boundaries)"},
        "config": {"workload": "deom_spin_boson_drude_L12_K5 (BASELINE.json configs[3])", "nmax": nmax, "K": 5,
                   "L": 12, "dt": 0.002, "steps": steps},
        "note": "value / batched: device-resident state, HIP events over `steps` RK4 steps (value: the banded "
                "persistent launch DEOMSolver.run takes for one hierarchy; batched: 4 stage launches per step); "
                "run_steps_per_s_end_to_end: DEOMSolver.run incl. table setup and transfers",
    }


def time_reduce_one_rank(dev, reps=50):
    """One 1 MiB RCCL reduce(sum) (the 256 x 256 c128 2DES grid) on a one-rank communicator through the C-ABI
    (qd_comm_init / qd_reduce_sum), HIP events on the launch stream: the per-grid RCCL launch cost that the 8-GPU
    projection adds (one rank cannot time the xGMI transfer itself)."""
    import ctypes
    import torch
    from pyqed_amd import _lib
    lib = _lib.load()
    uid = ctypes.create_string_buffer(128)
    # RCCL prints its version banner to stdout at communicator init: send fd 1 to stderr meanwhile, so that stdout
    # carries only the bench's JSON line
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        _lib.check(lib.qd_comm_unique_id(uid), "qd_comm_unique_id")
        _lib.check(lib.qd_comm_init(1, 0, uid), "qd_comm_init")
    finally:
        os.dup2(saved, 1)
        os.close(saved)
    try:
        x = torch.zeros(256 * 256, dtype=torch.complex128, device=dev)
        st = _lib.stream_ptr(dev)
        for _ in range(5):
            _lib.check(lib.qd_reduce_sum(x.data_ptr(), x.numel(), 0, st), "qd_reduce_sum")
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            _lib.check(lib.qd_reduce_sum(x.data_ptr(), x.numel(), 0, st), "qd_reduce_sum")
        e1.record()
        torch.cuda.synchronize(dev)
        return e0.elapsed_time(e1) / reps
    finally:
        _lib.check(lib.qd_comm_destroy(), "qd_comm_destroy")


def _band_case(ns, L, npsd=3):
    """A compute-heavy hierarchy for the tier-band model: GUE H / sqrt(ns), Q = diag(linspace(-1, 1)), one Drude bath
    (npsd Pade terms), rho0 = |0><0|."""
    import sympy as sp
    from pyqed_amd.deom import Bath, DEOMSolver
    w = sp.symbols(r"\omega", real=True)
    bath3 = Bath([2 * 0.3 * w / (1.0 + w ** 2)], w, [1.0], [npsd], [0] * (npsd + 1))
    rng = np.random.default_rng(ns)
    a = rng.standard_normal((ns, ns)) + 1j * rng.standard_normal((ns, ns))
    H = (a + a.conj().T) / 2 / np.sqrt(ns)
    Q = np.diag(np.linspace(-1, 1, ns)).astype(complex)
    rb = np.zeros((ns, ns), complex)
    rb[0, 0] = 1
    return (f"ns{ns}_L{L}_K{npsd + 1}", DEOMSolver(H, None, bath3, np.array([Q]), None, None, None, L), rb, 0.002)


def _deom_banded_cases():
    """(name, solver, rho0, dt) of the tier-banded leg: BASELINE.json configs[3] (spin-boson, ns = 2, L = 12, K = 5,
    6188 ADOs) and two compute-heavy hierarchies whose per-ADO work is ns^3 (_band_case: ns = 96 and 128, L = 8, K = 4:
    495 ADOs, 70 / 124 MB) -- the tiled MFMA stage kernel.  tools/deom_band_model.py runs the model on others."""
    import sympy as sp
    from pyqed_amd.deom import Bath, DEOMSolver
    w = sp.symbols(r"\omega", real=True)
    sx = np.array([[0, 1], [1, 0]], complex)
    sz = np.diag([1.0, -1.0]).astype(complex)
    r0 = np.zeros((2, 2), complex)
    r0[0, 0] = 1
    bath = Bath([2 * 0.5 * 1.0 * w / (1.0 + w ** 2)], w, [1.0], [4], [0] * 5)
    cases = [("spin_boson_L12_K5 (configs[3])", DEOMSolver(sz + sx, None, bath, np.array([sx]), None, None, None, 12),
              r0, 0.002)]
    for ns, L in ((96, 8), (128, 8)):
        cases.append(_band_case(ns, L))
    return cases


XGMI_LINK_GBS = 153.0     # one xGMI link per direction (MI355X: 7 links per GPU), the band model's transfer rate
RCCL_LATENCY_US = 10.0    # assumed per-exchange latency floor of a small RCCL send / recv or all-gather over xGMI


def deom_band_model(dev, sh, single_ms, reps=24):
    """Per-band model of one hierarchy tier-banded over len(sh.plans) GPUs, from quantities one
    GPU can measure: each band's RK4 stage timed ALONE (qd_deom_stage on its own rows, HIP events, `reps` stages),
    and the bytes each band receives per stage.  Per stage the bands run concurrently, then exchange halos:
        T_stage = max_b t_stage(b) + max_b max_q bytes(q -> b) / XGMI_LINK_GBS + latency
    (point-to-point: every peer arrives over its own link, so the largest single transfer bounds the exchange; the
    all-gather variant moves (n - 1) export sets over one ring link), four exchanges per RK4 step.  The projected
    speed-up is the unbanded one-GPU step time over 4 T_stage; latency = 0 and RCCL_LATENCY_US bracket it."""
    import torch
    ns = sh.solver.nsys
    row = ns * ns * 16
    stream = torch.cuda.current_stream(dev)
    t_band = []
    for b in sh.bands:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for k in range(4):
            b.stage(k, 0, 1e-6, 0j, 0j)
        e0.record(stream)
        for k in range(reps):
            b.stage(k % 4, 0, 1e-6, 0j, 0j)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        t_band.append(e0.elapsed_time(e1) / reps * 1e-3)
    recv_peer = [max([c for (_, c) in p.recv.values()] or [0]) * row for p in sh.plans]
    recv_tot = [len(p.halo) * row for p in sh.plans]
    export = max(len(np.unique(np.concatenate(list(p.send.values())))) if p.send else 0 for p in sh.plans) * row
    n = len(sh.plans)
    link = XGMI_LINK_GBS * 1e9
    comp = max(t_band)
    p2p = max(recv_peer) / link
    ring = (n - 1) * export / link
    out = {"bands": n, "band_stage_us": [round(t * 1e6, 2) for t in t_band],
           "max_band_stage_us": round(comp * 1e6, 2),
           "halo_bytes_per_stage_max": max(recv_tot), "largest_peer_transfer_bytes": max(recv_peer),
           "allgather_export_bytes": export, "xgmi_link_GBs": XGMI_LINK_GBS, "latency_us_assumed": RCCL_LATENCY_US,
           "one_gpu_unbanded_ms_per_step": round(single_ms, 4)}
    for tag, xfer in (("p2p", p2p), ("allgather", ring)):
        for lat in (0.0, RCCL_LATENCY_US * 1e-6):
            step = 4 * (comp + xfer + lat)
            key = f"{tag}_{'lat' if lat else 'nolat'}"
            out[key] = {"ms_per_step": round(step * 1e3, 4), "speedup": round(single_ms / (step * 1e3), 3)}
    return out


def bench_deom_banded(dev, world, rank, steps=40, cases=None):
    """ONE hierarchy tier-banded over the ranks (BASELINE.json configs[3]: "ADOs sharded over
    8xMI355X via xGMI"): one band per rank, one RCCL all-gather of the bands' export rows per RK4 stage
    (deom_shard.CollectiveExchange), HIP stage kernels per band.  World > 1: timed `steps` RK4 steps of
    device-resident bands between barriers + device syncs, max over ranks.  World 1: the 8-band per-band model
    (deom_band_model: each band's stage timed alone, halo bytes over one xGMI link, four exchanges per step) against the
    unbanded qd_deom_rk4 rate of the same hierarchy, plus the loopback run of all 8 bands on this GPU (serialised
    bands and device-copy exchanges: the correctness harness's cost, not a multi-GPU time)."""
    import torch
    import torch.distributed as dist
    from pyqed_amd.deom_shard import ShardedDEOM, run_bands
    out = {}
    for name, sol, rho0, dt in (cases if cases is not None else _deom_banded_cases()):
        sol.check_()
        sol.init_()
        single = None
        if rank == 0:   # the unbanded kernel sequence on this GPU, device-resident state, HIP events
            Qm = np.asarray(sol.coupling, dtype=complex).reshape(-1, sol.nsys, sol.nsys)
            single = 1e3 / _deom_event_rate(dev, sol, sol.bath, np.asarray(sol.system, complex), Qm, 1, steps, dt)
        nb = world if world > 1 else 8
        # compute-heavy hierarchies exchange point to point (each peer's rows over its own link: the model's p2p
        # form); the small-state bench hierarchy with one all-gather per stage
        exch = "p2p" if sol.nsys >= 32 else "allgather"
        sh = ShardedDEOM(sol, nbands=nb, loopback=world == 1, device=dev, exchange=exch)
        fs, fc = sh.setup(dt, steps)
        run_bands(sh.bands, sh.exchange, rho0, dt, 2, fs, fc)          # warm-up
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        run_bands(sh.bands, sh.exchange, rho0, dt, steps, fs, fc)
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        ns = sol.nsys
        halo = [len(p.halo) for p in sh.plans]
        own = [p.n_own for p in sh.plans]
        ent = {"nmax": sol.nmax, "ns": ns, "K": sol.nind, "L": sol.lmax, "bands": nb,
               "max_halo_over_owned": round(max(h / o for h, o in zip(halo, own)), 3),
               "state_bytes": sol.nmax * ns * ns * 16}
        if world > 1:
            ent.update({"exchange": ("RCCL all-gather per stage" if exch == "allgather" else
                                     "RCCL point-to-point halo exchange per stage"),
                        "ms_per_step": round(el / steps * 1e3, 4),
                        "steps": steps, "ado_steps_per_s": round(sol.nmax * steps / el, 1)})
            if exch == "allgather":
                ent["allgather_bytes_per_stage"] = sh.exchange.bytes_per_exchange
            if single is not None:
                ent["one_gpu_unbanded_ms_per_step"] = round(single, 4)
        else:
            ent["loopback_ms_per_step"] = round(el / steps * 1e3, 4)
            ent["loopback_note"] = "8 bands serialised on one GPU with device-copy exchanges (correctness harness)"
            ent["model_8gpu"] = deom_band_model(dev, sh, single)
        out[name] = ent
    return out


def bench_deom_corr4(dev, nw=32, T=0.5):
    """DEOMSolver.correlation_4op_3t at the bench hierarchy (L = 12, K = 5, n = nmax ns^2 = 24,752; SURVEY §8(f)
    rank 2) on an nw x nw (w_x, w_y) grid, signature 'lccc': the Krylov form (pyqed_amd/deom_krylov.py: multi-shift
    Krylov solves of P and P^T on the stencil kernel, Taylor-substep e^{PT}), wall clock of the whole call after a
    warm-up call.  The reference's eigen form would diagonalise the 9.8 GB dense P (O(n^3) ~ 6e13 flop on the host):
    not run, so there is no CPU baseline for this leg."""
    import torch
    import sympy as sp
    from pyqed_amd.deom import Bath, DEOMSolver
    w = sp.symbols(r"\omega", real=True)
    bath = Bath([2 * 0.5 * w / (1.0 + w ** 2)], w, [1.0], [4], [0] * 5)
    sx = np.array([[0, 1], [1, 0]], complex)
    sz = np.diag([1.0, -1.0]).astype(complex)
    sol = DEOMSolver(sz + sx, None, bath, np.array([sx]), None, None, None, 12)
    rho0 = np.array([[1, 0], [0, 0]], complex)
    wx = np.linspace(-4.1, 4.3, nw)   # grids clear of w = 0 (the steady-state pole)
    wy = np.linspace(-3.7, 4.9, nw)
    sol.correlation_4op_3t(sz, sx, sx, sz, rho0, T, wx[:4], wy[:4], lcr="lccc")   # warm-up (tables, kernels)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    c = sol.correlation_4op_3t(sz, sx, sx, sz, rho0, T, wx, wy, lcr="lccc")
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    assert np.all(np.isfinite(c))
    info = {k: v for k, v in sol.last_corr4.items() if k != "method"}
    res = {"value": round(nw * nw / el, 2), "unit": "(w_x, w_y) points/s (one correlation_4op_3t call, L=12 K=5)",
           "seconds": round(el, 3), "grid": [nw, nw], "T": T, "method": sol.last_corr4["method"], **info,
           "note": "eigen form of the reference (eig of the 24,752^2 P) not run: no CPU baseline"}
    if "stencil_vector_applications" in info:
        # the stencil kernel's roofline over the call -- algorithmic bytes per vector application
        # (read x, write y: 2 n 16 B) plus the tables once per launch (coef 3K, damp, minus / plus per ADO), over the
        # call's wall time (so a lower bound: the call also runs the Arnoldi basis passes, the small solves and the
        # host checkpoints); and the Arnoldi orthogonalisation's own traffic for the record: the j + 1 basis vectors read
        # twice per step by the delayed CGS2 (deom_krylov.ARNOLDI_DCGS2), four times by the plain CGS2 loop
        from pyqed_amd import deom_krylov
        nmax, K, n = sol.nmax, sol.nind, sol.nmax * 4
        per_vec = 2 * n * 16
        per_launch = nmax * (3 * K * 16 + 16 + 2 * K * 4)
        stencil = info["stencil_vector_applications"] * per_vec + info["stencil_launches"] * per_launch
        kr, kl = info.get("krylov_dim_right", 0), info.get("krylov_dim_left", 0)
        passes = 2 if deom_krylov.ARNOLDI_DCGS2 else 4
        cgs2 = sum(passes * k * (k + 1) // 2 * n * 16 for k in (kr, kl))
        res["roofline"] = {"bound": "hbm", "kernel": "qd_deom_apply (stencil)",
                           "achieved": round(stencil / el / 1e9, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": round(stencil / el / 1e9 / HBM_PEAK_GBS, 4),
                           "bytes_per_vector_application": per_vec, "table_bytes_per_launch": per_launch,
                           "arnoldi_basis_bytes": cgs2, "arnoldi_basis_passes_per_step": passes,
                           "note": "stencil algorithmic bytes / the whole call's wall time: the call is bound by its "
                                   "thousands of dependent small launches (Arnoldi steps, Taylor terms), not by HBM"}
    return res


def cpu_baseline_deom(budget_s=8.0):
    import sympy as sp
    from oracle import deom as od
    from pyqed_amd.deom import Bath
    w = sp.symbols(r"\omega", real=True)
    bath = Bath([2 * 0.5 * 1.0 * w / (1.0 + w ** 2)], w, [1.0], [4], [0] * 5)
    sx = np.array([[0, 1], [1, 0]], complex)
    sz = np.diag([1.0, -1.0]).astype(complex)
    rho0 = np.zeros((2, 2), complex)
    rho0[0, 0] = 1
    t0 = time.perf_counter()
    od.run(sz + sx, np.zeros((2, 2)), lambda t: 0, np.array([sx]), np.zeros((1, 2, 2)), lambda t: 0,
           (bath.etal, bath.etar, bath.etaa, bath.expn), 12, rho0, 0.01, 1)
    el = time.perf_counter() - t0
    return {"value": round(1 / el, 4), "unit": "RK4 steps/s", "cores": 1, "kind": "port",
            "sample": f"1 RK4 step of the NumPy restatement of DEOMSolver.run at L=12, K=5 in {el:.1f}s"}


_T0 = time.perf_counter()


def progress(msg):
    """One line per leg on stderr (stdout carries only the JSON line): long runs under a profiler show activity."""
    print(f"[bench {time.perf_counter() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)
    maps = os.environ.get("BENCH_MAPS")   # diagnostics: the process's library map, to resolve a crash's frames
    if maps:
        try:
            with open("/proc/self/maps") as fi, open(maps, "w") as fo:
                fo.write(fi.read())
        except OSError:
            pass


def write_detail(out, path):
    """Every leg's full record (per-leg configs, notes, PMC traffic, cpu_baseline samples) goes to a side file; the
    stdout line carries the compact summary (the driver keeps only the tail of stdout)."""
    if not path:
        path = os.path.join(ROOT, "gpurun_out", "bench_detail.json")
    try:
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
        return os.path.relpath(path, ROOT)
    except OSError as e:
        return f"not written ({e})"


def _pick(d, *keys):
    return {k: d[k] for k in keys if isinstance(d, dict) and k in d}


def _roof(r):
    return _pick(r, "bound", "kernel", "achieved", "peak", "unit", "frac", "traffic")


def _cpu(c):
    return _pick(c, "value", "unit", "cores", "kind", "sample") if isinstance(c, dict) else None


def compact_line(out, detail):
    """The one JSON line of the contract: the headline (Lindblad N = 128) with its roofline and cpu_baseline, then
    the 2DES half of BASELINE's metric, then one short entry per secondary leg; `detail` names the side file."""
    line = {k: out[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "timing",
                                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config") if k in out}
    sec = out.get("secondary", {})
    tw = sec.get("2des")
    if isinstance(tw, dict) and "error" not in tw:
        t = _pick(tw, "value", "unit", "ms_per_grid")
        t["members"] = tw["config"]["ensemble_members"]
        t["grid"] = tw["config"]["grid"]
        t["roofline"] = _roof(tw["roofline"])
        if "cpu_baseline" in tw:
            t["cpu_baseline"] = _cpu(tw["cpu_baseline"])
        if "shard_1of8" in tw:
            sh = tw["shard_1of8"]
            t["shard_1of8"] = {"members": sh["members"], "ms_per_grid": sh["ms_per_grid"],
                               "frac": sh["roofline"]["frac"],
                               "projected_8gpu_speedup_compute_only": sh["projected_8gpu_speedup_compute_only"],
                               "projected_8gpu_speedup_reduce_serial": sh.get("projected_8gpu_speedup_reduce_serial")}
        if isinstance(tw.get("t2scan"), dict):
            ts = tw["t2scan"]
            t["t2scan"] = {"value": ts["value"], "n_t2": ts["config"]["n_t2"], "ms_per_scan": ts["ms_per_scan"],
                           "frac": ts["roofline"]["frac"]}
        line["twodes"] = t
    r = out["roofline"]
    line["roofline"] = dict(_roof(r), flop_per_dm_step=r["flop_per_dm_step"], nominal_frac=r["nominal_frac"],
                            launch_ms=r["launch_ms"])
    if "cpu_baseline" in out:
        line["cpu_baseline"] = _cpu(out["cpu_baseline"])
    line["batch_sweep"] = {b: {"dm_steps_per_s": v["dm_steps_per_s"], "frac": v["roofline"]["frac"]}
                           for b, v in out.get("batch_sweep", {}).items()}
    s2 = {}
    for name, leg in sec.items():
        if name == "2des":
            continue
        if not isinstance(leg, dict) or "error" in leg:
            s2[name] = leg if isinstance(leg, dict) else None
            continue
        if name == "deom_banded":
            s2[name] = {}
            for k, v in leg.items():
                e = _pick(v, "nmax", "bands", "ms_per_step")
                m = v.get("model_8gpu")
                if isinstance(m, dict):
                    e["model_8gpu_speedup"] = {"p2p": m["p2p_lat"]["speedup"], "p2p_nolat": m["p2p_nolat"]["speedup"]}
                s2[name][k] = e
            continue
        e = _pick(leg, "value", "unit")
        if "roofline" in leg:
            e["frac"] = leg["roofline"]["frac"]
        if isinstance(leg.get("cpu_baseline"), dict):
            e["cpu"] = leg["cpu_baseline"].get("value")
        b = leg.get("batched")
        if isinstance(b, dict):
            e["batched"] = {k: b[k] for k in ("hierarchies", "wavepackets", "batch", "ado_steps_per_s",
                                              "wavepacket_steps_per_s", "dm_steps_per_s") if k in b}
            if "roofline" in b:
                e["batched"]["frac"] = b["roofline"]["frac"]
        if isinstance(leg.get("stretch_npsd5"), dict):
            e["stretch_steps_per_s"] = leg["stretch_npsd5"]["steps_per_s"]
        s2[name] = e
    line["secondary"] = s2
    line["detail"] = detail
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256, help="density matrices per GPU")
    ap.add_argument("--N", type=int, default=128)
    ap.add_argument("--nc", type=int, default=1)
    ap.add_argument("--dt", type=float, default=1e-3)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--general", action="store_true",
                    help="force the general (non-Hermitian) GLF kernel instead of the Hermitian one")
    ap.add_argument("--ens", type=int, default=65536,
                    help="2DES disorder-ensemble members (total; strong scaling: enough work to split 8 ways; "
                         "65,536 leaves each of 8 ranks 8,192 members, 0.2 ms per grid)")
    ap.add_argument("--ens-reps", type=int, default=50)   # >= 8 ms timed even for an 8-way shard
    ap.add_argument("--no-2des", action="store_true")
    ap.add_argument("--t2", type=int, default=16, help="2DES waiting times per scan (0 = skip the scan leg)")
    ap.add_argument("--t2-reps", type=int, default=3)
    ap.add_argument("--spo-steps", type=int, default=1000)
    ap.add_argument("--no-spo", action="store_true")
    ap.add_argument("--no-spo3", action="store_true")
    ap.add_argument("--deom-steps", type=int, default=200)
    ap.add_argument("--deom-batch", type=int, default=64)
    ap.add_argument("--no-deom", action="store_true")
    ap.add_argument("--no-deom-banded", action="store_true", help="skip the tier-banded DEOM leg")
    ap.add_argument("--no-deom-corr4", action="store_true", help="skip the bench-hierarchy correlation_4op_3t leg")
    ap.add_argument("--deom-banded-ranks", action="store_true",
                    help="world > 1: also run ONE hierarchy tier-banded over the ranks (RCCL all-gather per stage)")
    ap.add_argument("--no-redfield", action="store_true")
    ap.add_argument("--no-reduce", action="store_true",
                    help="skip the one-rank RCCL reduce timing of the 2DES projection (its communicator init crashes "
                         "under rocprofv3 --pmc)")
    ap.add_argument("--no-superop", action="store_true")
    ap.add_argument("--detail", default=None,
                    help="side file for every leg's full record (default gpurun_out/bench_detail.json)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from pyqed_amd import lindblad_rk4

    N, nc, B = args.N, args.nc, args.batch
    H, cs = synthetic_lindblad(N, nc=nc)
    rho0 = random_pure_states(B, N, seed=2 + rank)
    Ht = torch.from_numpy(H).to(dev)
    Ct = torch.from_numpy(np.array(cs)).to(dev) if nc else None
    rho = torch.from_numpy(rho0).to(dev)

    herm = not args.general and N <= 128  # pure states are exactly Hermitian
    kname = f"lindblad_rk4_kernel<{min(128, N)},{'herm' if herm else 'general'}>"

    stream = torch.cuda.current_stream(dev)
    # smaller batches (B in {1, 64, 256}), event-timed on the launch stream, BEFORE the headline's
    # warm-up: the GPU leaves idle clocks over tens of ms (tools/lindblad_launch_overhead.py: a 20-step launch after
    # 20 ms idle runs 0.825 ms per step against 0.726 queued behind other work), and a 5-step warm-up alone does not
    # cover that ramp, so real work of this leg runs first and the headline is timed at the clocks a running job has
    # (profiles/r04/lindblad/launch_overhead.txt).  The auto dispatch runs B = 64 (Hermitian states, 16 <= B < 192) on
    # the Hermitian pair-block split path and B = 1 as one single-trajectory launch; each entry's flops are its own
    # path's (Hermitian GLF form / general GLF form)
    from pyqed_amd import _lib
    from pyqed_amd.oqs import HERM_SPLIT_MIN_BATCH
    batch_sweep = {}
    # untimed: ~30 ms of B = 64 work first, so that neither timed leg runs through the idle-clock ramp (the B = 1 leg
    # measured 47.x k steps/s as the first work of the process against 49.7k behind other work)
    lindblad_rk4(Ht, Ct, rho[:64].clone(), args.dt, 100, hermitian=False if args.general else None)
    torch.cuda.synchronize(dev)
    for Bs in (1, 64):
        rs = rho[:Bs].clone()
        _lib.take_path()
        lindblad_rk4(Ht, Ct, rs, args.dt, 2, hermitian=False if args.general else None)
        torch.cuda.synchronize(dev)
        taken = _lib.take_path()
        # B = 1 of Hermitian states runs the Hermitian single launch (glf_single_herm_kernel), B = 64 the Hermitian
        # pair-block split path: both execute the Hermitian form's flops
        hsingle = "glf_single_herm" in taken
        hs = hsingle or (Bs >= HERM_SPLIT_MIN_BATCH and not args.general and N <= 128)
        ss = 300   # ~90 ms of B = 64 work: a measured leg that also carries the GPU out of idle clocks
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        lindblad_rk4(Ht, Ct, rs, args.dt, ss, hermitian=False if args.general else None)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        sec = e0.elapsed_time(e1) / 1e3
        fl = lindblad_executed_flops_per_step(N, nc, True) if hsingle else lindblad_flops_per_step(N, nc, hs)
        tf = fl * Bs * ss / sec / 1e12
        batch_sweep[str(Bs)] = {
            "dm_steps_per_s": round(Bs * ss / sec, 1), "us_per_step": round(sec / ss * 1e6, 2),
            "path": ("Hermitian single-trajectory launch (glf_single_herm_kernel, executed Hermitian-form flops)"
                     if hsingle else "Hermitian pair-block split (glf_split_hk)" if hs else
                     "single-trajectory tile launch (glf_single_kernel)" if Bs == 1 and N in (32, 64, 128) and nc <= 2
                     else "glf split-K (general kernel)"),
            "paths_taken": taken,
            "roofline": {"bound": "mfma", "achieved": round(tf, 3), "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(tf / FP64_MFMA_PEAK_TFLOPS, 4), "flop_per_dm_step": fl,
                         "traffic": (measured_traffic("glf_single_herm_kernel<1,true>_b1" if hsingle else
                                                      "glf_single_kernel<4,1,true,true>_b1", ss)
                                     if (Bs, N, nc) == (1, 128, 1) else None)}}
    single_rate = batch_sweep["1"]["dm_steps_per_s"]

    progress("lindblad batch sweep done")

    # warm-up
    lindblad_rk4(Ht, Ct, rho, args.dt, args.warmup, hermitian=herm)
    torch.cuda.synchronize(dev)

    # the headline is the MEDIAN of HEADLINE_REPS timed regions, each EXACTLY args.steps steps of the
    # whole batch bracketed by a barrier + torch.cuda.synchronize() on both sides, each rep's time the max over ranks
    # (the reps continue the same trajectories: every rep is the same work, steps args.steps * k .. * (k + 1))
    samples, kern_samples = [], []
    for _ in range(HEADLINE_REPS):
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        ev0.record(stream)
        lindblad_rk4(Ht, Ct, rho, args.dt, args.steps, hermitian=herm)
        ev1.record(stream)
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
        if world > 1:
            dist.barrier()
        t = torch.tensor([wall], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        samples.append(float(t.item()))
        kern_samples.append(ev0.elapsed_time(ev1) / 1e3)
    wall_max = float(np.median(samples))
    kern_s = float(np.median(kern_samples))

    # sanity: trace preserved (cheap, outside the timed region)
    tr = torch.diagonal(rho, dim1=1, dim2=2).sum(-1)
    tr_err = float((tr - 1).abs().max().item())

    progress("lindblad headline leg done")
    twodes = None
    if not args.no_2des:
        twodes, sig, ens_in = bench_2des(dev, world, rank, args.ens, args.ens_reps)
        if rank == 0:
            twodes["signal_abs_max"] = float(sig.abs().max().item())
        if world == 1 and args.ens >= 8:
            # the 8-GPU expectation from one GPU: an 8-way member shard timed alone (its reduce is pipelined
            # behind the next grid's compute at N > 1, so the shard's compute bounds the per-grid time)
            shard, _, _ = bench_2des(dev, 1, 0, args.ens // 8, args.ens_reps)
            # reduce model: the 1 MiB grid over ONE 153 GB/s xGMI link; pipelined behind the next
            # grid's compute it is hidden (the compute-only figure), serialised it adds to every grid
            red_ms = 256 * 256 * 16 / XGMI_LINK_GBS / 1e6
            twodes["shard_1of8"] = {
                "members": args.ens // 8, "ms_per_grid": shard["ms_per_grid"],
                "event_ms_per_grid": shard["event_ms_per_grid"], "roofline": shard["roofline"],
                "projected_8gpu_speedup_compute_only": round(twodes["ms_per_grid"] / shard["ms_per_grid"], 3),
                "projected_8gpu_speedup_reduce_serial": round(twodes["ms_per_grid"] / (shard["ms_per_grid"] + red_ms),
                                                              3),
                "reduce_model_ms": round(red_ms, 4),
                "reduce_model": "1 MiB reduce(sum) to rank 0 over one 153 GB/s xGMI link per grid: hidden when "
                                "pipelined behind the next grid (compute_only), added when serialised (reduce_serial)"}
            # (round 3 also printed a "serial reduce" projection from a 1 MiB reduce on a ONE-rank communicator: that
            # moves no bytes over xGMI, so it priced nothing and is gone; the driver's 8-GPU run measures the reduce)
            if not args.no_reduce:
                try:
                    twodes["shard_1of8"]["one_rank_reduce_launch_ms"] = round(time_reduce_one_rank(dev), 4)
                    twodes["shard_1of8"]["one_rank_reduce_note"] = ("1 MiB ncclReduce on a one-rank communicator: RCCL "
                                                                    "launch cost only, no xGMI transfer")
                except Exception as e:  # noqa: BLE001 (informational)
                    twodes["shard_1of8"]["reduce_error"] = f"{type(e).__name__}: {e}"
        if args.t2 > 0:
            twodes["t2scan"] = bench_2des_t2scan(dev, world, rank, args.ens, args.t2, args.t2_reps)

    # the remaining legs run no collective: a failure in one is reported in its place (stderr + an "error" entry)
    # and cannot take the primary line or another rank down with it
    def guarded(fn, *a):
        try:
            return fn(*a)
        except Exception as e:  # noqa: BLE001
            import traceback
            traceback.print_exc()
            return {"error": f"{type(e).__name__}: {e}"}

    def pair(r):
        return r if isinstance(r, tuple) else (r, None)

    progress("2des legs done")
    redfield = None
    if not args.no_redfield:
        redfield, rf_sol = pair(guarded(bench_redfield, dev, args.steps, B))

    progress("redfield leg done")
    superop = None
    if not args.no_superop:
        superop, so_in = pair(guarded(bench_superop, dev))

    progress("superop leg done")
    spo = None
    if not args.no_spo:
        spo = guarded(bench_spo2, dev, args.spo_steps)

    progress("spo2 leg done")
    spo3 = None
    if not args.no_spo3:
        spo3 = guarded(bench_spo3, dev)

    progress("spo3 leg done")
    deom = None
    if not args.no_deom:
        deom = guarded(bench_deom, dev, args.deom_steps, args.deom_batch)

    # one hierarchy tier-banded over the ranks (collective: every rank takes part; world 1: 8-band loopback)
    # At world > 1 it is opt-in (--deom-banded-ranks): a collective leg cannot be guarded per rank (one rank's
    # exception would leave the others waiting in the all-gather), and the halo is 2.5x the owned rows at 8 bands, so
    # it is a capacity tool, not a speed-up, for the bench hierarchy.  World 1 runs the 8-band loopback.
    progress("deom leg done")
    deom_corr4 = None
    if world == 1 and not args.no_deom and not args.no_deom_corr4:
        deom_corr4 = guarded(bench_deom_corr4, dev)
        progress("deom corr4 leg done")
    deom_banded = None
    if not args.no_deom and not args.no_deom_banded:
        if world > 1:
            if args.deom_banded_ranks:
                deom_banded = bench_deom_banded(dev, world, rank)
        else:
            deom_banded = guarded(bench_deom_banded, dev, world, rank)

    if rank == 0:
        total_dm_steps = B * args.steps * world
        value = total_dm_steps / wall_max
        # the headline roofline counts the flops the kernel EXECUTES: the Hermitian kernel skips
        # the redundant (C r)C^+ tiles below the diagonal, so its executed count (1 + n_c + 36/64 n_c GEMMs per RHS)
        # is the algorithm's minimum for the Hermitian GLF form; the nominal Hermitian-form count is a side key
        flops = lindblad_executed_flops_per_step(N, nc, herm) * B * args.steps
        achieved = flops / kern_s / 1e12
        nominal = lindblad_flops_per_step(N, nc, herm) * B * args.steps / kern_s / 1e12
        out = {
            "metric": "density-matrix steps/sec (N=128 Lindblad) + 2DES grid-points/sec at 1/2/4/8 GPU",
            "value": round(value, 3),
            "unit": "density-matrix steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall_max / args.steps * 1e3, 4),
            "timing": {"reps": HEADLINE_REPS, "statistic": "median over reps of (max over ranks of the wall time of "
                                                           "one timed region of exactly `steps` steps)",
                       "ms_per_step_samples": [round(x / args.steps * 1e3, 4) for x in samples]},
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "c128",
            "data": "synthetic (seeded GUE H, Ginibre collapse op, random pure states)",
            "config": {
                "workload": "lindblad_n128_rk4_fp64 (BASELINE.json configs[1])",
                "N": N, "n_c_ops": nc, "batch_per_gpu": B, "global_batch": B * world, "dt": args.dt,
                "parallelism": f"replicas x{world} (independent density matrices per rank, no collective)",
            },
            "roofline": {
                "bound": "mfma",
                "kernel": kname,
                "kernel_symbol": (f"qd::lindblad_rk4_kernel<{min(128, N)}, {'true, true' if herm else 'false, false'}>"
                                  " (rocprofv3 name)"),
                "achieved": round(achieved, 3),
                "peak": FP64_MFMA_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(achieved / FP64_MFMA_PEAK_TFLOPS, 4),
                "traffic": measured_traffic(kname, B * args.steps)
                if (N, nc) == (128, 1) else None,
                "traffic_unit": "HBM bytes per launch (PMC FETCH_SIZE+WRITE_SIZE, calibrated; profiles/pmc_traffic.json)",
                "flop_per_dm_step": lindblad_executed_flops_per_step(N, nc, herm),
                "flop_note": "achieved / frac count the executed MFMA work per DM-step (flop_per_dm_step; the "
                             "Hermitian kernel skips the 28 redundant 16 x 16 tiles of each (C r)C^+ below the "
                             "diagonal, confirmed by the F64 MFMA op counters in profiles/); nominal_* count the "
                             "Hermitian GLF form 4 x (1 + 2 n_c) x 8 N^3",
                "nominal_flop_per_dm_step": lindblad_flops_per_step(N, nc, herm),
                "nominal_tflops": round(nominal, 3),
                "nominal_frac": round(nominal / FP64_MFMA_PEAK_TFLOPS, 4),
                "general_path_equiv_tflops": round(lindblad_flops_per_step(N, nc) * B * args.steps / kern_s / 1e12, 3),
                "launch_ms": round(kern_s * 1e3, 3),
                "launch_ms_samples": [round(x * 1e3, 3) for x in kern_samples],
            },
            "single_trajectory_steps_per_s": round(single_rate, 2),
            "batch_sweep": batch_sweep,
            "trace_err": tr_err,
        }
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline(N, nc, args.dt)
        if twodes is not None:
            if world == 1 and not args.no_cpu:
                twodes["cpu_baseline"] = cpu_baseline_2des(*ens_in)
            out.setdefault("secondary", {})["2des"] = twodes
        if redfield is not None:
            if world == 1 and not args.no_cpu and "error" not in redfield:
                redfield["cpu_baseline"] = cpu_baseline_redfield(rf_sol)
            out.setdefault("secondary", {})["redfield"] = redfield
        if superop is not None:
            if world == 1 and not args.no_cpu and "error" not in superop:
                superop["cpu_baseline"] = cpu_baseline_superop(*so_in)
            out.setdefault("secondary", {})["superop"] = superop
        if spo is not None:
            if world == 1 and not args.no_cpu and "error" not in spo:
                spo["cpu_baseline"] = cpu_baseline_spo2()
            out.setdefault("secondary", {})["spo2"] = spo
        if spo3 is not None:
            if world == 1 and not args.no_cpu and "error" not in spo3:
                spo3["cpu_baseline"] = cpu_baseline_spo3()
            out.setdefault("secondary", {})["spo3"] = spo3
        if deom is not None:
            if world == 1 and not args.no_cpu and "error" not in deom:
                deom["cpu_baseline"] = cpu_baseline_deom()
            out.setdefault("secondary", {})["deom"] = deom
        if deom_corr4 is not None:
            out.setdefault("secondary", {})["deom_corr4"] = deom_corr4
        if deom_banded is not None:
            out.setdefault("secondary", {})["deom_banded"] = deom_banded
        detail = write_detail(out, args.detail)
        print(json.dumps(compact_line(out, detail)), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
