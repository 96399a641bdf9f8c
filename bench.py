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

FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X dense FP64 matrix peak (spec)
HBM_PEAK_GBS = 8000.0


def lindblad_flops_per_step(N: int, nc: int) -> float:
    # 4 RK4 stages x (2 + 2*nc) complex N^3 GEMMs x 8 real flop per complex MAC
    return 4.0 * (2 + 2 * nc) * 8.0 * N ** 3


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

    from oracle import lindblad as olb  # input synthesis only (seeded); compute is libqdyn
    from pyqed_amd import lindblad_rk4

    N, nc, B = args.N, args.nc, args.batch
    H, cs = olb.synthetic_lindblad(N, nc=nc)
    rho0 = olb.random_pure_states(B, N, seed=2 + rank)
    Ht = torch.from_numpy(H).to(dev)
    Ct = torch.from_numpy(np.array(cs)).to(dev) if nc else None
    rho = torch.from_numpy(rho0).to(dev)

    # warm-up
    lindblad_rk4(Ht, Ct, rho, args.dt, args.warmup)
    torch.cuda.synchronize(dev)

    stream = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    lindblad_rk4(Ht, Ct, rho, args.dt, args.steps)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    kern_s = ev0.elapsed_time(ev1) / 1e3

    t = torch.tensor([wall], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall_max = float(t.item())

    # sanity: trace preserved (cheap, outside the timed region)
    tr = torch.diagonal(rho, dim1=1, dim2=2).sum(-1)
    tr_err = float((tr - 1).abs().max().item())

    # single-trajectory latency (B=1), informational
    r1 = rho[:1].clone()
    lindblad_rk4(Ht, Ct, r1, args.dt, 2)
    torch.cuda.synchronize(dev)
    s1 = 20
    ta = time.perf_counter()
    lindblad_rk4(Ht, Ct, r1, args.dt, s1)
    torch.cuda.synchronize(dev)
    single_rate = s1 / (time.perf_counter() - ta)

    if rank == 0:
        total_dm_steps = B * args.steps * world
        value = total_dm_steps / wall_max
        flops = lindblad_flops_per_step(N, nc) * B * args.steps
        achieved = flops / kern_s / 1e12
        out = {
            "metric": "density-matrix steps/sec (N=128 Lindblad) + 2DES grid-points/sec at 1/2/4/8 GPU",
            "value": round(value, 3),
            "unit": "density-matrix steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall_max / args.steps * 1e3, 4),
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
                "kernel": "lindblad_rk4_kernel<128>",
                "achieved": round(achieved, 3),
                "peak": FP64_MFMA_PEAK_TFLOPS,
                "unit": "TFLOP/s",
                "frac": round(achieved / FP64_MFMA_PEAK_TFLOPS, 4),
                "traffic": None,
                "flop_per_dm_step": lindblad_flops_per_step(N, nc),
                "launch_ms": round(kern_s * 1e3, 3),
            },
            "single_trajectory_steps_per_s": round(single_rate, 2),
            "trace_err": tr_err,
        }
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline(N, nc, args.dt)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
