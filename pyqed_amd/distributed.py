"""Multi-GPU helpers: one process per GPU, torch.distributed (backend "nccl" = RCCL on ROCm).

The hot path shards only where units are independent:
  * 2DES disorder ensemble: members split into contiguous ranges, each rank evaluates its
    partial (t3, t1) grid, ONE reduce(sum) of the 1 MiB grid to rank 0 (strong scaling); a sequence of
    grids pipelines those reduces behind the next grid's compute (ReducePipeline);
    a waiting-time scan reduces its [n2, n3, n1] stack in buckets, each bucket's reduce overlapped
    with the next bucket's compute (sharded_sum_buckets);
  * Lindblad / DEOM / SPO batches: independent replicas per rank, no collective.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_range(n: int, rank: int, world_size: int) -> tuple[int, int]:
    """Contiguous, balanced [lo, hi) slice of n units for `rank` (sizes differ by at most 1)."""
    if n < 0 or world_size < 1 or not (0 <= rank < world_size):
        raise ValueError(f"bad shard request n={n} rank={rank} world={world_size}")
    return n * rank // world_size, n * (rank + 1) // world_size


def _real_view(t: torch.Tensor) -> torch.Tensor:
    """Collectives run on the real view of complex buffers (same storage): dist.reduce, unlike all_reduce,
    does not convert complex tensors itself, and RCCL has no complex datatype."""
    return torch.view_as_real(t) if t.is_complex() else t


def sharded_sum(local_fn, n_units: int, dst: int | None = 0, group=None) -> torch.Tensor:
    """Evaluate local_fn(lo, hi) -> tensor on this rank's shard of n_units and sum over ranks with one
    collective: reduce to `dst` (dst=None: all_reduce).  Single process: local_fn(0, n_units)."""
    rank, ws = world()
    lo, hi = shard_range(n_units, rank, ws)
    out = local_fn(lo, hi)
    if ws > 1:
        if dst is None:
            dist.all_reduce(_real_view(out), op=dist.ReduceOp.SUM, group=group)
        else:
            dist.reduce(_real_view(out), dst=dst, op=dist.ReduceOp.SUM, group=group)
    return out


def sharded_sum_buckets(local_fn, n_units: int, out: torch.Tensor, buckets, dst: int = 0, group=None):
    """Bucketed, overlapped variant of sharded_sum for a stacked output (e.g. a 2DES waiting-time scan).

    For each bucket (a slice along axis 0 of `out`): local_fn(lo, hi, bucket) fills out[bucket] with this
    rank's member-shard partial sum, then the bucket is reduced to `dst` asynchronously, so the reduce of
    bucket b overlaps the compute of bucket b+1 (the collective runs on RCCL's own stream).  All reduces
    are waited for before returning.  Single process: local_fn(0, n_units, bucket) per bucket.
    """
    rank, ws = world()
    lo, hi = shard_range(n_units, rank, ws)
    works = []
    for b in buckets:
        local_fn(lo, hi, b)
        if ws > 1:
            works.append(dist.reduce(_real_view(out[b]), dst=dst, op=dist.ReduceOp.SUM, group=group,
                                     async_op=True))
    for w in works:
        w.wait()
    return out


class ReducePipeline:
    """Sum-reduce a SEQUENCE of per-rank partial grids to `dst`, each reduce overlapping the compute of the next
    grid (one reduce per grid, hidden behind compute instead of serialised after it).

    Grids rotate over `depth` output buffers.  next_buffer() returns the buffer for the next grid after making the
    current stream wait (stream-side, no host block) for the reduce that last used it; submit(buf) issues that
    grid's reduce asynchronously on RCCL's stream (which first waits for the compute already queued on the current
    stream); finish() makes the current stream wait for every outstanding reduce.  Rank `dst` then holds the sum of
    every grid in the buffer it was computed in.  Single process: no collective, the buffers just rotate."""

    def __init__(self, shape, dtype, device, depth: int = 2, dst: int = 0, group=None):
        self.bufs = [torch.empty(shape, dtype=dtype, device=device) for _ in range(max(1, depth))]
        self.works = [None] * len(self.bufs)
        self.dst, self.group = dst, group
        self.rank, self.ws = world()
        self.i = 0

    def next_buffer(self) -> torch.Tensor:
        j = self.i % len(self.bufs)
        if self.works[j] is not None:
            self.works[j].wait()
            self.works[j] = None
        return self.bufs[j]

    def submit(self, buf: torch.Tensor):
        j = self.i % len(self.bufs)
        if buf is not self.bufs[j]:
            raise ValueError("submit() takes the buffer next_buffer() returned")
        if self.ws > 1:
            self.works[j] = dist.reduce(_real_view(buf), dst=self.dst, op=dist.ReduceOp.SUM, group=self.group,
                                        async_op=True)
        self.i += 1

    def finish(self):
        for j, w in enumerate(self.works):
            if w is not None:
                w.wait()
                self.works[j] = None


def ensemble_2des(lam, alpha, Mt, beta, t3, t1, dst=0, group=None):
    """Ensemble-summed 2DES grid over all ranks (each rank: its member shard on its GPU)."""
    from .response import response2d_ensemble
    dev = torch.device("cuda", torch.cuda.current_device())
    n3, n1 = len(t3), len(t1)

    def local(lo, hi):
        if hi <= lo:
            return torch.zeros((n3, n1), dtype=torch.complex128, device=dev)
        return response2d_ensemble(lam[lo:hi], alpha[lo:hi], Mt[lo:hi], beta[lo:hi], t3, t1, device=dev)

    return sharded_sum(local, len(lam), dst=dst, group=group)
