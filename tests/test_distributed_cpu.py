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
