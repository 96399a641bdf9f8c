"""Probe for the round-3 report that RCCL communicator init crashes under `rocprofv3 --pmc`.

    python tools/rccl_pmc_probe.py qd      one-rank communicator through libqdyn's C-ABI (qd_comm_init / qd_reduce_sum)
    python tools/rccl_pmc_probe.py torch   one-rank torch.distributed "nccl" (RCCL) process group + reduce
Run each under `rocprofv3 --pmc FETCH_SIZE -- python3 tools/rccl_pmc_probe.py MODE` and without the profiler: a
failure in both modes under the profiler only points at the profiler / RCCL pairing, not at qd_comm.hip."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "qd"
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
x = torch.ones(256 * 256, dtype=torch.complex128, device=dev)
if mode == "qd":
    from pyqed_amd import _lib
    lib = _lib.load()
    uid = ctypes.create_string_buffer(128)
    print("qd: unique id", flush=True)
    _lib.check(lib.qd_comm_unique_id(uid), "qd_comm_unique_id")
    print("qd: comm init", flush=True)
    _lib.check(lib.qd_comm_init(1, 0, uid), "qd_comm_init")
    print("qd: reduce", flush=True)
    for _ in range(3):
        _lib.check(lib.qd_reduce_sum(x.data_ptr(), x.numel(), 0, _lib.stream_ptr(dev)), "qd_reduce_sum")
    torch.cuda.synchronize(dev)
    _lib.check(lib.qd_comm_destroy(), "qd_comm_destroy")
else:
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    print("torch: init_process_group nccl", flush=True)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    print("torch: reduce", flush=True)
    for _ in range(3):
        dist.reduce(x, dst=0)
    torch.cuda.synchronize(dev)
    dist.destroy_process_group()
print(f"{mode}: ok, x[0] = {complex(x[0].item())}", flush=True)
