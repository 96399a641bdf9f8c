"""Control for the PMC-pass crash (profiles/r05/runtime/pmc_crash.md): the banded-DEOM loopback leg's launch pattern
without libqdyn -- many small index_select gathers and device-to-device row copies between a few dozen buffers, on the
current stream and on a side stream -- for rocprofv3 --pmc.  Prints one line per 2000 launches."""
import os
import sys

import torch

dev = torch.device("cuda", 0)
n_iter = int(sys.argv[1]) if len(sys.argv) > 1 else 6000
maps = os.environ.get("BENCH_MAPS")
bufs = [torch.zeros((700 + 13 * i, 2, 2), dtype=torch.complex128, device=dev) for i in range(24)]
idx = [torch.randint(0, 700, (40 + i,), device=dev) for i in range(24)]
side = torch.cuda.Stream(dev)
launches = 0
for it in range(n_iter):
    a, b = bufs[it % 24], bufs[(it * 7 + 3) % 24]
    g = torch.index_select(a, 0, idx[it % 24])
    b[:g.shape[0]].copy_(g)
    launches += 2
    if it % 50 == 0:
        with torch.cuda.stream(side):
            t = torch.empty((1 << (12 + it % 8), 2), dtype=torch.complex128, device=dev)
            t.zero_()
        launches += 1
    if it % 1000 == 0:
        torch.cuda.synchronize()
        print(f"iter {it} launches {launches}", flush=True)
        if maps:
            with open("/proc/self/maps") as fi, open(maps, "w") as fo:
                fo.write(fi.read())
torch.cuda.synchronize()
print(f"done {launches} launches", flush=True)
