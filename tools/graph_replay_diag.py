"""Graph-replay diagnosis of captured Lindblad calls (profiles/r06/graph/replay_diag.txt).

usage: python tools/graph_replay_diag.py   (QDYN_LIB=... to compare library builds)
For three shapes and every Lindblad path: capture one call, replay it twice per sequence (null stream, with and
without a host sync between the replays, then the side stream) and print max |x - ref| against two direct calls.
A torch-only graph replayed the same way is the control."""
import sys, numpy as np, torch
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
from oracle import lindblad as olb
from pyqed_amd import lindblad_rk4, _lib
from conftest import qd_option
dev = torch.device("cuda", 0)
m = lambda a, b: float((a - b).abs().max())
A = torch.randn(512, 512, dtype=torch.complex128, device=dev) / 40
v0 = torch.randn(512, 512, dtype=torch.complex128, device=dev)
v = v0.clone(); s0 = torch.cuda.Stream(dev)
with torch.cuda.stream(s0):
    v = v0.clone()
    for _ in range(12): v = torch.tanh(v @ A)
torch.cuda.synchronize(); vref = v.clone()
vx = v0.clone(); g0 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g0, stream=s0):
    w = vx
    for _ in range(6): w = torch.tanh(w @ A)
    vx.copy_(w)
outs = []
for _ in range(4):
    vx.copy_(v0); g0.replay(); g0.replay(); torch.cuda.synchronize(); outs.append(m(vx, vref))
for _ in range(4):
    with torch.cuda.stream(s0):
        vx.copy_(v0); g0.replay(); g0.replay()
    torch.cuda.synchronize(); outs.append(m(vx, vref))
print("torch-only graph:", outs, flush=True)
for N, B in [(128, 1), (64, 1), (32, 256)]:
    H, cs = olb.synthetic_lindblad(N, nc=1)
    Ht, Ct = torch.from_numpy(H).to(dev), torch.from_numpy(np.array(cs)).to(dev)
    r0 = torch.from_numpy(olb.random_pure_states(B, N, seed=12)).to(dev)
    s = torch.cuda.Stream(dev)
    for herm in (True, False):
        for path in ("auto", "split", "persistent", "single"):
            with qd_option("glf_path", path):
                ref = r0.clone(); torch.cuda.synchronize()
                with torch.cuda.stream(s):
                    for _ in range(2):
                        lindblad_rk4(Ht, Ct, ref, 1e-3, 6, hermitian=herm, stream=s.cuda_stream)
                torch.cuda.synchronize()
                x = r0.clone(); torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                _lib.take_path()
                with torch.cuda.graph(g, stream=s):
                    lindblad_rk4(Ht, Ct, x, 1e-3, 6, hermitian=herm, stream=s.cuda_stream)
                pth = _lib.take_path()
            outs = []
            for sync in (False, False, True, True):
                x.copy_(r0)
                g.replay()
                if sync:
                    torch.cuda.synchronize()
                g.replay()
                torch.cuda.synchronize()
                outs.append(x.clone())
            for _ in range(4):   # copy and replays on the side stream
                with torch.cuda.stream(s):
                    x.copy_(r0)
                    g.replay()
                    g.replay()
                torch.cuda.synchronize()
                outs.append(x.clone())
            print(f"N={N} B={B} herm={herm} path={path} captured={pth!r} vs direct:",
                  " ".join(f"{m(o, ref):.2e}" for o in outs), flush=True)
            del g
