"""Host-side conversion helpers (inputs may be numpy, scipy.sparse, np.matrix or torch)."""
from __future__ import annotations

import numpy as np
import torch

try:
    import scipy.sparse as _sp
except Exception:  # pragma: no cover
    _sp = None


def default_device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("pyqed_amd needs a ROCm GPU (torch.cuda.is_available() is False); "
                           "there is no CPU fallback")
    return torch.device("cuda", torch.cuda.current_device())


def issparse(a) -> bool:
    return _sp is not None and _sp.issparse(a)


def to_numpy(a, dtype=None) -> np.ndarray:
    if isinstance(a, torch.Tensor):
        a = a.detach().cpu().numpy()
    elif issparse(a):
        a = a.toarray()
    a = np.asarray(a)
    if dtype is not None:
        a = a.astype(dtype, copy=False)
    return a


def to_device(a, device=None, dtype=torch.complex128) -> torch.Tensor:
    """Contiguous device tensor of the given dtype (complex128 by default)."""
    device = device or default_device()
    if isinstance(a, torch.Tensor):
        return a.to(device=device, dtype=dtype).contiguous()
    npdt = {torch.complex128: np.complex128, torch.float64: np.float64,
            torch.int32: np.int32, torch.int64: np.int64}[dtype]
    return torch.from_numpy(np.ascontiguousarray(to_numpy(a, npdt))).to(device)


def stack_ops(ops, n, device=None) -> torch.Tensor | None:
    if ops is None or len(ops) == 0:
        return None
    out = torch.empty((len(ops), n, n), dtype=torch.complex128, device=device or default_device())
    for i, op in enumerate(ops):
        a = to_numpy(op, np.complex128)
        if a.shape != (n, n):
            raise ValueError(f"operator {i} has shape {a.shape}, expected {(n, n)}")
        out[i] = torch.from_numpy(np.ascontiguousarray(a)).to(out.device)
    return out
