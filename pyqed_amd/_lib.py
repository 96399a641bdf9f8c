"""ctypes binding of libqdyn.so (the C-ABI declared in include/qdyn.h).

The product path has exactly one compute backend: the HIP kernels in this
library.  There is no CPU fallback — if the library is missing or a call fails,
a RuntimeError/ValueError is raised.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("QDYN_LIB", os.path.join(_HERE, "libqdyn.so"))

QD_OK = 0
QD_EINVAL = -1
QD_EHIP = -2
QD_ERCCL = -3
QD_ENOMEM = -4
QD_EBUSY = -5

# process options (include/qdyn.h QD_OPT_*)
QD_OPT_COOP_LAUNCH = 0
QD_OPT_FAKE_TIMEOUT = 1
QD_OPT_GLF_PATH = 2
QD_OPT_IDLE_CAP_MIB = 3
GLF_PATHS = {"auto": 0, "single": 1, "split": 2, "persistent": 3}

c_int = ctypes.c_int
c_double = ctypes.c_double
c_long = ctypes.c_long
c_size_t = ctypes.c_size_t
c_void_p = ctypes.c_void_p
c_char_p = ctypes.c_char_p

# name -> (restype, argtypes); must list every symbol of include/qdyn.h
SIGNATURES = {
    "qd_version": (c_int, []),
    "qd_last_error": (c_char_p, []),
    "qd_init": (c_int, [c_int]),
    "qd_device_count": (c_int, [ctypes.POINTER(c_int)]),
    "qd_shutdown": (c_int, []),
    "qd_synchronize": (c_int, [c_void_p]),
    "qd_workspace_stats": (c_int, [ctypes.POINTER(c_size_t), ctypes.POINTER(c_size_t)]),
    "qd_set_option": (c_int, [c_int, c_int]),
    "qd_get_option": (c_int, [c_int, ctypes.POINTER(c_int)]),
    "qd_take_path": (c_int, [ctypes.c_char_p, c_size_t]),
    "qd_lindblad_rk4": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_double, c_int,
                                c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p]),
    "qd_lindblad_rk4_herm": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_double, c_int,
                                     c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p]),
    "qd_glf_rk4_herm": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_double, c_int,
                                c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p]),
    "qd_glf_rk4": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int, c_double,
                           c_int, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p]),
    "qd_basis_transform": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]),
    "qd_spo2_run_ex": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                               c_void_p, c_void_p]),
    "qd_spo2_run": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "qd_spo_expv": (c_int, [c_void_p, c_int, c_long, c_int, c_double, c_void_p, c_void_p, c_void_p]),
    "qd_spo_expm": (c_int, [c_void_p, c_int, c_long, c_int, c_double, c_void_p, c_void_p, c_void_p]),
    "qd_spo2_run_batch": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p,
                                  c_void_p]),
    "qd_spo1d_run": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                             c_void_p]),
    "qd_deom_rk4": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                            c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_double, c_int,
                            c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "qd_deom_rk4_ado_major": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_double, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "qd_deom_rk4_banded": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int,
                                   c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_double, c_int,
                                   c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    "qd_cgs_project": (c_int, [c_void_p, ctypes.c_long, c_int, c_int, c_void_p, c_void_p, c_void_p, ctypes.c_long,
                               c_void_p]),
    "qd_cgs_normalize": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    "qd_arnoldi_dcgs2_step": (c_int, [c_void_p, c_long, c_int, c_int, c_void_p, c_void_p, c_long, c_void_p, c_void_p,
                                      c_void_p]),
    "qd_shifted_hessenberg_solve": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_double, c_void_p, c_void_p,
                                            c_void_p]),
    "qd_deom_apply": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_double, c_int, c_void_p]),
    "qd_deom_stage": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p,
                              c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_double,
                              c_double, c_double, c_double, c_int, c_double, c_void_p, c_int, c_int, c_void_p]),
    "qd_gather_rows": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p]),
    "qd_deom_trace": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "qd_heom_chain_euler": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_double, c_double, c_double,
                                    c_double, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "qd_sandwich": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p]),
    "qd_sos_propagator": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p]),
    "qd_response_cube": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int,
                                 c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p]),
    "qd_response2d_ensemble_uniform": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_double,
                                               c_double, c_int, c_double, c_double, c_int, c_void_p, c_int,
                                               c_void_p]),
    "qd_response2d_ensemble": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_int,
                                       c_void_p, c_int, c_void_p, c_int, c_void_p]),
    "qd_response2d_t2scan": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_double,
                                     c_double, c_int, c_void_p, c_int, c_double, c_double, c_int, c_void_p, c_int,
                                     c_void_p]),
    "qd_response2d_t2_dims": (c_int, [c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "qd_response2d_t2_operands": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_double,
                                          c_double, c_int, c_double, c_double, c_int, c_void_p, c_void_p, c_void_p]),
    "qd_response2d_ensemble_rect": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                            c_void_p, c_double, c_double, c_int, c_void_p, c_double, c_double, c_int,
                                            c_int, c_void_p, c_int, c_void_p]),
    "qd_response2d_t2_operands_rect": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p,
                                               c_void_p, c_void_p, c_int, c_int, c_double, c_double, c_int, c_double,
                                               c_double, c_int, c_void_p, c_void_p, c_void_p]),
    "qd_response2d_t2_apply": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int,
                                       c_void_p, c_int, c_void_p]),
    "qd_comm_unique_id": (c_int, [c_void_p]),
    "qd_comm_init": (c_int, [c_int, c_int, c_void_p]),
    "qd_reduce_sum": (c_int, [c_void_p, c_size_t, c_int, c_void_p]),
    "qd_comm_destroy": (c_int, []),
    "qd_resolvent_grid2d": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p, c_int,
                                    c_void_p, c_void_p]),
    "qd_resolvent_sum": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p]),
    "qd_tdse_rk4": (c_int, [c_void_p, c_void_p, c_int, c_int, c_double, c_int, c_int, c_void_p, c_void_p, c_int,
                            c_void_p, c_void_p]),
    "qd_tdse_driven_rk4": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_double, c_int,
                                   c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "qd_photon_echo": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p,
                               c_int, c_void_p, c_int, c_void_p, c_int, c_double, c_void_p, c_void_p]),
    "qd_fft_axis": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_double, c_void_p, c_double, c_void_p]),
    "qd_dft2": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_int, c_double,
                        c_void_p, c_void_p]),
    "qd_spo3_run": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p,
                            c_void_p]),
    "qd_spo3_run_axes": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int,
                                 c_int, c_void_p, c_void_p]),
    "qd_superop_from_glf": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "qd_superop_lindblad": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "qd_superop_rk4": (c_int, [c_void_p, c_void_p, c_int, c_int, c_double, c_int, c_void_p, c_int, c_void_p,
                               c_void_p, c_int, c_void_p]),
    "qd_lindblad_driven_rk4": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int,
                                       c_double, c_int, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p]),
}

_lib = None
_lock = threading.Lock()
_inited_devices: set[int] = set()


def load() -> ctypes.CDLL:
    """Load libqdyn.so (idempotent).  Raises RuntimeError if it is absent."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"libqdyn.so not found at {LIB_PATH}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (make -C pyqed_amd/csrc)")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def last_error() -> str:
    msg = load().qd_last_error()
    return msg.decode() if msg else ""


def check(rc: int, what: str) -> None:
    if rc == QD_OK:
        return
    msg = last_error()
    if rc == QD_EINVAL:
        raise ValueError(f"{what}: {msg}")
    raise RuntimeError(f"{what} failed (code {rc}): {msg}")


def ensure_device(device: torch.device) -> None:
    """qd_init once per device (checks the gfx950 target)."""
    if device.type != "cuda":
        raise RuntimeError(f"pyqed_amd computes on the GPU only; got device {device}")
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if idx in _inited_devices:
        return
    lib = load()
    with torch.cuda.device(idx):
        check(lib.qd_init(idx), "qd_init")
    _inited_devices.add(idx)


def set_option(opt: int, value: int) -> int:
    """Set a process option (qd_set_option); returns the previous value."""
    lib = load()
    prev = c_int(0)
    check(lib.qd_get_option(opt, ctypes.byref(prev)), "qd_get_option")
    check(lib.qd_set_option(opt, int(value)), "qd_set_option")
    return prev.value


def take_path() -> str:
    """The kernel paths this thread's library calls took since the last take_path() (qd_take_path)."""
    buf = ctypes.create_string_buffer(4096)
    check(load().qd_take_path(buf, len(buf)), "qd_take_path")
    return buf.value.decode()


def stream_ptr(device: torch.device | None = None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t: torch.Tensor | None) -> int | None:
    if t is None:
        return None
    if not t.is_contiguous():
        raise ValueError("pyqed_amd: tensor must be contiguous")
    return t.data_ptr()
