"""The C-ABI library loads and exports every symbol include/qdyn.h declares (no GPU calls)."""
import ctypes
import os
import re

from conftest import ROOT


def declared_symbols():
    syms = set()
    inc = os.path.join(ROOT, "include")
    for f in os.listdir(inc):
        if f.endswith(".h"):
            txt = open(os.path.join(inc, f)).read()
            txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
            syms |= set(re.findall(r"\b(qd_[a-z0-9_]+)\s*\(", txt))
    return syms


def test_library_exports_every_declared_symbol():
    from pyqed_amd import _lib
    lib = ctypes.CDLL(_lib.LIB_PATH)
    syms = declared_symbols()
    assert "qd_lindblad_rk4" in syms
    missing = [s for s in sorted(syms) if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_covers_header():
    from pyqed_amd import _lib
    assert declared_symbols() == set(_lib.SIGNATURES)


def test_version_and_error_string():
    from pyqed_amd import _lib
    lib = _lib.load()
    assert lib.qd_version() >= 100
    # argument validation happens before any HIP call -> safe without a GPU
    rc = lib.qd_lindblad_rk4(None, None, 0, None, 1, 4, 0.1, 1, None, 0, None, None, 0, None)
    assert rc == _lib.QD_EINVAL
    assert "non-null" in _lib.last_error()


def test_process_options_env_and_setter():
    """The library's only run-time switches (include/qdyn.h QD_OPT_*): read once from the environment at load,
    changeable with qd_set_option, out-of-range options / path values rejected; qd_take_path starts empty.  No GPU
    call is made."""
    import subprocess
    import sys
    from pyqed_amd import _lib
    code = ("import ctypes; from pyqed_amd import _lib; lib = _lib.load(); v = ctypes.c_int(); "
            "[lib.qd_get_option(o, ctypes.byref(v)) or print(v.value) for o in (0, 1, 2)]")
    env = dict(os.environ, QD_COOP_LAUNCH="0", QD_TEST_FAKE_TIMEOUT="1", QD_GLF_PATH="2")
    out = subprocess.run([sys.executable, "-c", code], env=env, cwd=ROOT, capture_output=True, text=True, check=True)
    assert out.stdout.split() == ["0", "1", "2"]
    env = {k: v for k, v in os.environ.items() if k not in ("QD_COOP_LAUNCH", "QD_TEST_FAKE_TIMEOUT", "QD_GLF_PATH")}
    out = subprocess.run([sys.executable, "-c", code], env=env, cwd=ROOT, capture_output=True, text=True, check=True)
    assert out.stdout.split() == ["1", "0", "0"]
    prev = _lib.set_option(_lib.QD_OPT_GLF_PATH, _lib.GLF_PATHS["split"])
    try:
        assert _lib.set_option(_lib.QD_OPT_GLF_PATH, prev) == _lib.GLF_PATHS["split"]
    finally:
        _lib.load().qd_set_option(_lib.QD_OPT_GLF_PATH, prev)
    lib = _lib.load()
    assert lib.qd_set_option(99, 0) == _lib.QD_EINVAL
    assert lib.qd_set_option(_lib.QD_OPT_GLF_PATH, 7) == _lib.QD_EINVAL
    assert _lib.take_path() == ""


def test_library_reads_no_other_environment_switch():
    """dispatch reads no A/B environment variables -- the only QD_* names the library's sources
    hold as strings are the three QD_OPT_* variables, and the Python package reads none."""
    import glob
    names = set()
    for f in glob.glob(os.path.join(ROOT, "pyqed_amd", "csrc", "*.hip")) + \
            glob.glob(os.path.join(ROOT, "pyqed_amd", "csrc", "*.hpp")):
        names |= set(re.findall(r'"(QD_[A-Z0-9_]+)"', open(f).read()))
    assert names <= {"QD_COOP_LAUNCH", "QD_TEST_FAKE_TIMEOUT", "QD_GLF_PATH"}, sorted(names)
    py = set()
    for f in glob.glob(os.path.join(ROOT, "pyqed_amd", "*.py")):
        py |= set(re.findall(r'environ(?:\.get)?[\[(]"(QD_[A-Z0-9_]+)"', open(f).read()))
    assert not py, sorted(py)
