"""Physical-unit Fourier transforms (drop-in for pyqed/fft.py) computed in libqdyn."""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from ._util import default_device


def _fft_axis(a, axis, inverse, scale, freq, x0, shift=True):
    dev = default_device()
    _lib.ensure_device(dev)
    a = np.asarray(a, dtype=complex)
    axis = axis % a.ndim
    n = a.shape[axis]
    outer = int(np.prod(a.shape[:axis], dtype=np.int64))
    inner = int(np.prod(a.shape[axis + 1:], dtype=np.int64))
    t = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    f = torch.from_numpy(np.ascontiguousarray(freq, dtype=float)).to(dev) if freq is not None else None
    with torch.cuda.device(dev):
        rc = _lib.load().qd_fft_axis(t.data_ptr(), outer, n, inner, int(inverse), int(shift), float(scale),
                                     _lib.ptr(f), float(x0), _lib.stream_ptr(dev))
    _lib.check(rc, "qd_fft_axis")
    return t.cpu().numpy()


def _normalize_axis(axis, ndim):
    """numpy's normalize_axis_index (fft.py:41 / :78): an out-of-range axis raises AxisError."""
    if not -ndim <= axis < ndim:
        raise np.exceptions.AxisError(axis, ndim)
    return axis % ndim


_NORM_SCALE = {None: lambda n: 1.0, "backward": lambda n: 1.0, "ortho": lambda n: 1.0 / np.sqrt(n),
               "forward": lambda n: 1.0 / n}


def fft(a, x=None, axis=-1, **kwargs):
    """fft.py:11-68: g(w) = fftshift(FFT(a)) dx exp(-i w x0), freq = 2 pi fftshift(fftfreq(n, dx)).

    Any length (numpy.fft takes every n).  ``**kwargs`` are forwarded as the reference forwards them to
    ``np.fft.fft`` (fft.py:49): ``norm`` (None / 'backward' / 'ortho' / 'forward') scales the transform; ``n`` pads or
    truncates the axis, after which the reference multiplies the length-n result by a phase built from the
    ORIGINAL length and fails to broadcast unless n equals it -- that ValueError is reproduced here.  Anything else
    raises the TypeError numpy raises for an unknown keyword."""
    a = np.asarray(a)
    axis = _normalize_axis(axis, a.ndim)
    nx = a.shape[axis]
    if x is None:
        x = np.arange(nx)
    dx = x[1] - x[0]
    kw = dict(kwargs)
    norm = kw.pop("norm", None)
    n = kw.pop("n", None)
    if kw:
        raise TypeError(f"fft() got an unexpected keyword argument '{next(iter(kw))}'")
    if norm not in _NORM_SCALE:
        raise ValueError(f'Invalid norm value {norm}; should be "backward", "ortho" or "forward".')
    if n is not None:
        n = int(n)
        if n < 1:
            raise ValueError(f"Invalid number of FFT data points ({n}) specified.")
        if n != nx and n != 1:
            # np.fft.fft(a, n) has n points along `axis`; the reference's exp(-i freq x0) has nx (fft.py:53-61)
            shape = list(a.shape)
            shape[axis] = n
            raise ValueError(f"operands could not be broadcast together with shapes {tuple(shape)} ({nx},)")
    freq = 2. * np.pi * np.fft.fftshift(np.fft.fftfreq(nx, d=dx))
    if n == 1 and nx != 1:
        # np.fft.fft(a, n=1) keeps a[0] along the axis, and the reference's phase broadcasts it to nx points:
        # a[0] dx exp(-i freq x0).  That is exactly the length-nx transform of a[0] placed at index 0 (the FFT of a
        # delta is the constant a[0]; every other term is an exact zero), so the GPU path serves it unchanged.
        z = np.zeros(a.shape, dtype=complex)
        sl = [slice(None)] * a.ndim
        sl[axis] = slice(0, 1)
        z[tuple(sl)] = a[tuple(sl)]
        a, nx = z, 1
    scale = dx * _NORM_SCALE[norm](nx)
    return _fft_axis(a, axis, False, scale, freq, float(np.real(x[0]))), freq


def ifft(a, x=None, axis=-1):
    """fft.py:70-102: g = fftshift(IFFT(a)) dx n exp(+i w x0), any length (the unnormalised inverse kernel times dx,
    which is the reference's ifft(a) * dx * n)."""
    a = np.asarray(a)
    axis = _normalize_axis(axis, a.ndim)
    nx = a.shape[axis]
    if x is None:
        x = np.arange(nx)
    dx = x[1] - x[0]
    freq = 2. * np.pi * np.fft.fftshift(np.fft.fftfreq(nx, d=dx))
    return _fft_axis(a, axis, True, dx, freq, float(np.real(x[0]))), freq


def fft2(f, dx=1, dy=1):
    """fft.py:104-126 (freqy uses nx, as the reference)."""
    nx, ny = f.shape
    g = _fft_axis(f, 1, False, 1.0, None, 0.0)
    g = _fft_axis(g, 0, False, dx * dy, None, 0.0)
    freqx = 2. * np.pi * np.fft.fftshift(np.fft.fftfreq(nx, d=dx))
    freqy = 2. * np.pi * np.fft.fftshift(np.fft.fftfreq(nx, d=dy))
    return freqx, freqy, g


def _dft2(x, y, f, kx, ky, weight):
    dev = default_device()
    _lib.ensure_device(dev)
    d = lambda v: torch.from_numpy(np.ascontiguousarray(np.real(v), dtype=float).reshape(-1)).to(dev)
    ft = torch.from_numpy(np.ascontiguousarray(np.asarray(f, dtype=complex))).to(dev)
    xs, ys, kxs, kys = d(x), d(y), d(kx), d(ky)
    out = torch.empty((kxs.numel(), kys.numel()), dtype=torch.complex128, device=dev)
    with torch.cuda.device(dev):
        rc = _lib.load().qd_dft2(xs.data_ptr(), xs.numel(), ys.data_ptr(), ys.numel(), ft.data_ptr(), kxs.data_ptr(),
                                 kxs.numel(), kys.data_ptr(), kys.numel(), float(weight), out.data_ptr(),
                                 _lib.stream_ptr(dev))
    _lib.check(rc, "qd_dft2")
    return out.cpu().numpy()


def dft(x, f, k):
    """fft.py:128-141: g(k) = sum f e^{-i k x} dx (the reference also plots; not here)."""
    dx = (x[1] - x[0]).real
    return _dft2(x, [0.0], np.asarray(f).reshape(1, -1), k, [0.0], dx)[:, 0]


def dft2(x, y, f, kx, ky):
    """fft.py:144-160 with X, Y = meshgrid(x, y) ('xy'): f has shape (len(y), len(x))."""
    dx = x[1] - x[0]
    dy = y[1] - y[0]
    return _dft2(x, y, f, kx, ky, dx * dy)
