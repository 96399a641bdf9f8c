"""NumPy restatement of pyqed/fft.py fft / ifft (test infrastructure only: the checker for pyqed_amd.fft).

Follows pyqed/fft.py:11-68 (fft: numpy FFT along `axis` with the caller's kwargs, fftshift, times dx, times
exp(-i freq x0) along that axis) and :70-102 (ifft: numpy inverse FFT times dx n, exp(+i freq x0)).
"""
import numpy as np


def _phase(g, axis, ph):
    g = np.moveaxis(g, axis, -1) * ph                      # fft.py:55-61 (swapaxes, multiply, swap back)
    return np.moveaxis(g, -1, axis)


def fft(a, x=None, axis=-1, **kwargs):
    a = np.asarray(a)
    axis = axis % a.ndim
    nx = a.shape[axis]
    if x is None:
        x = np.arange(nx)
    dx = x[1] - x[0]
    g = np.fft.fftshift(np.fft.fft(a, axis=axis, **kwargs), axes=(axis,)) * dx
    freq = 2. * np.pi * np.fft.fftshift(np.fft.fftfreq(nx, d=dx))
    return _phase(g, axis, np.exp(-1j * freq * x[0])), freq


def ifft(a, x=None, axis=-1):
    a = np.asarray(a)
    axis = axis % a.ndim
    nx = a.shape[axis]
    if x is None:
        x = np.arange(nx)
    dx = x[1] - x[0]
    g = np.fft.fftshift(np.fft.ifft(a, axis=axis), axes=(axis,)) * dx * nx
    freq = 2. * np.pi * np.fft.fftshift(np.fft.fftfreq(nx, d=dx))
    return _phase(g, axis, np.exp(1j * freq * x[0])), freq
