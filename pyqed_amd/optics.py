"""Laser pulses that drive the time-dependent propagators (host side).

Mirror of pyqed.optics.Pulse (optics.py:229-310, the pulse the driven solvers take): a Gaussian
envelope times a carrier; `efield(t)` returns the real field.  The drivers evaluate `efield` on
the host once per step block and hand the values to the GPU kernels.
"""
from __future__ import annotations

import numpy as np

AU2FS = 2.41888432651e-2                 # pyqed/units.py:2
AU2EV = 27.2116                          # pyqed/units.py:8
FINE_STRUCTURE = 0.0072973525693         # pyqed/units.py:36
AU2W_PER_CM2 = 3.50944758e16             # pyqed/units.py:46


def intensity_to_field(I):
    """optics.py:22-39: peak field (a.u.) of intensity I (W/cm^2)."""
    return np.sqrt(2. * I * 4. * np.pi / AU2W_PER_CM2 / FINE_STRUCTURE)


class Pulse:
    """optics.py:229 Pulse: E(t) = Re[A exp(-(t-tc)^2 / 2 tau^2) exp(-i omegac (t-tc))]."""

    def __init__(self, omegac=3. / AU2EV, tau=5. / AU2FS, tc=0, delay=0., amplitude=0.001, intensity=None, cep=0.,
                 beta=0, polarization=None):
        self.delay = delay
        self.tc = tc
        self.tau = tau
        self.fwhm = tau * 2.3548200450309493
        self.sigma = tau
        self.omegac = omegac
        self.unit = 'au'
        self.amplitude = amplitude if intensity is None else intensity_to_field(intensity)
        self.cep = cep
        self.bandwidth = 1. / tau
        self.duration = 2. * tau
        self.beta = beta
        self.ndim = 1
        self.polarization = polarization

    def envelop(self, t):
        return self.amplitude * np.exp(-(t - self.tc) ** 2 / 2. / self.tau ** 2)

    def spectrum(self, omega):
        return self.amplitude * self.tau * np.sqrt(2. * np.pi) * np.exp(-(omega - self.omegac) ** 2 * self.tau ** 2 / 2.)

    def field(self, t):
        return self.efield(t)

    def efield(self, t, return_complex=False):
        E = self.amplitude * np.exp(-(t - self.tc) ** 2 / 2. / self.sigma ** 2) * np.exp(-1j * self.omegac * (t - self.tc))
        return np.real(E)
