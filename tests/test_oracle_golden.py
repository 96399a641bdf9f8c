"""Pin the CPU oracle against golden vectors produced by the real reference."""
import numpy as np
import pytest

from conftest import load_golden, relerr
from oracle import lindblad as olb

# oracle vs reference: same fp64 arithmetic up to summation order
TOL = 1e-12


@pytest.mark.parametrize("name", ["lindblad_n4", "lindblad_n16", "lindblad_n40_noc", "lindblad_n128"])
def test_lindblad_oracle_matches_reference(name):
    g = load_golden(name)
    Nt = int(g["Nt"])
    obs, rholist, rho = olb.lindblad(g["H"], g["rho0"], list(g["C"]), list(g["E"]), Nt, float(g["dt"]))
    assert obs.shape == g["observables"].shape
    assert relerr(obs, g["observables"]) < TOL
    if "rholist" in g:
        assert relerr(np.array(rholist), g["rholist"]) < TOL
    else:
        assert relerr(rho, g["rho_final"]) < TOL
    assert np.allclose(g["times"], np.arange(Nt + 1) * float(g["dt"]))
