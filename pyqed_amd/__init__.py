"""pyqed_amd — MI355X-native propagators behind pyqed's solver class surface.

Hot path (HIP, libqdyn.so): Lindblad RK4, ....
"""
from .deom import Bath, DEOMSolver
from .mol import Result, load_result
from .wpd import SPO, SPO2, SPO2NH, SPO3
from .oqs import HEOMSolver, LindbladSolver, RedfieldSolver, glf_rk4, lindblad_rk4
from .superoperator import Lindblad_solver

__all__ = ["HEOMSolver", "Lindblad_solver", "Bath", "DEOMSolver", "SPO", "SPO2", "SPO2NH", "SPO3", "Result", "load_result", "LindbladSolver", "RedfieldSolver", "glf_rk4", "lindblad_rk4"]
__version__ = "0.1.0"
