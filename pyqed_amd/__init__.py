"""pyqed_amd — MI355X-native propagators behind pyqed's solver class surface.

Hot path (HIP, libqdyn.so): Lindblad RK4, ....
"""
from .mol import Result, load_result
from .oqs import LindbladSolver, RedfieldSolver, glf_rk4, lindblad_rk4

__all__ = ["Result", "load_result", "LindbladSolver", "RedfieldSolver", "glf_rk4", "lindblad_rk4"]
__version__ = "0.1.0"
