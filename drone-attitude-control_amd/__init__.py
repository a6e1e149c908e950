"""MI355X-native batched NMPC engine for the drone attitude-control hot path.

Replaces `AcadosOcpSolver.solve()` of BroilerCompiler/drone-attitude-control
(src/force_model/controller.py:32, src/jerk_model/controller.py:33) with hand-written HIP
kernels for gfx950 behind a C-ABI (include/nmpc.h, lib/libnmpc_hip.so) and an
acados_template-compatible Python façade (`acados`).

Importing this package never falls back to the CPU: the solver classes load the HIP
library on construction and raise NmpcError when it (or a GPU) is unavailable.
"""
from . import params  # noqa: F401
from ._lib import NmpcError  # noqa: F401
from .acados import (AcadosModel, AcadosOcp, AcadosOcpSolver, AcadosSim,  # noqa: F401
                     AcadosSimSolver)

__all__ = ["AcadosModel", "AcadosOcp", "AcadosOcpSolver", "AcadosSim", "AcadosSimSolver",
           "NmpcError", "params"]
