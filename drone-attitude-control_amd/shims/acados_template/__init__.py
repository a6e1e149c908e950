"""`acados_template` drop-in: the MI355X engine's façade under acados_template's name
(see shims/README.md)."""
from drone_attitude_control_amd.acados import (ACADOS_INFTY, AcadosModel, AcadosOcp,  # noqa: F401
                                               AcadosOcpSolver, AcadosSim, AcadosSimSolver)
