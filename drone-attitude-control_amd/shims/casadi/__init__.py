"""`casadi` drop-in for the reference's model files: the SX subset of
drone_attitude_control_amd.casadi_shim (see shims/README.md)."""
from drone_attitude_control_amd.casadi_shim import (SX, atan2, cos, exp, fabs, inf, log, pi,  # noqa: F401
                                                    sin, sqrt, tan, tanh, vertcat)

__version__ = "3.6.7-nmpc-shim"
