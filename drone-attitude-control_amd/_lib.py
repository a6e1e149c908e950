"""ctypes binding of the C-ABI in include/nmpc.h (libnmpc_hip.so).

This is the binding a maintainer of the reference would add in place of acados_template's
ctypes layer over `libacados_ocp_solver_<model>.so`. There is no CPU
fallback: if the HIP library is missing or no GPU is visible, every entry point raises.
"""
import ctypes
import os

import numpy as np

from . import build as _build

LIB_PATH = _build.LIB

NMPC_FP64, NMPC_FP32 = 0, 1
NMPC_DYN_CONTINUOUS_AFFINE, NMPC_DYN_DISCRETE_AFFINE = 0, 1
NMPC_IRK, NMPC_ERK = 0, 1
NMPC_COST_SCALING_TIME_STEPS, NMPC_COST_SCALING_NONE = 0, 1
NMPC_ABI_VERSION = 2

STATUS_TEXT = {0: "success", 1: "failure", 2: "maximum number of iterations reached",
               3: "minimum step size in QP solver reached", 4: "qp solver failed"}

_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int)


class OcpDesc(ctypes.Structure):
    _fields_ = [
        ("abi_version", ctypes.c_int), ("name", ctypes.c_char_p),
        ("nx", ctypes.c_int), ("nu", ctypes.c_int), ("N", ctypes.c_int),
        ("ny", ctypes.c_int), ("ny_e", ctypes.c_int),
        ("dyn_type", ctypes.c_int), ("A", _dp), ("B", _dp), ("c", _dp),
        ("integrator_type", ctypes.c_int), ("num_stages", ctypes.c_int), ("num_steps", ctypes.c_int),
        ("tf", ctypes.c_double),
        ("W", _dp), ("Vx", _dp), ("Vu", _dp), ("W_e", _dp), ("Vx_e", _dp),
        ("yref", _dp), ("yref_e", _dp), ("cost_scaling", ctypes.c_int),
        ("nbu", ctypes.c_int), ("idxbu", _ip), ("lbu", _dp), ("ubu", _dp),
        ("nbx", ctypes.c_int), ("idxbx", _ip), ("lbx", _dp), ("ubx", _dp),
        ("nbx_e", ctypes.c_int), ("idxbx_e", _ip), ("lbx_e", _dp), ("ubx_e", _dp),
        ("x0", _dp),
        ("qp_solver_iter_max", ctypes.c_int), ("qp_solver_tol_comp", ctypes.c_double),
        ("qp_solver_tol_res", ctypes.c_double), ("qp_solver_mu0", ctypes.c_double),
        ("qp_solver_polish_mu", ctypes.c_double), ("qp_solver_polish_steps", ctypes.c_int),
    ]


NMPC_PLANT_MODEL, NMPC_PLANT_CRAZYFLIE_FORCE, NMPC_PLANT_CRAZYFLIE_JERK = 0, 1, 2


class ClosedLoopDesc(ctypes.Structure):
    _fields_ = [
        ("plant", ctypes.c_int), ("ref_table", _dp),
        ("ref_rows", ctypes.c_int), ("ref_cols", ctypes.c_int), ("ref_period", ctypes.c_int),
        ("offsets", ctypes.POINTER(ctypes.c_int32)), ("x_init", _dp),
        ("instance_base", ctypes.c_longlong), ("seed", ctypes.c_ulonglong),
        ("noise_std", ctypes.c_double), ("noise_dims", ctypes.c_int),
        ("noise_table", _dp), ("noise_len", ctypes.c_int),
        ("cost_stage", ctypes.c_int), ("ncl", ctypes.c_int), ("w_cl", _dp), ("aed_dims", ctypes.c_int),
        ("mass", ctypes.c_double), ("g", ctypes.c_double), ("dt", ctypes.c_double), ("dt_conv", ctypes.c_double),
        ("substeps", ctypes.c_int),
    ]


# every symbol include/nmpc.h declares, with (restype, argtypes)
SIGNATURES = {
    "nmpc_abi_version": (ctypes.c_int, []),
    "nmpc_device_count": (ctypes.c_int, []),
    "nmpc_last_error_global": (ctypes.c_char_p, []),
    "nmpc_create": (ctypes.c_int, [ctypes.POINTER(OcpDesc), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   ctypes.POINTER(ctypes.c_void_p)]),
    "nmpc_destroy": (None, [ctypes.c_void_p]),
    "nmpc_last_error": (ctypes.c_char_p, [ctypes.c_void_p]),
    "nmpc_set_stream": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "nmpc_get_stream": (ctypes.c_void_p, [ctypes.c_void_p]),
    "nmpc_get_model": (ctypes.c_int, [ctypes.c_void_p, _dp, _dp, _dp]),
    "nmpc_set": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_char_p, _dp, ctypes.c_int]),
    "nmpc_get": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_char_p, _dp, ctypes.c_int]),
    "nmpc_set_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, _dp, ctypes.c_size_t]),
    "nmpc_get_batch": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, _dp, ctypes.c_size_t]),
    "nmpc_get_batch_int": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int32),
                                          ctypes.c_size_t]),
    "nmpc_device_ptr": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]),
    "nmpc_solve": (ctypes.c_int, [ctypes.c_void_p]),
    "nmpc_solve_async": (ctypes.c_int, [ctypes.c_void_p]),
    "nmpc_synchronize": (ctypes.c_int, [ctypes.c_void_p]),
    "nmpc_get_cost": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, _dp]),
    "nmpc_get_stats": (ctypes.c_int, [ctypes.c_void_p, _dp, ctypes.c_int]),
    "nmpc_get_launch_info": (ctypes.c_int, [ctypes.c_void_p, _ip, ctypes.c_int]),
    "nmpc_closed_loop_init": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ClosedLoopDesc)]),
    "nmpc_closed_loop_run": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "nmpc_closed_loop_stats": (ctypes.c_int, [ctypes.c_void_p, _dp, ctypes.c_int]),
    "nmpc_closed_loop_instance_stats": (ctypes.c_int, [ctypes.c_void_p, _dp, ctypes.c_size_t]),
    "nmpc_closed_loop_get_state": (ctypes.c_int, [ctypes.c_void_p, _dp, ctypes.c_size_t]),
    "nmpc_closed_loop_set_outputs": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    "nmpc_closed_loop_iter_log": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32), ctypes.c_size_t]),
    "nmpc_sim_plant": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                      ctypes.c_double, _dp, _dp, _dp]),
}

_LIB = None


class NmpcError(RuntimeError):
    pass


def load(path=None):
    """Load libnmpc_hip.so (building it first if the sources are newer). Raises if absent."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    # NMPC_LIB: an experimental build of the same library (tools/, tuning runs only)
    p = path or os.environ.get("NMPC_LIB") or LIB_PATH
    if not os.path.exists(p):
        try:
            _build.build()
        except Exception as e:  # noqa: BLE001
            raise NmpcError(f"HIP library {p} is missing and could not be built: {e}") from e
    lib = ctypes.CDLL(p)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.nmpc_abi_version() != NMPC_ABI_VERSION:
        raise NmpcError("libnmpc_hip.so ABI version mismatch")
    if path is None:
        _LIB = lib
    return lib


def dptr(a):
    return a.ctypes.data_as(_dp) if a is not None else None


def iptr(a):
    return a.ctypes.data_as(_ip) if a is not None else None


def f64(a, shape=None):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float64))
    return a.reshape(shape) if shape is not None else a
