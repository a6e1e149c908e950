"""acados_template-compatible façade over the HIP engine (the reference's hot-path interface).

Mirrors the subset of `acados_template` the reference uses on its hot path
(call sites force_model/ocp.py:21-122, force_model/controller.py:25-54,
jerk_model/ocp.py:20-123, jerk_model/controller.py:26-56):

    AcadosModel, AcadosOcp (.model/.cost/.constraints/.solver_options/.dims),
    AcadosOcpSolver(ocp, json_file=..., verbose=False)
        .set(stage, 'yref' | 'lbx' | 'ubx', value)   .solve() -> status
        .get(stage, 'x' | 'u')   .get_cost()   .print_statistics()   .solve_for_x0(x0)
        .get_stats('qp_iter' | 'sqp_iter' | 'time_tot' | 'status')
    AcadosSim, AcadosSimSolver(sim).set('x'|'u', v) .solve() .get('x') .simulate(x=, u=)

Same names, argument meaning and error behaviour (status codes of src/Readme.md:14-20;
unknown fields / wrong sizes raise). Extension: every solver carries a batch dimension
(`batch=` at construction, `instance=` on set/get, set_batch/get_batch) so the same object
drives one trajectory (the reference) or thousands (the batched engine).

Dynamics must be affine in (x, u) — true for both reference controller models
(force_model/dynamics.py:32-37, jerk_model/dynamics.py:35-42). They are given either as
numeric `model.A_c, model.B_c, model.c_c`, or as `f_expl_expr` objects that expose
`affine_coefficients(x, u)` (the CasADi-SX shim, drone_attitude_control_amd.casadi_shim),
or as a Python callable f(x, u) that is probed and checked for affinity. The integrator
sensitivities are then computed natively by the library (nmpc_create).
"""
import ctypes
import json

import numpy as np

from . import _lib
from ._lib import NmpcError

ACADOS_INFTY = 1e10  # acados's default "infinite" bound magnitude used by acados_template


class AcadosModel:
    def __init__(self):
        self.name = None
        self.x = None
        self.u = None
        self.xdot = None
        self.f_expl_expr = None
        self.f_impl_expr = None
        # numeric affine form x' = A_c x + B_c u + c_c (alternative to symbolic f_expl_expr)
        self.A_c = None
        self.B_c = None
        self.c_c = None
        # discrete affine form x+ = A x + B u + c (integrator_type 'DISCRETE')
        self.disc_dyn_A = None
        self.disc_dyn_B = None
        self.disc_dyn_c = None


def _dim(v):
    if v is None:
        return None
    if hasattr(v, "size1"):
        return int(v.size1())
    if hasattr(v, "shape"):
        return int(v.shape[0])
    return len(v)


def affine_form(model):
    """(A_c, B_c, c_c) of an affine model, from numeric fields, the SX shim, or probing."""
    if model.A_c is not None:
        A = np.atleast_2d(np.asarray(model.A_c, float))
        B = np.atleast_2d(np.asarray(model.B_c, float))
        c = np.asarray(model.c_c if model.c_c is not None else np.zeros(A.shape[0]), float).ravel()
        return A, B, c
    f = model.f_expl_expr
    if hasattr(f, "affine_coefficients"):
        return f.affine_coefficients(model.x, model.u)
    if callable(f):
        nx, nu = _dim(model.x), _dim(model.u)
        c = np.asarray(f(np.zeros(nx), np.zeros(nu)), float).ravel()
        A = np.stack([np.asarray(f(np.eye(nx)[i], np.zeros(nu)), float).ravel() - c for i in range(nx)], 1)
        B = np.stack([np.asarray(f(np.zeros(nx), np.eye(nu)[i]), float).ravel() - c for i in range(nu)], 1)
        rng = np.random.default_rng(0)
        for _ in range(3):
            x, u = rng.normal(size=nx), rng.normal(size=nu)
            if not np.allclose(np.asarray(f(x, u), float).ravel(), A @ x + B @ u + c, rtol=1e-9, atol=1e-9):
                raise NotImplementedError("model dynamics are not affine in (x, u); the engine solves LQ-OCPs")
        return A, B, c
    raise NotImplementedError("cannot extract affine dynamics from model.f_expl_expr")


class AcadosOcpDims:
    def __init__(self):
        self.nx = None
        self.nu = None
        self.N = None
        self.ny = None
        self.ny_e = None


class AcadosOcpCost:
    def __init__(self):
        self.cost_type = "LINEAR_LS"
        self.cost_type_e = "LINEAR_LS"
        self.W = None
        self.W_e = None
        self.Vx = None
        self.Vu = None
        self.Vx_e = None
        self.yref = None
        self.yref_e = None


class AcadosOcpConstraints:
    def __init__(self):
        self.constr_type = "BGH"
        self.constr_type_e = "BGH"
        self.lbu = np.zeros(0)
        self.ubu = np.zeros(0)
        self.idxbu = np.zeros(0, dtype=int)
        self.lbx = np.zeros(0)
        self.ubx = np.zeros(0)
        self.idxbx = np.zeros(0, dtype=int)
        self.lbx_e = np.zeros(0)
        self.ubx_e = np.zeros(0)
        self.idxbx_e = np.zeros(0, dtype=int)
        self.x0 = None


class AcadosOcpOptions:
    def __init__(self):
        self.qp_solver = "PARTIAL_CONDENSING_HPIPM"
        self.hessian_approx = "GAUSS_NEWTON"
        self.integrator_type = "ERK"
        self.nlp_solver_type = "SQP"
        self.print_level = 0
        self.N_horizon = None
        self.tf = None
        self.sim_method_num_stages = 4
        self.sim_method_num_steps = 1
        self.qp_solver_iter_max = 50
        self.qp_tol = None
        self.qp_solver_tol_comp = None
        self.qp_solver_tol_stat = None
        self.qp_solver_mu0 = None
        # engine extensions (no acados counterpart): exact-finish threshold and active-set steps,
        # None = library defaults (1 and 12 on fp64 handles), threshold < 0 = off
        # (include/nmpc.h qp_solver_polish_mu / qp_solver_polish_steps)
        self.qp_solver_polish_mu = None
        self.qp_solver_polish_steps = None
        self.cost_scaling = "time_steps"   # acados default: stage cost x time step


class AcadosOcp:
    def __init__(self):
        self.model = AcadosModel()
        self.dims = AcadosOcpDims()
        self.cost = AcadosOcpCost()
        self.constraints = AcadosOcpConstraints()
        self.solver_options = AcadosOcpOptions()
        self.code_export_directory = "c_generated_code"

    def to_dict(self):
        d = {"name": self.model.name, "dims": vars(self.dims).copy()}
        for sec in ("cost", "constraints", "solver_options"):
            d[sec] = {k: (v.tolist() if isinstance(v, np.ndarray) else v)
                      for k, v in vars(getattr(self, sec)).items()}
        return d


def _arr(v, n=None, dtype=float):
    a = np.ascontiguousarray(np.asarray(v if v is not None else [], dtype=dtype).ravel())
    if n is not None and a.size != n:
        raise ValueError(f"expected {n} values, got {a.size}")
    return a


def describe_ocp(ocp):
    """Numeric description of an AcadosOcp as the engine consumes it (no GPU needed):
    dynamics (continuous affine + integrator, or discrete), LINEAR_LS weights/selectors,
    bounds with acados's infinity mapped to none, horizon, tolerances. Raises for anything
    outside the supported class (the reference's OCPs, force_model/ocp.py:21-93,
    jerk_model/ocp.py:20-92, are inside it)."""
    opts, cost, cons, model = ocp.solver_options, ocp.cost, ocp.constraints, ocp.model
    if cost.cost_type != "LINEAR_LS" or cost.cost_type_e != "LINEAR_LS":
        raise NotImplementedError("only LINEAR_LS costs are supported (force_model/ocp.py:28-29)")
    if opts.hessian_approx != "GAUSS_NEWTON":
        raise NotImplementedError("only GAUSS_NEWTON Hessians are supported")
    if opts.nlp_solver_type not in ("SQP", "SQP_RTI"):
        raise NotImplementedError(f"nlp_solver_type {opts.nlp_solver_type}")
    N = opts.N_horizon if opts.N_horizon is not None else ocp.dims.N
    if N is None or opts.tf is None:
        raise ValueError("solver_options.N_horizon and solver_options.tf must be set")
    if cons.x0 is None:
        raise NotImplementedError("the engine pins x0 at stage 0 (constraints.x0 must be set)")
    if opts.integrator_type == "DISCRETE":
        A, B, c = (np.atleast_2d(np.asarray(model.disc_dyn_A, float)),
                   np.atleast_2d(np.asarray(model.disc_dyn_B, float)),
                   np.asarray(model.disc_dyn_c, float).ravel())
        dyn_type, integ = _lib.NMPC_DYN_DISCRETE_AFFINE, _lib.NMPC_ERK
    else:
        A, B, c = affine_form(model)
        dyn_type = _lib.NMPC_DYN_CONTINUOUS_AFFINE
        integ = {"IRK": _lib.NMPC_IRK, "ERK": _lib.NMPC_ERK}.get(opts.integrator_type)
        if integ is None:
            raise NotImplementedError(f"integrator_type {opts.integrator_type}")
    nx, nu = B.shape
    W = np.atleast_2d(np.asarray(cost.W, float))
    W_e = np.atleast_2d(np.asarray(cost.W_e, float)) if cost.W_e is not None else np.zeros((0, 0))

    def bounds(lb, ub, idx):
        idx = _arr(idx, None, np.int32)
        lb, ub = _arr(lb, idx.size), _arr(ub, idx.size)
        # acados_template's ACADOS_INFTY magnitude means "no bound"
        lb = np.where(np.abs(lb) >= ACADOS_INFTY, -1e30, lb)
        ub = np.where(np.abs(ub) >= ACADOS_INFTY, 1e30, ub)
        return lb, ub, idx

    lbu, ubu, idxbu = bounds(cons.lbu, cons.ubu, cons.idxbu)
    lbx, ubx, idxbx = bounds(cons.lbx, cons.ubx, cons.idxbx)
    lbx_e, ubx_e, idxbx_e = bounds(cons.lbx_e, cons.ubx_e, cons.idxbx_e)
    return dict(
        name=model.name or "ocp", nx=nx, nu=nu, N=int(N), ny=W.shape[0], ny_e=W_e.shape[0],
        dyn_type=dyn_type, A=A, B=B, c=c, integrator_type=integ,
        integrator=opts.integrator_type, num_stages=int(opts.sim_method_num_stages),
        num_steps=int(opts.sim_method_num_steps), tf=float(opts.tf),
        W=W, Vx=np.asarray(cost.Vx, float), Vu=np.asarray(cost.Vu, float), W_e=W_e,
        Vx_e=np.asarray(cost.Vx_e, float) if cost.Vx_e is not None else np.zeros((0, nx)),
        yref=cost.yref, yref_e=cost.yref_e, cost_scaling=opts.cost_scaling,
        lbu=lbu, ubu=ubu, idxbu=idxbu, lbx=lbx, ubx=ubx, idxbx=idxbx,
        lbx_e=lbx_e, ubx_e=ubx_e, idxbx_e=idxbx_e, x0=_arr(cons.x0, nx),
        qp_solver_iter_max=int(opts.qp_solver_iter_max or 0),
        # acados's qp_tol sets every QP tolerance (stat/eq/ineq/comp) unless one is given
        qp_solver_tol_comp=float(opts.qp_solver_tol_comp or (opts.qp_tol or 0.0) or 0.0),
        qp_solver_tol_res=float(opts.qp_solver_tol_stat or (opts.qp_tol or 0.0) or 0.0),
        qp_solver_mu0=float(opts.qp_solver_mu0 or 0.0),
        qp_solver_polish_mu=float(getattr(opts, "qp_solver_polish_mu", None) or 0.0),
        qp_solver_polish_steps=int(getattr(opts, "qp_solver_polish_steps", None) or 0))


class AcadosOcpSolver:
    """Batched drop-in for acados_template.AcadosOcpSolver (force_model/ocp.py:95-96)."""

    def __init__(self, acados_ocp, json_file=None, verbose=False, build=True, generate=True,
                 *, batch=1, device=0, precision="fp64"):
        ocp = acados_ocp
        self.lib = _lib.load()
        D = describe_ocp(ocp)
        nx, nu, N, ny, ny_e = D["nx"], D["nu"], D["N"], D["ny"], D["ny_e"]
        self.nx, self.nu, self.N, self.ny, self.ny_e = nx, nu, N, ny, ny_e
        self.batch = int(batch)
        self.name = D["name"]
        self.precision = precision
        prec = {"fp64": _lib.NMPC_FP64, "fp32": _lib.NMPC_FP32}[precision]

        keep = {}

        def P(name, v, n=None, dtype=float):
            keep[name] = _arr(v, n, dtype)
            return _lib.iptr(keep[name]) if dtype is np.int32 else _lib.dptr(keep[name])

        d = _lib.OcpDesc()
        d.abi_version = _lib.NMPC_ABI_VERSION
        keep["name"] = self.name.encode()
        d.name = keep["name"]
        d.nx, d.nu, d.N, d.ny, d.ny_e = nx, nu, N, ny, ny_e
        d.dyn_type = D["dyn_type"]
        d.A, d.B, d.c = P("A", D["A"], nx * nx), P("B", D["B"], nx * nu), P("c", D["c"], nx)
        d.integrator_type = D["integrator_type"]
        d.num_stages = D["num_stages"]
        d.num_steps = D["num_steps"]
        d.tf = D["tf"]
        d.W, d.Vx, d.Vu = P("W", D["W"], ny * ny), P("Vx", D["Vx"], ny * nx), P("Vu", D["Vu"], ny * nu)
        if ny_e:
            d.W_e, d.Vx_e = P("W_e", D["W_e"], ny_e * ny_e), P("Vx_e", D["Vx_e"], ny_e * nx)
        if D["yref"] is not None:
            d.yref = P("yref", D["yref"], ny)
        if D["yref_e"] is not None and ny_e:
            d.yref_e = P("yref_e", D["yref_e"], ny_e)
        d.cost_scaling = (_lib.NMPC_COST_SCALING_TIME_STEPS if D["cost_scaling"] == "time_steps"
                          else _lib.NMPC_COST_SCALING_NONE)
        d.nbu, d.idxbu = D["idxbu"].size, P("idxbu", D["idxbu"], None, np.int32)
        d.lbu, d.ubu = P("lbu", D["lbu"]), P("ubu", D["ubu"])
        d.nbx, d.idxbx = D["idxbx"].size, P("idxbx", D["idxbx"], None, np.int32)
        d.lbx, d.ubx = P("lbx", D["lbx"]), P("ubx", D["ubx"])
        d.nbx_e, d.idxbx_e = D["idxbx_e"].size, P("idxbx_e", D["idxbx_e"], None, np.int32)
        d.lbx_e, d.ubx_e = P("lbx_e", D["lbx_e"]), P("ubx_e", D["ubx_e"])
        d.x0 = P("x0", D["x0"], nx)
        d.qp_solver_iter_max = D["qp_solver_iter_max"]
        d.qp_solver_tol_comp = D["qp_solver_tol_comp"]
        d.qp_solver_tol_res = D["qp_solver_tol_res"]
        d.qp_solver_mu0 = D["qp_solver_mu0"]
        d.qp_solver_polish_mu = D["qp_solver_polish_mu"]
        d.qp_solver_polish_steps = D["qp_solver_polish_steps"]
        h = ctypes.c_void_p()
        rc = self.lib.nmpc_create(ctypes.byref(d), self.batch, int(device), prec, ctypes.byref(h))
        if rc != 0:
            raise NmpcError(f"nmpc_create failed ({rc}): {self.lib.nmpc_last_error_global().decode()}")
        self._h = h
        self._keep = keep
        self._status = 0
        self.acados_ocp = ocp
        if json_file:
            with open(json_file, "w") as f:
                json.dump(ocp.to_dict(), f, indent=1, default=str)

    # -------------------------------------------------------------- helpers
    def _check(self, rc, what):
        if rc < 0:
            raise NmpcError(f"{what}: {self.lib.nmpc_last_error(self._h).decode()}")
        return rc

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            try:
                self.lib.nmpc_destroy(h)
            except Exception:  # noqa: BLE001
                pass
            self._h = None

    # -------------------------------------------------------------- acados surface
    def set(self, stage_, field_, value_, instance=-1):
        """ocp_solver.set(k, 'yref', v) (force_model/ocp.py:120-122); set(0, 'lbx'/'ubx', x0)
        (force_model/controller.py:30-31). `instance` (extension): -1 = all instances."""
        v = _arr(value_)
        rc = self.lib.nmpc_set(self._h, int(instance), int(stage_), field_.encode(), _lib.dptr(v), v.size)
        self._check(rc, f"set({stage_}, '{field_}')")

    def get(self, stage_, field_, instance=0):
        n = {"x": self.nx, "u": self.nu}.get(field_)
        if n is None:
            raise NmpcError(f"get: unknown field '{field_}'")
        out = np.zeros(n)
        rc = self.lib.nmpc_get(self._h, int(instance), int(stage_), field_.encode(), _lib.dptr(out), n)
        self._check(rc, f"get({stage_}, '{field_}')")
        return out

    def solve(self):
        """Returns the acados status (max over instances): 0 ok, 2 max iter, 4 QP failure."""
        rc = self.lib.nmpc_solve(self._h)
        self._status = self._check(rc, "solve")
        return self._status

    def solve_for_x0(self, x0_bar, fail_on_nonzero_status=True, print_stats_on_failure=True):
        self.set(0, "lbx", x0_bar)
        self.set(0, "ubx", x0_bar)
        status = self.solve()
        if status != 0:
            if print_stats_on_failure:
                self.print_statistics()
            if fail_on_nonzero_status:
                raise NmpcError(f"acados acados_ocp_solver returned status {status}")
        return self.get(0, "u")

    def get_cost(self, instance=0):
        out = ctypes.c_double()
        self._check(self.lib.nmpc_get_cost(self._h, int(instance), ctypes.byref(out)), "get_cost")
        return out.value

    def get_status(self, instance=None):
        st = self.get_batch_int("status")
        return int(st.max()) if instance is None else int(st[instance])

    def get_stats(self, field_):
        s = np.zeros(5)
        self._check(self.lib.nmpc_get_stats(self._h, _lib.dptr(s), 5), "get_stats")
        if field_ == "qp_iter":
            return self.get_batch_int("qp_iter") if self.batch > 1 else int(self.get_batch_int("qp_iter")[0])
        if field_ == "sqp_iter":
            return 1
        if field_ == "time_tot":
            return float(s[3]) * 1e-3
        if field_ == "status":
            return self.get_status()
        if field_ in ("fast_listed", "fast_parked"):   # the last fast solve waited for (batched extension)
            s7 = np.zeros(7)
            self._check(self.lib.nmpc_get_stats(self._h, _lib.dptr(s7), 7), "get_stats")
            return int(s7[5 if field_ == "fast_listed" else 6])
        raise NmpcError(f"get_stats: unknown field '{field_}'")

    def print_statistics(self):
        s = np.zeros(5)
        self._check(self.lib.nmpc_get_stats(self._h, _lib.dptr(s), 5), "print_statistics")
        print(f"\niter\tqp_status\tqp_iter (max/mean)\ttime [ms]\n"
              f"1\t{self._status} ({_lib.STATUS_TEXT.get(self._status, '?')})\t"
              f"{int(s[0])}/{s[1]:.2f}\t\t\t{s[3]:.3f}\n"
              f"instances with status != 0: {int(s[2])} of {self.batch}")

    # -------------------------------------------------------------- batched extension
    def set_batch(self, field_, values):
        v = _arr(values)
        self._check(self.lib.nmpc_set_batch(self._h, field_.encode(), _lib.dptr(v), v.size), f"set_batch('{field_}')")

    def get_batch(self, field_):
        shape = {"x": (self.batch, self.N + 1, self.nx), "u": (self.batch, self.N, self.nu)}.get(field_)
        if shape is None:
            raise NmpcError(f"get_batch: unknown field '{field_}'")
        out = np.zeros(shape)
        self._check(self.lib.nmpc_get_batch(self._h, field_.encode(), _lib.dptr(out), out.size),
                    f"get_batch('{field_}')")
        return out

    def get_batch_int(self, field_):
        out = np.zeros(self.batch, dtype=np.int32)
        self._check(self.lib.nmpc_get_batch_int(self._h, field_.encode(),
                                                out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), out.size),
                    f"get_batch_int('{field_}')")
        return out

    def device_ptr(self, field_):
        p = ctypes.c_void_p()
        self._check(self.lib.nmpc_device_ptr(self._h, field_.encode(), ctypes.byref(p)), "device_ptr")
        return p.value

    def solve_async(self):
        return self._check(self.lib.nmpc_solve_async(self._h), "solve_async")

    def synchronize(self):
        return self._check(self.lib.nmpc_synchronize(self._h), "synchronize")

    def set_stream(self, stream_ptr):
        return self._check(self.lib.nmpc_set_stream(self._h, ctypes.c_void_p(stream_ptr)), "set_stream")

    def launch_info(self):
        out = (ctypes.c_int * 9)()
        self._check(self.lib.nmpc_get_launch_info(self._h, out, 9), "launch_info")
        return {"instances_per_wave": out[0], "workgroups": out[1], "threads": out[2], "lds_bytes": out[3],
                "kernel": {0: "ipm_kernel", 1: "ipm_lpc_kernel", 2: "cond_ipm_kernel", 3: "ipm_lpi_kernel"}.get(out[4], str(out[4])),
                "structure": {0: "dense", 1: "force", 2: "jerk", 3: "quad13"}.get(out[5], str(out[5])),
                "closed_loop_kernel": {0: "fused", 1: "cl_fast_kernel", 2: "cl_lock_kernel"}.get(out[6], str(out[6])),
                "active_set_max": out[7],
                # what nmpc_solve runs: the fp64 fast path (sf_kernel: unconstrained solution on the shared
                # factorisation, fin64_kernel: active-set finish; full IPM only for what they leave) or `kernel`
                "solve_kernel": "sf_kernel" if out[8] else {0: "ipm_kernel", 1: "ipm_lpc_kernel", 2: "cond_ipm_kernel",
                                                            3: "ipm_lpi_kernel"}.get(out[4], str(out[4]))}

    def discrete_model(self):
        A = np.zeros((self.nx, self.nx))
        B = np.zeros((self.nx, self.nu))
        c = np.zeros(self.nx)
        self._check(self.lib.nmpc_get_model(self._h, _lib.dptr(A), _lib.dptr(B), _lib.dptr(c)), "get_model")
        return A, B, c


# ---------------------------------------------------------------------------- simulator
class AcadosSimOptions:
    def __init__(self):
        self.T = None
        self.integrator_type = "ERK"
        self.num_stages = 4
        self.num_steps = 1


class AcadosSim:
    def __init__(self):
        self.model = AcadosModel()
        self.solver_options = AcadosSimOptions()


class AcadosSimSolver:
    """AcadosSimSolver for the reference plant (src/plant.py:27-43), stepped on the device.

    Supported models: the 2-D Crazyflie plant x=[px,pz,vx,vz], u=[theta,F_d]; the model must
    expose `plant_mass` and `plant_g` (set by drone_attitude_control_amd.models.PlantModel or
    recovered by the CasADi shim). ERK with 1 or 4 stages (force_model/ocp.py:98-104,
    jerk_model/ocp.py:97-104).
    """

    def __init__(self, acados_sim, json_file=None, verbose=False, build=True, generate=True, *, device=0):
        self.lib = _lib.load()
        sim = acados_sim
        opts = sim.solver_options
        if opts.integrator_type != "ERK" or int(opts.num_stages) not in (1, 4) or int(opts.num_steps) != 1:
            raise NotImplementedError("plant simulator: ERK with 1 or 4 stages, 1 step")
        m = sim.model
        mass = getattr(m, "plant_mass", None)
        g = getattr(m, "plant_g", None)
        if (mass is None or g is None) and m.f_expl_expr is not None and hasattr(m.f_expl_expr, "affine_coefficients"):
            # CasADi-SX model (the reference's plant.py through the shim): recognise the plant
            from .casadi_shim import crazyflie_plant_params
            mass, g = crazyflie_plant_params(m.f_expl_expr, m.x, m.u)
        if mass is None or g is None:
            raise NotImplementedError("AcadosSimSolver supports the 2-D Crazyflie plant model (src/plant.py)")
        self.mass, self.g = float(mass), float(g)
        self.T = float(opts.T)
        self.stages = int(opts.num_stages)
        self.device = int(device)
        self._x = np.zeros(4)
        self._u = np.zeros(2)
        self._xn = np.zeros(4)

    def set(self, field_, value_):
        v = _arr(value_)
        if field_ == "x":
            self._x = _arr(v, 4)
        elif field_ == "u":
            self._u = _arr(v, 2)
        else:
            raise NmpcError(f"AcadosSimSolver.set: unknown field '{field_}'")

    def solve(self):
        rc = self.lib.nmpc_sim_plant(self.device, 1, self.stages, self.T, self.mass, self.g,
                                     _lib.dptr(self._x), _lib.dptr(self._u), _lib.dptr(self._xn))
        if rc != 0:
            raise NmpcError(f"nmpc_sim_plant: {self.lib.nmpc_last_error_global().decode()}")
        return 0

    def get(self, field_):
        if field_ != "x":
            raise NmpcError(f"AcadosSimSolver.get: unknown field '{field_}'")
        return self._xn.copy()

    def simulate(self, x=None, u=None):
        if x is not None:
            self.set("x", x)
        if u is not None:
            self.set("u", u)
        self.solve()
        return self.get("x")
