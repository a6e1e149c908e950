"""ctypes loader for oracle/c/riccati_ipm.c (test infrastructure only; see oracle/__init__.py).

`build()` compiles the plain-C fp64 Riccati IPM with gcc into oracle/build/ (git-ignored,
shipped to the GPU box with the snapshot). It is the CPU baseline ("port") that bench.py
times on the host cores, and a second stage-wise implementation for the tests.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "c", "riccati_ipm.c")
LIB = os.path.join(HERE, "build", "libriccati_ipm.so")
# x86-64-v3 (AVX2+FMA) runs on both this container's Xeon and the GPU box's EPYC hosts
CFLAGS = ["-O3", "-march=x86-64-v3", "-fopenmp", "-shared", "-fPIC", "-std=c99"]


def build(force=False):
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    if not force and os.path.exists(LIB) and os.path.getmtime(LIB) >= os.path.getmtime(SRC):
        return LIB
    subprocess.check_call(["gcc", *CFLAGS, SRC, "-o", LIB, "-lm"])
    return LIB


class _Desc(ctypes.Structure):
    _fields_ = [
        ("nx", ctypes.c_int), ("nu", ctypes.c_int), ("N", ctypes.c_int),
        ("ny", ctypes.c_int), ("ny_e", ctypes.c_int),
        ("A", ctypes.c_void_p), ("B", ctypes.c_void_p), ("c", ctypes.c_void_p),
        ("H", ctypes.c_void_p), ("G", ctypes.c_void_p),
        ("He", ctypes.c_void_p), ("Ge", ctypes.c_void_p),
        ("lb0", ctypes.c_void_p), ("ub0", ctypes.c_void_p),
        ("lb", ctypes.c_void_p), ("ub", ctypes.c_void_p),
        ("lbe", ctypes.c_void_p), ("ube", ctypes.c_void_p),
        ("tol_comp", ctypes.c_double), ("tol_res", ctypes.c_double), ("mu0", ctypes.c_double),
        ("max_iter", ctypes.c_int), ("polish_mu", ctypes.c_double), ("polish_steps", ctypes.c_int),
    ]


INF = 1e30
# include/nmpc.h defaults of the exact finish (fp64 handles): first attempt once mu <= 1 (at the
# start for mu0 <= 1), at most 12 active-set steps per attempt
DEFAULT_POLISH_MU = 1.0
DEFAULT_POLISH_STEPS = 12


def stage_qp_data(spec):
    """Stage-wise QP data (H, G, He, Ge, bounds) built from the OcpSpec, the oracle's way."""
    nx, nu = spec.nx, spec.nu
    s = spec.scaling()
    V = np.hstack([spec.Vx, spec.Vu])
    H = s[0] * V.T @ spec.W @ V
    G = -s[0] * V.T @ spec.W
    He = s[spec.N] * spec.Vx_e.T @ spec.W_e @ spec.Vx_e
    Ge = -s[spec.N] * spec.Vx_e.T @ spec.W_e
    lb = np.full(nx + nu, -INF)
    ub = np.full(nx + nu, INF)
    lb[nx + spec.idxbu] = spec.lbu
    ub[nx + spec.idxbu] = spec.ubu
    lb0, ub0 = lb.copy(), ub.copy()
    lb[spec.idxbx] = spec.lbx
    ub[spec.idxbx] = spec.ubx
    lbe = np.full(nx, -INF)
    ube = np.full(nx, INF)
    if len(spec.idxbx_e):
        lbe[spec.idxbx_e] = spec.lbx_e
        ube[spec.idxbx_e] = spec.ubx_e
    return dict(H=H, G=G, He=He, Ge=Ge, lb0=lb0, ub0=ub0, lb=lb, ub=ub, lbe=lbe, ube=ube)


class RiccatiIpmRef:
    def __init__(self, spec, tol_comp=1e-15, tol_res=1e-12, mu0=1e-2, max_iter=50, polish_mu=0.0,
                 polish_steps=None):
        self.lib = ctypes.CDLL(build())
        self.lib.riccati_ipm_solve_batch.restype = ctypes.c_int
        self.lib.riccati_ipm_max_threads.restype = ctypes.c_int
        self.spec = spec
        q = stage_qp_data(spec)
        self._keep = {k: np.ascontiguousarray(v, dtype=np.float64) for k, v in q.items()}
        for k in ("A", "B", "c"):
            self._keep[k] = np.ascontiguousarray(getattr(spec, k), dtype=np.float64)
        p = lambda k: self._keep[k].ctypes.data
        self.desc = _Desc(spec.nx, spec.nu, spec.N, spec.ny, spec.nx,
                          p("A"), p("B"), p("c"), p("H"), p("G"), p("He"), p("Ge"),
                          p("lb0"), p("ub0"), p("lb"), p("ub"), p("lbe"), p("ube"),
                          tol_comp, tol_res, mu0, max_iter, polish_mu,
                          DEFAULT_POLISH_STEPS if polish_steps is None else polish_steps)

    @classmethod
    def for_options(cls, spec, o, precision="fp64"):
        """The oracle configured like the engine handle of an OCP with solver options `o`
        (include/nmpc.h defaults: tol_comp 1e-15, tol_res 1e-12, exact finish from mu <= 1 with
        <= 12 active-set steps on fp64 handles, none on fp32; a negative threshold switches it off)."""
        pm = getattr(o, "qp_solver_polish_mu", None) or 0.0
        pm = 0.0 if pm < 0 or precision != "fp64" else (pm or DEFAULT_POLISH_MU)
        ps = getattr(o, "qp_solver_polish_steps", None) or DEFAULT_POLISH_STEPS
        return cls(spec, tol_comp=o.qp_solver_tol_comp or 1e-15, tol_res=o.qp_solver_tol_stat or 1e-12,
                   polish_mu=pm, polish_steps=ps)

    def max_threads(self):
        """Host threads this process may use: the CPU affinity mask, capped by OMP_NUM_THREADS
        (the GPU box exports 16 = its CPU share although nproc shows the whole machine)."""
        n = len(os.sched_getaffinity(0))
        env = os.environ.get("OMP_NUM_THREADS")
        if env and env.isdigit() and int(env) > 0:
            n = min(n, int(env))
        return max(1, n)

    def solve(self, x0, yref, nthreads=None):
        """x0: (B, nx); yref: (B, N*ny + ny_e). Returns X (B,N+1,nx), U (B,N,nu), status, iters."""
        sp = self.spec
        x0 = np.ascontiguousarray(x0, dtype=np.float64).reshape(-1, sp.nx)
        B = x0.shape[0]
        yref = np.ascontiguousarray(yref, dtype=np.float64).reshape(B, -1)
        assert yref.shape[1] == sp.N * sp.ny + sp.nx
        X = np.zeros((B, sp.N + 1, sp.nx))
        U = np.zeros((B, sp.N, sp.nu))
        st = np.zeros(B, dtype=np.int32)
        it = np.zeros(B, dtype=np.int32)
        rc = self.lib.riccati_ipm_solve_batch(
            ctypes.byref(self.desc), B, ctypes.c_void_p(x0.ctypes.data), ctypes.c_void_p(yref.ctypes.data),
            ctypes.c_void_p(X.ctypes.data), ctypes.c_void_p(U.ctypes.data),
            ctypes.c_void_p(st.ctypes.data), ctypes.c_void_p(it.ctypes.data),
            int(nthreads) if nthreads else self.max_threads())
        if rc < 0:
            raise ValueError("riccati_ipm_solve_batch rejected the problem dimensions")
        return X, U, st, it

    def __del__(self):
        if getattr(self, "_fast", None):
            self.lib.riccati_fast_tables_free(ctypes.c_void_p(self._fast))
            self._fast = None

    def solve_fast(self, x0, yref, wsmax=16, nthreads=None):
        """The engine's fp64 general solve, restated (riccati_ipm_solve_batch_fast): the unconstrained
        solution on the shared factorisation, primal-dual active-set rounds on W from its violations, the
        dual fallback, the full IPM + exact finish for what is left. Returns X, U, status, iters and the
        counters {solves, unconstrained, set, set_steps, full, failed, flops, full_newton}."""
        sp = self.spec
        x0 = np.ascontiguousarray(x0, dtype=np.float64).reshape(-1, sp.nx)
        B = x0.shape[0]
        yref = np.ascontiguousarray(yref, dtype=np.float64).reshape(B, -1)
        assert yref.shape[1] == sp.N * sp.ny + sp.nx
        X = np.zeros((B, sp.N + 1, sp.nx))
        U = np.zeros((B, sp.N, sp.nu))
        st = np.zeros(B, dtype=np.int32)
        it = np.zeros(B, dtype=np.int32)
        cnt = np.zeros(8)
        p = lambda a: ctypes.c_void_p(a.ctypes.data)
        if getattr(self, "_fast", None) is None:   # the factorisation and W, once per OCP (setup, untimed)
            self.lib.riccati_fast_tables_create.restype = ctypes.c_void_p
            self._fast = self.lib.riccati_fast_tables_create(ctypes.byref(self.desc))
            if not self._fast:
                raise ValueError("riccati_fast_tables_create rejected the problem dimensions")
        rc = self.lib.riccati_ipm_solve_batch_fast(
            ctypes.byref(self.desc), ctypes.c_void_p(self._fast), B, p(x0), p(yref), p(X), p(U), p(st), p(it), p(cnt), int(wsmax),
            int(nthreads) if nthreads else self.max_threads())
        if rc < 0:
            raise ValueError("riccati_ipm_solve_batch_fast rejected the problem dimensions")
        keys = ("solves", "unconstrained", "set", "set_steps", "full", "failed", "flops", "full_newton")
        return X, U, st, it, dict(zip(keys, cnt.tolist()))


class _ClDesc(ctypes.Structure):
    _fields_ = [
        ("plant", ctypes.c_int), ("table", ctypes.c_void_p),
        ("rows", ctypes.c_int), ("cols", ctypes.c_int), ("period", ctypes.c_int),
        ("cost_stage", ctypes.c_int), ("ncl", ctypes.c_int), ("aed_dims", ctypes.c_int),
        ("noise_dims", ctypes.c_int), ("substeps", ctypes.c_int),
        ("wcl", ctypes.c_void_p),
        ("mass", ctypes.c_double), ("g", ctypes.c_double), ("dt", ctypes.c_double), ("dt_conv", ctypes.c_double),
        ("noise", ctypes.c_void_p), ("noise_len", ctypes.c_int),
        ("noise_std", ctypes.c_double), ("seed", ctypes.c_ulonglong), ("inst_base", ctypes.c_longlong),
        ("inst_ids", ctypes.c_void_p), ("wsmax", ctypes.c_int),
    ]


# largest active set of the device's lean closed loop per model (nmpc_cl_fast.hip cl_fast_wsmax):
# mode 1 restates the same cap
WSMAX = {"quad13": 16, "jerk": 16, "force": 32}


class ClosedLoopRef:
    """CPU restatement of the device closed loop (nmpc_closed_loop_run; oracle/c/riccati_ipm.c
    riccati_ipm_closed_loop): per instance and step the yref window from the shared reference
    table at row (offset + step) % period (force_model/ocp.py:117-122), x0 pinned to the state
    (force_model/controller.py:29-31), the solve (controller.py:32), cost (controller.py:40-41),
    AED numerator (store_results.py:233-236) and the plant with its noise draw.

    model: "force" | "jerk" | "quad13" (plants: Crazyflie + force converter, Crazyflie + jerk
    converter, the controller's own discrete model). mode 0 = the oracle (every QP solved cold
    to its exact solution); mode 1 = the GPU's algorithm (warm-started fast finish on the shared
    factorisation, full solves only where it fails) — the closed-loop CPU baseline. Noise: the
    injected `noise_table` [batch, steps] if given, else the device's Philox stream
    (seed, instance_base + b or instance_ids[b], step) x noise_std."""

    PLANTS = {"quad13": 0, "force": 1, "jerk": 2}

    def __init__(self, spec, model, table, offsets, x_init, mode=0, noise_table=None, seed=42, instance_base=0,
                 noise_std=None, tol_comp=None, tol_res=None, polish_mu=DEFAULT_POLISH_MU,
                 polish_steps=DEFAULT_POLISH_STEPS, period=None, instance_ids=None, cost_stage=None):
        from . import params as P
        self.ipm = RiccatiIpmRef(spec, tol_comp=tol_comp or 1e-15, tol_res=tol_res or 1e-12, polish_mu=polish_mu,
                                 polish_steps=polish_steps)
        self.lib = self.ipm.lib
        self.lib.riccati_ipm_closed_loop.restype = ctypes.c_int
        self.spec, self.model, self.mode = spec, model, int(mode)
        nx, N = spec.nx, spec.N
        self.batch = len(offsets)
        keep = self._keep = {
            "table": np.ascontiguousarray(table, dtype=np.float64),
            "offsets": np.ascontiguousarray(offsets, dtype=np.int32),
            "wcl": np.array([1e2] * 3 + [1e0] * 3 if model == "quad13" else list(P.W_CL), dtype=np.float64),
        }
        self.state = np.ascontiguousarray(x_init, dtype=np.float64).reshape(self.batch, nx).copy()
        self.acc = np.zeros((self.batch, 4))
        self.act = np.zeros((self.batch, (N + 1) * (nx + spec.nu)), dtype=np.int8)
        self.failed = np.zeros(self.batch, dtype=np.uint8)
        self.step = 0
        self.counters = np.zeros(10)
        d = self.desc = _ClDesc()
        d.plant = self.PLANTS[model]
        d.table = keep["table"].ctypes.data
        d.rows, d.cols = keep["table"].shape
        d.period = int(period or P.N_SIM)
        d.cost_stage = (1 if model == "jerk" else 0) if cost_stage is None else int(cost_stage)
        d.ncl = keep["wcl"].size
        d.aed_dims = 3 if model == "quad13" else 2
        d.noise_dims = 6 if model == "quad13" else nx
        d.substeps = P.CTRLS_PER_SAMPLE
        d.wcl = keep["wcl"].ctypes.data
        d.mass, d.g, d.dt, d.dt_conv = P.MASS, P.GRAVITY_ACC, P.DT, P.DT_CONV
        if noise_table is not None:
            keep["noise"] = np.ascontiguousarray(noise_table, dtype=np.float64).reshape(self.batch, -1)
            d.noise, d.noise_len = keep["noise"].ctypes.data, keep["noise"].shape[1]
        d.noise_std = P.NOISE if noise_std is None else float(noise_std)
        d.seed, d.inst_base = int(seed), int(instance_base)
        d.wsmax = WSMAX.get(model, 8)
        if instance_ids is not None:   # global ids of a subset of instances (Philox stream)
            keep["ids"] = np.ascontiguousarray(instance_ids, dtype=np.int64)
            d.inst_ids = keep["ids"].ctypes.data

    def run(self, steps, nthreads=None, logs=False):
        """Advance `steps` steps. logs=True returns per-step (u0 [B, steps, nu], state after the
        step [B, steps, nx], status [B, steps], path [B, steps]: 0 fast unconstrained, 1 fast
        active-set steps, 2 full solve)."""
        sp, B = self.spec, self.batch
        lg = None
        if logs:
            lg = (np.zeros((B, steps, sp.nu)), np.zeros((B, steps, sp.nx)), np.zeros((B, steps), dtype=np.int32),
                  np.zeros((B, steps), dtype=np.int32))
        p = lambda a: ctypes.c_void_p(a.ctypes.data) if a is not None else None
        rc = self.lib.riccati_ipm_closed_loop(
            ctypes.byref(self.ipm.desc), ctypes.byref(self.desc), B, self.step, int(steps),
            p(self._keep["offsets"]), p(self.state), p(self.acc), p(self.act), p(self.failed), self.mode,
            *(p(a) for a in (lg or (None,) * 4)), p(self.counters),
            int(nthreads) if nthreads else self.ipm.max_threads())
        if rc < 0:
            raise ValueError("riccati_ipm_closed_loop rejected the problem")
        self.step += steps
        return lg

    def stats(self):
        """Counters: solves, fast unconstrained, fast active-set accepted, fast active-set steps,
        full solves, failures, FP64 flops of the paths taken, Newton systems of the full solves,
        (mode 0) solutions whose active set the dense KKT pass corrected / could not settle."""
        k = ("solves", "fast_unconstrained", "fast_set", "fast_set_steps", "full", "failed", "flops", "full_newton",
             "kkt_corrected", "kkt_unsettled")
        return dict(zip(k, self.counters.tolist()))
