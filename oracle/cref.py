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
