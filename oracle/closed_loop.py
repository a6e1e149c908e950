"""Closed-loop restatements of the reference drivers (test infrastructure only).

Follows, line by line in behaviour:
  * force loop   `src/force_model/controller.py:8-56`
  * jerk loop    `src/jerk_model/controller.py:8-58`
  * converters   `src/force_model/dynamics.py:54-79`, `src/jerk_model/dynamics.py:59-83`
  * plant        `src/plant.py:27-33`; simulators `force_model/ocp.py:98-115` (AcadosSim ERK,
                 4 stages = RK4 over dt) and `jerk_model/ocp.py:97-116` (ERK 1 stage = Euler
                 over dt_conv, 10 sub-steps); one scalar N(0, noise) draw per MPC step added to
                 every state component (`ocp.py:114-115`)
  * metric       `src/store_results.py:233-236` (calc_aed)
The QP solve is `oracle.qp.solve_ocp` (exact, KKT-certified) unless a different `solve`
callable is passed (the GPU closed-loop tests pass the HIP engine and compare).
"""
import numpy as np

from . import params as P
from . import qp as Q


def plant_f(x, u):
    """plant.py:27-33: x=[px,pz,vx,vz], u=[theta, F_d]."""
    theta, Fd = u
    return np.array([x[2], x[3], 1 / P.MASS * Fd * np.sin(theta),
                     1 / P.MASS * Fd * np.cos(theta) - P.GRAVITY_ACC])


def rk4_step(x, u, h):
    k1 = plant_f(x, u)
    k2 = plant_f(x + 0.5 * h * k1, u)
    k3 = plant_f(x + 0.5 * h * k2, u)
    k4 = plant_f(x + h * k3, u)
    return x + h / 6.0 * (k1 + 2 * k2 + 2 * k3 + k4)


def euler_step(x, u, h):
    return x + h * plant_f(x, u)


def force_convert(u_tilde):
    """force_model/dynamics.py:65-70 (single u): theta = atan2(Fx, Fz), F_d = |F|."""
    F_x, F_z = u_tilde
    return np.array([np.arctan2(F_x, F_z), np.sqrt(F_x * F_x + F_z * F_z)])


def jerk_convert(h, a_i):
    """jerk_model/dynamics.py:76-83: 10 sub-steps a <- a + h*dt_conv (sequential adds; the
    first call turns the list a_i into a new ndarray, later calls mutate it in place —
    SURVEY A.4), then theta/F_d from F = m*a at every sub-step."""
    a = np.asarray(a_i, dtype=float).copy()
    u = np.zeros((P.CTRLS_PER_SAMPLE, 2))
    for j in range(P.CTRLS_PER_SAMPLE):
        a = a + h * P.DT_CONV
        F_x = P.MASS * a[0]
        F_z = P.MASS * a[1]
        u[j, 0] = np.arctan2(F_x, F_z)
        u[j, 1] = np.sqrt(F_x * F_x + F_z * F_z)
    return u, a


class NoiseStream:
    """Scalar draws in call order (np.random.normal(0, noise) at ocp.py:114 / :115)."""

    def __init__(self, draws=None):
        self.draws = draws
        self.i = 0

    def __call__(self):
        if self.draws is None:
            return 0.0
        v = float(self.draws[self.i])
        self.i += 1
        return v


def _default_solve(spec):
    def solve(x0, yref, yref_e):
        out = Q.solve_ocp(spec, x0, yref, yref_e)
        if not out["certified"]:
            raise RuntimeError("oracle QP not certified")
        return out["X"], out["U"]
    return solve


def force_follow_trajectory(spec, xref, uref, x0, noise, n_steps=P.N_SIM, solve=None):
    """force_model/controller.py:8-56. Returns (closedLoopCost, Xsim, a, U_opt_plant, U_ctrl)."""
    solve = solve or _default_solve(spec)
    N = spec.N
    Xsim = np.zeros((n_steps + 1, 4))
    U_opt_plant = np.zeros((n_steps, 2))
    U_ctrl = np.zeros((n_steps, 2))
    a = np.zeros((n_steps, 2))
    cost_total = 0.0
    Xsim[0] = x0
    Wcl = np.diag(P.W_CL)
    for it in range(n_steps):
        yref, yref_e = Q.yref_window(xref, uref, it, N)          # ocp.py:117-122
        X, U = solve(Xsim[it].copy(), yref, yref_e)               # controller.py:29-32
        u0 = U[0]                                                 # :37
        U_ctrl[it] = u0
        a[it] = u0 / P.MASS                                       # :38
        X_opt = X[0]                                              # :39 get(0,'x') == x0_bar
        e = X_opt[:4] - xref[it, :4]
        cost = e @ Wcl @ e                                        # :40-41
        U_opt_plant[it] = force_convert(u0)                       # :44
        Xsim[it + 1] = rk4_step(Xsim[it], U_opt_plant[it], P.DT) + noise()   # :47-48
        cost_total += cost
    return cost_total, Xsim, a, U_opt_plant, U_ctrl


def jerk_follow_trajectory(spec, xref, uref, x0, noise, n_steps=P.N_SIM, solve=None):
    """jerk_model/controller.py:8-58. Returns (closedLoopCost, Xsim, a, U_opt_plant, U_ctrl)."""
    solve = solve or _default_solve(spec)
    N = spec.N
    Xsim = np.zeros((n_steps + 1, 4))
    U_opt_plant = np.zeros((n_steps, 2))
    U_ctrl = np.zeros((n_steps, 2))
    a = np.zeros((n_steps, 2))
    cost_total = 0.0
    a_i = np.array([0.0, P.GRAVITY_ACC])                          # :23
    Xsim[0] = x0
    Wcl = np.diag(P.W_CL)
    for it in range(n_steps):
        yref, yref_e = Q.yref_window(xref, uref, it, N)
        x0_bar = np.hstack((Xsim[it], a_i))                       # :30
        X, U = solve(x0_bar, yref, yref_e)
        u0 = U[0]                                                 # :38
        U_ctrl[it] = u0
        X_opt = X[1]                                              # :39 get(1,'x')
        e = X_opt[:4] - xref[it, :4]
        cost = e @ Wcl @ e                                        # :40-41
        u_tmp, a_i = jerk_convert(u0, a_i)                        # :44
        a[it] = a_i                                               # :45
        U_opt_plant[it] = u_tmp[-1]                               # :46
        x_i = Xsim[it]
        for j in range(P.CTRLS_PER_SAMPLE):                       # jerk_model/ocp.py:109-113
            x_i = euler_step(x_i, u_tmp[j], P.DT_CONV)
        Xsim[it + 1] = x_i + noise()                              # jerk_model/ocp.py:115-116
        cost_total += cost
    return cost_total, Xsim, a, U_opt_plant, U_ctrl


def calc_aed(pref, psim):
    """store_results.py:233-236 — mean of elementwise |diff| (not a Euclidean norm)."""
    return float(np.mean(np.sqrt((pref - psim) ** 2)))
