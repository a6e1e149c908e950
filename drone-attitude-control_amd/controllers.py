"""Closed-loop drivers over the façade — the reference's callers of the hot path.

`force_follow_trajectory` / `jerk_follow_trajectory` keep the reference's loop structure
(src/force_model/controller.py:8-56, src/jerk_model/controller.py:8-58) and its quirks
(cost on get(0,'x') / get(1,'x'), one scalar noise draw per step added to every state,
sequential acceleration sub-steps of the jerk converter), but every QP solve and every
plant step runs on the GPU through AcadosOcpSolver / AcadosSimSolver. The batched on-device
closed loop (all instances, all steps, one launch) is `batched.ClosedLoop`.
"""
import numpy as np

from .acados import AcadosSim, AcadosSimSolver, AcadosOcpSolver, NmpcError
from .models import PlantModel, force_ocp, jerk_ocp
from .params import DroneData, ExperimentParameters


def _noise_source(noise, rng):
    p = ExperimentParameters()
    if callable(noise):
        return noise
    if noise:
        return (lambda: rng.normal(0, p.noise)) if rng is not None else (lambda: np.random.normal(0, p.noise))
    return lambda: 0.0


def _plant_sim(T, stages):
    sim = AcadosSim()
    sim.model = PlantModel().model
    sim.solver_options.T = T
    sim.solver_options.integrator_type = "ERK"
    sim.solver_options.num_stages = stages
    return AcadosSimSolver(sim)


def force_convert(u_tilde):
    """force_model/dynamics.py:54-79 (single u): theta = atan2(Fx, Fz), F_d = |F|."""
    F_x, F_z = u_tilde
    return np.array([np.arctan2(F_x, F_z), np.sqrt(F_x * F_x + F_z * F_z)])


def jerk_convert(h, a_i):
    """jerk_model/dynamics.py:59-83: a <- a + h*dt_conv at each of the 10 sub-steps."""
    p, dd = ExperimentParameters(), DroneData()
    a = np.asarray(a_i, dtype=float).copy()
    u = np.zeros((p.ctrls_per_sample, 2))
    for j in range(p.ctrls_per_sample):
        a = a + h * p.dt_conv
        F_x, F_z = dd.MASS * a[0], dd.MASS * a[1]
        u[j, 0] = np.arctan2(F_x, F_z)
        u[j, 1] = np.sqrt(F_x * F_x + F_z * F_z)
    return u, a


def force_follow_trajectory(xref, uref, x0, noise, verbose=True, N=None, n_steps=None, rng=None):
    """force_model/controller.py:8-56 on the engine. Returns (cost, Xsim, a, U_opt_plant)."""
    p, dd = ExperimentParameters(), DroneData()
    N = N or p.N_horizon
    n_steps = n_steps or p.N
    draw = _noise_source(noise, rng)
    solver = AcadosOcpSolver(force_ocp(N))
    sim = _plant_sim(p.dt, 4)
    Xsim = np.zeros((n_steps + 1, 4))
    U_opt_plant = np.zeros((n_steps, 2))
    a = np.zeros((n_steps, 2))
    total = 0.0
    Xsim[0] = x0
    Wcl = np.diag([1e2, 1e2, 1e0, 1e0])
    for it in range(n_steps):
        for k in range(N):                                           # ocp.py:117-122
            solver.set(k, "yref", np.hstack((xref[it + k], uref[it + k])))
        solver.set(N, "yref", xref[it + N])
        x0_bar = Xsim[it]
        solver.set(0, "lbx", x0_bar)
        solver.set(0, "ubx", x0_bar)
        status = solver.solve()
        if status != 0:
            solver.print_statistics()
            raise NmpcError(f"Failed in iteration {it}\nacados acados_ocp_solver returned status {status}")
        u0 = solver.get(0, "u")
        a[it] = u0 / dd.MASS
        X_opt = solver.get(0, "x")
        e = X_opt[:4] - xref[it, :4]
        cost = e @ Wcl @ e
        U_opt_plant[it] = force_convert(u0)
        sim.set("u", U_opt_plant[it])
        sim.set("x", Xsim[it])
        sim.solve()
        Xsim[it + 1] = sim.get("x") + draw()
        if verbose:
            print(f"{it}: U_opt [theta F_d]: {np.round(U_opt_plant[it], 2)} X: {np.round(Xsim[it], 2)} C: {cost}")
        total += cost
    return total, Xsim, a, U_opt_plant


def jerk_follow_trajectory(xref, uref, x0, noise, verbose=True, N=None, n_steps=None, rng=None):
    """jerk_model/controller.py:8-58 on the engine. Returns (cost, Xsim, a, U_opt_plant)."""
    p, dd = ExperimentParameters(), DroneData()
    N = N or p.N_horizon
    n_steps = n_steps or p.N
    draw = _noise_source(noise, rng)
    solver = AcadosOcpSolver(jerk_ocp(N))
    sim = _plant_sim(p.dt_conv, 1)
    Xsim = np.zeros((n_steps + 1, 4))
    U_opt_plant = np.zeros((n_steps, 2))
    a = np.zeros((n_steps, 2))
    total = 0.0
    a_i = np.array([0.0, dd.GRAVITY_ACC])
    Xsim[0] = x0
    Wcl = np.diag([1e2, 1e2, 1e0, 1e0])
    for it in range(n_steps):
        for k in range(N):
            solver.set(k, "yref", np.hstack((xref[it + k], uref[it + k])))
        solver.set(N, "yref", xref[it + N])
        x0_bar = np.hstack((Xsim[it], a_i))
        solver.set(0, "lbx", x0_bar)
        solver.set(0, "ubx", x0_bar)
        status = solver.solve()
        if status != 0:
            solver.print_statistics()
            raise NmpcError(f"Failed in iteration {it}\nacados acados_ocp_solver returned status {status}")
        u0 = solver.get(0, "u")
        X_opt = solver.get(1, "x")
        e = X_opt[:4] - xref[it, :4]
        cost = e @ Wcl @ e
        u_tmp, a_i = jerk_convert(u0, a_i)
        a[it] = a_i
        U_opt_plant[it] = u_tmp[-1]
        x_i = Xsim[it]
        for j in range(p.ctrls_per_sample):                          # jerk_model/ocp.py:109-113
            sim.set("u", u_tmp[j])
            sim.set("x", x_i)
            sim.solve()
            x_i = sim.get("x")
        Xsim[it + 1] = x_i + draw()
        if verbose:
            print(f"{it}: U_opt [h_x h_z]: {np.round(u0, 2)} X: {np.round(np.hstack((Xsim[it], a_i)), 2)} "
                  f"C: {np.round(cost, 5)}")
        total += cost
    return total, Xsim, a, U_opt_plant


def calc_aed(pref, psim):
    """store_results.py:233-236."""
    return float(np.mean(np.sqrt((pref - psim) ** 2)))
