"""Batched Monte-Carlo closed loops on the device.

`workload(...)` builds the synthetic batched inputs of SURVEY §8d deterministically for the
GLOBAL instance set (every rank generates the same arrays and takes its slice, so results
do not depend on how instances are sharded):
  * reference table: gen_circle_traj(500, N, 6, 2, [0, 0], 1) (generate_trajectory.py:7-28),
    or its 3-D extension for quad13;
  * start rows k_b ~ U{0..499}; x0_b = ref[k_b] + N(0, 0.02) on positions, N(0, 0.05) on
    velocities (clipped inside the bounds); jerk: a0 = [0, g] + N(0, 0.1); quad13: hover +
    perturbations on p/v/q/omega;
  * instance 0 starts like main.py (x0 = [1, 0, 0, 0.62], main.py:45) for force/jerk.
`ClosedLoop` binds a solver handle to the on-device closed loop of the C-ABI
(nmpc_closed_loop_*): prepare (yref window + x0 pinning) -> solve -> advance (cost, AED,
converter + plant + Philox noise), all resident in HBM.
"""
import ctypes

import numpy as np

from . import _lib
from .acados import AcadosOcpSolver, NmpcError
from .models import OCPS, gen_circle_traj, quad13_reference
from .params import DroneData, ExperimentParameters

dd = DroneData()
p = ExperimentParameters()

DEFAULT_N = {"force": 20, "jerk": 40, "quad13": 20}
PLANTS = {"force": _lib.NMPC_PLANT_CRAZYFLIE_FORCE, "jerk": _lib.NMPC_PLANT_CRAZYFLIE_JERK,
          "quad13": _lib.NMPC_PLANT_MODEL}


def reference_table(model, N):
    if model == "quad13":
        return quad13_reference(p.N, N)                     # (500+N) x 17
    ref = gen_circle_traj(p.N, N, 6, 2)                     # (500+N) x 8
    return ref[:, :6] if model == "force" else ref          # force: [x(4), u(2)], jerk: [x(6), u(2)]


def workload(model, N, batch_global, seed=42, main_like_first=True):
    """Global synthetic batch: (table, offsets int32 [B], x_init [B, nx])."""
    table = reference_table(model, N)
    rng = np.random.default_rng(seed)
    B = batch_global
    offsets = rng.integers(0, p.N, B).astype(np.int32)
    if model == "quad13":
        x = table[offsets, :13].copy()
        x[:, 0:3] += rng.normal(0, 0.02, (B, 3))
        x[:, 3:6] += rng.normal(0, 0.05, (B, 3))
        x[:, 7:10] += rng.normal(0, 0.01, (B, 3))
        x[:, 10:13] += rng.normal(0, 0.05, (B, 3))
        x[:, 0:3] = np.clip(x[:, 0:3], -1.14, 1.14)
        x[:, 3:6] = np.clip(x[:, 3:6], -0.95, 0.95)
        return table, offsets, x
    x = table[offsets, :4].copy()
    x[:, 0:2] += rng.normal(0, 0.02, (B, 2))
    x[:, 2:4] += rng.normal(0, 0.05, (B, 2))
    x[:, 0:2] = np.clip(x[:, 0:2], -1.14, 1.14)
    x[:, 2:4] = np.clip(x[:, 2:4], -0.95, 0.95)
    if main_like_first:
        offsets[0] = 0
        x[0] = [1.0, 0.0, 0.0, 0.62]
    if model == "jerk":
        a = np.array([0.0, dd.GRAVITY_ACC]) + rng.normal(0, 0.1, (B, 2))
        if main_like_first:
            a[0] = [0.0, dd.GRAVITY_ACC]
        x = np.hstack([x, a])
    return table, offsets, x


NY = {"force": (6, 4), "jerk": (8, 6), "quad13": (17, 13)}


def first_step_qps(model, N, table, offsets, x_init):
    """The QPs the closed loop solves at step 0 (what cl_prepare_kernel builds on the device):
    x0 = x_init, yref_k = table[t + k, :ny] (k < N), yref_N = table[t + N, :ny_e], t = offset.
    Returns (x0 [B, nx], yref [B, N*ny + ny_e])."""
    ny, nye = NY[model]
    offsets = np.asarray(offsets)
    rows = offsets[:, None] + np.arange(N)[None, :]
    Y = np.concatenate([table[rows, :ny].reshape(len(offsets), -1), table[offsets + N, :nye]], axis=1)
    return np.asarray(x_init, dtype=np.float64), Y


class ClosedLoop:
    """Device closed loop of `batch` instances of `model` on one GPU."""

    def __init__(self, model, batch, N=None, device=0, precision="fp64", table=None, offsets=None,
                 x_init=None, instance_base=0, seed=42, noise_std=None, noise_table=None, cost_stage=None):
        """cost_stage: the state the closed-loop cost is taken at (0: x_0 as force_model/controller.py:39,
        1: x_1 as jerk_model/controller.py:39); default by model."""
        self.model = model
        self.N = N or DEFAULT_N[model]
        self.batch = batch
        if table is None:
            table, offsets, x_init = workload(model, self.N, batch, seed)
        self.solver = AcadosOcpSolver(OCPS[model](self.N), batch=batch, device=device, precision=precision)
        self.lib = self.solver.lib
        nx = self.solver.nx
        keep = {
            "table": np.ascontiguousarray(table, dtype=np.float64),
            "offsets": np.ascontiguousarray(offsets, dtype=np.int32),
            "x": np.ascontiguousarray(x_init, dtype=np.float64).reshape(batch, nx),
        }
        d = _lib.ClosedLoopDesc()
        d.plant = PLANTS[model]
        d.ref_table = _lib.dptr(keep["table"])
        d.ref_rows, d.ref_cols = keep["table"].shape
        d.ref_period = p.N
        self.period = p.N                                # start row of step s: (offset + s) % period
        d.offsets = keep["offsets"].ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
        d.x_init = _lib.dptr(keep["x"])
        d.instance_base = int(instance_base)
        d.seed = int(seed)
        d.noise_std = p.noise if noise_std is None else float(noise_std)
        d.noise_dims = 6 if model == "quad13" else nx
        if noise_table is not None:
            keep["noise"] = np.ascontiguousarray(noise_table, dtype=np.float64).reshape(batch, -1)
            d.noise_table = _lib.dptr(keep["noise"])
            d.noise_len = keep["noise"].shape[1]
        d.cost_stage = (1 if model == "jerk" else 0) if cost_stage is None else int(cost_stage)
        if model == "quad13":
            w = np.array([1e2] * 3 + [1e0] * 3)
        else:
            w = np.array([1e2, 1e2, 1e0, 1e0])               # controller.py:40-41
        keep["w"] = w
        d.ncl, d.w_cl = w.size, _lib.dptr(w)
        d.aed_dims = 2 if model != "quad13" else 3
        d.mass, d.g, d.dt, d.dt_conv = dd.MASS, dd.GRAVITY_ACC, p.dt, p.dt_conv
        d.substeps = p.ctrls_per_sample
        rc = self.lib.nmpc_closed_loop_init(self.solver._h, ctypes.byref(d))
        if rc != 0:
            raise NmpcError(f"nmpc_closed_loop_init: {self.lib.nmpc_last_error(self.solver._h).decode()}")
        self._keep = keep

    def run(self, steps, sync=True):
        rc = self.lib.nmpc_closed_loop_run(self.solver._h, int(steps), 1 if sync else 0)
        if rc != 0:
            raise NmpcError(f"nmpc_closed_loop_run: {self.lib.nmpc_last_error(self.solver._h).decode()}")

    def set_outputs(self, on=True):
        """Opt in to the lean loop's trajectory outputs (nmpc_closed_loop_set_outputs): after each later run the
        solver's get / get_batch return every instance's last-step solution (x_0 = the state that step started
        from), status and qp_iter. Off by default: the loop reads only u_0 / x_1 (controller.py:37-41)."""
        rc = self.lib.nmpc_closed_loop_set_outputs(self.solver._h, 1 if on else 0)
        if rc != 0:
            raise NmpcError(f"nmpc_closed_loop_set_outputs: {self.lib.nmpc_last_error(self.solver._h).decode()}")

    def stats(self):
        out = np.zeros(10)
        rc = self.lib.nmpc_closed_loop_stats(self.solver._h, _lib.dptr(out), 10)
        if rc != 0:
            raise NmpcError(f"nmpc_closed_loop_stats: {self.lib.nmpc_last_error(self.solver._h).decode()}")
        return {"cost_sum": out[0], "aed_sum": out[1], "failed": out[2], "instance_steps": out[3],
                "solve_kernel_ms": out[4], "solve_launches": int(out[5]), "mean_qp_iter": out[6],
                "steps": int(out[7]), "parked": int(out[8]), "fast_launches": int(out[9])}

    def instance_stats(self):
        """Per-instance [cost sum, AED numerator, failed solves, steps] (batch x 4)."""
        out = np.zeros((self.batch, 4))
        rc = self.lib.nmpc_closed_loop_instance_stats(self.solver._h, _lib.dptr(out), out.size)
        if rc != 0:
            raise NmpcError(f"nmpc_closed_loop_instance_stats: {self.lib.nmpc_last_error(self.solver._h).decode()}")
        return out

    def iter_log(self):
        """Per-step solve record (env NMPC_ITER_LOG set before the run), each [steps, batch]: the fused
        kernels' last launch (NMPC_CL_FAST=0): (finish steps, IPM iterations, status); the lean loop's
        last run (nmpc_cl_fast.hip): (active-set steps, status, wall-clock ticks of the step: wall_clock64,
        100 MHz on MI355X)."""
        steps = int(self.lib.nmpc_closed_loop_iter_log(self.solver._h, None, 0))
        if steps <= 0:
            raise NmpcError("nmpc_closed_loop_iter_log: no log (set NMPC_ITER_LOG before the run)")
        buf = np.zeros((steps, self.batch), dtype=np.int32)
        rc = self.lib.nmpc_closed_loop_iter_log(self.solver._h, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                                buf.size)
        if rc < 0:
            raise NmpcError(f"nmpc_closed_loop_iter_log: {self.lib.nmpc_last_error(self.solver._h).decode()}")
        return buf & 0xFF, (buf >> 8) & 0xFF, buf >> 16

    def state(self):
        out = np.zeros((self.batch, self.solver.nx))
        rc = self.lib.nmpc_closed_loop_get_state(self.solver._h, _lib.dptr(out), out.size)
        if rc != 0:
            raise NmpcError(f"nmpc_closed_loop_get_state: {self.lib.nmpc_last_error(self.solver._h).decode()}")
        return out


def flops_per_iter(nx, nu, N):
    """Algorithmic flops of one Riccati-IPM iteration (SURVEY §8d formula)."""
    nz = nx + nu
    per_stage = (2 * nx * nx * nz + 2 * nx * nz * nz + nu ** 3 / 3 + 2 * nu * nu * nx + 2 * nu * nx * nx
                 + 2 * (2 * nx * nz + 2 * nu * nx + 2 * nx * nx) + 40 * nz)
    return N * per_stage


def unconstrained_solve_flops(nx, nu, N, ny, ny_e):
    """FP64 flops of the fast solve's unconstrained path per QP, as oracle/c/riccati_ipm.c
    riccati_ipm_solve_batch_fast counts them: the gradient G yref (2 n m per stage, n = nx + nu rows for
    k < N, nx for the terminal stage) and the Riccati recursion on the shared factorisation."""
    nz = nx + nu
    grad = N * 2 * nz * ny + 2 * nx * ny_e
    return grad + N * (2 * nx * nx + 2 * nx * nz + 2 * nu * nu + 4 * nu * nx + 2 * nx * nz)


def bytes_per_step(nx, nu, N, ny, ny_e, itemsize=8):
    """Algorithmic HBM bytes of one instance-step: inputs x0 + yref window,
    outputs the full x/u trajectory."""
    return (nx + N * ny + ny_e + N * nu + (N + 1) * nx) * itemsize
