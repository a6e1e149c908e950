"""GPU parity of the condensed MFMA family (csrc/nmpc_cond.hip, NMPC_KERNEL=cond) and of the
dimension-generic path: any (nx, nu) without a compiled stage-wise kernel runs there.

Expected values: the KKT-certified dense oracle (oracle/qp.py) — golden cases of the reference
models (tests/golden/qp_cases.npz) and seeded random stable LTI OCPs built here (nx=5, nu=3
and others), which no other kernel family is compiled for. Bar: 1e-6 relative (fp64), as for
the stage-wise families; fp32 3e-2.
"""
import os

import numpy as np
import pytest

from drone_attitude_control_amd import AcadosOcpSolver
from drone_attitude_control_amd.acados import AcadosOcp
from drone_attitude_control_amd.models import OCPS
from oracle import models, qp

pytestmark = pytest.mark.gpu

TOL64, TOL32 = 1e-6, 3e-2


def rel_err(X, U, Xr, Ur):
    scale = np.maximum(1.0, np.maximum(np.abs(Xr).max(axis=(-2, -1)), np.abs(Ur).max(axis=(-2, -1))))
    err = np.maximum(np.abs(X - Xr).max(axis=(-2, -1)), np.abs(U - Ur).max(axis=(-2, -1)))
    return err / scale


def make(ocp, batch, precision="fp64", kernel="cond"):
    if kernel:
        os.environ["NMPC_KERNEL"] = kernel
    try:
        return AcadosOcpSolver(ocp, batch=batch, precision=precision)
    finally:
        os.environ.pop("NMPC_KERNEL", None)


@pytest.fixture(scope="module")
def cases(golden_dir):
    return np.load(os.path.join(golden_dir, "qp_cases.npz"))


@pytest.mark.parametrize("key,precision", [("force_N20", "fp64"), ("force_N30", "fp64"), ("jerk_N30", "fp64"),
                                           ("force_N20", "fp32"), ("jerk_N30", "fp32"), ("quad13_N20", "fp32")])
def test_condensed_matches_oracle(key, precision, cases):
    name, N = key.split("_N")
    N = int(N)
    x0, y = cases[key + "_x0"], cases[key + "_yref"]
    s = make(OCPS[name](N), x0.shape[0], precision)
    assert s.launch_info()["kernel"] == "cond_ipm_kernel"
    s.set_batch("x0", x0)
    s.set_batch("yref", y)
    st = s.solve()
    status = s.get_batch_int("status")
    assert (status == 0).all(), (st, status, s.get_batch_int("qp_iter"))
    e = rel_err(s.get_batch("x"), s.get_batch("u"), cases[key + "_X"], cases[key + "_U"])
    it = s.get_batch_int("qp_iter")
    print(f"cond {key} {precision}: max rel err {e.max():.3e}, iters mean {it.mean():.2f} max {it.max()}")
    assert e.max() < (TOL64 if precision == "fp64" else TOL32), e.max()


def random_lti(nx, nu, N, seed):
    """A seeded random stable discrete LTI OCP (spectral radius 0.98), LINEAR_LS tracking cost,
    input boxes on every input and state boxes on every other state. Returns the façade OCP
    (integrator_type DISCRETE) and the oracle's OcpSpec of the same problem."""
    rng = np.random.default_rng(seed)
    Q, _ = np.linalg.qr(rng.normal(size=(nx, nx)))
    A = Q @ np.diag(rng.uniform(0.6, 0.98, nx)) @ Q.T + 0.05 * rng.normal(size=(nx, nx))
    A *= 0.98 / max(0.98, np.abs(np.linalg.eigvals(A)).max())
    B = rng.normal(size=(nx, nu)) * 0.3
    c = rng.normal(size=nx) * 0.02
    ny = nx + nu
    w = np.concatenate([rng.uniform(0.5, 2.0, nx), rng.uniform(0.05, 0.3, nu)])
    Vx = np.zeros((ny, nx))
    Vx[:nx] = np.eye(nx)
    Vu = np.zeros((ny, nu))
    Vu[nx:] = np.eye(nu)
    idxbx = np.arange(0, nx, 2)
    ocp = AcadosOcp()
    ocp.model.name = f"lti_{nx}x{nu}"
    ocp.model.disc_dyn_A, ocp.model.disc_dyn_B, ocp.model.disc_dyn_c = A, B, c
    ocp.cost.W = np.diag(w)
    ocp.cost.W_e = np.diag(w[:nx])
    ocp.cost.Vx, ocp.cost.Vu, ocp.cost.Vx_e = Vx, Vu, np.eye(nx)
    ocp.cost.yref, ocp.cost.yref_e = np.zeros(ny), np.zeros(nx)
    ocp.constraints.lbu, ocp.constraints.ubu, ocp.constraints.idxbu = -np.ones(nu), np.ones(nu), np.arange(nu)
    ocp.constraints.lbx, ocp.constraints.ubx = -2.0 * np.ones(idxbx.size), 2.0 * np.ones(idxbx.size)
    ocp.constraints.idxbx = idxbx
    ocp.constraints.x0 = np.zeros(nx)
    o = ocp.solver_options
    o.integrator_type = "DISCRETE"
    o.N_horizon, o.tf = N, 0.1 * N
    o.cost_scaling = "none"
    spec = models.OcpSpec(name=ocp.model.name, nx=nx, nu=nu, N=N, h=0.1, A_c=None, B_c=None, c_c=None,
                          integrator=None, W=np.diag(w), W_e=np.diag(w[:nx]), Vx=Vx, Vu=Vu, Vx_e=np.eye(nx),
                          lbu=-np.ones(nu), ubu=np.ones(nu), idxbu=np.arange(nu), lbx=-2.0 * np.ones(idxbx.size),
                          ubx=2.0 * np.ones(idxbx.size), idxbx=idxbx, cost_scaling="none", A=A, B=B, c=c)
    return ocp, spec, rng


@pytest.mark.parametrize("nx,nu,N", [(5, 3, 10), (3, 1, 25), (8, 5, 12), (7, 2, 30)])
def test_random_lti_dimension_generic(nx, nu, N):
    """No stage-wise kernel is compiled for these (nx, nu): nmpc_create picks the condensed
    family by itself (no env override) and the solutions match the certified oracle."""
    ocp, spec, rng = random_lti(nx, nu, N, seed=100 * nx + nu)
    B = 48
    x0 = rng.uniform(-1.5, 1.5, (B, nx))
    Y = rng.normal(0, 1.0, (B, N * (nx + nu) + nx))
    s = make(ocp, B, kernel=None)
    assert s.launch_info()["kernel"] == "cond_ipm_kernel"
    s.set_batch("x0", x0)
    s.set_batch("yref", Y)
    s.solve()
    status = s.get_batch_int("status")
    Xg, Ug, ok = [], [], []
    for b in range(B):
        o = qp.solve_ocp(spec, x0[b], Y[b, :N * (nx + nu)].reshape(N, nx + nu), Y[b, N * (nx + nu):])
        ok.append(o["certified"])
        Xg.append(o["X"])
        Ug.append(o["U"])
    ok = np.array(ok)
    assert ok.mean() > 0.9
    assert (status[ok] == 0).all(), status
    e = rel_err(s.get_batch("x")[ok], s.get_batch("u")[ok], np.array(Xg)[ok], np.array(Ug)[ok])
    print(f"random LTI nx={nx} nu={nu} N={N}: max rel err {e.max():.3e}, iters {s.get_batch_int('qp_iter').mean():.1f}")
    assert e.max() < TOL64, e.max()


@pytest.mark.parametrize("B", [1, 5, 1024])
def test_condensed_ragged_and_full_batches(B, golden_dir):
    """Ragged tails (B not a multiple of the workgroup) and the BASELINE config 2 batch."""
    from drone_attitude_control_amd.batched import first_step_qps, workload
    g = np.load(os.path.join(golden_dir, "bench_samples.npz"))
    table, off, x = workload("force", 20, 1024, seed=42)
    X0, Y = first_step_qps("force", 20, table, off, x)
    s = make(OCPS["force"](20), B)
    s.set_batch("x0", X0[:B])
    s.set_batch("yref", Y[:B])
    s.solve()
    assert (s.get_batch_int("status") == 0).all()
    idx = g["force_N20_B1024_idx"]
    keep = idx < B
    e = rel_err(s.get_batch("x")[idx[keep]], s.get_batch("u")[idx[keep]], g["force_N20_B1024_X"][keep],
                g["force_N20_B1024_U"][keep])
    assert e.max() < TOL64
