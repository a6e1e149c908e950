"""Controller models as discrete box-constrained LQ-OCPs (test infrastructure only).

Restates what acados builds from the reference's OCP description:
  * dynamics  — force: `force_model/dynamics.py:32-37` (x=[px,pz,vx,vz], u=[Fx,Fz]),
                jerk:  `jerk_model/dynamics.py:35-42` (x=[px,pz,vx,vz,ax,az], u=[hx,hz]);
  * discretisation — force: IRK (`force_model/ocp.py:85`, acados default Gauss-Legendre,
                4 stages), jerk: ERK with 1 stage (`jerk_model/ocp.py:86-87`) = explicit Euler;
                step h = tf/N = dt (`ocp.py:92-93`);
  * cost      — LINEAR_LS (`ocp.py:28-58`): stage k<N  s_k * 1/2 |Vx x + Vu u - yref_k|^2_W,
                terminal 1/2 |Vx_e x - yref_N|^2_We; acados scales the stage cost by the time
                step (s_k = h) and the terminal by 1 [ext, SURVEY Appendix B.1];
  * bounds    — u at stages 0..N-1, x at 1..N-1; stage 0 pins x0 (`ocp.py:62-78`,
                `controller.py:29-31`); no terminal bounds (lbx_e never set).

The discretisation here is the closed-form exact map (scipy expm of the augmented
generator) because Gauss-Legendre with s stages is exact whenever the augmented generator
is nilpotent of index <= 2s+1 — asserted below. The product code computes the same
matrices a different way (Butcher-tableau collocation solve), so the two cross-check.

`quad13` (nx=13, nu=4) has no reference counterpart: it is the synthetic hover-linearised
3-D quadrotor (p, v, q=[qw,qx,qy,qz], omega) that realises BASELINE.json's metric
dimensions. Inputs are the mass-normalised collective thrust and the
three body angular accelerations (well-scaled; torque = J * alpha).
"""
from dataclasses import dataclass, field

import numpy as np
import scipy.linalg

from . import params as P


@dataclass
class OcpSpec:
    name: str
    nx: int
    nu: int
    N: int
    h: float
    A_c: np.ndarray
    B_c: np.ndarray
    c_c: np.ndarray
    integrator: tuple          # ("IRK", stages) | ("ERK", stages)
    W: np.ndarray              # ny x ny
    W_e: np.ndarray            # nx x nx
    Vx: np.ndarray             # ny x nx
    Vu: np.ndarray             # ny x nu
    Vx_e: np.ndarray           # nx x nx
    lbu: np.ndarray
    ubu: np.ndarray
    idxbu: np.ndarray
    lbx: np.ndarray
    ubx: np.ndarray
    idxbx: np.ndarray
    lbx_e: np.ndarray = field(default_factory=lambda: np.zeros(0))
    ubx_e: np.ndarray = field(default_factory=lambda: np.zeros(0))
    idxbx_e: np.ndarray = field(default_factory=lambda: np.zeros(0, dtype=int))
    cost_scaling: str = "time_steps"
    A: np.ndarray = None
    B: np.ndarray = None
    c: np.ndarray = None

    @property
    def ny(self):
        return self.nx + self.nu

    def scaling(self):
        """Per-stage cost factors s_0..s_N."""
        s = np.ones(self.N + 1)
        if self.cost_scaling == "time_steps":
            s[: self.N] = self.h
        return s


def discretize(A_c, B_c, c_c, h, integrator):
    """Exact discrete map for affine dynamics x' = A_c x + B_c u + c_c with u held over h."""
    nx, nu = B_c.shape
    kind, stages = integrator
    if kind == "ERK" and stages == 1:
        # explicit Euler: one RK stage (jerk_model/ocp.py:86-87)
        return np.eye(nx) + h * A_c, h * B_c, h * c_c
    n = nx + nu + 1
    G = np.zeros((n, n))
    G[:nx, :nx] = A_c
    G[:nx, nx:nx + nu] = B_c
    G[:nx, -1] = c_c
    if kind == "IRK":
        # Gauss-Legendre s-stage is exact iff G is nilpotent of index <= 2s+1.
        Gk = np.eye(n)
        for _ in range(2 * stages + 1):
            Gk = Gk @ G
        assert np.allclose(Gk, 0.0), "oracle restates GL-IRK only where it is exact"
    elif kind == "ERK" and stages == 4:
        # classic RK4 on affine dynamics = 4th-order Taylor polynomial of the generator
        E = np.eye(n)
        term = np.eye(n)
        for k in range(1, 5):
            term = term @ (G * h) / k
            E = E + term
        return E[:nx, :nx], E[:nx, nx:nx + nu], E[:nx, -1]
    else:
        raise NotImplementedError(integrator)
    E = scipy.linalg.expm(G * h)
    return E[:nx, :nx], E[:nx, nx:nx + nu], E[:nx, -1]


def _ls_selectors(nx, nu):
    ny = nx + nu
    Vx = np.zeros((ny, nx))
    Vx[:nx] = np.eye(nx)
    Vu = np.zeros((ny, nu))
    Vu[nx:] = np.eye(nu)
    return Vx, Vu


def _finish(spec):
    spec.A, spec.B, spec.c = discretize(spec.A_c, spec.B_c, spec.c_c, spec.h, spec.integrator)
    return spec


def force_model(N=P.N_HORIZON, cost_scaling="time_steps"):
    """force_model/dynamics.py:32-37 + force_model/ocp.py:21-96."""
    nx, nu = 4, 2
    A_c = np.zeros((nx, nx))
    A_c[0, 2] = A_c[1, 3] = 1.0
    B_c = np.zeros((nx, nu))
    B_c[2, 0] = B_c[3, 1] = 1.0 / P.MASS
    c_c = np.array([0.0, 0.0, 0.0, -P.GRAVITY_ACC])
    Vx, Vu = _ls_selectors(nx, nu)
    W = np.diag(list(P.W_X_FORCE) + [P.W_U] * nu)          # ocp.py:38-46
    spec = OcpSpec(
        name="controllerModel_force", nx=nx, nu=nu, N=N, h=P.DT,
        A_c=A_c, B_c=B_c, c_c=c_c, integrator=("IRK", 4),
        W=W, W_e=np.diag(P.W_X_FORCE), Vx=Vx, Vu=Vu, Vx_e=np.eye(nx),
        lbu=np.array([P.MIN_F, P.MIN_F]), ubu=np.array([P.MAX_F, P.MAX_F]), idxbu=np.arange(nu),
        lbx=np.array([P.MIN_P_X, P.MIN_P_Z, P.MIN_V_X, P.MIN_V_Z]),
        ubx=np.array([P.MAX_P_X, P.MAX_P_Z, P.MAX_V_X, P.MAX_V_Z]), idxbx=np.arange(nx),
        cost_scaling=cost_scaling)
    return _finish(spec)


def jerk_model(N=P.N_HORIZON, cost_scaling="time_steps"):
    """jerk_model/dynamics.py:35-42 + jerk_model/ocp.py:20-95."""
    nx, nu = 6, 2
    A_c = np.zeros((nx, nx))
    A_c[0, 2] = A_c[1, 3] = A_c[2, 4] = A_c[3, 5] = 1.0
    B_c = np.zeros((nx, nu))
    B_c[4, 0] = B_c[5, 1] = 1.0
    c_c = np.array([0.0, 0.0, 0.0, -P.GRAVITY_ACC, 0.0, 0.0])
    Vx, Vu = _ls_selectors(nx, nu)
    W = np.diag(list(P.W_X_JERK) + [P.W_U] * nu)
    spec = OcpSpec(
        name="controllerModel_jerk", nx=nx, nu=nu, N=N, h=P.DT,
        A_c=A_c, B_c=B_c, c_c=c_c, integrator=("ERK", 1),
        W=W, W_e=np.diag(P.W_X_JERK), Vx=Vx, Vu=Vu, Vx_e=np.eye(nx),
        lbu=np.array([P.MIN_JERK, P.MIN_JERK]), ubu=np.array([P.MAX_JERK, P.MAX_JERK]),
        idxbu=np.arange(nu),
        lbx=np.array([P.MIN_P_X, P.MIN_P_Z, P.MIN_V_X, P.MIN_V_Z, P.MIN_A_X, P.MIN_A_Z]),
        ubx=np.array([P.MAX_P_X, P.MAX_P_Z, P.MAX_V_X, P.MAX_V_Z, P.MAX_A_X, P.MAX_A_Z]),
        idxbx=np.arange(nx), cost_scaling=cost_scaling)
    return _finish(spec)


# quad13 input bounds: collective thrust acceleration in [0, T/W * g]; body angular
# acceleration bounded well inside the URDF torque limit (L*KF*RPM_max^2 / J ~ 500 rad/s^2)
QUAD13_ALPHA_MAX = 100.0
QUAD13_OMEGA_MAX = 10.0


def quad13_model(N=20, cost_scaling="time_steps"):
    """Synthetic hover-linearised quadrotor: x=[p(3), v(3), q(4), w(3)], u=[aT, alpha(3)].

    p' = v;  v' = [2g qy, -2g qx, aT - g];  q' = [0, wx/2, wy/2, wz/2];  w' = alpha.
    """
    nx, nu = 13, 4
    g = P.GRAVITY_ACC
    A_c = np.zeros((nx, nx))
    A_c[0, 3] = A_c[1, 4] = A_c[2, 5] = 1.0          # p' = v
    A_c[3, 8] = 2 * g                                # vx' = 2 g qy
    A_c[4, 7] = -2 * g                               # vy' = -2 g qx
    A_c[7, 10] = A_c[8, 11] = A_c[9, 12] = 0.5       # q' = 1/2 w
    B_c = np.zeros((nx, nu))
    B_c[5, 0] = 1.0                                  # vz' = aT - g
    B_c[10, 1] = B_c[11, 2] = B_c[12, 3] = 1.0       # w' = alpha
    c_c = np.zeros(nx)
    c_c[5] = -g
    Vx, Vu = _ls_selectors(nx, nu)
    w_x = [1e2] * 3 + [1e0] * 3 + [1e0] * 4 + [1e-1] * 3
    w_u = [1e-1] + [1e-2] * 3
    W = np.diag(w_x + w_u)
    inf_box = [P.MIN_P_X] * 3, [P.MAX_P_X] * 3
    lbx = np.array(inf_box[0] + [P.MIN_V_X] * 3 + [-QUAD13_OMEGA_MAX] * 3)
    ubx = np.array(inf_box[1] + [P.MAX_V_X] * 3 + [QUAD13_OMEGA_MAX] * 3)
    idxbx = np.array([0, 1, 2, 3, 4, 5, 10, 11, 12])
    spec = OcpSpec(
        name="quad13", nx=nx, nu=nu, N=N, h=P.DT,
        A_c=A_c, B_c=B_c, c_c=c_c, integrator=("IRK", 4),
        W=W, W_e=np.diag(w_x), Vx=Vx, Vu=Vu, Vx_e=np.eye(nx),
        lbu=np.array([0.0] + [-QUAD13_ALPHA_MAX] * 3),
        ubu=np.array([P.THRUST2WEIGHT * g] + [QUAD13_ALPHA_MAX] * 3), idxbu=np.arange(nu),
        lbx=lbx, ubx=ubx, idxbx=idxbx, cost_scaling=cost_scaling)
    return _finish(spec)


MODELS = {"force": force_model, "jerk": jerk_model, "quad13": quad13_model}


def quad13_reference(n_rows, N_horizon):
    """3-D extension of the reference circle for quad13: the x-z circle of
    generate_trajectory.py:7-28 with y = 0, level attitude q = [1,0,0,0], w = 0 and hover
    thrust aT = g. Returns (n_rows + N_horizon) x 17."""
    from .trajectory import gen_circle_traj
    base = gen_circle_traj(n_rows, N_horizon, nx=6, nu=2)
    ref = np.zeros((base.shape[0], 17))
    ref[:, 0] = base[:, 0]
    ref[:, 2] = base[:, 1]
    ref[:, 3] = base[:, 2]
    ref[:, 5] = base[:, 3]
    ref[:, 6] = 1.0
    ref[:, 13] = P.GRAVITY_ACC
    return ref
