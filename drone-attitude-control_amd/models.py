"""OCP builders for the controller models, written against the acados-compatible façade.

`force_ocp` / `jerk_ocp` follow the reference's `OCP.create_ocp` + `create_ocp_solver`
(force_model/ocp.py:21-96 with dynamics force_model/dynamics.py:32-47;
jerk_model/ocp.py:20-95 with dynamics jerk_model/dynamics.py:35-52) field for field.
`quad13_ocp` is the synthetic nx=13, nu=4 hover-linearised quadrotor that realises the
headline metric's dimensions (BASELINE.json) — it has no reference counterpart.
`PlantModel` mirrors src/plant.py:8-43 for AcadosSimSolver.
"""
import numpy as np

from .acados import AcadosModel, AcadosOcp
from .params import DroneData, ExperimentParameters

dd = DroneData()
p = ExperimentParameters()


def _ls(ocp, nx, nu, w_x, w_x_e, w_u):
    ny = nx + nu
    ocp.cost.cost_type = "LINEAR_LS"
    ocp.cost.cost_type_e = "LINEAR_LS"
    Q = np.diag(w_x)
    R = np.diag(w_u)
    ocp.cost.W = np.block([[Q, np.zeros((nx, nu))], [np.zeros((nu, nx)), R]])
    ocp.cost.W_e = np.diag(w_x_e)
    ocp.cost.Vx = np.zeros((ny, nx))
    ocp.cost.Vx[:nx, :] = np.eye(nx)
    ocp.cost.Vu = np.zeros((ny, nu))
    ocp.cost.Vu[nx:, :] = np.eye(nu)
    ocp.cost.Vx_e = np.eye(nx)
    ocp.cost.yref = np.zeros((ny,))
    ocp.cost.yref_e = np.zeros((nx,))


def force_model():
    """ControllerModel of force_model/dynamics.py:22-47: x=[px,pz,vx,vz], u=[Fx,Fz],
    x' = [vx, vz, Fx/m, Fz/m - g]."""
    m = AcadosModel()
    m.name = "controllerModel_force"
    m.A_c = np.zeros((4, 4))
    m.A_c[0, 2] = m.A_c[1, 3] = 1.0
    m.B_c = np.zeros((4, 2))
    m.B_c[2, 0] = m.B_c[3, 1] = 1.0 / dd.MASS
    m.c_c = np.array([0.0, 0.0, 0.0, -dd.GRAVITY_ACC])
    m.x = np.zeros(4)
    m.u = np.zeros(2)
    return m


def jerk_model():
    """ControllerModel of jerk_model/dynamics.py:22-52: x=[px,pz,vx,vz,ax,az], u=[hx,hz]."""
    m = AcadosModel()
    m.name = "controllerModel_jerk"
    m.A_c = np.zeros((6, 6))
    m.A_c[0, 2] = m.A_c[1, 3] = m.A_c[2, 4] = m.A_c[3, 5] = 1.0
    m.B_c = np.zeros((6, 2))
    m.B_c[4, 0] = m.B_c[5, 1] = 1.0
    m.c_c = np.array([0.0, 0.0, 0.0, -dd.GRAVITY_ACC, 0.0, 0.0])
    m.x = np.zeros(6)
    m.u = np.zeros(2)
    return m


def force_ocp(N=p.N_horizon):
    """force_model/ocp.py:21-93."""
    ocp = AcadosOcp()
    ocp.code_export_directory = "c_generated_code_acados_ocp"
    ocp.model = force_model()
    nx, nu = 4, 2
    _ls(ocp, nx, nu, [1e2, 1e2, 1e0, 1e0], [1e2, 1e2, 1e0, 1e0], [1e-1] * nu)
    c = ocp.constraints
    c.constr_type = c.constr_type_e = "BGH"
    c.lbu = np.array([dd.min_F, dd.min_F])
    c.ubu = np.array([dd.max_F, dd.max_F])
    c.idxbu = np.array([0, 1])
    c.lbx = np.array([dd.min_p_x, dd.min_p_z, dd.min_v_x, dd.min_v_z])
    c.ubx = np.array([dd.max_p_x, dd.max_p_z, dd.max_v_x, dd.max_v_z])
    c.idxbx = np.array([0, 1, 2, 3])
    c.x0 = np.zeros(nx)
    o = ocp.solver_options
    o.qp_solver = "PARTIAL_CONDENSING_HPIPM"
    o.hessian_approx = "GAUSS_NEWTON"
    o.integrator_type = "IRK"
    o.nlp_solver_type = "SQP"
    o.print_level = 0
    o.N_horizon = N
    o.tf = p.dt * N
    return ocp


def jerk_ocp(N=p.N_horizon):
    """jerk_model/ocp.py:20-92."""
    ocp = AcadosOcp()
    ocp.code_export_directory = "c_generated_code_acados_ocp"
    ocp.model = jerk_model()
    nx, nu = 6, 2
    _ls(ocp, nx, nu, [1e2, 1e2, 1e0, 1e0, 0, 0], [1e2, 1e2, 1e0, 1e0, 0, 0], [1e-1] * nu)
    c = ocp.constraints
    c.constr_type = c.constr_type_e = "BGH"
    c.lbu = np.array([dd.min_jerk, dd.min_jerk])
    c.ubu = np.array([dd.max_jerk, dd.max_jerk])
    c.idxbu = np.array([0, 1])
    c.lbx = np.array([dd.min_p_x, dd.min_p_z, dd.min_v_x, dd.min_v_z, dd.min_a_x, dd.min_a_z])
    c.ubx = np.array([dd.max_p_x, dd.max_p_z, dd.max_v_x, dd.max_v_z, dd.max_a_x, dd.max_a_z])
    c.idxbx = np.array([0, 1, 2, 3, 4, 5])
    c.x0 = np.zeros(nx)
    o = ocp.solver_options
    o.qp_solver = "PARTIAL_CONDENSING_HPIPM"
    o.hessian_approx = "GAUSS_NEWTON"
    o.integrator_type = "ERK"
    o.sim_method_num_stages = 1
    o.nlp_solver_type = "SQP"
    o.print_level = 0
    o.N_horizon = N
    o.tf = p.dt * N
    return ocp


QUAD13_ALPHA_MAX = 100.0
QUAD13_OMEGA_MAX = 10.0


def quad13_model():
    """x=[p(3), v(3), q=[qw,qx,qy,qz], w(3)], u=[aT, alpha(3)] linearised at hover:
    p' = v, v' = [2g qy, -2g qx, aT - g], q' = [0, w/2], w' = alpha."""
    g = dd.GRAVITY_ACC
    m = AcadosModel()
    m.name = "quad13"
    A = np.zeros((13, 13))
    A[0, 3] = A[1, 4] = A[2, 5] = 1.0
    A[3, 8] = 2 * g
    A[4, 7] = -2 * g
    A[7, 10] = A[8, 11] = A[9, 12] = 0.5
    B = np.zeros((13, 4))
    B[5, 0] = 1.0
    B[10, 1] = B[11, 2] = B[12, 3] = 1.0
    c = np.zeros(13)
    c[5] = -g
    m.A_c, m.B_c, m.c_c = A, B, c
    m.x = np.zeros(13)
    m.u = np.zeros(4)
    return m


def quad13_ocp(N=20):
    g = dd.GRAVITY_ACC
    ocp = AcadosOcp()
    ocp.model = quad13_model()
    nx, nu = 13, 4
    w_x = [1e2] * 3 + [1e0] * 3 + [1e0] * 4 + [1e-1] * 3
    _ls(ocp, nx, nu, w_x, w_x, [1e-1] + [1e-2] * 3)
    c = ocp.constraints
    c.lbu = np.array([0.0] + [-QUAD13_ALPHA_MAX] * 3)
    c.ubu = np.array([dd.THRUST2WEIGHT_RATIO * g] + [QUAD13_ALPHA_MAX] * 3)
    c.idxbu = np.arange(4)
    c.lbx = np.array([dd.min_p_x] * 3 + [dd.min_v_x] * 3 + [-QUAD13_OMEGA_MAX] * 3)
    c.ubx = np.array([dd.max_p_x] * 3 + [dd.max_v_x] * 3 + [QUAD13_OMEGA_MAX] * 3)
    c.idxbx = np.array([0, 1, 2, 3, 4, 5, 10, 11, 12])
    c.x0 = np.zeros(nx)
    o = ocp.solver_options
    o.integrator_type = "IRK"
    o.sim_method_num_stages = 4
    o.N_horizon = N
    o.tf = p.dt * N
    # IPM tolerances (solver options, like acados's qp_solver_tol_*): the well-conditioned quad13
    # OCP meets the 1e-6 parity bar with > 300x margin at mu <= 1e-12 (max
    # deviation 3e-9 on the golden cases, 7e-11 on the 8192 bench instances, vs ~1e-15 / 1e-12
    # solves); the force OCP (condition ~4e4) keeps the library default 1e-15 / 1e-12
    o.qp_solver_tol_comp = 1e-12
    o.qp_solver_tol_stat = 1e-10
    return ocp


OCPS = {"force": force_ocp, "jerk": jerk_ocp, "quad13": quad13_ocp}


class PlantModel:
    """src/plant.py:8-43: x=[px,pz,vx,vz], u=[theta,F_d],
    x' = [vx, vz, F_d sin(theta)/m, F_d cos(theta)/m - g]. `noise` is ignored (plant.py:10)."""

    def __init__(self, noise=True):
        self.model = AcadosModel()
        self.model.name = "plantModel"
        self.model.x = np.zeros(4)
        self.model.u = np.zeros(2)
        self.model.plant_mass = dd.MASS
        self.model.plant_g = dd.GRAVITY_ACC


def gen_circle_traj(N, N_horizon, nx, nu, center=(0.0, 0.0), radius=1.0):
    """Reference table of generate_trajectory.py:7-28 (host-side copy for the drivers)."""
    ref = np.empty((N + N_horizon, nx + nu), dtype=float)
    omega = 2 * np.pi / p.T
    i = np.linspace(0, p.T, N)
    ref[:N, 0] = center[0] + radius * np.cos(omega * i)
    ref[:N, 1] = center[1] + radius * np.sin(omega * i)
    ref[:N, 2] = -radius * omega * np.sin(omega * i)
    ref[:N, 3] = radius * omega * np.cos(omega * i)
    if nx in (4, 6):
        ref[:N, 4] = -radius * omega ** 2 * np.cos(omega * i)
        ref[:N, 5] = -radius * omega ** 2 * np.sin(omega * i) + dd.GRAVITY_ACC
    else:
        raise ValueError("Invalid dimensions")
    if nx == 6:
        ref[:N, 6] = 0
        ref[:N, 7] = 0
    ref[N:] = ref[:N_horizon]
    return ref


def quad13_reference(n_rows, N_horizon):
    """3-D extension of the reference circle for quad13 (y = 0, level attitude, hover thrust)."""
    base = gen_circle_traj(n_rows, N_horizon, nx=6, nu=2)
    ref = np.zeros((base.shape[0], 17))
    ref[:, 0] = base[:, 0]
    ref[:, 2] = base[:, 1]
    ref[:, 3] = base[:, 2]
    ref[:, 5] = base[:, 3]
    ref[:, 6] = 1.0
    ref[:, 13] = dd.GRAVITY_ACC
    return ref
