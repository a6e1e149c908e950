"""GPU parity tests of the HIP engine (run on the MI355X box with `pytest -m gpu`).

Every test goes through the C-ABI (libnmpc_hip.so) via the façade. Expected values come
from the KKT-certified dense oracle (tests/golden/qp_cases.npz, oracle/qp.py) and the
plain-C Riccati IPM (oracle/c). Tolerance (BASELINE.json north_star): 1e-6 relative on the
x/u trajectories, measured as max|z_gpu - z_ref| / max(1, max|z_ref|) per instance, fp64.
fp32 handles: the IPM in fp32, then the exact finish (nmpc_cl_fast.hip fin32_*: z_0 = [T_x | V_y][x0; yref]
+ v_c on the f32 matrix cores, PDAS / dual active-set steps on the fp64 W with fp64 acceptance). Their bar
TOL32 = 2e-5: the finish returns the exact solution of the fp32-rounded data, whose
distance from the fp64 solution is the rounding of z_0 (a few fp32 ulps of |T_x x0| + |V_y yref| ~ 1-10)
carried through W[:, S] W_SS^-1 — not amplified by cond(W_SS) ~ 4e4, since W and the solves are fp64.
Measured max 4.6e-6 (force), 1.6e-6 (jerk), 4.2e-6 (quad13); the fp32 IPM alone was 1e-4 .. 1e-2.
"""
import os

import numpy as np
import pytest

from drone_attitude_control_amd import AcadosOcpSolver
from drone_attitude_control_amd.models import OCPS
from oracle import cref, models, qp

pytestmark = pytest.mark.gpu

KEYS = ["force_N20", "force_N30", "jerk_N40", "jerk_N30", "quad13_N20"]
TOL64 = 1e-6
TOL32 = 2e-5


@pytest.fixture(scope="module")
def cases(golden_dir):
    return np.load(os.path.join(golden_dir, "qp_cases.npz"))


def split(key):
    name, N = key.split("_N")
    return name, int(N)


def rel_err(X, U, Xr, Ur):
    scale = np.maximum(1.0, np.maximum(np.abs(Xr).max(axis=(-2, -1)), np.abs(Ur).max(axis=(-2, -1))))
    err = np.maximum(np.abs(X - Xr).max(axis=(-2, -1)), np.abs(U - Ur).max(axis=(-2, -1)))
    return err / scale


def solve_batch(key, cases, precision="fp64", reps=1, ipw=None, kernel=None, structure=True, fast=True, env=None):
    """kernel: None (default family: lane-per-component), "wave" (wavefront-per-instance,
    with ipw instances per wavefront) or "lpc" — an explicit family also selects that family's full
    IPM for the solve; structure=False forces the dense lane-per-component kernel instead of the
    model-structure-specialised one. fast=False: the full IPM + exact finish instead of the fp64 fast
    solve (sf_kernel + fin64_kernel, NMPC_SOLVE_FAST=0). env: extra environment for the handle's
    lifetime (read at create and at each solve)."""
    name, N = split(key)
    x0 = np.tile(cases[key + "_x0"], (reps, 1))
    y = np.tile(cases[key + "_yref"], (reps, 1))
    set_env = dict(env or {})
    if ipw:
        set_env["NMPC_IPW"] = str(ipw)
    if kernel:
        set_env["NMPC_KERNEL"] = kernel
    if not structure:
        set_env["NMPC_STRUCT"] = "0"
    if not fast:
        set_env["NMPC_SOLVE_FAST"] = "0"
    os.environ.update(set_env)
    try:
        s = AcadosOcpSolver(OCPS[name](N), batch=x0.shape[0], precision=precision)
        s.set_batch("x0", x0)
        s.set_batch("yref", y)
        st = s.solve()
    finally:
        for k_ in set_env:
            os.environ.pop(k_, None)
    return s, st



@pytest.mark.parametrize("key", KEYS)
def test_batch_parity_fp64(key, cases):
    """The fp64 solve (the fast path: unconstrained solution on the shared factorisation, sf_kernel, then the
    active-set finish, fin64_kernel) against the certified oracle, with the same Newton-system counts as the C
    restatement of that algorithm (riccati_ipm_solve_batch_fast) — and the full IPM + exact finish
    (NMPC_SOLVE_FAST=0) with the counts of the C cold solve (+-1 from rounding order)."""
    name, N = split(key)
    o = OCPS[name](N).solver_options   # the OCP's IPM tolerances (quad13 sets its own) + exact finish
    R = cref.RiccatiIpmRef.for_options(models.MODELS[name](N), o)
    for fast in (True, False):
        s, st = solve_batch(key, cases, fast=fast)
        assert st == 0
        assert s.launch_info()["solve_kernel"] == ("sf_kernel" if fast else s.launch_info()["kernel"])
        X, U = s.get_batch("x"), s.get_batch("u")
        e = rel_err(X, U, cases[key + "_X"], cases[key + "_U"])
        assert e.max() < TOL64, (fast, e.max())
        if fast:
            _, _, stc, itc, cnt = R.solve_fast(cases[key + "_x0"], cases[key + "_yref"], wsmax=cref.WSMAX[name])
            assert cnt["full"] == 0
        else:
            _, _, stc, itc = R.solve(cases[key + "_x0"], cases[key + "_yref"])
        it = s.get_batch_int("qp_iter")
        assert np.abs(it - itc).max() <= (0 if fast else 1), (fast, it, itc)


@pytest.mark.parametrize("key", ["force_N20", "jerk_N40", "quad13_N20"])
def test_fast_solve_parks_take_the_full_solve(key, cases):
    """The fast solve's last resort: with the dual fallback off (NMPC_CLF_NO_GI=1) every instance whose PDAS
    rounds do not settle parks, and the full IPM (ipm_lpc_kernel in list mode, cold) solves it; the batch still
    matches the certified oracle, and the parked instances carry the full solve's Newton-system counts."""
    s, st = solve_batch(key, cases, env={"NMPC_CLF_NO_GI": "1"})
    assert st == 0 and s.launch_info()["solve_kernel"] == "sf_kernel"
    e = rel_err(s.get_batch("x"), s.get_batch("u"), cases[key + "_X"], cases[key + "_U"])
    assert e.max() < TOL64, e.max()


RT_KEYS = ["force_N10", "force_N3", "jerk_N20", "quad13_N30"]


@pytest.mark.parametrize("key", RT_KEYS)
@pytest.mark.parametrize("no_gi", [False, True])
def test_fast_solve_runtime_horizons(key, no_gi, golden_dir):
    """The fast solve at horizons without a compiled (fully unrolled) sf_kernel: the runtime-horizon variants
    (four-stage two-slot LDS ring, the register ring indexed at run time; N = 3 is a single slot, shorter than a
    chunk). Against the certified oracle on tests/golden/qp_cases_rt.npz (make_qp_golden.py qp_rt), with the
    C restatement's Newton-system counts; no_gi: the dual fallback off, so unsettled instances park and take
    the list-mode full IPM."""
    cases = np.load(os.path.join(golden_dir, "qp_cases_rt.npz"))
    name, N = split(key)
    env = {"NMPC_CLF_NO_GI": "1"} if no_gi else None
    s, st = solve_batch(key, cases, env=env)
    assert s.launch_info()["solve_kernel"] == "sf_kernel"
    assert st == 0
    e = rel_err(s.get_batch("x"), s.get_batch("u"), cases[key + "_X"], cases[key + "_U"])
    assert e.max() < TOL64, e.max()
    if not no_gi:
        R = cref.RiccatiIpmRef.for_options(models.MODELS[name](N), OCPS[name](N).solver_options)
        _, _, stc, itc, cnt = R.solve_fast(cases[key + "_x0"], cases[key + "_yref"], wsmax=cref.WSMAX[name])
        assert cnt["full"] == 0
        assert np.array_equal(s.get_batch_int("qp_iter"), itc)


def _hip():
    """The HIP runtime libnmpc_hip.so already loaded (same soname: the same runtime and device context)."""
    import ctypes
    from drone_attitude_control_amd import _lib
    _lib.load()
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipStreamCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    return hip


@pytest.mark.parametrize("key", ["force_N20", "jerk_N40", "quad13_N20"])
def test_solve_async_is_complete_in_stream_order(key, cases):
    """nmpc_solve_async on a caller's stream (nmpc_set_stream), then hipMemcpyAsync of the device x / u on that
    stream and a plain hipStreamSynchronize — no nmpc_synchronize, no host step of the engine in between. With
    the dual fallback off (NMPC_CLF_NO_GI=1) instances park, so the copy is correct only if the parked
    instances' full IPM ran in stream order before it (src/force_model/controller.py:32-39: solve() returns a
    finished solution). Twice back to back: the second solve's copies are final too."""
    import ctypes
    name, N = split(key)
    x0, y = cases[key + "_x0"], cases[key + "_yref"]
    B = x0.shape[0]
    os.environ["NMPC_CLF_NO_GI"] = "1"
    hip = _hip()
    stream = ctypes.c_void_p()
    assert hip.hipStreamCreate(ctypes.byref(stream)) == 0
    try:
        s = AcadosOcpSolver(OCPS[name](N), batch=B)
        assert s.launch_info()["solve_kernel"] == "sf_kernel"
        s.set_stream(stream.value)
        s.set_batch("x0", x0)
        s.set_batch("yref", y)
        s.solve()                       # stages the inputs in HBM (and one complete solve)
        for rep in range(2):
            X = np.zeros((B, N + 1, s.nx))
            U = np.zeros((B, N, s.nu))
            st = np.zeros(B, dtype=np.int32)
            s.solve_async()
            for host, field in ((X, "x"), (U, "u"), (st, "status")):
                assert hip.hipMemcpyAsync(host.ctypes.data, s.device_ptr(field), host.nbytes, 2, stream) == 0
            assert hip.hipStreamSynchronize(stream) == 0
            assert (st == 0).all(), st
            e = rel_err(X, U, cases[key + "_X"], cases[key + "_U"])
            assert e.max() < TOL64, (rep, e.max())
        s.synchronize()
        parked, listed = s.get_stats("fast_parked"), s.get_stats("fast_listed")
        print(f"{key}: listed {listed}, parked {parked} of {B}")
        if name == "force":
            assert parked > 0, "the test needs parked instances"
        s.set_stream(0)
    finally:
        os.environ.pop("NMPC_CLF_NO_GI", None)
        hip.hipStreamDestroy(stream)


@pytest.mark.parametrize("key", ["force_N20", "jerk_N40"])
@pytest.mark.parametrize("ipw", [1, 2, 4])
def test_instance_packing_variants(key, ipw, cases):
    """Every compiled lane-group width of the wavefront-per-instance family gives the same
    answer (tail groups included)."""
    s, st = solve_batch(key, cases, reps=1, ipw=ipw, kernel="wave")
    assert s.launch_info()["instances_per_wave"] == ipw
    assert st == 0
    e = rel_err(s.get_batch("x"), s.get_batch("u"), cases[key + "_X"], cases[key + "_U"])
    assert e.max() < TOL64


@pytest.mark.parametrize("key", KEYS)
@pytest.mark.parametrize("precision", ["fp64", "fp32"])
def test_kernel_families_agree(key, precision, cases):
    """Lane-per-component (default) and wavefront-per-instance kernels: same statuses, same
    iterates to rounding, both within the oracle bar."""
    a, sa = solve_batch(key, cases, precision=precision, kernel="lpc")
    b, sb = solve_batch(key, cases, precision=precision, kernel="wave")
    assert a.launch_info()["instances_per_wave"] == 64 // (a.nx + a.nu)
    assert (a.get_batch_int("status") == b.get_batch_int("status")).all()
    tol = TOL64 if precision == "fp64" else TOL32
    ea = rel_err(a.get_batch("x"), a.get_batch("u"), cases[key + "_X"], cases[key + "_U"])
    eb = rel_err(b.get_batch("x"), b.get_batch("u"), cases[key + "_X"], cases[key + "_U"])
    assert ea.max() < tol and eb.max() < tol, (ea.max(), eb.max())


@pytest.mark.parametrize("key", KEYS)
def test_structure_specialised_matches_dense(key, cases):
    """The model-structure-specialised lane-per-component kernel (chosen whenever that family
    runs: every shipped model fits its compiled [A B] mask and diagonal cost) and the dense one
    agree to rounding."""
    a, sa = solve_batch(key, cases, kernel="lpc")
    b, sb = solve_batch(key, cases, kernel="lpc", structure=False)
    assert a.launch_info()["structure"] == split(key)[0]
    assert b.launch_info()["structure"] == "dense"
    assert sa == 0 and sb == 0
    # both follow the same algorithm, but FMA order (sparse vs dense products) perturbs the
    # step-length heuristics, so the iterate paths agree to the solver tolerance, not bitwise;
    # 1e-7 is 10x inside the oracle bar each of them meets
    for f in ("x", "u"):
        A, B = a.get_batch(f), b.get_batch(f)
        assert np.abs(A - B).max() <= 1e-7 * max(1.0, np.abs(B).max())
    ea = rel_err(a.get_batch("x"), a.get_batch("u"), cases[key + "_X"], cases[key + "_U"])
    eb = rel_err(b.get_batch("x"), b.get_batch("u"), cases[key + "_X"], cases[key + "_U"])
    assert ea.max() < TOL64 and eb.max() < TOL64


@pytest.mark.parametrize("key", ["force_N20", "force_N30", "jerk_N40", "jerk_N30"])
@pytest.mark.parametrize("precision", ["fp64", "fp32"])
@pytest.mark.parametrize("W", [1, 3, 64])
def test_lane_per_instance_family(key, precision, W, cases):
    """The lane-per-instance kernels (nmpc_ipm_lpi.hip, one lane = one instance, W instances per
    wavefront — 1, a ragged 3 and a full 64) against the certified oracle, with the same
    iteration counts as the C baseline (same algorithm, +-1 from rounding order)."""
    os.environ["NMPC_LPI_W"] = str(W)
    try:
        s, st = solve_batch(key, cases, precision=precision, kernel="lpi")
    finally:
        os.environ.pop("NMPC_LPI_W", None)
    assert s.launch_info()["kernel"] == "ipm_lpi_kernel"
    assert s.launch_info()["instances_per_wave"] == W
    status = s.get_batch_int("status")
    assert (status == 0).all(), status
    e = rel_err(s.get_batch("x"), s.get_batch("u"), cases[key + "_X"], cases[key + "_U"])
    assert e.max() < (TOL64 if precision == "fp64" else TOL32), e.max()
    if precision == "fp64":
        name, N = split(key)
        _, _, _, itc = cref.RiccatiIpmRef(models.MODELS[name](N)).solve(cases[key + "_x0"], cases[key + "_yref"])
        assert np.abs(s.get_batch_int("qp_iter") - itc).max() <= 1


def test_default_family_is_batch_aware(cases):
    """quad13 always runs lane-per-component; the small force model switches to it only when
    the batch fills enough wavefronts (nmpc_ipm.hip kernel_kind)."""
    key = "force_N20"
    s, _ = solve_batch(key, cases)
    assert s.launch_info()["kernel"] == "ipm_kernel"
    s, _ = solve_batch(key, cases, reps=8192 // cases[key + "_x0"].shape[0] + 1)
    assert s.launch_info()["kernel"] == "ipm_lpc_kernel"
    s, _ = solve_batch("quad13_N20", cases)
    assert s.launch_info()["kernel"] == "ipm_lpc_kernel"


def test_ragged_batch(cases):
    key = "force_N20"
    name, N = split(key)
    for B in (1, 3, 37):
        s = AcadosOcpSolver(OCPS[name](N), batch=B)
        s.set_batch("x0", cases[key + "_x0"][:B])
        s.set_batch("yref", cases[key + "_yref"][:B])
        assert s.solve() == 0
        e = rel_err(s.get_batch("x"), s.get_batch("u"), cases[key + "_X"][:B], cases[key + "_U"][:B])
        assert e.max() < TOL64


def test_acados_call_pattern_and_cost(cases):
    """The reference's own per-stage call sequence (ocp.py:117-122, controller.py:29-39)."""
    key = "jerk_N30"
    name, N = split(key)
    spec = models.MODELS[name](N)
    s = AcadosOcpSolver(OCPS[name](N))
    for b in range(4):
        y = cases[key + "_yref"][b]
        for k in range(N):
            s.set(k, "yref", y[k * spec.ny:(k + 1) * spec.ny])
        s.set(N, "yref", y[N * spec.ny:])
        s.set(0, "lbx", cases[key + "_x0"][b])
        s.set(0, "ubx", cases[key + "_x0"][b])
        assert s.solve() == 0
        X = np.array([s.get(k, "x") for k in range(N + 1)])
        U = np.array([s.get(k, "u") for k in range(N)])
        assert rel_err(X, U, cases[key + "_X"][b], cases[key + "_U"][b]) < TOL64
        assert s.get_cost() == pytest.approx(float(cases[key + "_cost"][b]), rel=1e-8, abs=1e-10)
    assert s.get_stats("sqp_iter") == 1 and s.get_stats("qp_iter") > 0


def test_errors_behave_like_acados(cases):
    s = AcadosOcpSolver(OCPS["force"](20))
    with pytest.raises(Exception):
        s.set(0, "yref", np.zeros(5))          # wrong size
    with pytest.raises(Exception):
        s.set(0, "not_a_field", np.zeros(6))
    with pytest.raises(Exception):
        s.get(0, "x")                          # nothing solved yet
    s.set(0, "lbx", np.zeros(4))
    s.set(0, "ubx", np.ones(4))
    with pytest.raises(Exception, match="lbx != ubx"):
        s.solve()


@pytest.mark.parametrize("name", ["force", "jerk", "quad13"])
def test_discrete_model_matches_oracle(name):
    """The library's native integrator sensitivities (Butcher collocation) == oracle."""
    s = AcadosOcpSolver(OCPS[name](20))
    A, B, c = s.discrete_model()
    spec = models.MODELS[name](20)
    assert np.allclose(A, spec.A, rtol=1e-12, atol=1e-14)
    assert np.allclose(B, spec.B, rtol=1e-12, atol=1e-14)
    assert np.allclose(c, spec.c, rtol=1e-12, atol=1e-14)


@pytest.mark.parametrize("key", ["force_N20", "jerk_N40", "quad13_N20"])
def test_fp32_throughput_config(key, cases):
    """fp32 (BASELINE config 3's precision): every golden case converges (status 0) and stays
    within the fp32 bar of the exact fp64 solution."""
    s, st = solve_batch(key, cases, precision="fp32")
    status = s.get_batch_int("status")
    assert (status == 0).all(), status
    e = rel_err(s.get_batch("x"), s.get_batch("u"), cases[key + "_X"], cases[key + "_U"])
    print(f"fp32 {key}: max rel err {e.max():.3e}, median {np.median(e):.3e}")
    assert e.max() < TOL32, e.max()


BENCH = [("force", 20, 1024, "fp64"), ("force", 20, 8192, "fp32"), ("force", 20, 8192, "fp64"),
         ("jerk", 40, 4096, "fp64"), ("quad13", 20, 8192, "fp64")]


@pytest.mark.parametrize("name,N,B,precision", BENCH)
def test_bench_size_batch_matches_certified_sample(name, N, B, precision, golden_dir):
    """BASELINE.json configs at full size: the bench's first-step QPs for the WHOLE batch
    (batched.workload seed 42 -> first_step_qps) solved in one launch of the engine's default
    kernel; 64 instances spread over the batch against KKT-certified oracle solutions
    (tests/golden/bench_samples.npz, make_bench_samples.py). fp64 bar 1e-6, fp32 bar TOL32."""
    from drone_attitude_control_amd.batched import first_step_qps, workload
    g = np.load(os.path.join(golden_dir, "bench_samples.npz"))
    key = f"{name}_N{N}_B{B}"
    table, off, x = workload(name, N, B, seed=42)
    X0, Y = first_step_qps(name, N, table, off, x)
    s = AcadosOcpSolver(OCPS[name](N), batch=B, precision=precision)
    s.set_batch("x0", X0)
    s.set_batch("yref", Y)
    s.solve()
    status = s.get_batch_int("status")
    idx = g[key + "_idx"]
    assert g[key + "_certified"].all()
    assert (status[idx] == 0).all()
    # the bench workload keeps every first step feasible: the whole batch converges
    assert (status == 0).mean() >= (0.999 if precision == "fp32" else 1.0), np.flatnonzero(status)
    e = rel_err(s.get_batch("x")[idx], s.get_batch("u")[idx], g[key + "_X"], g[key + "_U"])
    print(f"{key} {precision} {s.launch_info()['kernel']}: max rel err {e.max():.3e}")
    assert e.max() < (TOL64 if precision == "fp64" else TOL32), e.max()


def test_force_acados_recorded_states_batch(golden_dir):
    """The 239 force steps acados recorded (experiment_data/img/example_acc_trajectory_component.pdf,
    tests/golden/reference_plots.npz), each QP posed from acados's own plotted state with the window at
    its sample (src/force_model/ocp.py:117-122, controller.py:29-32), solved as one GPU batch: x/u match
    the oracle's certified exact solutions to 1e-6. tests/test_reference_plots.py shows that acados's u0
    at each of these steps is an interior point of the same QP with complementarity <= 1e-6, so the
    engine returns, step by step, the exact solution of the QP acados solved."""
    from oracle import acados_termination as AT
    plots = np.load(os.path.join(golden_dir, "reference_plots.npz"))
    ref = np.load(os.path.join(golden_dir, "circle_ref.npz"))["nh30_nx6"]
    spec = models.force_model(30)
    X0, Y, Xr, Ur = [], [], [], []
    for t, x, _ in AT.force_recorded_steps(plots):
        y, ye = qp.yref_window(ref[:, :4], ref[:, 4:6], t, 30)
        m = AT.StepModel(spec, x, y, ye)
        X0.append(x)
        Y.append(np.concatenate([y.ravel(), ye]))
        Xr.append(m.Q.states(m.U))
        Ur.append(m.U.reshape(30, 2))
    assert len(X0) == 239
    s = AcadosOcpSolver(OCPS["force"](30), batch=len(X0))
    s.set_batch("x0", np.array(X0))
    s.set_batch("yref", np.array(Y))
    assert s.solve() == 0
    e = rel_err(s.get_batch("x"), s.get_batch("u"), np.array(Xr), np.array(Ur))
    print(f"acados-recorded force states: max rel err {e.max():.3e} ({s.launch_info()['kernel']})")
    assert e.max() < TOL64, e.max()


EDGE_KERNELS = [("lpc", "fp64"), ("wave", "fp64"), ("lpc", "fp32"), ("wave", "fp32")]


@pytest.mark.parametrize("kernel,precision", EDGE_KERNELS)
def test_edge_cases_match_oracle(kernel, precision):
    """The oracle's edge cases (tests/test_oracle.py::test_qp_oracle_edge_cases) on the GPU:
    an instance perturbed above the circle whose input saturates exactly on MIN_F, and an
    initial state exactly on the 1.2 m position bound; both kernel families, fp64 and fp32."""
    from oracle import trajectory
    from oracle import params as Pm
    spec = models.force_model(20)
    ref = trajectory.gen_circle_traj(500, 20, 6, 2)
    y, ye = qp.yref_window(ref[:, :4], ref[:, 4:6], 100, 20)
    X0 = np.array([ref[100, :4] + 0.05, [1.2, 0.0, 0.0, 0.5]])
    sols = [qp.solve_ocp(spec, x0, y, ye) for x0 in X0]
    assert all(o["certified"] for o in sols)
    os.environ["NMPC_KERNEL"] = kernel
    try:
        s = AcadosOcpSolver(OCPS["force"](20), batch=2, precision=precision)
    finally:
        os.environ.pop("NMPC_KERNEL", None)
    assert s.launch_info()["kernel"] == ("ipm_lpc_kernel" if kernel == "lpc" else "ipm_kernel")
    s.set_batch("x0", X0)
    s.set_batch("yref", np.tile(np.concatenate([y.ravel(), ye]), (2, 1)))
    assert s.solve() == 0
    X, U = s.get_batch("x"), s.get_batch("u")
    tol = TOL64 if precision == "fp64" else TOL32
    e = rel_err(X, U, np.array([o["X"] for o in sols]), np.array([o["U"] for o in sols]))
    assert e.max() < tol, e.max()
    # saturation exactly on the bound (to the solver tolerance), never beyond it
    slack = 1e-6 if precision == "fp64" else 1e-4
    assert U[0].min() == pytest.approx(Pm.MIN_F, abs=slack)
    assert U.max() <= Pm.MAX_F + slack and U.min() >= Pm.MIN_F - slack
    assert X[1, 1:-1, 0].max() <= 1.2 + slack
    assert X[1, 0, 0] == pytest.approx(1.2, abs=1e-15 if precision == "fp64" else 1e-7)


def test_infeasible_instance_reports_status(cases):
    """quad13 with |vx| = 1.6 > 1: x_1 cannot satisfy the velocity bound -> nonzero status,
    no crash, and the feasible neighbours in the same launch are unaffected."""
    key = "quad13_N20"
    x0 = cases[key + "_x0"][:8].copy()
    x0[3, 3] = 1.6
    s = AcadosOcpSolver(OCPS["quad13"](20), batch=8)
    s.set_batch("x0", x0)
    s.set_batch("yref", cases[key + "_yref"][:8])
    st = s.solve()
    status = s.get_batch_int("status")
    assert st != 0 and status[3] in (2, 4)
    good = np.arange(8) != 3
    assert (status[good] == 0).all()
    e = rel_err(s.get_batch("x")[good], s.get_batch("u")[good], cases[key + "_X"][:8][good],
                cases[key + "_U"][:8][good])
    assert e.max() < TOL64


def test_full_size_batch_properties(cases):
    """BASELINE headline size (quad13, N=20, B=8192): every instance converges, duplicated
    instances give bitwise-identical answers, and a sample matches the oracle."""
    key = "quad13_N20"
    reps = 8192 // cases[key + "_x0"].shape[0] + 1
    s, st = solve_batch(key, cases, reps=reps)
    B = s.batch
    assert st == 0
    X, U = s.get_batch("x"), s.get_batch("u")
    n0 = cases[key + "_x0"].shape[0]
    assert np.array_equal(X[:n0], X[n0:2 * n0]) and np.array_equal(U[:n0], U[-n0:] if B % n0 == 0 else U[:n0])
    e = rel_err(X[:n0], U[:n0], cases[key + "_X"], cases[key + "_U"])
    assert e.max() < TOL64


def test_plant_simulator_matches_oracle():
    from drone_attitude_control_amd import AcadosSim, AcadosSimSolver
    from drone_attitude_control_amd.models import PlantModel
    from oracle import closed_loop as CL
    rng = np.random.default_rng(5)
    for stages, T, ref in ((4, 0.02, CL.rk4_step), (1, 0.002, CL.euler_step)):
        sim = AcadosSim()
        sim.model = PlantModel().model
        sim.solver_options.T = T
        sim.solver_options.num_stages = stages
        ss = AcadosSimSolver(sim)
        for _ in range(5):
            x = rng.normal(size=4)
            u = np.array([rng.normal(0, 0.5), abs(rng.normal(0.3, 0.1))])
            assert np.allclose(ss.simulate(x=x, u=u), ref(x, u, T), rtol=1e-13, atol=1e-15)


@pytest.mark.parametrize("kernel", ["lpc", "wave", None])
def test_factorisation_failure_keeps_last_iterate(kernel, cases, golden_dir):
    """A closed-loop jerk instance pushed past the position bound (tests/golden/qp_failure.npz,
    make_failure_case.py): x_1 cannot be feasible, F_uu loses positive definiteness at the C
    oracle's iteration 9 -> status 4 with the iterate from the start of that iteration, finite
    (no NaN handed to the plant), and the other instances of the launch are unaffected."""
    f = np.load(os.path.join(golden_dir, "qp_failure.npz"))
    key = "jerk_N40"
    x0 = np.vstack([f[key + "_x0"], cases[key + "_x0"][:3]])
    y = np.vstack([f[key + "_yref"], cases[key + "_yref"][:3]])
    # kernel None: the fp64 fast solve, whose active-set finish cannot settle this QP (the dual fallback finds
    # it infeasible, the certificate does not prove it), so it parks and takes the full IPM in list mode
    if kernel:
        os.environ["NMPC_KERNEL"] = kernel
    try:
        s = AcadosOcpSolver(OCPS["jerk"](40), batch=4)
    finally:
        os.environ.pop("NMPC_KERNEL", None)
    s.set_batch("x0", x0)
    s.set_batch("yref", y)
    assert s.solve() == 4
    status, it = s.get_batch_int("status"), s.get_batch_int("qp_iter")
    assert list(status) == [4, 0, 0, 0]
    # the handle runs the exact finish (fp64 default): its attempts count in qp_iter, so the
    # iteration count is the oracle's with the same options (the failing iterate is the IPM's)
    _, _, stc, itc = cref.RiccatiIpmRef.for_options(models.MODELS["jerk"](40), OCPS["jerk"](40).solver_options).solve(
        f[key + "_x0"], f[key + "_yref"], nthreads=1)
    assert stc[0] == 4 and it[0] == itc[0], (it[0], itc[0])
    X, U = s.get_batch("x"), s.get_batch("u")
    assert np.isfinite(X).all() and np.isfinite(U).all()
    assert rel_err(X[:1], U[:1], f[key + "_X"], f[key + "_U"]).max() < TOL64
    assert rel_err(X[1:], U[1:], cases[key + "_X"][:3], cases[key + "_U"][:3]).max() < TOL64


@pytest.mark.parametrize("kernel", ["lpc", "wave", None])
@pytest.mark.parametrize("name,N", [("jerk", 40), ("quad13", 20)])
def test_infeasibility_certificate_on_gpu(kernel, name, N, golden_dir):
    """Closed-loop QPs past a position bound (tests/golden/qp_infeasible.npz): the kernels' interval
    certificate ends them before the first iteration — status 4, 0 iterations, the oracle's
    initial point — next to feasible instances of the same launch that solve normally. kernel None: the
    fp64 fast solve, whose finish (fin64_kernel) runs the same certificate and parks such an instance for
    the full solve's list mode, which returns that status and initial point."""
    f = np.load(os.path.join(golden_dir, "qp_infeasible.npz"))
    d = np.load(os.path.join(golden_dir, "qp_cases.npz"))
    key = f"{name}_N{N}"
    gkey = key if key + "_x0" in d else f"{name}_N30"
    n = f[key + "_x0"].shape[0]
    x0 = np.vstack([f[key + "_x0"], d[gkey + "_x0"][:3]]) if gkey == key else f[key + "_x0"]
    y = np.vstack([f[key + "_yref"], d[gkey + "_yref"][:3]]) if gkey == key else f[key + "_yref"]
    if kernel:
        os.environ["NMPC_KERNEL"] = kernel
    try:
        s = AcadosOcpSolver(OCPS[name](N), batch=x0.shape[0])
    finally:
        os.environ.pop("NMPC_KERNEL", None)
    s.set_batch("x0", x0)
    s.set_batch("yref", y)
    s.solve()
    st, it = s.get_batch_int("status"), s.get_batch_int("qp_iter")
    assert (st[:n] == 4).all() and (it[:n] == 0).all(), (st, it)
    X, U = s.get_batch("x"), s.get_batch("u")
    assert rel_err(X[:n], U[:n], f[key + "_X"], f[key + "_U"]).max() < 1e-12
    if gkey == key:
        assert (st[n:] == 0).all()
        assert rel_err(X[n:], U[n:], d[key + "_X"][:3], d[key + "_U"][:3]).max() < TOL64
