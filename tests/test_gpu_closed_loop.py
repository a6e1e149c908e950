"""GPU closed-loop parity: the reference's follow_trajectory loops (force/jerk) with every QP
solve and plant step on the GPU, over the whole seed-42 main.py run (500 steps, force then
jerk on one noise stream, x0 = [1, 0, 0, 0.62], main.py:43-46), against
  * the oracle's restatement (tests/golden/closed_loop.npz, make_qp_golden.py closed_loop), and
  * for jerk at the reference default N = 30, acados's own recorded run
    (tests/golden/reference_plots.npz, extracted from experiment_data/img/*.pdf).
Bars: states 1e-6 absolute (the solve bar, BASELINE north_star), closed-loop cost and AED 1e-6
relative (f4: controller.py:40-41,54, store_results.py:233-236).
"""
import os

import numpy as np
import pytest

from drone_attitude_control_amd import controllers

pytestmark = pytest.mark.gpu

STEPS = 500


@pytest.fixture(scope="module")
def data(golden_dir):
    return (np.load(os.path.join(golden_dir, "closed_loop.npz")),
            np.load(os.path.join(golden_dir, "noise_seed42.npy")),
            np.load(os.path.join(golden_dir, "circle_ref.npz")))


def stream(noise):
    it = iter(noise)
    return lambda: float(next(it))


@pytest.mark.parametrize("N", [20, 30])
def test_force_and_jerk_closed_loop(data, N):
    """The façade loop (nmpc_set / nmpc_solve / nmpc_get per step, nmpc_sim_plant per plant step)."""
    cl, noise, refs = data
    ref = refs[f"nh{N}_nx6"]
    draw = stream(noise)
    x0 = np.array([1.0, 0, 0, 0.62])
    c, X, a, Up = controllers.force_follow_trajectory(ref[:, :4], ref[:, 4:6], x0, draw, verbose=False,
                                                      N=N, n_steps=STEPS)
    assert np.abs(X - cl[f"force_N{N}_X"]).max() < 1e-6
    assert np.abs(Up - cl[f"force_N{N}_Uplant"]).max() < 1e-6
    assert c == pytest.approx(float(cl[f"force_N{N}_cost"]), rel=1e-6)
    assert controllers.calc_aed(ref[:STEPS, :2], X[:STEPS, :2]) == pytest.approx(float(cl[f"force_N{N}_aed"]),
                                                                                 rel=1e-6)
    c, X, a, Up = controllers.jerk_follow_trajectory(ref[:, :6], ref[:, 6:], x0, draw, verbose=False,
                                                     N=N, n_steps=STEPS)
    assert np.abs(X - cl[f"jerk_N{N}_X"]).max() < 1e-6
    assert np.abs(a - cl[f"jerk_N{N}_a"]).max() < 1e-6
    assert c == pytest.approx(float(cl[f"jerk_N{N}_cost"]), rel=1e-6)
    assert controllers.calc_aed(ref[:STEPS, :2], X[:STEPS, :2]) == pytest.approx(float(cl[f"jerk_N{N}_aed"]),
                                                                                 rel=1e-6)


def _device_loop(model, N, refs_noise, B=5):
    """nmpc_closed_loop_* (prepare -> solve -> advance, all on the device) for a batch whose
    instance 0 is main.py's run with the seed-42 noise stream injected (force draws 0..499,
    jerk 500..999); the other instances start elsewhere on the circle."""
    from drone_attitude_control_amd.batched import ClosedLoop, reference_table
    noise = refs_noise
    table = reference_table(model, N)
    offsets = np.array([0, 10, 100, 250, 400][:B], dtype=np.int32)
    x = table[offsets, :4].copy()
    x[0] = [1.0, 0, 0, 0.62]
    if model == "jerk":
        x = np.hstack([x, np.tile([0.0, 9.81], (B, 1))])
    nt = np.zeros((B, STEPS))
    nt[0] = noise[:STEPS] if model == "force" else noise[STEPS:2 * STEPS]
    return ClosedLoop(model, B, N=N, table=table, offsets=offsets, x_init=x, noise_table=nt)


@pytest.mark.parametrize("N", [20, 30])
@pytest.mark.parametrize("model", ["force", "jerk"])
def test_device_closed_loop_matches_oracle(data, N, model):
    """All 500 steps on the device; instance 0's states after every step and its accumulated
    closed-loop cost / AED numerator (f4) against the oracle."""
    cl_gold, noise, refs = data
    loop = _device_loop(model, N, noise)
    states = []
    for _ in range(STEPS):
        loop.run(1)
        states.append(loop.state()[0, :4].copy())
    X = np.array(states)
    Xg = cl_gold[f"{model}_N{N}_X"]
    assert np.abs(X - Xg[1:STEPS + 1]).max() < 1e-6
    st = loop.stats()
    assert st["failed"] == 0 and st["instance_steps"] == 5 * STEPS
    per = loop.instance_stats()
    assert per[0, 0] == pytest.approx(float(cl_gold[f"{model}_N{N}_cost"]), rel=1e-6)
    assert per[0, 1] / (STEPS * 2) == pytest.approx(float(cl_gold[f"{model}_N{N}_aed"]), rel=1e-6)
    assert per[0, 3] == STEPS
    assert st["cost_sum"] == pytest.approx(per[:, 0].sum(), rel=1e-12)


def test_device_jerk_loop_matches_acados_run(data, golden_dir):
    """Instance 0 of the device jerk loop (N = 30, the reference default) against the plotted
    acados run itself: positions, velocities and accelerations at every plotted sample."""
    _, noise, _ = data
    plots = np.load(os.path.join(golden_dir, "reference_plots.npz"))
    loop = _device_loop("jerk", 30, noise, B=1)
    states = [loop.state()[0].copy()]
    for _ in range(STEPS - 1):
        loop.run(1)
        states.append(loop.state()[0].copy())
    S = np.array(states)          # S[t] = Xsim[t] (+ a before step t)
    fig = "example_jerk_trajectory_component"
    for j, col, tol in ((0, 0, 1e-6), (1, 1, 1e-6), (4, 2, 1e-6), (5, 3, 1e-6)):
        p = plots[f"{fig}__p{j}"]
        i = np.round(p[:, 0] / 0.02).astype(int)
        assert np.abs(S[i, col] - p[:, 1]).max() < tol, j
    # a[t] is the acceleration after step t = the state's a-part before step t + 1
    for j, col in ((10, 4), (11, 5)):
        p = plots[f"{fig}__p{j}"]
        i = np.round(p[:, 0] / 0.02).astype(int)
        ok = i < STEPS - 1
        assert np.abs(S[i[ok] + 1, col] - p[ok, 1]).max() < 1e-5


@pytest.mark.parametrize("model", ["force", "quad13"])
def test_device_sharding_invariance(model):
    """Two shards (instance_base 0 and 4) reproduce one 8-instance closed loop exactly: the
    device noise is keyed by the global instance id, so results do not depend on
    how instances are split over GPUs."""
    from drone_attitude_control_amd.batched import ClosedLoop, DEFAULT_N
    from drone_attitude_control_amd.sharding import rank_workload
    N = DEFAULT_N[model]
    table, off, x, _ = rank_workload(model, N, 8, 1, 0, seed=7)
    full = ClosedLoop(model, 8, N=N, table=table, offsets=off, x_init=x, instance_base=0, seed=7)
    full.run(5)
    parts = []
    for r in range(2):
        t, o, xr, base = rank_workload(model, N, 4, 2, r, seed=7)
        cl = ClosedLoop(model, 4, N=N, table=t, offsets=o, x_init=xr, instance_base=base, seed=7)
        cl.run(5)
        parts.append(cl.state())
    assert np.abs(np.vstack(parts) - full.state()).max() <= 1e-12


def test_batched_closed_loop_survives_infeasible_steps():
    """The bench's jerk workload (seed 42, B=4096, N=40) drives instance 1202 past the 1.2 m
    position bound at step 18 (tests/golden/qp_failure.npz): that solve reports status 4, the
    instance continues on the last finite iterate, and every closed-loop statistic stays finite
    (before the fix a NaN step reached the plant and the cost sum became NaN)."""
    from drone_attitude_control_amd.batched import ClosedLoop
    loop = ClosedLoop("jerk", 4096, N=40, seed=42)
    loop.run(23)
    st = loop.stats()
    assert st["failed"] >= 1
    assert np.isfinite(st["cost_sum"]) and np.isfinite(st["aed_sum"])
    assert np.isfinite(loop.state()).all()


def test_solve_after_closed_loop_uses_host_inputs(data):
    """After a device closed loop rewrote the engine's x0 / yref buffers, a plain nmpc_solve
    with no new set() calls solves the host-staged problem again, not the loop's last window."""
    from oracle import models, qp
    cl_gold, noise, refs = data
    loop = _device_loop("force", 20, noise, B=1)
    s = loop.solver
    ref = refs["nh20_nx6"]
    yref, ye = qp.yref_window(ref[:, :4], ref[:, 4:6], 7, 20)
    x0 = ref[7, :4] + 0.01
    s.set_batch("x0", x0[None])
    s.set_batch("yref", np.concatenate([yref.ravel(), ye])[None])
    assert s.solve() == 0
    u1 = s.get_batch("u").copy()
    loop.run(3)
    assert s.solve() == 0
    assert np.array_equal(s.get_batch("u"), u1)
    o = qp.solve_ocp(models.force_model(20), x0, yref, ye)
    assert np.abs(u1[0] - o["U"]).max() < 1e-6


@pytest.mark.parametrize("model,N,B,kernel", [("quad13", 20, 1000, None), ("force", 20, 777, "wave"),
                                              ("force", 20, 777, "lpc"), ("jerk", 40, 301, None)])
def test_fused_closed_loop_matches_per_step(model, N, B, kernel):
    """The fused closed loop (steps inside the solve kernel, nmpc_closed_loop_run's default for the
    lane-per-component and wavefront families, with warm-started active sets) gives the per-step
    loop's results (one prepare / solve / advance launch per step, NMPC_CL_FUSED=0): states,
    per-instance cost / AED sums and failure counts, over 70 steps (two fused launches, 64 + 6
    steps), ragged batches."""
    from drone_attitude_control_amd.batched import ClosedLoop

    def run(fused):
        if kernel:
            os.environ["NMPC_KERNEL"] = kernel
        os.environ["NMPC_CL_FUSED"] = "1" if fused else "0"
        try:
            cl = ClosedLoop(model, B, N=N, seed=7)
            cl.run(70)
            return cl.state(), cl.instance_stats(), cl.stats()
        finally:
            os.environ.pop("NMPC_KERNEL", None)
            os.environ.pop("NMPC_CL_FUSED", None)

    xs, ins, sts = run(False)
    xf, inf, stf = run(True)
    # fused: two launches of the solve kernel (64 + 6 steps), or the lean loop's rounds (quad13, jerk)
    assert sts["solve_launches"] == 70 and 1 <= stf["solve_launches"] <= 70 and stf["steps"] == 70
    assert np.array_equal(ins[:, 2:], inf[:, 2:])            # failures, steps per instance
    # certified solutions reached by different paths (warm-started active sets, no finish after a
    # failed step in the fused loop) agree to rounding, far inside the 1e-6 solve bar
    assert np.allclose(xf, xs, rtol=1e-9, atol=1e-9), np.abs(xf - xs).max()
    assert np.allclose(inf[:, :2], ins[:, :2], rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("model,N,B", [("quad13", 20, 3000), ("jerk", 40, 1001), ("force", 20, 2049)])
def test_shared_factorisation_paths_match_full_factorisation(model, N, B):
    """The exact finish's shortcuts on the handle's shared factorisation — the fast finish (the
    unconstrained LQ solution, explicit from the closed loop's tables or by the recursion
    (NMPC_EXPLICIT=0), then active-set steps on the projected inverse Hessian (off: NMPC_WSET=0),
    skipping certificate, initial point and IPM) and lqr_back (inside the finish loop) — and factoring
    every finish step (NMPC_LQR=0) all give the oracle's closed loop (oracle/c/riccati_ipm.c mode 0:
    cold exact solves, active sets confirmed by a dense KKT solve): states to 1e-6 relative (the solve
    bar), per-instance cost / AED sums to 1e-6 relative, failure counts exactly, over 40 steps of the
    lane-per-component fused closed loop (two launches: 25 + 15), and the same for the lean closed loop
    (nmpc_cl_fast.hip: the fast path as its own kernel, parked instances solved in list mode). (The
    paths agree with each other to
    ~1e-8, not to rounding: the penalised finish of a full factorisation decides a held bound's
    multiplier sign on z - b, which resolves small multipliers of low-curvature inputs less finely than
    the active-set steps' displacement test.)"""
    from drone_attitude_control_amd.batched import ClosedLoop, workload
    from drone_attitude_control_amd.models import OCPS
    from oracle import cref, models

    def run(env):
        os.environ.update(env, NMPC_KERNEL="lpc")
        try:
            cl = ClosedLoop(model, B, N=N, seed=11)
            cl.run(25)
            cl.run(15)
            return cl.state(), cl.instance_stats()
        finally:
            for k in list(env) + ["NMPC_KERNEL"]:
                os.environ.pop(k, None)

    table, off, x = workload(model, N, B, 11)
    o = OCPS[model](N).solver_options
    ref = cref.ClosedLoopRef(getattr(models, f"{model}_model")(N), model, table, off, x, mode=0, seed=11,
                             tol_comp=o.qp_solver_tol_comp, tol_res=o.qp_solver_tol_stat)
    ref.run(40)
    # the fused lane-per-component kernel's switches (NMPC_CL_FAST=0: not the lean loop) and the lean
    # loop itself (nmpc_cl_fast.hip, default for quad13 / jerk; forced for force)
    for env in ({"NMPC_LQR": "0", "NMPC_CL_FAST": "0"}, {"NMPC_CL_FAST": "0"}, {"NMPC_FAST": "0", "NMPC_CL_FAST": "0"},
                {"NMPC_FAST": "2", "NMPC_CL_FAST": "0"}, {"NMPC_EXPLICIT": "0", "NMPC_CL_FAST": "0"},
                {"NMPC_WSET": "0", "NMPC_CL_FAST": "0"}, {"NMPC_CL_FAST": "1"}):
        x1, s1 = run(env)
        assert np.array_equal(s1[:, 2:], ref.acc[:, 2:]), env
        err = np.abs(x1 - ref.state).max(1) / np.maximum(1.0, np.abs(ref.state).max(1))
        assert err.max() < 1e-6, (env, err.max())
        np.testing.assert_allclose(s1[:, :2], ref.acc[:, :2], rtol=1e-6, atol=1e-12, err_msg=str(env))


@pytest.mark.parametrize("model,N,B", [("quad13", 20, 2048), ("force", 20, 1024), ("jerk", 40, 1024)])
def test_lean_loop_trajectory_outputs_are_opt_in(model, N, B):
    """The lean loop writes no trajectory by default (the loop reads only u_0 / x_1, controller.py:37-41);
    nmpc_closed_loop_set_outputs(1) turns the last step's write-back on. Results are the same either way
    (states and per-instance sums bit for bit), the default leaves nothing to read, and the opted-in outputs
    are each instance's last-step solution: x_0 the state that step started from, the trajectory the oracle's
    QP solution from that state and window (1e-6 relative), the status the oracle's."""
    from drone_attitude_control_amd.batched import ClosedLoop, first_step_qps, workload
    from drone_attitude_control_amd._lib import NmpcError
    from oracle import cref, models
    table, off, x = workload(model, N, B, 42)
    a = ClosedLoop(model, B, N=N, table=table, offsets=off, x_init=x, seed=42)
    b = ClosedLoop(model, B, N=N, table=table, offsets=off, x_init=x, seed=42)
    b.set_outputs(True)
    k = 7
    a.run(k - 1)       # the same launch split for both (a launch boundary flushes the sums and may move an
    a.run(1)           # instance between the lockstep and the single-instance code: last-bit differences)
    b.run(k - 1)
    xs = b.state()
    b.run(1)
    assert np.array_equal(a.state(), b.state())
    assert np.array_equal(a.instance_stats(), b.instance_stats())
    with pytest.raises(NmpcError):
        a.solver.get_batch("x")
    X, U = b.solver.get_batch("x"), b.solver.get_batch("u")
    st = b.solver.get_batch_int("status")
    assert np.array_equal(X[:, 0], xs)
    idx = np.arange(0, B, max(1, B // 97))
    x0s, Y = first_step_qps(model, N, table, (np.asarray(off)[idx] + k - 1) % b.period, xs[idx])
    Xr, Ur, str_, _ = cref.RiccatiIpmRef(models.MODELS[model](N)).solve(x0s, Y)
    assert np.array_equal(st[idx], str_)
    ok = str_ == 0
    assert ok.sum() >= len(idx) - 2
    scale = np.maximum(1.0, np.maximum(np.abs(Xr).max(axis=(-2, -1)), np.abs(Ur).max(axis=(-2, -1))))
    err = np.maximum(np.abs(X[idx] - Xr).max(axis=(-2, -1)), np.abs(U[idx] - Ur).max(axis=(-2, -1))) / scale
    assert err[ok].max() < 1e-6, err.max()
