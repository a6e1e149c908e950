"""GPU parity of the exact path bench.py times: the default closed loop — the lean loop
(nmpc_cl_fast.hip: explicit unconstrained solution, warm-started PDAS steps on the projected inverse
Hessian, the dual active-set fallback, the interval certificate, the list-mode full solve for what
is left) — at the BASELINE sizes, on the bench's
own seed-42 workload (batched.workload: start rows, initial states, Philox noise keyed by the
global instance id) and launch boundaries (3 warm-up steps, then 10 regions of 20), against

  * the committed oracle closed loops (tests/golden/closed_loop_bench.npz,
    make_closed_loop_bench.py: oracle/c/riccati_ipm.c mode 0, every QP solved cold to its exact
    solution and the active set confirmed by a dense KKT solve) for 256 instances per workload —
    every instance with a failed solve, the ones with the most full solves, and evenly spaced
    others — at every region boundary;
  * the C restatement of the GPU's algorithm (mode 1, run here on the host) for every instance of
    the batch at the final boundary.

Reference loop: src/force_model/controller.py:25-54 (jerk_model/controller.py:26-56; the
quad13 instances close the loop through the controller's own model). Bars: states 1e-6 per
instance relative to max(1, |x|) (BASELINE north_star's solve bar), per-instance closed-loop
cost and AED numerator 1e-6 relative, failed (status 4) solves per region exactly.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

WORKLOADS = [("quad13", 20, 8192), ("force", 20, 8192), ("jerk", 40, 4096)]
REGIONS = [3] + [20] * 10


def _rel(a, b):
    """per-instance max |a - b| / max(1, max |b|) over the last axis"""
    return (np.abs(a - b).max(-1) / np.maximum(1.0, np.abs(b).max(-1)))


@pytest.fixture(scope="module")
def golden(golden_dir):
    return np.load(os.path.join(golden_dir, "closed_loop_bench.npz"))


@pytest.mark.timeout(300)
@pytest.mark.parametrize("model,N,B", WORKLOADS)
def test_bench_closed_loop_matches_oracle(golden, model, N, B):
    from drone_attitude_control_amd.batched import ClosedLoop, workload
    from oracle import cref, models
    from drone_attitude_control_amd.models import OCPS
    key = f"{model}_N{N}_B{B}"
    sel = golden[f"{key}_sel"]
    assert list(golden["checkpoints"]) == list(np.cumsum(REGIONS))
    loop = ClosedLoop(model, B, N=N, seed=42)             # bench.py's workload and defaults
    info = loop.solver.launch_info()
    assert info["kernel"] in ("ipm_lpc_kernel", "ipm_kernel")
    # the lean loop bench.py times (quad13: the lockstep MFMA kernel)
    assert info["closed_loop_kernel"] == ("cl_lock_kernel" if model == "quad13" else "cl_fast_kernel")
    states, sums = [], []
    for n in REGIONS:
        loop.run(n)
        states.append(loop.state())
        sums.append(loop.instance_stats())
    S, A = np.array(states), np.array(sums)
    Sg, Ag, Fg = golden[f"{key}_states"], golden[f"{key}_sums"], golden[f"{key}_failed"]

    # oracle goldens (256 instances, every region boundary)
    err = _rel(S[:, sel], Sg)
    assert err.max() < 1e-6, (err.max(), sel[np.unravel_index(err.argmax(), err.shape)[1]])
    fails_region = np.diff(np.concatenate([np.zeros((1, len(sel))), A[:, sel, 2]]), axis=0)
    fails_gold = np.add.reduceat(Fg, np.concatenate([[0], np.cumsum(REGIONS)[:-1]]), axis=1).T
    assert np.array_equal(fails_region, fails_gold)
    assert np.array_equal(A[:, sel, 3], Ag[:, :, 3])
    for j in (0, 1):                                       # cost, AED numerator
        np.testing.assert_allclose(A[:, sel, j], Ag[:, :, j], rtol=1e-6, atol=1e-12)

    # every instance of the batch against the C restatement of the GPU's algorithm
    table, off, x = workload(model, N, B, 42)
    o = OCPS[model](N).solver_options
    ref = cref.ClosedLoopRef(getattr(models, f"{model}_model")(N), model, table, off, x, mode=1, seed=42,
                             tol_comp=o.qp_solver_tol_comp, tol_res=o.qp_solver_tol_stat)
    ref.run(sum(REGIONS))
    err = _rel(S[-1], ref.state)
    assert err.max() < 1e-6, (err.max(), int(err.argmax()))
    assert np.array_equal(A[-1, :, 2:], ref.acc[:, 2:])
    np.testing.assert_allclose(A[-1, :, :2], ref.acc[:, :2], rtol=1e-6, atol=1e-12)


@pytest.mark.timeout(300)
def test_force_config2_one_wave_variant_matches_oracle(monkeypatch):
    """BASELINE config 2 (force N=20 B=1024 fp64) runs the one-wavefront-per-SIMD variant (CLF_ONE: batch <= the
    device's SIMD count; its sweep pivots unrolled). Its states, sums and failures equal the default variant's
    (NMPC_CLF_ONE=0) bit for bit — the arithmetic is the same — and every instance matches the C restatement of
    the algorithm (oracle mode 1) over 43 steps."""
    from drone_attitude_control_amd.batched import ClosedLoop, workload
    from drone_attitude_control_amd.models import OCPS
    from oracle import cref, models
    B, N, steps = 1024, 20, (3, 20, 20)

    def run(one):
        monkeypatch.setenv("NMPC_CLF_ONE", one)
        loop = ClosedLoop("force", B, N=N, seed=42)
        for n in steps:
            loop.run(n)
        return loop.state(), loop.instance_stats()

    S1, A1 = run("1")
    S0, A0 = run("0")
    assert np.array_equal(S1, S0) and np.array_equal(A1, A0)
    table, off, x = workload("force", N, B, 42)
    o = OCPS["force"](N).solver_options
    ref = cref.ClosedLoopRef(models.force_model(N), "force", table, off, x, mode=1, seed=42,
                             tol_comp=o.qp_solver_tol_comp, tol_res=o.qp_solver_tol_stat)
    ref.run(sum(steps))
    err = _rel(S1, ref.state)
    assert err.max() < 1e-6, (err.max(), int(err.argmax()))
    assert np.array_equal(A1[:, 2:], ref.acc[:, 2:])
    np.testing.assert_allclose(A1[:, :2], ref.acc[:, :2], rtol=1e-6, atol=1e-12)


@pytest.mark.timeout(300)
def test_jerk_lockstep_variant_matches_oracle():
    """The jerk shape's lockstep kernel (opt-in, NMPC_CLF_LOCK=1: cl_lock_kernel with the jerk converter plant
    evaluated per instance in the four-instance layout and the cost on x_1 gathered from the MFMA tiles;
    src/jerk_model/controller.py:26-56) on a ragged batch of 1030 over 43 steps (3 + 40): states, sums and
    failure counts against the C restatement of the GPU's algorithm (mode 1) over the whole batch."""
    from drone_attitude_control_amd.batched import ClosedLoop, workload
    from oracle import cref, models
    from drone_attitude_control_amd.models import OCPS
    os.environ["NMPC_CLF_LOCK"] = "1"
    try:
        cl = ClosedLoop("jerk", 1030, N=40, seed=7)
        assert cl.solver.launch_info()["closed_loop_kernel"] == "cl_lock_kernel"
        cl.run(3)
        cl.run(40)
        x, acc = cl.state(), cl.instance_stats()
    finally:
        os.environ.pop("NMPC_CLF_LOCK", None)
    table, off, x0 = workload("jerk", 40, 1030, 7)
    o = OCPS["jerk"](40).solver_options
    ref = cref.ClosedLoopRef(models.jerk_model(40), "jerk", table, off, x0, mode=1, seed=7,
                             tol_comp=o.qp_solver_tol_comp, tol_res=o.qp_solver_tol_stat)
    ref.run(43)
    assert _rel(x, ref.state).max() < 1e-6, _rel(x, ref.state).max()
    assert np.array_equal(acc[:, 2:], ref.acc[:, 2:])
    np.testing.assert_allclose(acc[:, :2], ref.acc[:, :2], rtol=1e-6, atol=1e-12)


@pytest.mark.timeout(300)
def test_quad13_cost_on_x1_runs_the_single_instance_loop():
    """quad13 with the closed-loop cost on x_1 (cost_stage 1, the jerk loop's choice, jerk_model/controller.py:39):
    the lockstep kernel gathers x_1 for the jerk shape only, so this configuration runs cl_fast_kernel, and its
    per-instance cost sums (taken at x_1) match the C restatement (mode 1, cost_stage 1) over a ragged batch of
    1030 and 23 steps (3 + 20); the cost differs from the x_0 loop's (the lockstep path once charged
    it at x_0 silently)."""
    from drone_attitude_control_amd.batched import ClosedLoop, workload
    from oracle import cref, models
    from drone_attitude_control_amd.models import OCPS
    cl = ClosedLoop("quad13", 1030, N=20, seed=9, cost_stage=1)
    assert cl.solver.launch_info()["closed_loop_kernel"] == "cl_fast_kernel"
    cl.run(3)
    cl.run(20)
    x, acc = cl.state(), cl.instance_stats()
    table, off, x0 = workload("quad13", 20, 1030, 9)
    o = OCPS["quad13"](20).solver_options
    ref = cref.ClosedLoopRef(models.quad13_model(20), "quad13", table, off, x0, mode=1, seed=9, cost_stage=1,
                             tol_comp=o.qp_solver_tol_comp, tol_res=o.qp_solver_tol_stat)
    ref.run(23)
    assert _rel(x, ref.state).max() < 1e-6, _rel(x, ref.state).max()
    assert np.array_equal(acc[:, 2:], ref.acc[:, 2:])
    np.testing.assert_allclose(acc[:, :2], ref.acc[:, :2], rtol=1e-6, atol=1e-12)
    ref0 = cref.ClosedLoopRef(models.quad13_model(20), "quad13", table, off, x0, mode=1, seed=9, cost_stage=0,
                              tol_comp=o.qp_solver_tol_comp, tol_res=o.qp_solver_tol_stat)
    ref0.run(23)
    assert np.abs(ref0.acc[:, 0] - acc[:, 0]).max() > 1e-6


@pytest.mark.timeout(300)
@pytest.mark.parametrize("model,N,B", [("quad13", 20, 4096), ("jerk", 40, 2048)])
def test_claim_order_changes_only_the_schedule(model, N, B):
    """The lean loop's claim order (NMPC_CLF_ORDER, read per run: the previous launch's warm-start and
    rare-path instances first; nmpc_cl_fast.hip claim_order) moves instances between wavefronts and
    rounds, never between paths: each instance runs lockstep (quad13: cl_lock_kernel) until its first
    rare step, or whole on one wavefront (jerk: cl_fast_kernel), whatever its place in the order. Five
    launches in each order from the same workload: states and per-instance sums bit for bit."""
    from drone_attitude_control_amd.batched import ClosedLoop
    out = []
    for order in ("0", "1"):
        os.environ["NMPC_CLF_ORDER"] = order
        try:
            cl = ClosedLoop(model, B, N=N, seed=11)
            kernel = cl.solver.launch_info()["closed_loop_kernel"]
            assert kernel == ("cl_lock_kernel" if model == "quad13" else "cl_fast_kernel")
            for n in (3, 20, 20, 20, 20):
                cl.run(n)
            out.append((cl.state(), cl.instance_stats(), cl.stats()["parked"]))
        finally:
            os.environ.pop("NMPC_CLF_ORDER", None)
    (x0, a0, p0), (x1, a1, p1) = out
    assert np.array_equal(x0, x1), np.abs(x0 - x1).max()
    assert np.array_equal(a0, a1), np.abs(a0 - a1).max()
    assert p0 == p1


@pytest.mark.timeout(300)
@pytest.mark.parametrize("model,N,B,no_gi,gclaim", [("quad13", 20, 4096, "0", None), ("jerk", 40, 2048, "0", None),
                                                   ("force", 20, 2048, "1", None), ("force", 20, 2048, "1", "0")])
def test_host_round_paths_agree(model, N, B, no_gi, gclaim, monkeypatch):
    """The host-driven round's two forms: the default — the lean kernel draws the chunk's noise
    itself (gen_noise) and its last wavefront stores the park count into the pinned word (report_exit) — and
    the noise kernel + a copy of the count (NMPC_CLF_NOISE_KERNEL=1, NMPC_CLF_PARK_COPY=1), with one or two
    early phase-2 wavefronts (NMPC_LOCK_WORKERS) and with the warm-started instances through lockstep instead of
    straight to phase 2 (NMPC_LOCK_DIRECT=0), and force's device-wide claim in instance order instead of the
    batch-wide claim order (NMPC_CLF_GORDER=0) — schedule only. With NMPC_CLF_NO_GI=1 steps park, so the
    host reads nonzero park counts (force, whose saturating inputs need the fallback); force's device-wide claim
    keeps the noise kernel, so its per-workgroup claim (NMPC_CLF_GCLAIM=0) is the case where the list-mode solves
    read the kernel-drawn noise. Five launches each: states, per-instance sums and parked counts bit for bit (with
    parks: counts exact, states and sums to 1e-12 — the parked solves' list order is not deterministic)."""
    from drone_attitude_control_amd.batched import ClosedLoop
    monkeypatch.setenv("NMPC_CLF_NO_GI", no_gi)
    if gclaim is not None:
        monkeypatch.setenv("NMPC_CLF_GCLAIM", gclaim)
    arms = [{}, {"NMPC_CLF_NOISE_KERNEL": "1", "NMPC_CLF_PARK_COPY": "1"}, {"NMPC_LOCK_WORKERS": "1"},
            {"NMPC_LOCK_DIRECT": "0"}, {"NMPC_CLF_GORDER": "0"}]
    out = []
    for env in arms:
        for k in ("NMPC_CLF_NOISE_KERNEL", "NMPC_CLF_PARK_COPY", "NMPC_LOCK_WORKERS", "NMPC_LOCK_DIRECT", "NMPC_CLF_GORDER"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        cl = ClosedLoop(model, B, N=N, seed=5)
        parked = 0
        for n in (3, 20, 20, 20, 20):
            cl.run(n)
            parked += cl.stats()["parked"]
        out.append((cl.state(), cl.instance_stats(), parked))
    x0, a0, p0 = out[0]
    if no_gi == "1":
        assert p0 > 0
    for x1, a1, p1 in out[1:]:
        assert p0 == p1
        if no_gi == "1":
            # the parked steps' full solves: the park list is filled by atomics, and the list-mode kernel picks a
            # wavefront's finish path over all the instances it holds (ipm_lpc_kernel: refine_back when every
            # group refines), so a parked instance's solution depends on its list neighbours to rounding
            np.testing.assert_allclose(x1, x0, rtol=1e-12, atol=1e-12)
            np.testing.assert_allclose(a1[:, :2], a0[:, :2], rtol=1e-12, atol=1e-12)
            assert np.array_equal(a1[:, 2:], a0[:, 2:])
        else:
            assert np.array_equal(x0, x1), np.abs(x0 - x1).max()
            assert np.array_equal(a0, a1), np.abs(a0 - a1).max()


TOL_CL32 = 1e-5        # fp32 lean loop, force (BASELINE config 3), DESIGN.md §6 (measured 1.4e-6)
TOL_CL32_LOOP = 1e-3   # fp32 lean loop, quad13 / jerk: a few loop-sensitive instances (measured 2.6e-4 / 5.2e-4)


TOL_CL32_PARKED = 5e-2   # fp32 lean loop whose parked steps take the fp32 IPM (no exact finish), include/nmpc.h


@pytest.mark.timeout(300)
def test_fp32_parked_steps_take_the_fp32_ipm(golden, monkeypatch):
    """The fp32 lean loop's fallback, forced: NMPC_CLF_NO_GI=1 parks every step the PDAS rounds do not settle
    (no dual fallback), so those steps run the fp32 list-mode IPM, which has no exact finish (include/nmpc.h).
    Force N=20 B=8192 fp32 (BASELINE config 3's workload) against the exact fp64 oracle loop: parks happen, step
    counts stay exact, and the states stay within the fp32 IPM's accuracy carried through the loop
    (TOL_CL32_PARKED) — the measured size of the difference the default path (0 parks) does not have."""
    from drone_attitude_control_amd.batched import ClosedLoop
    monkeypatch.setenv("NMPC_CLF_NO_GI", "1")
    key = "force_N20_B8192"
    sel = golden[f"{key}_sel"]
    loop = ClosedLoop("force", 8192, N=20, seed=42, precision="fp32")
    states, sums, parked = [], [], 0
    for n in REGIONS[:4]:
        loop.run(n)
        parked += loop.stats()["parked"]
        states.append(loop.state())
        sums.append(loop.instance_stats())
    S, A = np.array(states), np.array(sums)
    err = _rel(S[:, sel], golden[f"{key}_states"][:4])
    print(f"fp32 {key} closed loop with parks: parked {parked}, max state err {err.max():.3e}, "
          f"median {np.median(err):.3e}, instances above 1e-5: {(err.max(0) > 1e-5).sum()} of {len(sel)}")
    assert parked > 0
    assert np.array_equal(A[:, sel, 3], golden[f"{key}_sums"][:4, :, 3])
    assert np.median(err) < 1e-5
    assert err.max() < TOL_CL32_PARKED


@pytest.mark.timeout(300)
@pytest.mark.parametrize("model,N,B", [("force", 20, 8192), ("quad13", 20, 8192), ("jerk", 40, 4096)])
def test_fp32_closed_loop_matches_oracle(golden, model, N, B):
    """fp32 handles on the lean loop (BASELINE config 3 is force N=20, B=8192, fp32): fp32 tables and
    explicit form, fp64 W, set solves and acceptance (nmpc_cl_fast.hip ClfTol). Against the exact oracle
    loop (mode 0, closed_loop_bench.npz, fp64) on the bench's own seed-42 workload and launch
    boundaries. Force: states at every region boundary within TOL_CL32 relative (the fp32 data's rounding
    carried through the loop), cost / AED numerator within TOL_CL32, failed solves and step counts
    exactly. quad13 / jerk: median state error <= 1e-6, max TOL_CL32_LOOP (a few loop-sensitive instances),
    failures exactly for every instance that tracks the oracle to TOL_CL32 (>= 95 % of the failure-weighted
    sample)."""
    from drone_attitude_control_amd.batched import ClosedLoop
    key = f"{model}_N{N}_B{B}"
    sel = golden[f"{key}_sel"]
    loop = ClosedLoop(model, B, N=N, seed=42, precision="fp32")
    info = loop.solver.launch_info()
    assert info["closed_loop_kernel"] == "cl_fast_kernel", info
    states, sums, parked = [], [], 0
    for n in REGIONS:
        loop.run(n)
        parked += loop.stats()["parked"]
        states.append(loop.state())
        sums.append(loop.instance_stats())
    S, A = np.array(states), np.array(sums)
    Sg, Ag, Fg = golden[f"{key}_states"], golden[f"{key}_sums"], golden[f"{key}_failed"]
    err = _rel(S[:, sel], Sg)
    print(f"fp32 {key} closed loop: max state err {err.max():.3e}, median {np.median(err):.3e}, parked {parked}; "
          f"per region {np.array2string(err.max(1), precision=2)}")
    # force (BASELINE config 3): TOL_CL32 on every instance. quad13 / jerk: the same accuracy on all but a
    # few instances, where an fp32-rounded z_0 decides a bound within the fp32 acceptance band and the loop
    # carries the difference: median <= 1e-6, max < TOL_CL32_LOOP
    tol = TOL_CL32 if model == "force" else TOL_CL32_LOOP
    assert np.median(err) < 1e-6, np.median(err)
    assert err.max() < tol, (err.max(), sel[np.unravel_index(err.argmax(), err.shape)[1]])
    fails_region = np.diff(np.concatenate([np.zeros((1, len(sel))), A[:, sel, 2]]), axis=0)
    fails_gold = np.add.reduceat(Fg, np.concatenate([[0], np.cumsum(REGIONS)[:-1]]), axis=1).T
    assert np.array_equal(A[:, sel, 3], Ag[:, :, 3])
    if model == "force":
        assert np.array_equal(fails_region, fails_gold)
        tracked = np.ones(len(sel), bool)
    else:
        # failures (certified-infeasible QPs at a position bound) exactly for every instance that tracks the
        # oracle to TOL_CL32; an instance the fp32 data moved past a bound decision may fail at another step.
        # The sample is weighted toward failing instances (every instance with a failure is in it), the
        # loop-sensitive ones: at most 5 % of it (measured: quad13 <= 1 %, jerk 8 of 256)
        tracked = err.max(0) < TOL_CL32
        assert (~tracked).mean() <= 0.05, (~tracked).sum()
        assert np.array_equal(fails_region[:, tracked], fails_gold[:, tracked])
    for j in (0, 1):
        np.testing.assert_allclose(A[:, sel, j][:, tracked], Ag[:, :, j][:, tracked], rtol=tol, atol=1e-9)


@pytest.mark.timeout(300)
def test_force_fused_loop_families_agree():
    """The force model's three closed-loop paths — the lean loop (nmpc_cl_fast.hip, the default, with
    its list-mode fallback on the lane-per-component kernel), and the fused loops of the two kernel
    families (NMPC_CL_FAST=0: lane per component, LPC; wavefront per instance block) — on a ragged
    batch of 2049 over 70 steps (two launches, 64 + 6): states and per-instance sums agree to 1e-9,
    failure counts exactly, and all match the oracle."""
    from drone_attitude_control_amd.batched import ClosedLoop, workload
    from oracle import cref, models

    def run(kernel):
        env = {"NMPC_KERNEL": kernel, "NMPC_CL_FAST": "0"} if kernel else {}
        os.environ.update(env)
        try:
            cl = ClosedLoop("force", 2049, N=20, seed=5)
            if kernel:
                assert cl.solver.launch_info()["kernel"] == {"lpc": "ipm_lpc_kernel", "wave": "ipm_kernel"}[kernel]
            cl.run(70)
            return cl.state(), cl.instance_stats()
        finally:
            for k in env:
                os.environ.pop(k, None)

    xl, sl = run("lpc")
    for other in ("wave", None):
        xw, sw = run(other)
        assert np.array_equal(sl[:, 2:], sw[:, 2:]), other
        assert np.allclose(xl, xw, rtol=1e-9, atol=1e-9), (other, np.abs(xl - xw).max())
        assert np.allclose(sl[:, :2], sw[:, :2], rtol=1e-9, atol=1e-12), other
    table, off, x = workload("force", 20, 2049, 5)
    ref = cref.ClosedLoopRef(models.force_model(20), "force", table, off, x, mode=0, seed=5)
    ref.run(70)
    assert _rel(xl, ref.state).max() < 1e-6
    assert np.array_equal(sl[:, 2:], ref.acc[:, 2:])
    np.testing.assert_allclose(sl[:, :2], ref.acc[:, :2], rtol=1e-6, atol=1e-12)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("sync", [True, False])
def test_lean_loop_list_mode_fallback_with_forced_parks(sync):
    """The lean loop's list-mode fallback (nmpc_api.cpp clf_run -> ipm_lpc_kernel in list mode, the path
    whose idle lanes once read an unset noise column, nmpc_ipm_lpc.hip list mode) forced by the test knob
    NMPC_CLF_NO_GI=1: without the dual active-set fallback every force step whose PDAS run does not
    settle parks and gets the full solve. Force (saturating inputs, src/force_model/ocp.py:64-68), a
    ragged batch of 2049 over 40 steps in three runs (3 + 20 + 17, reference loop
    src/force_model/controller.py:25-54): parks happen, and states / sums match the exact oracle loop
    (mode 0) at 1e-6 with the failure counts exact. sync=False: nmpc_closed_loop_run(.., sync = 0) enqueues
    every round with its park count read on the device (no host wait inside the run); the same results."""
    from drone_attitude_control_amd.batched import ClosedLoop, workload
    from oracle import cref, models
    os.environ["NMPC_CLF_NO_GI"] = "1"
    try:
        cl = ClosedLoop("force", 2049, N=20, seed=5)
        assert cl.solver.launch_info()["closed_loop_kernel"] == "cl_fast_kernel"
        parked = 0
        for n in (3, 20, 17):
            cl.run(n, sync=sync)
            st = cl.stats()
            parked += st["parked"]
            if not sync:   # every possible round was enqueued: n + 1 fast launches
                assert st["fast_launches"] == n + 1, st
        x, acc = cl.state(), cl.instance_stats()
    finally:
        os.environ.pop("NMPC_CLF_NO_GI", None)
    assert parked > 0
    table, off, x0 = workload("force", 20, 2049, 5)
    ref = cref.ClosedLoopRef(models.force_model(20), "force", table, off, x0, mode=0, seed=5)
    ref.run(40)
    assert _rel(x, ref.state).max() < 1e-6, _rel(x, ref.state).max()
    assert np.array_equal(acc[:, 2:], ref.acc[:, 2:])
    np.testing.assert_allclose(acc[:, :2], ref.acc[:, :2], rtol=1e-6, atol=1e-12)


_ITER_LOG_RUN = r"""
import json, os, sys
import numpy as np
sys.path.insert(0, os.environ["ROOT"])
from drone_attitude_control_amd.batched import ClosedLoop
cl = ClosedLoop("force", 2049, N=20, seed=5)
cl.run(3)
cl.run(20)
st = cl.stats()
it, s, kc = cl.iter_log()
raw = it.astype(np.int64) | (s.astype(np.int64) << 8) | (kc.astype(np.int64) << 16)
print(json.dumps({"rows": int(it.shape[0]), "parked": st["parked"],
                  "marked": int((raw[:-2] == -1).sum()), "state": cl.state().tolist()}))
"""


@pytest.mark.timeout(300)
def test_lean_loop_iter_log_survives_list_mode():
    """NMPC_ITER_LOG with parks (the list-mode launch once resized the lean loop's log
    bookkeeping without reallocating it, so run(3) then run(20) wrote past the buffer): in a fresh
    process (the env switch is read once), force B=2049 with NMPC_CLF_NO_GI=1, run(3) then run(20):
    the log has 20 + 2 rows, the parked steps carry the -1 marker (one per parked solve), and the
    states match the exact oracle loop (mode 0)."""
    import json
    import subprocess
    import sys
    from drone_attitude_control_amd.batched import workload
    from oracle import cref, models
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, NMPC_ITER_LOG="1", NMPC_CLF_NO_GI="1", ROOT=root)
    out = subprocess.run([sys.executable, "-c", _ITER_LOG_RUN], env=env, capture_output=True, text=True,
                         timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["rows"] == 22
    assert r["parked"] > 0 and r["marked"] == r["parked"], (r["parked"], r["marked"])
    table, off, x0 = workload("force", 20, 2049, 5)
    ref = cref.ClosedLoopRef(models.force_model(20), "force", table, off, x0, mode=0, seed=5)
    ref.run(23)
    assert _rel(np.array(r["state"]), ref.state).max() < 1e-6
