"""CPU tests: the oracle against acados's own recorded run.

The reference holds one artefact that acados produced: the plots of the seed-42 `main.py`
run (`experiment_data/img/example_{acc,jerk}_*.pdf`, `main.py:43-46`; acc = force model).
`tests/golden/extract_reference_plots.py` recovered the plotted polylines as data
(`tests/golden/reference_plots.npz`): the component figures plot Xsim, a and the plant
inputs (theta, F_d) against t = arange(0, T, dt) (`store_results.py:148-191`), so each
surviving vertex is one closed-loop sample, quantised to ~3e-8 in data units.

What these tests establish:
  * the extraction is exact to plot precision (the plotted reference circle equals
    generate_trajectory.py's, ~2e-8);
  * the jerk closed loop of the oracle — exact QP per step, cost_scaling "time_steps"
     — reproduces acados's 500 recorded steps to < 1e-6 in position,
    velocity, theta and F_d; with cost_scaling "none" it misses by > 5e-2, so the plots
    decide App. B.1 for "time_steps";
  * the force closed loop agrees with acados exactly at step 0; from step 1 on acados stops
    its interior-point iteration with a weakly active input bound (multiplier ~2e-4) a few
    1e-3 inside the bound — complementarity t*lambda ~ 6e-7, i.e. acados's 1e-6 termination —
    where the exact QP solution sits on the bound. The trajectory deviation stays bounded
    (< 1e-3 m over 500 steps).
"""
import os

import numpy as np
import pytest

from oracle import closed_loop as CL
from oracle import models, qp

DT = 0.02


@pytest.fixture(scope="module")
def plots(golden_dir):
    return np.load(os.path.join(golden_dir, "reference_plots.npz"))


@pytest.fixture(scope="module")
def gold(golden_dir):
    return np.load(os.path.join(golden_dir, "closed_loop.npz"))


def series(plots, fig, j):
    p = plots[f"{fig}__p{j}"]
    idx = p[:, 0] / DT
    assert np.abs(idx - np.round(idx)).max() < 1e-5        # every vertex is a sample
    return np.round(idx).astype(int), p[:, 1]


FORCE = "example_acc_trajectory_component"
JERK = "example_jerk_trajectory_component"


def test_extraction_reproduces_reference_circle(plots, golden_dir):
    ref = np.load(os.path.join(golden_dir, "circle_ref.npz"))["nh30_nx6"]
    # dotted deepskyblue paths: XRef columns (store_results.py:163-177)
    for fig, pairs in ((FORCE, [(2, 0), (3, 1), (6, 2), (7, 3)]),
                       (JERK, [(2, 0), (3, 1), (6, 2), (7, 3), (8, 4), (9, 5)])):
        for j, col in pairs:
            assert tuple(plots[f"{fig}__p{j}_meta"][1:]) == (2, 1)
            i, y = series(plots, fig, j)
            tol = 3e-7 if col >= 4 else 5e-8
            assert np.abs(ref[i, col] - y).max() < tol, (fig, j)


def test_jerk_closed_loop_matches_acados_run(plots, gold):
    """Oracle golden (N=30, time_steps) vs the recorded acados jerk run, all 500 steps."""
    X, a, Up = gold["jerk_N30_X"], gold["jerk_N30_a"], gold["jerk_N30_Uplant"]
    for j, arr, col, tol in ((0, X, 0, 1e-6), (1, X, 1, 1e-6), (4, X, 2, 1e-6), (5, X, 3, 1e-6),
                             (10, a, 0, 1e-5), (11, a, 1, 1e-5), (12, Up, 0, 1e-6), (13, Up, 1, 1e-6)):
        i, y = series(plots, JERK, j)
        assert i.max() == 499
        err = np.abs(arr[i, col] - y).max()
        assert err < tol, (j, err)


def test_cost_scaling_decided_by_plots(plots, golden_dir):
    """The untested App. B.1 assumption, checked: the jerk run under cost_scaling='none'
    misses acados's recorded positions by centimetres."""
    noise = np.load(os.path.join(golden_dir, "noise_seed42.npy"))
    ref = np.load(os.path.join(golden_dir, "circle_ref.npz"))["nh30_nx6"]
    ns = CL.NoiseStream(noise)
    ns.i = 500                                     # force consumed the first 500 draws
    _, X, _, _, _ = CL.jerk_follow_trajectory(models.jerk_model(30, cost_scaling="none"), ref[:, :6], ref[:, 6:],
                                              np.array([1.0, 0, 0, 0.62]), ns)
    i, y = series(plots, JERK, 0)
    assert np.abs(X[i, 0] - y).max() > 5e-2


def test_force_closed_loop_vs_acados_run(plots, gold):
    X, Up = gold["force_N30_X"], gold["force_N30_Uplant"]
    i8, th = series(plots, FORCE, 8)
    i9, fd = series(plots, FORCE, 9)
    assert i8[0] == 0 and i9[0] == 0
    # step 0: identical QP, identical answer
    assert abs(Up[0, 0] - th[0]) < 1e-6 and abs(Up[0, 1] - fd[0]) < 1e-6
    # bounded deviation over the whole run
    for j, col in ((0, 0), (1, 1)):
        i, y = series(plots, FORCE, j)
        assert np.abs(X[i, col] - y).max() < 1e-3
    for j, col in ((4, 2), (5, 3)):
        i, y = series(plots, FORCE, j)
        assert np.abs(X[i, col] - y).max() < 1e-2


@pytest.fixture(scope="module")
def force_steps(plots, golden_dir):
    """Every recorded force sample re-posed from acados's own state: [(t, StepModel, u0_acados)]."""
    from oracle import acados_termination as AT
    ref = np.load(os.path.join(golden_dir, "circle_ref.npz"))["nh30_nx6"]
    spec = models.force_model(30)
    out = []
    for t, x, u in AT.force_recorded_steps(plots):
        yref, ye = qp.yref_window(ref[:, :4], ref[:, 4:6], t, 30)
        out.append((t, AT.StepModel(spec, x, yref, ye), u))
    return out


ACADOS_TOL_COMP = 1e-6     # acados's default complementarity tolerance [ext]


def test_force_u0_bound_gaps_every_step(force_steps):
    """Every recorded step at which the exact QP (re-posed from acados's plotted state) holds an input
    of u0 on its bound: acados's u0 lies inside that bound (to plot precision) at a gap t with
    t * lambda* <= acados's complementarity tolerance. 196 such (step, bound) pairs over 239 steps;
    the largest product is 8.8e-7 (step 146)."""
    assert len(force_steps) == 239
    prods = []
    for t, m, u in force_steps:
        nC = m.Q.C.shape[0]
        for c in range(m.nu):
            for row, gap in ((c, u[c] - m.Q.lo[c]), (nC + c, m.Q.hi[c] - u[c])):
                if m.lam[row] > 0:
                    assert gap > -2e-8, (t, c, gap)
                    prods.append(gap * m.lam[row])
    assert len(prods) == 196
    assert max(prods) <= ACADOS_TOL_COMP


def test_force_every_step_is_an_acados_interior_point(force_steps):
    """The per-step pin of the force oracle to acados: at every one of the 239 recorded
    samples, acados's u0 equals the u0 of an interior point of the oracle's exact QP whose complementarity
    s_i * lambda_i is at most 1e-6 at every one-sided bound (the first-order fit refined by Gauss-Newton on
    the nonlinear weighted KKT system), to 1e-8 (plot quantisation ~3e-8). acados therefore solved the same
    QP as the oracle and stopped at its default tolerance; the trajectory drift of
    test_force_closed_loop_vs_acados_run is that stopping point carried through the loop."""
    worst, n_exact = 0.0, 0
    for t, m, u in force_steps:
        e, mu, (U, s, lam) = m.interior_point_fit(u, ACADOS_TOL_COMP)
        assert e < 1e-8, (t, e)
        assert (s * lam).max() <= ACADOS_TOL_COMP * (1 + 1e-9) and s.min() > 0 and lam.min() > 0
        worst = max(worst, e)
        n_exact += np.abs(m.u0 - u).max() < 1e-6
    assert n_exact == 21        # steps where acados's u0 is the exact solution to 1e-6 outright


def test_force_acados_tolerance_is_tight(force_steps):
    """The fit needs acados's tolerance: with complementarity capped at 5e-7, the hardest steps (largest
    measured t * lambda) cannot be reproduced — 29 of the 239 steps fail at that cap."""
    by_t = {t: (m, u) for t, m, u in force_steps}
    for t in (146, 36, 106):
        m, u = by_t[t]
        e, _, _ = m.interior_point_fit(u, 5e-7)
        assert e > 1e-5, (t, e)


def test_force_step_fit_rejects_a_wrong_oracle(plots, golden_dir):
    """Control: the same fit against an oracle with the other cost scaling (SURVEY App. B.1 'none')
    fails — acados's inputs are not an interior point of that QP at tolerance 1e-6."""
    from oracle import acados_termination as AT
    ref = np.load(os.path.join(golden_dir, "circle_ref.npz"))["nh30_nx6"]
    spec = models.force_model(30, cost_scaling="none")
    bad = 0
    steps = AT.force_recorded_steps(plots)[:8]
    for t, x, u in steps:
        yref, ye = qp.yref_window(ref[:, :4], ref[:, 4:6], t, 30)
        e, _, _ = AT.StepModel(spec, x, yref, ye).interior_point_fit(u, ACADOS_TOL_COMP, iters=10)
        bad += e > 1e-6
    assert bad >= 7


def test_force_step1_is_acados_termination(plots, golden_dir):
    """Step 1: the state acados reached equals ours (to 1e-8), so both solve the same QP.
    The exact solution has F_x on its lower bound with multiplier ~2.3e-4; acados's plotted
    input lies t ~ 2.7e-3 inside that bound, t * lambda ~ 6e-7 — an interior point stopped at
    complementarity ~1e-6 (acados's default tolerance), not a different problem."""
    ref = np.load(os.path.join(golden_dir, "circle_ref.npz"))["nh30_nx6"]

    def at(j, t):
        i, y = series(plots, FORCE, j)
        return y[np.where(i == t)[0][0]]

    x1 = np.array([at(0, 1), at(1, 1), at(4, 1), at(5, 1)])
    spec = models.force_model(30)
    yref, ye = qp.yref_window(ref[:, :4], ref[:, 4:6], 1, 30)
    Q = qp.CondensedQP(spec, x1, yref, ye)
    U, ml, mu_, ok = Q.polish(*Q.ipm()[:5])
    assert ok
    assert U[0] == pytest.approx(spec.lbu[0], abs=1e-12)          # F_x on its lower bound
    lam = ml[0]
    assert 1e-4 < lam < 5e-4
    th, fd = at(8, 1), at(9, 1)
    fx_acados = fd * np.sin(th)
    t = fx_acados - spec.lbu[0]
    assert 1e-3 < t < 5e-3
    assert 1e-7 < t * lam < 2e-6
    # the other input component agrees to plot precision
    assert fd * np.cos(th) == pytest.approx(U[1], abs=1e-5)
