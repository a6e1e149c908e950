"""The C oracle's closed loop (oracle/c/riccati_ipm.c riccati_ipm_closed_loop) on CPU:

  * pinned to the existing oracle chain: main.py's seed-42 run (force then jerk on one noise
    stream, x0 = [1, 0, 0, 0.62], src/main.py:43-46; src/force_model/controller.py:8-56,
    src/jerk_model/controller.py:8-58) reproduces tests/golden/closed_loop.npz — the numpy
    restatement whose jerk run matches acados's own recorded run (test_reference_plots.py);
  * mode 1 (the GPU's warm-started fast finish, restated) gives mode 0's exact closed loops;
  * it reproduces the committed bench-workload goldens (tests/golden/closed_loop_bench.npz) that
    the GPU parity test (test_gpu_bench_parity.py) checks the device against.
"""
import os

import numpy as np
import pytest

from oracle import cref, models

REGIONS = [3] + [20] * 10


@pytest.fixture(scope="module")
def mainpy(golden_dir):
    return (np.load(os.path.join(golden_dir, "closed_loop.npz")),
            np.load(os.path.join(golden_dir, "noise_seed42.npy")),
            np.load(os.path.join(golden_dir, "circle_ref.npz")))


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("N", [20, 30])
@pytest.mark.parametrize("model", ["force", "jerk"])
def test_main_py_run(mainpy, model, N, mode):
    gold, noise, refs = mainpy
    ref = refs[f"nh{N}_nx6"]
    table = ref[:, :6] if model == "force" else ref
    x0 = np.array([[1.0, 0, 0, 0.62] + ([0.0, 9.81] if model == "jerk" else [])])
    nt = (noise[:500] if model == "force" else noise[500:1000])[None]
    spec = getattr(models, f"{model}_model")(N)
    cl = cref.ClosedLoopRef(spec, model, table, np.array([0]), x0, mode=mode, noise_table=nt)
    u, xs, st, _ = cl.run(500, logs=True)
    X = gold[f"{model}_N{N}_X"]
    assert np.abs(xs[0, :, :4] - X[1:501]).max() < 1e-9
    assert (st == 0).all()
    assert cl.acc[0, 0] == pytest.approx(float(gold[f"{model}_N{N}_cost"]), rel=1e-9)
    assert cl.acc[0, 1] / 1000 == pytest.approx(float(gold[f"{model}_N{N}_aed"]), rel=1e-9)
    if model == "jerk":
        assert np.abs(xs[0, :, 4:] - gold[f"jerk_N{N}_a"]).max() < 1e-9


@pytest.mark.parametrize("model,N,B", [("quad13", 20, 8192), ("force", 20, 8192), ("jerk", 40, 4096)])
def test_bench_goldens(golden_dir, model, N, B):
    """64 of the golden instances (the first 32 — failures and bound riders first — and 32 spaced):
    mode 0 reproduces the committed checkpoints, mode 1 agrees with them."""
    from drone_attitude_control_amd.batched import workload
    from drone_attitude_control_amd.models import OCPS
    g = np.load(os.path.join(golden_dir, "closed_loop_bench.npz"))
    key = f"{model}_N{N}_B{B}"
    sel = g[f"{key}_sel"]
    pick = np.unique(np.concatenate([np.arange(32), np.linspace(32, len(sel) - 1, 32).astype(int)]))
    ids = sel[pick]
    table, off, x = workload(model, N, B, 42)
    o = OCPS[model](N).solver_options
    for mode in (0, 1):
        cl = cref.ClosedLoopRef(getattr(models, f"{model}_model")(N), model, table, off[ids], x[ids], mode=mode,
                                instance_ids=ids, tol_comp=o.qp_solver_tol_comp, tol_res=o.qp_solver_tol_stat)
        S, A = [], []
        for n in REGIONS:
            cl.run(n)
            S.append(cl.state.copy())
            A.append(cl.acc.copy())
        S, A = np.array(S), np.array(A)
        Sg, Ag = g[f"{key}_states"][:, pick], g[f"{key}_sums"][:, pick]
        tol = 1e-12 if mode == 0 else 1e-8
        err = np.abs(S - Sg).max(-1) / np.maximum(1.0, np.abs(Sg).max(-1))
        assert err.max() < tol, (mode, err.max())
        assert np.array_equal(A[..., 2:], Ag[..., 2:])
        np.testing.assert_allclose(A[..., :2], Ag[..., :2], rtol=tol, atol=1e-12)


def test_philox_stream_matches_its_definition():
    """The Philox noise of a subset (instance_ids) equals the full batch's stream for those ids:
    a subset reproduces the full batch's closed loops (what the goldens rely on)."""
    from drone_attitude_control_amd.batched import workload
    table, off, x = workload("quad13", 20, 64, 3)
    spec = models.quad13_model(20)
    full = cref.ClosedLoopRef(spec, "quad13", table, off, x, mode=1, seed=3)
    full.run(30)
    ids = np.array([5, 17, 63])
    sub = cref.ClosedLoopRef(spec, "quad13", table, off[ids], x[ids], mode=1, seed=3, instance_ids=ids)
    sub.run(30)
    assert np.array_equal(sub.state, full.state[ids])
    assert np.array_equal(sub.acc, full.acc[ids])
