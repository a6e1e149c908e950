"""Generate QP / closed-loop golden vectors from the CPU oracle (oracle/).

    python tests/golden/make_qp_golden.py

Inputs are seeded synthetic instances built on the reference's own circle table
(tests/golden/circle_ref.npz, generated from generate_trajectory.py by make_golden.py) and
the seed-42 noise stream (main.py:44). Expected outputs are the oracle's KKT-certified
exact QP solutions (oracle/qp.py) and its closed-loop restatement (oracle/closed_loop.py).
These fixtures pin the HIP engine to the oracle; the oracle itself is pinned to the
reference through the fixtures of make_golden.py and to acados's own recorded run through
tests/golden/reference_plots.npz (extract_reference_plots.py).

    python tests/golden/make_qp_golden.py [qp] [qp_rt] [closed_loop]
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import closed_loop as CL  # noqa: E402
from oracle import models, qp  # noqa: E402

CASES = [("force", 20), ("force", 30), ("jerk", 40), ("jerk", 30), ("quad13", 20)]
PER_CASE = 48
# horizons the fast solve has no compiled (fully unrolled) kernel for: its runtime-horizon sf_kernel variants
# (N = 3: a single LDS slot, N below the chunk of 4 stages) — qp_cases_rt.npz
CASES_RT = [("force", 10), ("force", 3), ("jerk", 20), ("quad13", 30)]
PER_CASE_RT = 32


def reference_table(name, N):
    refs = np.load(os.path.join(HERE, "circle_ref.npz"))
    if f"nh{N}_nx6" in refs:
        base = refs[f"nh{N}_nx6"]
    else:   # a horizon the reference fixture does not hold: the same table (generate_trajectory.py:7-28)
        from oracle.trajectory import gen_circle_traj
        base = gen_circle_traj(500, N, 6, 2)
    if name == "force":
        return base[:, :4], base[:, 4:6]
    if name == "jerk":
        return base[:, :6], base[:, 6:]
    r = models.quad13_reference(500, N)
    return r[:, :13], r[:, 13:]


def perturbed_x0(name, xr, t, rng):
    x0 = xr[t].copy()
    x0[:2] += rng.normal(0, 0.05, 2)
    if name == "force":
        x0[2:4] += rng.normal(0, 0.1, 2)
        x0[2:4] = np.clip(x0[2:4], -0.95, 0.95)
    elif name == "jerk":
        x0[2:4] += rng.normal(0, 0.1, 2)
        x0[2:4] = np.clip(x0[2:4], -0.95, 0.95)
        x0[4:6] += rng.normal(0, 0.3, 2)
    else:
        x0[2] += rng.normal(0, 0.1)
        x0[3:6] += rng.normal(0, 0.1, 3)
        x0[3:6] = np.clip(x0[3:6], -0.9, 0.9)
        x0[7:10] += rng.normal(0, 0.02, 3)
        x0[10:13] += rng.normal(0, 0.2, 3)
    x0[:2] = np.clip(x0[:2], -1.15, 1.15)
    return x0


def qp_cases(cases=CASES, per_case=PER_CASE, seed=20251121, fname="qp_cases.npz"):
    out = {}
    rng = np.random.default_rng(seed)
    for name, N in cases:
        spec = models.MODELS[name](N)
        xr, ur = reference_table(name, N)
        X0, Y, XS, US, COST = [], [], [], [], []
        while len(X0) < per_case:
            t = int(rng.integers(0, 500))
            x0 = perturbed_x0(name, xr, t, rng)
            yref, yref_e = qp.yref_window(xr, ur, t, N)
            sol = qp.solve_ocp(spec, x0, yref, yref_e)
            if not sol["certified"]:
                continue
            X0.append(x0)
            Y.append(np.concatenate([yref.ravel(), yref_e]))
            XS.append(sol["X"])
            US.append(sol["U"])
            COST.append(sol["cost"])
        key = f"{name}_N{N}"
        out[key + "_x0"] = np.array(X0)
        out[key + "_yref"] = np.array(Y)
        out[key + "_X"] = np.array(XS)
        out[key + "_U"] = np.array(US)
        out[key + "_cost"] = np.array(COST)
        print(key, "done")
    np.savez_compressed(os.path.join(HERE, fname), **out)
    print("wrote", fname)


def closed_loops():
    """The whole seed-42 main.py run (main.py:43-46): force for all 500 steps
    (params.py:119), then jerk continuing the same noise stream, x0 = [1, 0, 0, 0.62], at the
    reference default N_horizon = 30 (params.py:121) and at the BASELINE N = 20. Stored per
    run: Xsim (501 x 4), the controller inputs U, the plant inputs (theta, F_d), a, the
    closed-loop cost (controller.py:40-41,54) and the AED (store_results.py:233-236, as
    main.py:23 computes it from ref[:N_sim] and Xsim[:N_sim])."""
    noise = np.load(os.path.join(HERE, "noise_seed42.npy"))
    refs = np.load(os.path.join(HERE, "circle_ref.npz"))
    cl = {}
    for N in (20, 30):
        ref = refs[f"nh{N}_nx6"]
        x0 = np.array([1.0, 0, 0, 0.62])
        ns = CL.NoiseStream(noise)
        for name, run, xr, ur in (("force", CL.force_follow_trajectory, ref[:, :4], ref[:, 4:6]),
                                  ("jerk", CL.jerk_follow_trajectory, ref[:, :6], ref[:, 6:])):
            c, X, a, Up, Uc = run(models.MODELS[name](N), xr, ur, x0, ns)
            k = f"{name}_N{N}"
            cl[k + "_X"], cl[k + "_U"], cl[k + "_Uplant"], cl[k + "_a"], cl[k + "_cost"] = X, Uc, Up, a, c
            cl[k + "_aed"] = CL.calc_aed(ref[:500, :2], X[:500, :2])
        cl[f"noise_used_N{N}"] = np.array(ns.i)
        print("closed loops N", N, "done")
    np.savez_compressed(os.path.join(HERE, "closed_loop.npz"), **cl)
    print("wrote closed_loop.npz")


def main():
    what = sys.argv[1:] or ["qp", "qp_rt", "closed_loop"]
    if "qp" in what:
        qp_cases()
    if "qp_rt" in what:
        qp_cases(CASES_RT, PER_CASE_RT, 20261018, "qp_cases_rt.npz")
    if "closed_loop" in what:
        closed_loops()


if __name__ == "__main__":
    main()
