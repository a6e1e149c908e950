"""Golden closed loops of the bench workloads (tests/golden/closed_loop_bench.npz).

The batched Monte-Carlo closed loop bench.py times (batched.workload(model, N, B, seed=42): start
rows, initial states, the device's Philox noise stream, shared reference table) restated by the
C oracle (oracle/c/riccati_ipm.c riccati_ipm_closed_loop, mode 0: every QP solved cold to its
exact, KKT-accepted solution) for a subset of instances, at the bench's launch boundaries
(3 warm-up steps, then 10 regions of 20: checkpoints after 3, 23, ..., 203 steps):

  * every instance whose closed loop has a failed (status 4) solve,
  * the instances with the most full solves in the GPU's algorithm (oracle mode 1: the
    warm-started fast finish; they ride state bounds or leave the feasible set),
  * evenly spaced others, up to 256 per workload.

Stored per workload: sel (instance indices), states [12][n][nx] and per-instance sums
[12][n][4] (cost, AED numerator, failed solves, steps) at the checkpoints, and the failed-step
indices. The closed loop of an instance depends only on its own start row, initial state and
noise (Philox keyed by the global instance id), so a subset reproduces the full batch's loops.

    python tests/golden/make_closed_loop_bench.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

WORKLOADS = (("quad13", 20, 8192), ("force", 20, 8192), ("jerk", 40, 4096))
CHECKPOINTS = [3] + [20] * 10          # bench.py: --warmup 3, --repeats 10 x --steps 20
NSEL = 256


def oracle_loop(model, N, table, offsets, x_init, mode, ids=None, seed=42):
    from drone_attitude_control_amd.models import OCPS
    from oracle import cref, models
    spec = getattr(models, f"{model}_model")(N)
    o = OCPS[model](N).solver_options
    return cref.ClosedLoopRef(spec, model, table, offsets, x_init, mode=mode, seed=seed, instance_ids=ids,
                              tol_comp=o.qp_solver_tol_comp, tol_res=o.qp_solver_tol_stat)


def run_checkpoints(loop):
    states, sums, status = [], [], []
    for n in CHECKPOINTS:
        _, _, st, _ = loop.run(n, logs=True)
        states.append(loop.state.copy())
        sums.append(loop.acc.copy())
        status.append(st)
    return np.array(states), np.array(sums), np.concatenate(status, axis=1)


def select(model, N, B):
    from drone_attitude_control_amd.batched import workload
    table, off, x = workload(model, N, B, 42)
    fast = oracle_loop(model, N, table, off, x, mode=1)
    _, _, st, path = fast.run(sum(CHECKPOINTS), logs=True)
    fails = np.flatnonzero((st != 0).any(1))
    full = (path == 2).sum(1)
    order = [i for i in np.argsort(-full, kind="stable") if i not in set(fails)]
    sel = list(fails) + order[:64]
    rest = [i for i in np.linspace(0, B - 1, NSEL).astype(int) if i not in set(sel)]
    sel = np.array(sorted(set(sel + rest[:max(0, NSEL - len(sel))])), dtype=np.int64)
    return table, off, x, sel


def main():
    out = {}
    for model, N, B in WORKLOADS:
        table, off, x, sel = select(model, N, B)
        ref = oracle_loop(model, N, table, off[sel], x[sel], mode=0, ids=sel)
        S, A, st = run_checkpoints(ref)
        alt = oracle_loop(model, N, table, off[sel], x[sel], mode=1, ids=sel)
        S1, A1, st1 = run_checkpoints(alt)
        print(f"{model} N={N} B={B}: {len(sel)} instances, {int((st != 0).sum())} failed solves; "
              f"oracle mode 0 vs mode 1: states {np.abs(S1 - S).max():.2e}, "
              f"sums {np.abs(A1 - A).max() / max(1.0, np.abs(A).max()):.2e} rel, "
              f"failed steps equal {np.array_equal(st != 0, st1 != 0)}; dense KKT pass: "
              f"{ref.stats()['kkt_corrected']:.0f} sets corrected, {ref.stats()['kkt_unsettled']:.0f} unsettled")
        key = f"{model}_N{N}_B{B}"
        out[f"{key}_sel"] = sel
        out[f"{key}_states"] = S
        out[f"{key}_sums"] = A
        out[f"{key}_failed"] = (st != 0).astype(np.int8)
    out["checkpoints"] = np.cumsum(CHECKPOINTS)
    np.savez_compressed(os.path.join(HERE, "closed_loop_bench.npz"), **out)


if __name__ == "__main__":
    main()
