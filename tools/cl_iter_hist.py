"""Per-step solve statistics along the bench's device closed loop (tuning aid).

    python tools/cl_iter_hist.py --model quad13 --batch 8192 --steps 20 [--polish-steps 12]

At every step the closed loop's current states (nmpc_closed_loop_get_state) and yref windows are
solved again on a second handle, so the per-instance qp_iter / status of the step and the solve
kernel's duration are visible (the closed loop itself keeps only sums). One JSON line per step."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from drone_attitude_control_amd import AcadosOcpSolver  # noqa: E402
from drone_attitude_control_amd.batched import ClosedLoop, first_step_qps, workload  # noqa: E402
from drone_attitude_control_amd.models import OCPS  # noqa: E402
from drone_attitude_control_amd.params import ExperimentParameters  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="quad13")
    ap.add_argument("--N", type=int, default=20)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--precision", default="fp64")
    ap.add_argument("--polish-mu", type=float, default=None)
    ap.add_argument("--polish-steps", type=int, default=None)
    ap.add_argument("--kernel", default=None)
    ap.add_argument("--dump", default="", help="npz path: the QPs of instances above --dump-iter")
    ap.add_argument("--dump-iter", type=int, default=6)
    args = ap.parse_args()
    dump = {"x0": [], "yref": [], "iters": [], "step": []}
    period = ExperimentParameters().N
    table, off, x = workload(args.model, args.N, args.batch, seed=42)
    cl = ClosedLoop(args.model, args.batch, N=args.N, precision=args.precision, table=table, offsets=off, x_init=x)
    ocp = OCPS[args.model](args.N)
    if args.polish_mu is not None:
        ocp.solver_options.qp_solver_polish_mu = args.polish_mu
    if args.polish_steps is not None:
        ocp.solver_options.qp_solver_polish_steps = args.polish_steps
    if args.kernel:
        os.environ["NMPC_KERNEL"] = args.kernel
    s = AcadosOcpSolver(ocp, batch=args.batch, precision=args.precision)
    os.environ.pop("NMPC_KERNEL", None)
    for step in range(args.steps):
        X0, Y = first_step_qps(args.model, args.N, table, (np.asarray(off) + step) % period, cl.state())
        s.set_batch("x0", X0)
        s.set_batch("yref", Y)
        s.solve()
        s.solve()   # second launch on the same inputs: its time is the one reported
        it, st = s.get_batch_int("qp_iter"), s.get_batch_int("status")
        vals, cnt = np.unique(it, return_counts=True)
        print(json.dumps({"step": step, "kernel_ms": s.get_stats("time_tot") * 1e3,
                          "mean_iter": float(it.mean()), "max_iter": int(it.max()),
                          "hist": {int(v): int(c) for v, c in zip(vals, cnt)}, "status": np.bincount(st).tolist()}),
              flush=True)
        sel = np.nonzero(it > args.dump_iter)[0]
        dump["x0"] += list(X0[sel])
        dump["yref"] += list(Y[sel])
        dump["iters"] += list(it[sel])
        dump["step"] += [step] * len(sel)
        cl.run(1)
    if args.dump:
        np.savez(args.dump, **{k: np.array(v) for k, v in dump.items()})


if __name__ == "__main__":
    main()
