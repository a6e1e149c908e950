"""Dump the closed-loop QPs of the instances with the longest step chains (tuning aid, GPU).

    NMPC_ITER_LOG=1 python tools/dump_hard.py --model quad13 --out gpurun_out/hard_quad13.npz

Runs the bench workload's closed loop one fused step per launch (the same computation as longer
launches: the warm start and the noise are keyed by the global step), records every instance's state
before each step and the step's solve record, and saves for the `--worst` longest chains the QPs of
every step (x0, yref window) with their (finish steps, IPM iterations, status)."""
import argparse
import os
import sys

import numpy as np

os.environ.setdefault("NMPC_ITER_LOG", "1")
os.environ.setdefault("NMPC_CL_FAST", "0")   # the iteration log is the fused lane-per-component kernel's
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from drone_attitude_control_amd.batched import ClosedLoop, DEFAULT_N, first_step_qps, workload  # noqa: E402
from drone_attitude_control_amd.params import ExperimentParameters  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="quad13")
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--skip", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--worst", type=int, default=16)
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    N = DEFAULT_N[args.model]
    period = ExperimentParameters().N
    table, off, x = workload(args.model, N, args.batch, seed=42)
    cl = ClosedLoop(args.model, args.batch, N=N, table=table, offsets=off, x_init=x)
    if args.skip:
        cl.run(args.skip)
    states, logs = [], []
    for s in range(args.steps):
        states.append(cl.state())
        cl.run(1)
        fin, ipm, st = cl.iter_log()
        logs.append(np.stack([fin[0], ipm[0], st[0]], axis=1))
    states = np.array(states)            # [steps, B, nx]
    logs = np.array(logs)                # [steps, B, 3]
    cost = logs[:, :, 0] + 1.6 * logs[:, :, 1]
    chain = cost.sum(axis=0)
    worst = np.argsort(-chain)[:args.worst]
    X0, Y, L, S, I = [], [], [], [], []
    for b in worst:
        for s in range(args.steps):
            x0, y = first_step_qps(args.model, N, table, np.array([(off[b] + args.skip + s) % period]), states[s, b][None])
            X0.append(x0[0])
            Y.append(y[0])
            L.append(logs[s, b])
            S.append(s)
            I.append(b)
    np.savez(args.out, x0=np.array(X0), yref=np.array(Y), log=np.array(L), step=np.array(S), inst=np.array(I),
             chain=chain, mean_chain=chain.mean())
    print("worst chains", chain[worst].round(1).tolist(), "mean", round(float(chain.mean()), 2))


if __name__ == "__main__":
    main()
