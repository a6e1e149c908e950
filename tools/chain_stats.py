"""Step-chain statistics of the fused closed loop (tuning aid, needs a GPU).

    NMPC_ITER_LOG=1 python tools/chain_stats.py --model quad13 --batch 8192 --steps 20

Runs the bench workload's closed loop in one fused launch per chunk and reads the per-step solve
record (finish steps, IPM iterations, status). A wavefront's time in the fused loop is the sum over
steps of the most expensive of its lane groups' solves; the kernel's time is set by its longest
wavefront chains. Costs in sweep-pair units: a finish step 1 (sweeps A + B), an IPM iteration
`--ipm-cost` (A + B + C + D). One JSON line."""
import argparse
import json
import os
import sys

import numpy as np

os.environ.setdefault("NMPC_ITER_LOG", "1")
os.environ.setdefault("NMPC_CL_FAST", "0")   # the iteration log is the fused lane-per-component kernel's
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from drone_attitude_control_amd.batched import ClosedLoop, DEFAULT_N, workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="quad13")
    ap.add_argument("--N", type=int, default=None)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--skip", type=int, default=3, help="warm-up launch of this many steps first")
    ap.add_argument("--precision", default="fp64")
    ap.add_argument("--ipw", type=int, default=None, help="instances per wavefront (default: 64 // nz)")
    ap.add_argument("--ipm-cost", type=float, default=1.6)
    ap.add_argument("--worst", type=int, default=4, help="print the step records of the longest chains")
    ap.add_argument("--uniform", type=int, default=-1,
                    help="every instance a copy of this one, no noise: the kernel time without a tail")
    args = ap.parse_args()
    N = args.N or DEFAULT_N[args.model]
    if args.uniform >= 0:
        table, off, x = workload(args.model, N, args.batch, seed=42)
        u = args.uniform
        cl = ClosedLoop(args.model, args.batch, N=N, precision=args.precision, table=table,
                        offsets=np.full(args.batch, off[u], dtype=np.int32), x_init=np.repeat(x[u:u + 1], args.batch, 0),
                        noise_std=0.0)
    else:
        cl = ClosedLoop(args.model, args.batch, N=N, precision=args.precision)
    if args.skip:
        cl.run(args.skip)
    cl.run(args.steps)
    st = cl.stats()
    fin, ipm, status = cl.iter_log()
    cost = fin + args.ipm_cost * ipm                       # [steps, B]
    nz = cl.solver.nx + cl.solver.nu
    ipw = args.ipw or max(1, 64 // nz)
    B = args.batch
    W = (B + ipw - 1) // ipw
    pad = np.zeros((cost.shape[0], W * ipw))
    pad[:, :B] = cost
    wave_step = pad.reshape(cost.shape[0], W, ipw).max(axis=2)      # per step: max over the wave's groups
    wave_chain = wave_step.sum(axis=0)
    inst_chain = cost.sum(axis=0)
    hist_f = np.bincount(fin.ravel())
    hist_i = np.bincount(ipm.ravel())
    print(json.dumps({
        "model": args.model, "batch": B, "steps": int(cost.shape[0]), "ipw": ipw,
        "kernel_ms_per_step": st["solve_kernel_ms"] / max(1, st["steps"]),
        "solve_cost_mean": float(cost.mean()), "solve_cost_p99": float(np.percentile(cost, 99)),
        "solve_cost_max": float(cost.max()),
        "inst_chain_mean": float(inst_chain.mean()), "inst_chain_max": float(inst_chain.max()),
        "wave_chain_mean": float(wave_chain.mean()), "wave_chain_p99": float(np.percentile(wave_chain, 99)),
        "wave_chain_max": float(wave_chain.max()),
        "wave_step_sum_over_inst_mean": float(wave_chain.mean() / inst_chain.mean()),
        "finish_steps_hist": hist_f.tolist()[:40], "ipm_iter_hist": hist_i.tolist()[:40],
        "failed": int((status > 0).sum()), "status_hist": np.bincount(status.ravel()).tolist(),
        "frac_solves_one_finish_no_ipm": float(((fin == 1) & (ipm == 0)).mean()),
        "env": {k: v for k, v in os.environ.items() if k.startswith("NMPC_")},
        "worst": [{"inst": int(b), "chain": float(inst_chain[b]),
                   "steps": [[int(fin[s, b]), int(ipm[s, b]), int(status[s, b])] for s in range(cost.shape[0])
                             if cost[s, b] > 1]}
                  for b in np.argsort(-inst_chain)[:args.worst]],
    }))


if __name__ == "__main__":
    main()
