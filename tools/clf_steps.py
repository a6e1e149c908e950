"""Lean closed loop step record (tuning aid, needs a GPU): runs the bench workload with NMPC_ITER_LOG and
prints the distribution of per-step wall time (ns) and active-set steps, and the per-instance totals that
set a launch's time (the slowest wavefront).

    python tools/clf_steps.py --model force --batch 1024 --steps 20
"""
import argparse
import json
import os
import sys

import numpy as np

os.environ["NMPC_ITER_LOG"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from drone_attitude_control_amd.batched import ClosedLoop, DEFAULT_N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="force")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--regions", type=int, default=5)
    args = ap.parse_args()
    cl = ClosedLoop(args.model, args.batch, N=DEFAULT_N[args.model], seed=42)
    cl.run(args.warmup)
    out = []
    for _ in range(args.regions):
        cl.run(args.steps)
        it, st, kc = cl.iter_log()
        raw = lambda r: it[r].astype(np.int64) | (st[r].astype(np.int64) << 8) | (kc[r].astype(np.int64) << 16)
        t_start, t_end = raw(-2), raw(-1)           # the last two rows: each instance's start / end ticks
        life = (t_end - t_start) * 10
        rel0 = (t_start - t_start.min()) * 10
        rel1 = (t_end - t_start.min()) * 10
        it, st, kc = it[:-2], st[:-2], kc[:-2]
        cyc = kc.astype(np.int64) * 10   # ns (wall_clock64 ticks at 100 MHz)
        tot = cyc.sum(0)
        worst = int(tot.argmax())
        q = lambda a: [float(np.percentile(a, x)) for x in (50, 90, 99, 99.9, 100)]
        out.append({"kernel_ms_per_step": cl.stats()["solve_kernel_ms"] / args.steps,
                    "step_ns_p50_90_99_999_max": q(cyc.ravel()),
                    "instance_total_ns_p50_90_99_max": q(tot)[:3] + [int(tot.max())],
                    "instance_launch_ns_p50_90_99_max": q(life)[:3] + [int(life.max())],
                    "instance_start_ns_from_first_p0_50_90_100": [float(np.percentile(rel0, x)) for x in (0, 50, 90, 100)],
                    "instance_end_ns_from_first_p10_50_90_100": [float(np.percentile(rel1, x)) for x in (10, 50, 90, 100)],
                    "worst_instance": worst, "worst_steps_ns": cyc[:, worst].tolist(),
                    "worst_steps_iters": it[:, worst].tolist(),
                    "iters_hist": np.bincount(np.minimum(it.ravel(), 40)).tolist()})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
