"""Lean closed loop check (tuning aid, needs a GPU): the default closed loop (lean loop for quad13 /
jerk) against the C oracle's restatement of the same algorithm (mode 1) and the exact loop (mode 0),
on the bench workload; prints the max state error, failures, and the per-step time of the launches.

    python tools/clf_check.py --model quad13 --batch 8192 --steps 20
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from drone_attitude_control_amd.batched import ClosedLoop, DEFAULT_N, workload  # noqa: E402
from drone_attitude_control_amd.models import OCPS  # noqa: E402
from oracle import cref, models  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="quad13")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--repeats", type=int, default=3)
    ap.add_argument("--oracle", type=int, default=1)
    args = ap.parse_args()
    m, B = args.model, args.batch
    N = DEFAULT_N[m]
    cl = ClosedLoop(m, B, N=N, seed=42)
    t0 = time.perf_counter()
    cl.run(args.warmup)
    tw = time.perf_counter() - t0
    regions, kms, launches = [], [], []
    for _ in range(args.repeats):
        t0 = time.perf_counter()
        cl.run(args.steps)
        regions.append(time.perf_counter() - t0)
        st = cl.stats()
        kms.append(st["solve_kernel_ms"] / args.steps)
        launches.append(st["solve_launches"])
    out = {"model": m, "batch": B, "warmup_s": tw, "region_ms": [r * 1e3 for r in regions],
           "ms_per_step": float(np.median(regions)) / args.steps * 1e3, "kernel_ms_per_step": kms,
           "launches": launches, "steps_per_s": B * args.steps / float(np.median(regions)),
           "failed": cl.stats()["failed"]}
    if args.oracle:
        total = args.warmup + args.repeats * args.steps
        table, off, x = workload(m, N, B, 42)
        o = OCPS[m](N).solver_options
        for mode in (1, 0) if B <= 512 else (1,):
            ref = cref.ClosedLoopRef(getattr(models, f"{m}_model")(N), m, table, off, x, mode=mode, seed=42,
                                     tol_comp=o.qp_solver_tol_comp, tol_res=o.qp_solver_tol_stat)
            ref.run(total)
            s = cl.state()
            err = np.abs(s - ref.state).max(1) / np.maximum(1.0, np.abs(ref.state).max(1))
            acc = cl.instance_stats()
            out[f"mode{mode}"] = {"max_state_err": float(err.max()), "worst": int(err.argmax()),
                                  "fail_equal": bool(np.array_equal(acc[:, 2:], ref.acc[:, 2:])),
                                  "cost_rel": float(np.abs(acc[:, 0] - ref.acc[:, 0]).max() / max(1e-300, np.abs(ref.acc[:, 0]).max()))}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
