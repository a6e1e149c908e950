"""Lean closed loop phase cycles (tuning aid, needs a GPU): runs the bench workload on a timing build of
the library (-DNMPC_CLF_TIMING, build.build_experiment) with NMPC_CLF_CYCLES set, then prints where the
cycles of the timed runs go: per phase the total over instances and the share of the slowest instances.

    python tools/clf_phases.py --model force --batch 1024 --steps 20 --regions 3
"""
import argparse
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PHASES = ["prologue", "explicit+test", "pdas", "pdas.solve", "pdas.combo", "gi", "certificate", "outputs",
          "plant+cost", "record", "pdas_rounds", "gi_iters", "slow_steps", "steps", "gi.select", "gi.solve",
          "gi.combo", "gi.hupdate", "pdas.load_set", "pdas.check", "pdas.check.add_states", "pdas.signs",
          "pdas.count", "pdas.check.z"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="force")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--regions", type=int, default=3)
    args = ap.parse_args()
    path = os.path.join(tempfile.mkdtemp(), "cyc.bin")
    os.environ["NMPC_CLF_CYCLES"] = path
    if "NMPC_LIB" not in os.environ:
        from drone_attitude_control_amd import build
        os.environ["NMPC_LIB"] = build.build_experiment("timing", ["NMPC_CLF_TIMING"])
    from drone_attitude_control_amd.batched import ClosedLoop, DEFAULT_N
    cl = ClosedLoop(args.model, args.batch, N=DEFAULT_N[args.model], seed=42)
    cl.run(args.warmup)
    os.remove(path)
    kms = []
    for _ in range(args.regions):
        cl.run(args.steps)
        kms.append(cl.stats()["solve_kernel_ms"] / args.steps)
    cy = np.fromfile(path, dtype=np.uint64).astype(np.float64).reshape(args.regions, args.batch, len(PHASES)).sum(0)
    tot = cy[:, [0, 1, 2, 5, 6, 7, 8, 9]].sum(1)          # the disjoint phases
    order = np.argsort(-tot)
    top = order[:max(1, args.batch // 100)]
    out = {"model": args.model, "batch": args.batch, "kernel_ms_per_step": kms,
           "instance_cycles_p50_p90_p99_max": [float(np.percentile(tot, q)) for q in (50, 90, 99)] + [float(tot.max())],
           "all": {k: float(cy[:, i].sum()) for i, k in enumerate(PHASES)},
           "slowest_1pct": {k: float(cy[top, i].sum()) for i, k in enumerate(PHASES)},
           "worst": {k: float(cy[order[0], i]) for i, k in enumerate(PHASES)}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
