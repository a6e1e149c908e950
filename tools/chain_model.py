"""CPU model of the lean loop's critical chain (tuning aid): the oracle's mode-1 closed loop (the GPU's algorithm)
on the bench workload, per instance and launch the sum of its steps' active-set steps (PDAS rounds + dual-fallback
iterations; env RIC_PATH_COST), i.e. the rare-path work that sets a launch's length.

    python tools/chain_model.py --model quad13 --batch 8192 [--regions 3]
"""
import argparse
import json
import os
import sys

import numpy as np

os.environ["RIC_PATH_COST"] = "1"
CERT = float(os.environ.get("CERT", "0.5"))
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="quad13")
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--regions", type=int, default=3)
    args = ap.parse_args()
    import bench
    from drone_attitude_control_amd.batched import DEFAULT_N
    from drone_attitude_control_amd.sharding import rank_workload
    from oracle import cref, models
    N = DEFAULT_N[args.model]
    table, off, x, _ = rank_workload(args.model, N, args.batch, 1, 0, 42)
    tc, tr, pm, ps = bench.ipm_tolerances(args.model, N)
    cl = cref.ClosedLoopRef(models.MODELS[args.model](N), args.model, table, off, x, mode=1, seed=42,
                            tol_comp=tc, tol_res=tr, polish_mu=pm, polish_steps=ps)
    cl.run(args.warmup)
    out = []
    for _ in range(args.regions):
        _, _, _, path = cl.run(args.steps, logs=True)
        sets = (path >> 4) & 255
        certs = path >> 12
        chain = sets.sum(1)
        cost = sets + CERT * certs   # in PDAS-round units (env CERT: the certificate's cost per round)
        wc = cost.sum(1)
        out.append({"sets_total": int(sets.sum()), "chain_max": int(chain.max()), "chain_p999": float(np.percentile(chain, 99.9)),
                    "chain_p99": float(np.percentile(chain, 99)), "instances_with_sets": int((chain > 0).sum()),
                    "worst": int(chain.argmax()), "worst_steps": sets[chain.argmax()].tolist(),
                    "full": int(((path & 15) == 2).sum()), "certs_total": int(certs.sum()),
                    "cost_max": float(wc.max()), "cost_p999": float(np.percentile(wc, 99.9))})
    print(json.dumps({"model": args.model, "batch": args.batch, "warm_end": os.environ.get("RIC_WARM_END", "0"),
                      "regions": out}))


if __name__ == "__main__":
    main()
