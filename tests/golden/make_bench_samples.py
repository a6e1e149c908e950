"""Certified oracle solutions for a sample of the BASELINE-size bench workloads' first-step QPs.

    python tests/golden/make_bench_samples.py

For each BASELINE.json config solved on one GPU — force N=20 B=1024 (fp64) and B=8192 (fp32),
jerk N=40 B=4096, quad13 N=20 B=8192 — the global synthetic workload of bench.py
(batched.workload, seed 42) defines B first-step QPs (batched.first_step_qps). 64 instances,
spread over the batch (instance 0 = main.py's start, the rest seeded), are solved by the
KKT-certified dense oracle (oracle/qp.py). tests/test_gpu_solver.py solves the FULL batch on
the GPU and compares these instances.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from drone_attitude_control_amd.batched import first_step_qps, workload  # noqa: E402
from oracle import models, qp  # noqa: E402

CONFIGS = [("force", 20, 1024), ("force", 20, 8192), ("jerk", 40, 4096), ("quad13", 20, 8192)]
SAMPLE = 64


def main():
    out = {}
    for name, N, B in CONFIGS:
        table, offsets, x = workload(name, N, B, seed=42)
        X0, Y = first_step_qps(name, N, table, offsets, x)
        rng = np.random.default_rng(B * 1000 + N)
        idx = np.unique(np.concatenate([[0, B - 1], rng.choice(B, SAMPLE - 2, replace=False)]))[:SAMPLE]
        spec = models.MODELS[name](N)
        XS, US, ok = [], [], []
        for b in idx:
            y = Y[b]
            sol = qp.solve_ocp(spec, X0[b], y[:N * spec.ny].reshape(N, spec.ny), y[N * spec.ny:])
            ok.append(sol["certified"])
            XS.append(sol["X"])
            US.append(sol["U"])
        key = f"{name}_N{N}_B{B}"
        out[key + "_idx"] = idx.astype(np.int64)
        out[key + "_X"] = np.array(XS)
        out[key + "_U"] = np.array(US)
        out[key + "_certified"] = np.array(ok)
        print(key, "certified", int(np.sum(ok)), "of", len(idx))
    np.savez_compressed(os.path.join(HERE, "bench_samples.npz"), **out)


if __name__ == "__main__":
    main()
