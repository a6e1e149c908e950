"""Make tests/golden/qp_infeasible.npz: closed-loop QPs the interval certificate proves infeasible.

Input: the hard QPs dumped along the bench's device closed loops (tools/cl_iter_hist.py --dump,
gpurun_out/r2c_hard_{jerk,quad13}.npz: seed-42 workload, steps with > 6 Newton systems). Kept:
the instances whose QP the C oracle (oracle/c/riccati_ipm.c) proves infeasible before the first
iteration (status 4, 0 iterations), with the oracle's answer (the initial point).

    python tests/golden/make_infeasible_cases.py [gpurun_out]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import cref, models  # noqa: E402


def main(src):
    out = {}
    for name, N, keep in [("jerk", 40, 8), ("quad13", 20, 4)]:
        d = np.load(os.path.join(src, f"r2c_hard_{name}.npz"))
        spec = models.MODELS[name](N)
        X, U, st, it = cref.RiccatiIpmRef(spec).solve(d["x0"], d["yref"])
        sel = np.nonzero((st == 4) & (it == 0))[0][:keep]
        out[f"{name}_N{N}_x0"], out[f"{name}_N{N}_yref"] = d["x0"][sel], d["yref"][sel]
        out[f"{name}_N{N}_X"], out[f"{name}_N{N}_U"] = X[sel], U[sel]
        print(name, len(sel), "infeasible cases")
    np.savez(os.path.join(os.path.dirname(os.path.abspath(__file__)), "qp_infeasible.npz"), **out)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out"))
