"""Make tests/golden/qp_failure.npz: a closed-loop jerk OCP whose factorisation breaks down.

Input: gpurun_out/fail.npz from `python tools/fail_diag.py --model jerk --batch 4096` (GPU
closed loop, seed 42): the first instance whose solve returned status 4. Its x0 (the plant
state after 18 noisy closed-loop steps, px = 1.1992 against the 1.2 position bound) and yref
window are stored together with the C oracle's answer (oracle/c/riccati_ipm.c): status 4 — since
round 2 from the interval infeasibility certificate before the first iteration (x_1 cannot meet
the position bound), with the initial point as the iterate; before, F_uu lost positive
definiteness at iteration 9.

    python tests/golden/make_failure_case.py [gpurun_out/fail.npz]
    python tests/golden/make_failure_case.py --refresh   # same inputs, the current oracle's answer
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import cref, models  # noqa: E402


def main(src):
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "qp_failure.npz")
    if src == "--refresh":
        d = np.load(out)
        x0, y, N, step, off = d["jerk_N40_x0"][0], d["jerk_N40_yref"][0], 40, -1, -1
        spec = models.MODELS["jerk"](N)
    else:
        d = np.load(src)
        N = int(d["N"])
        step, off, x0 = int(d["step"][0]), int(d["offset"][0]), d["x0"][0]
        spec = models.MODELS["jerk"](N)
        table = d["table"]
        t = (off + step) % 500
        y = np.concatenate([table[t:t + N, :spec.ny].ravel(), table[t + N, :spec.nx]])
    X, U, st, it = cref.RiccatiIpmRef(spec).solve(x0[None], y[None], nthreads=1)
    assert st[0] == 4, st
    np.savez(out, jerk_N40_x0=x0[None], jerk_N40_yref=y[None], jerk_N40_X=X, jerk_N40_U=U,
             jerk_N40_status=st, jerk_N40_iters=it)
    print(f"{out}: step {step} offset {off} x0 {x0} -> status {st[0]} after {it[0]} iterations")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "fail.npz"))
