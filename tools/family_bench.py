"""Solve-kernel time per kernel family on the BASELINE configs' first-step QPs (tuning aid).

    python tools/family_bench.py [--families lpc,wave,cond] [--reps 10]

For each config the bench's global workload (batched.workload, seed 42) gives B first-step QPs
(batched.first_step_qps); every family solves them `reps` times and the median device time of
the solve kernel (HIP events, nmpc_get_stats) is printed with the mean IPM iterations, one JSON
line per (config, family)."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from drone_attitude_control_amd import AcadosOcpSolver  # noqa: E402
from drone_attitude_control_amd.batched import first_step_qps, workload  # noqa: E402
from drone_attitude_control_amd.models import OCPS  # noqa: E402

CONFIGS = [("force", 20, 1024, "fp64"), ("force", 20, 8192, "fp32"), ("force", 20, 8192, "fp64"),
           ("jerk", 40, 4096, "fp64"), ("quad13", 20, 8192, "fp64"), ("quad13", 20, 8192, "fp32")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--families", default="lpc,wave,cond")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--configs", default="")
    args = ap.parse_args()
    sel = [c for c in CONFIGS if not args.configs or f"{c[0]}{c[1]}_{c[2]}_{c[3]}" in args.configs.split(",")]
    for name, N, B, prec in sel:
        table, off, x = workload(name, N, B, seed=42)
        X0, Y = first_step_qps(name, N, table, off, x)
        for fam in args.families.split(","):
            os.environ["NMPC_KERNEL"] = fam
            try:
                s = AcadosOcpSolver(OCPS[name](N), batch=B, precision=prec)
            except Exception as e:  # noqa: BLE001
                print(json.dumps({"config": f"{name} N={N} B={B} {prec}", "family": fam, "error": str(e)[:200]}))
                continue
            finally:
                os.environ.pop("NMPC_KERNEL", None)
            s.set_batch("x0", X0)
            s.set_batch("yref", Y)
            ts = []
            for r in range(args.reps + 2):
                s.solve()
                st = np.zeros(5)
                s.lib.nmpc_get_stats(s._h, st.ctypes.data_as(__import__("ctypes").POINTER(__import__("ctypes").c_double)), 5)
                if r >= 2:
                    ts.append(st[3])
            status = s.get_batch_int("status")
            it = s.get_batch_int("qp_iter")
            print(json.dumps({"config": f"{name} N={N} B={B} {prec}", "family": fam,
                              "kernel": s.launch_info()["kernel"], "ms": float(np.median(ts)),
                              "ms_min": float(np.min(ts)), "mean_iter": float(it.mean()), "max_iter": int(it.max()),
                              "failed": int((status != 0).sum()), "launch": s.launch_info()}), flush=True)


if __name__ == "__main__":
    main()
