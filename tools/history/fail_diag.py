"""Find the first failed solve of a device closed loop and save its inputs (GPU diagnostic).

    python tools/fail_diag.py --model jerk --batch 4096 --steps 23 --out gpurun_out/fail.npz

Runs the closed loop one step at a time, reads the per-instance status/iteration arrays from
the device after every step, and stores (step, instance, status, iters, x0, offset) of every
failed solve plus the state trajectory of the failing instances, for replay on the CPU oracle.
"""
import argparse
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from drone_attitude_control_amd.batched import DEFAULT_N, ClosedLoop, workload  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="jerk")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=23)
    ap.add_argument("--precision", default="fp64")
    ap.add_argument("--out", default="gpurun_out/fail.npz")
    a = ap.parse_args()
    N = DEFAULT_N[a.model]
    table, offsets, x_init = workload(a.model, N, a.batch, 42)
    cl = ClosedLoop(a.model, a.batch, N=N, precision=a.precision, table=table, offsets=offsets,
                    x_init=x_init, seed=42)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]

    def dev_int(field):
        p = ctypes.c_void_p()
        assert cl.lib.nmpc_device_ptr(cl.solver._h, field.encode(), ctypes.byref(p)) == 0
        out = np.zeros(a.batch, np.int32)
        assert hip.hipMemcpy(out.ctypes.data, p, out.nbytes, 2) == 0
        return out

    rec = {"step": [], "inst": [], "status": [], "iters": [], "x0": [], "offset": []}
    states = [cl.state()]
    for s in range(a.steps):
        x0 = states[-1]
        cl.run(1, sync=True)
        st, it = dev_int("status"), dev_int("qp_iter")
        states.append(cl.state())
        bad = np.nonzero(st != 0)[0]
        nonfinite = int((~np.isfinite(states[-1])).any(axis=1).sum())
        print(f"step {s}: failed {bad.size} nonfinite-state {nonfinite} max_iter {it.max()} "
              f"mean_iter {it.mean():.2f}", flush=True)
        for b in bad:
            rec["step"].append(s)
            rec["inst"].append(int(b))
            rec["status"].append(int(st[b]))
            rec["iters"].append(int(it[b]))
            rec["x0"].append(x0[b].copy())
            rec["offset"].append(int(offsets[b]))
            print(f"   inst {b} status {st[b]} iters {it[b]} x0 {np.array2string(x0[b], precision=4)}")
    np.savez(a.out, **{k: np.array(v) for k, v in rec.items()}, table=table,
             states=np.array(states), N=N)


if __name__ == "__main__":
    main()
