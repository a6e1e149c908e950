"""Generate the golden fixtures under tests/golden/ from the reference itself.

Run once in the build container (the reference is NOT present on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What is imported from the reference (read-only, nothing is written there):
  * src/params.py            -> DroneData / ExperimentParameters constants (params.py:10-122)
  * src/generate_trajectory.py -> gen_circle_traj (generate_trajectory.py:7-28)
Both import with numpy + xml only. acados/casadi are absent, so the
QP solve itself cannot be run here; QP fixtures come from oracle/ (see make_qp_golden.py).

Outputs (small data files, inputs + expected outputs only):
  params.json                    scalar constants + URDF-derived inertia (for quad13)
  circle_ref.npz                 gen_circle_traj(500, Nh, nx, 2, [0,0], 1) for Nh in {20,30,40}, nx in {4,6}
  noise_seed42.npy               np.random.seed(42); 1000 x normal(0, 0.01)  (main.py:44, ocp.py:114)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SRC = "/root/reference/src"


def main():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF_SRC)
    import params  # noqa: E402  (reference module)
    import generate_trajectory  # noqa: E402  (reference module)

    dd = params.DroneData()
    p = params.ExperimentParameters()
    out = {
        "MASS": dd.MASS, "GRAVITY_ACC": dd.GRAVITY_ACC, "GRAVITY": dd.GRAVITY,
        "max_F": dd.max_F, "min_F": dd.min_F,
        "min_p_x": dd.min_p_x, "max_p_x": dd.max_p_x, "min_p_z": dd.min_p_z, "max_p_z": dd.max_p_z,
        "min_v_x": dd.min_v_x, "max_v_x": dd.max_v_x, "min_v_z": dd.min_v_z, "max_v_z": dd.max_v_z,
        "min_a_x": dd.min_a_x, "max_a_x": dd.max_a_x, "min_a_z": dd.min_a_z, "max_a_z": dd.max_a_z,
        "min_jerk": dd.min_jerk, "max_jerk": dd.max_jerk,
        "L": dd.L, "KF": dd.KF, "KM": dd.KM, "THRUST2WEIGHT_RATIO": dd.THRUST2WEIGHT_RATIO,
        "J_diag": [float(v) for v in np.diag(dd.J)],
        "URDF_MASS": float(dd._parse_urdf_parameters(dd.URDF_PATH)[0]),
        "T": p.T, "dt": p.dt, "dt_conv": p.dt_conv, "ctrls_per_sample": p.ctrls_per_sample,
        "N": p.N, "N_conv": p.N_conv, "N_horizon": p.N_horizon, "noise": p.noise,
    }
    with open(os.path.join(HERE, "params.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)

    refs = {}
    for nh in (20, 30, 40):
        for nx in (4, 6):
            refs[f"nh{nh}_nx{nx}"] = generate_trajectory.gen_circle_traj(
                p.N, nh, nx=nx, nu=2, center=[0, 0], radius=1)
    np.savez(os.path.join(HERE, "circle_ref.npz"), **refs)

    np.random.seed(42)
    noise = np.array([np.random.normal(0, p.noise) for _ in range(1000)])
    np.save(os.path.join(HERE, "noise_seed42.npy"), noise)
    print("wrote params.json, circle_ref.npz, noise_seed42.npy")


if __name__ == "__main__":
    main()
