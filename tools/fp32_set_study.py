"""fp32 arithmetic for the lean loop's active-set steps: how far from the exact fp64 solution
does z = z_0 + W[:, S] nu land when (a) W_SS and its solve are fp32, (b) as (a) plus one fp64 refinement of nu on
the fp64 W_SS rows, (c) (b) with the combination W[:, S] nu also in fp32 (fp32 W tiles). CPU study (numpy) on the
force model's bench-workload first-step QPs and their exact active sets (oracle/qp.py), W = M H^-1 M' from the
condensed problem (z = M U + m: the projected inverse Hessian the kernels use, nmpc_api.cpp lqr_wmat).

    python tools/fp32_set_study.py [--model force] [--n 512]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="force")
    ap.add_argument("--n", type=int, default=512)
    args = ap.parse_args()
    from drone_attitude_control_amd.batched import DEFAULT_N, first_step_qps
    from drone_attitude_control_amd.sharding import rank_workload
    from oracle import models, qp
    N = DEFAULT_N[args.model]
    spec = models.MODELS[args.model](N)
    nx, nu = spec.nx, spec.nu
    nz, ne = nx + nu, (N + 1) * (nx + nu)
    table, off, x, _ = rank_workload(args.model, N, args.n, 1, 0, 42)
    X0, Y = first_step_qps(args.model, N, table, off, x)
    ny = Y.shape[1] // 1
    rows = []
    for b in range(args.n):
        ysz = spec.W.shape[0]
        yref = Y[b][:N * ysz].reshape(N, ysz)
        yref_e = Y[b][N * ysz:]
        sol = qp.solve_ocp(spec, X0[b], yref, yref_e)
        if not sol["certified"]:
            continue
        c = qp.CondensedQP(spec, X0[b], yref, yref_e)
        nU = N * nu
        M = np.zeros((ne, nU))
        m = np.zeros(ne)
        for k in range(N + 1):
            M[k * nz:k * nz + nx] = c.Gam[k]
            m[k * nz:k * nz + nx] = c.Phi[k] @ X0[b] + c.d[k]
            if k < N:
                M[k * nz + nx:k * nz + nz, k * nu:(k + 1) * nu] = np.eye(nu)
        Hinv = np.linalg.inv(c.H)
        W = M @ Hinv @ M.T
        U0 = -Hinv @ c.g
        z0 = M @ U0 + m
        z = np.concatenate([np.concatenate([sol["X"][k], sol["U"][k] if k < N else np.zeros(nu)]) for k in range(N + 1)])
        # the active set: bounded decision elements on a bound (stage 0 states pinned, stage N inputs absent)
        S, bS = [], []
        for k in range(N + 1):
            for i in range(nz):
                if (k == 0 and i < nx) or (k == N and i >= nx):
                    continue
                lb, ub = -1e30, 1e30
                if i >= nx and i - nx in list(spec.idxbu):
                    j = list(spec.idxbu).index(i - nx)
                    lb, ub = spec.lbu[j], spec.ubu[j]
                elif i < nx and 0 < k < N and i in list(spec.idxbx):
                    j = list(spec.idxbx).index(i)
                    lb, ub = spec.lbx[j], spec.ubx[j]
                e = k * nz + i
                for bnd in (lb, ub):
                    if abs(bnd) < 1e20 and abs(z[e] - bnd) <= 1e-9 * (1 + abs(bnd)):
                        S.append(e)
                        bS.append(bnd)
        if not S:
            continue
        S = np.array(S)
        t = np.array(bS) - z0[S]
        Wss = W[np.ix_(S, S)]
        nu64 = np.linalg.solve(Wss, t)
        zref = z0 + W[:, S] @ nu64
        W32 = Wss.astype(np.float32)
        nu32 = np.linalg.solve(W32, t.astype(np.float32)).astype(np.float64)
        za = z0 + W[:, S] @ nu32
        r = t - Wss @ nu32
        nur = nu32 + np.linalg.solve(W32, r.astype(np.float32)).astype(np.float64)
        zb = z0 + W[:, S] @ nur
        zc = z0 + (W[:, S].astype(np.float32) @ nur.astype(np.float32)).astype(np.float64)
        sc = max(1.0, np.abs(zref).max())
        rows.append((len(S), np.linalg.cond(Wss), np.abs(za - zref).max() / sc, np.abs(zb - zref).max() / sc,
                     np.abs(zc - zref).max() / sc))
    R = np.array(rows)
    out = {"model": args.model, "N": N, "qps": len(R), "by_set_size": []}
    for lo, hi in ((1, 4), (5, 8), (9, 16), (17, 24), (25, 32), (33, 99)):
        sel = (R[:, 0] >= lo) & (R[:, 0] <= hi)
        if sel.any():
            out["by_set_size"].append({"m": f"{lo}-{hi}", "count": int(sel.sum()), "cond_max": float(R[sel, 1].max()),
                                       "fp32_solve_max": float(R[sel, 2].max()), "fp32_solve_1_refine_max": float(R[sel, 3].max()),
                                       "plus_fp32_combination_max": float(R[sel, 4].max())})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
