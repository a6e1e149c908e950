"""Exact solution of one NMPC step's QP, certified by KKT (test infrastructure only).

What is restated: `AcadosOcpSolver.solve()` as called at `force_model/controller.py:30-32`
and `jerk_model/controller.py:31-33` after `set_up_ocp` (`force_model/ocp.py:117-122`).
For the reference's LTI models with LINEAR_LS cost and box constraints, SQP-GN converges
after one QP, so solve() == the unique minimiser of the box-constrained LQ-OCP
(SURVEY §0 "Key simplification", Appendix B).

Method (deliberately different from the GPU's stage-wise Riccati recursion):
  1. condense: eliminate states, X = Phi x0 + Gamma U + d; dense H, g, C;
  2. Mehrotra predictor-corrector IPM on the dense QP (numpy Cholesky);
  3. active-set polish: solve the equality-constrained KKT system on the identified
     active set, then verify every KKT condition (stationarity, primal feasibility,
     dual sign, complementarity). A strictly convex QP (R > 0) has exactly one KKT point,
     so a passing certificate proves the solution exact to rounding.
"""
import numpy as np


class CondensedQP:
    """min 1/2 U'HU + g'U  s.t.  lo <= C U <= hi   (U = [u_0; ...; u_{N-1}])."""

    def __init__(self, spec, x0, yref, yref_e):
        nx, nu, N = spec.nx, spec.nu, spec.N
        A, B, c = spec.A, spec.B, spec.c
        s = spec.scaling()
        nU = N * nu
        # state maps: x_k = Phi_k x0 + Gam_k U + d_k
        Phi = [np.eye(nx)]
        Gam = [np.zeros((nx, nU))]
        d = [np.zeros(nx)]
        for k in range(N):
            G = A @ Gam[k]
            G[:, k * nu:(k + 1) * nu] += B
            Gam.append(G)
            Phi.append(A @ Phi[k])
            d.append(A @ d[k] + c)
        self.Phi, self.Gam, self.d = Phi, Gam, d
        x0 = np.asarray(x0, float)
        H = np.zeros((nU, nU))
        g = np.zeros(nU)
        const = 0.0
        for k in range(N + 1):
            if k < N:
                Psi = spec.Vx @ Gam[k]
                Psi[:, k * nu:(k + 1) * nu] += spec.Vu
                psi = spec.Vx @ (Phi[k] @ x0 + d[k]) - yref[k]
                Wk = s[k] * spec.W
            else:
                Psi = spec.Vx_e @ Gam[N]
                psi = spec.Vx_e @ (Phi[N] @ x0 + d[N]) - yref_e
                Wk = s[N] * spec.W_e
            H += Psi.T @ Wk @ Psi
            g += Psi.T @ Wk @ psi
            const += 0.5 * psi @ Wk @ psi
        rows, lo, hi = [], [], []
        for k in range(N):
            for j, i in enumerate(spec.idxbu):
                r = np.zeros(nU)
                r[k * nu + i] = 1.0
                rows.append(r)
                lo.append(spec.lbu[j])
                hi.append(spec.ubu[j])
        for k in range(1, N + 1):
            idx, lb, ub = ((spec.idxbx, spec.lbx, spec.ubx) if k < N
                           else (spec.idxbx_e, spec.lbx_e, spec.ubx_e))
            off = Phi[k] @ x0 + d[k]
            for j, i in enumerate(idx):
                rows.append(Gam[k][i].copy())
                lo.append(lb[j] - off[i])
                hi.append(ub[j] - off[i])
        self.H, self.g, self.const = H, g, const
        self.C = np.array(rows).reshape(-1, nU)
        self.lo, self.hi = np.array(lo), np.array(hi)
        self.spec, self.x0 = spec, x0

    def states(self, U):
        return np.array([self.Phi[k] @ self.x0 + self.Gam[k] @ U + self.d[k]
                         for k in range(self.spec.N + 1)])

    def cost(self, U):
        return 0.5 * U @ self.H @ U + self.g @ U + self.const

    # ---------------------------------------------------------------- IPM
    def ipm(self, tol=1e-13, max_iter=100):
        H, g, C, lo, hi = self.H, self.g, self.C, self.lo, self.hi
        m = C.shape[0]
        U = np.zeros(H.shape[0])
        CU = C @ U
        t_l = np.maximum(CU - lo, 1.0)
        t_u = np.maximum(hi - CU, 1.0)
        lam_l = np.ones(m)
        lam_u = np.ones(m)
        it = 0
        for it in range(1, max_iter + 1):
            CU = C @ U
            r_d = H @ U + g - C.T @ lam_l + C.T @ lam_u
            r_pl = CU - lo - t_l
            r_pu = hi - CU - t_u
            mu = (lam_l @ t_l + lam_u @ t_u) / (2 * m)
            scale = 1.0 + max(np.abs(g).max(), np.abs(H).max())
            if (mu < tol and np.abs(r_d).max() < tol * scale
                    and max(np.abs(r_pl).max(), np.abs(r_pu).max()) < tol * 10):
                break
            D = lam_l / t_l + lam_u / t_u
            K = H + C.T @ (D[:, None] * C)
            try:
                L = np.linalg.cholesky(K)
            except np.linalg.LinAlgError:
                # barrier terms ~1/mu swamp H at the very end: the iterate is already at
                # rounding level and the active-set polish below finishes the job
                break

            def solve(rc_l, rc_u):
                rhs = -(r_d + C.T @ ((rc_l + lam_l * r_pl) / t_l) - C.T @ ((rc_u + lam_u * r_pu) / t_u))
                dU = np.linalg.solve(L.T, np.linalg.solve(L, rhs))
                CdU = C @ dU
                dt_l = CdU + r_pl
                dt_u = -CdU + r_pu
                dl_l = (-rc_l - lam_l * dt_l) / t_l
                dl_u = (-rc_u - lam_u * dt_u) / t_u
                return dU, dt_l, dt_u, dl_l, dl_u

            def max_step(v, dv):
                neg = dv < 0
                return min(1.0, np.min(-v[neg] / dv[neg])) if neg.any() else 1.0

            aff = solve(lam_l * t_l, lam_u * t_u)
            a_aff = min(max_step(t_l, aff[1]), max_step(t_u, aff[2]),
                        max_step(lam_l, aff[3]), max_step(lam_u, aff[4]))
            mu_aff = ((t_l + a_aff * aff[1]) @ (lam_l + a_aff * aff[3])
                      + (t_u + a_aff * aff[2]) @ (lam_u + a_aff * aff[4])) / (2 * m)
            sigma = (mu_aff / mu) ** 3
            dU, dt_l, dt_u, dl_l, dl_u = solve(lam_l * t_l + aff[1] * aff[3] - sigma * mu,
                                              lam_u * t_u + aff[2] * aff[4] - sigma * mu)
            a = min(max_step(t_l, dt_l), max_step(t_u, dt_u),
                    max_step(lam_l, dl_l), max_step(lam_u, dl_u))
            a = min(1.0, 0.995 * a)
            U = U + a * dU
            t_l, t_u = t_l + a * dt_l, t_u + a * dt_u
            lam_l, lam_u = lam_l + a * dl_l, lam_u + a * dl_u
        return U, lam_l, lam_u, t_l, t_u, it

    # ---------------------------------------------------------------- polish + certificate
    def polish(self, U, lam_l, lam_u, t_l, t_u):
        H, g, C, lo, hi = self.H, self.g, self.C, self.lo, self.hi
        act_l = lam_l > t_l
        act_u = lam_u > t_u
        for _ in range(20):
            A = np.vstack([C[act_l], C[act_u]])
            b = np.concatenate([lo[act_l], hi[act_u]])
            n, na = H.shape[0], A.shape[0]
            K = np.zeros((n + na, n + na))
            K[:n, :n] = H
            K[:n, n:] = -A.T
            K[n:, :n] = -A
            rhs = np.concatenate([-g, -b])
            sol = np.linalg.lstsq(K, rhs, rcond=None)[0]
            Up = sol[:n]
            nu_ = sol[n:]       # multipliers: H U + g - A_l' nu_l + A_u' nu_u = 0 (sign below)
            nl = int(act_l.sum())
            ml = np.zeros_like(lam_l)
            mu_ = np.zeros_like(lam_u)
            ml[act_l] = nu_[:nl]
            mu_[act_u] = -nu_[nl:]
            CU = C @ Up
            viol_l = lo - CU
            viol_u = CU - hi
            bad_p_l = (~act_l) & (viol_l > 1e-11 * (1 + np.abs(lo)))
            bad_p_u = (~act_u) & (viol_u > 1e-11 * (1 + np.abs(hi)))
            bad_d_l = act_l & (ml < -1e-11)
            bad_d_u = act_u & (mu_ < -1e-11)
            if not (bad_p_l.any() or bad_p_u.any() or bad_d_l.any() or bad_d_u.any()):
                return Up, ml, mu_, True
            act_l = (act_l & ~bad_d_l) | bad_p_l
            act_u = (act_u & ~bad_d_u) | bad_p_u
        return U, lam_l, lam_u, False

    def kkt_residuals(self, U, ml, mu_):
        H, g, C, lo, hi = self.H, self.g, self.C, self.lo, self.hi
        CU = C @ U
        stat = H @ U + g - C.T @ ml + C.T @ mu_
        return {
            "stationarity": float(np.abs(stat).max()),
            "primal": float(max(0.0, (lo - CU).max(initial=0.0), (CU - hi).max(initial=0.0))),
            "dual": float(max(0.0, -ml.min(initial=0.0), -mu_.min(initial=0.0))),
            "complementarity": float(max(np.abs(ml * (CU - lo)).max(initial=0.0),
                                         np.abs(mu_ * (hi - CU)).max(initial=0.0))),
        }


def solve_ocp(spec, x0, yref, yref_e):
    """One NMPC step. Returns dict with X ((N+1) x nx, X[0] = x0), U (N x nu), cost
    (acados get_cost() semantics: 1/2-weighted, time-step-scaled), certified flag, kkt."""
    qp = CondensedQP(spec, x0, yref, yref_e)
    U, ll, lu, tl, tu, it = qp.ipm()
    Up, ml, mu_, ok = qp.polish(U, ll, lu, tl, tu)
    kkt = qp.kkt_residuals(Up, ml, mu_)
    scale = 1.0 + np.abs(qp.g).max() + np.abs(qp.H).max()
    certified = ok and kkt["stationarity"] < 1e-9 * scale and kkt["primal"] < 1e-9 \
        and kkt["dual"] < 1e-9
    return {
        "X": qp.states(Up), "U": Up.reshape(spec.N, spec.nu), "cost": float(qp.cost(Up)),
        "certified": bool(certified), "kkt": kkt, "ipm_iters": it,
        "U_ipm": U.reshape(spec.N, spec.nu),
    }


def yref_window(xref, uref, t, N):
    """set_up_ocp (force_model/ocp.py:117-122): yref_k = [xref[t+k], uref[t+k]] for k<N and
    yref_N = xref[t+N]."""
    yref = np.hstack([xref[t:t + N], uref[t:t + N]])
    return yref, np.asarray(xref[t + N], float)
