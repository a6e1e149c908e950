"""Where acados stops: the recorded force run re-posed step by step (TEST INFRASTRUCTURE ONLY).

The one acados force run the reference holds is the seed-42 `main.py` run plotted in
`experiment_data/img/example_acc_trajectory_component.pdf` (`src/main.py:43-46` ->
`src/force_model/controller.py:25-41`, `qp_solver='PARTIAL_CONDENSING_HPIPM'`, `nlp_solver_type='SQP'`,
`src/force_model/ocp.py:83-93`). The plot holds, for every surviving sample t, the full force state
Xsim[t] (`store_results.py:157-163`) and the plant input (theta, F_d)[t] that acados's u0 was converted
to (`controller.py:37-44`, converter `force_model/dynamics.py:64-69`). So each step's QP can be posed
again from acados's OWN state (`force_model/ocp.py:117-122`, x0 pinned as `controller.py:29-31`), which
removes the closed loop's drift from the comparison.

acados does not return the exact QP solution: SQP + HPIPM stop at the default tolerances (1e-6 on the
stationarity / equality / inequality / complementarity residuals, acados_template defaults [ext]). What
this module decides per step is whether acados's u0 is the exact solution displaced by an interior point
whose complementarity is at most `tau` for every one-sided bound:

  * exact solution z*, multipliers lambda* and slacks s* (`qp.CondensedQP`, certified by KKT);
  * first-order model of a terminated interior point: a bound i with complementarity mu_i sits
      - active (lambda*_i > 0): mu_i / lambda*_i inside its bound  (a shift of that bound),
      - inactive (slack s*_i): pushed by a barrier force mu_i / s*_i along its row;
    so u0 = u0* + J mu with J's columns the KKT sensitivities of u0 to those perturbations;
  * `fit`: the smallest-residual mu in [0, tau]^m (bounded least squares);
  * `weighted_point`: the nonlinear check — a primal-dual Newton solve of the QP's KKT system with
    s_i * lambda_i = mu_i exactly (mu_i = 0: the bound's ordinary complementarity) returns that
    interior point itself, whose u0 is compared with acados's.
The smallest tau that explains a step (`min_tau`) is that step's complementarity, measured.
"""
import numpy as np

from . import qp

DT = 0.02
FORCE_FIG = "example_acc_trajectory_component"
# store_results.py:157-191 for the force figure (4 axes): p0/p1 = XSim[:, 0/1] (positions),
# p4/p5 = XSim[:, 2/3] (velocities), p8 = theta, p9 = F_d
STATE_PATHS = (0, 1, 4, 5)
THETA_PATH, FD_PATH = 8, 9


def plot_series(plots, fig, j):
    """{sample index: value} of one plotted polyline; every vertex sits on t = k * dt."""
    p = plots[f"{fig}__p{j}"]
    idx = p[:, 0] / DT
    k = np.round(idx).astype(int)
    assert np.abs(idx - k).max() < 1e-5
    return dict(zip(k.tolist(), p[:, 1].tolist()))


def force_recorded_steps(plots):
    """[(t, x_t, u0_t)] for every sample t at which all four states and both plant inputs survive
    in the plot; u0 = (F_x, F_z) = F_d (sin theta, cos theta) inverts the converter
    (force_model/dynamics.py:64-69: theta = atan2(F_x, F_z), F_d = |F|)."""
    S = {j: plot_series(plots, FORCE_FIG, j) for j in STATE_PATHS + (THETA_PATH, FD_PATH)}
    common = sorted(set.intersection(*[set(s) for s in S.values()]))
    out = []
    for t in common:
        x = np.array([S[j][t] for j in STATE_PATHS])
        th, fd = S[THETA_PATH][t], S[FD_PATH][t]
        out.append((t, x, np.array([fd * np.sin(th), fd * np.cos(th)])))
    return out


class StepModel:
    """One step's QP (condensed, `qp.CondensedQP`), its exact certified solution and the first-order
    sensitivity of u0 to a complementarity mu_i at every finite one-sided bound."""

    def __init__(self, spec, x0, yref, yref_e):
        Q = qp.CondensedQP(spec, x0, yref, yref_e)
        U, ml, mu_, ok = Q.polish(*Q.ipm()[:5])
        assert ok, "exact solution not certified"
        self.Q, self.U, self.nu = Q, U, spec.nu
        # one-sided rows a_i U >= beta_i (lower: C, lo; upper: -C, -hi)
        a = np.vstack([Q.C, -Q.C])
        beta = np.concatenate([Q.lo, -Q.hi])
        lam = np.concatenate([ml, mu_])
        fin = np.isfinite(beta)
        self.a, self.beta, self.lam = a[fin], beta[fin], lam[fin]
        self.s = self.a @ U - self.beta
        self.active = self.lam > 0
        n = Q.H.shape[0]
        Aa = self.a[self.active]
        na = Aa.shape[0]
        K = np.zeros((n + na, n + na))
        K[:n, :n] = Q.H
        K[:n, n:] = -Aa.T
        K[n:, :n] = Aa
        Kinv = np.linalg.inv(K)[:self.nu]
        J = np.empty((self.nu, self.a.shape[0]))
        ia = np.where(self.active)[0]
        J[:, ia] = Kinv[:, n:] / self.lam[ia]                 # bound shift mu / lambda
        ii = np.where(~self.active)[0]
        J[:, ii] = (Kinv[:, :n] @ self.a[ii].T) / self.s[ii]   # barrier force mu / s along a_i
        self.J = J

    @property
    def u0(self):
        return self.U[:self.nu]

    def reach(self, tau):
        """Largest |u0 - u0*| component the first-order model allows with every mu_i <= tau."""
        return tau * max(np.clip(self.J, 0, None).sum(1).max(), -np.clip(self.J, None, 0).sum(1).min())

    def fit(self, u0_obs, tau):
        """(mu, residual): mu in [0, tau]^m with J mu closest to u0_obs - u0* (max-norm residual)."""
        from scipy.optimize import lsq_linear
        d = u0_obs - self.u0
        sc = max(np.abs(d).max(), 1e-12)
        r = lsq_linear(self.J * (tau / sc), d / sc, bounds=(0.0, 1.0), method="bvls", tol=1e-14)
        mu = r.x * tau
        return mu, float(np.abs(self.J @ mu - d).max())

    def min_tau(self, u0_obs, resid=2e-8, lo=1e-13, hi=1e-4):
        """Smallest tau (bisection, 2 % resolution) whose first-order model explains u0_obs to `resid`."""
        if self.fit(u0_obs, hi)[1] > resid:
            return np.inf
        while hi / lo > 1.02:
            m = np.sqrt(lo * hi)
            if self.fit(u0_obs, m)[1] <= resid:
                hi = m
            else:
                lo = m
        return hi

    def interior_point_fit(self, u0_obs, tau, iters=30, tol=1e-10):
        """Gauss-Newton over mu in [0, tau]^m on the nonlinear map mu -> u0(weighted_point(mu)),
        started from the first-order `fit`. At a weighted point the Newton system gives
        du/dmu_i = [K^-1 a_i / s_i]_u0 with K = H + a' diag(lam / s) a. Returns
        (residual max|u0(mu) - u0_obs|, mu, (U, s, lam))."""
        from scipy.optimize import lsq_linear
        mu, _ = self.fit(u0_obs, tau)
        H, a = self.Q.H, self.a
        for _ in range(iters):
            U, s, lam = self.weighted_point(mu)
            d = u0_obs - U[:self.nu]
            e = float(np.abs(d).max())
            if e < tol:
                break
            J = np.linalg.solve(H + a.T @ ((lam / s)[:, None] * a), a.T / s)[:self.nu]
            r = lsq_linear(J * (tau / e), d / e, bounds=(-mu / tau, (tau - mu) / tau), method="bvls", tol=1e-14)
            mu = np.clip(mu + r.x * tau, 0.0, tau)
        return e, mu, (U, s, lam)

    def weighted_point(self, mu, iters=200):
        """The interior point itself: primal-dual Newton on H U + g - a' lam = 0, a U - beta = s,
        s_i lam_i = mu_i (a target of max(mu_i, kappa), kappa driven to 1e-18), from a cold start.
        Returns (U, s, lam)."""
        H, g, a, beta = self.Q.H, self.Q.g, self.a, self.beta
        U = np.zeros(H.shape[0])
        s = np.maximum(a @ U - beta, 1.0)
        lam = np.ones_like(s)
        kappa = float(s @ lam) / s.size
        for _ in range(iters):
            kappa = max(0.2 * kappa, 1e-18)
            tgt = np.maximum(mu, kappa)
            r_d = H @ U + g - a.T @ lam
            r_p = a @ U - beta - s
            w = (tgt - s * lam - lam * r_p) / s
            K = H + a.T @ ((lam / s)[:, None] * a)
            dU = np.linalg.solve(K, -r_d + a.T @ w)
            ds = a @ dU + r_p
            dl = (tgt - s * lam - lam * ds) / s
            al = 1.0
            for v, dv in ((s, ds), (lam, dl)):
                neg = dv < 0
                if neg.any():
                    al = min(al, 0.99 * float(np.min(-v[neg] / dv[neg])))
            U, s, lam = U + al * dU, s + al * ds, lam + al * dl
            if kappa <= 1e-18 and al == 1.0 and np.abs(dU).max() < 1e-15 * (1 + np.abs(U).max()):
                break
        return U, s, lam
