/*
 * riccati_ipm.c — plain-C fp64 reference of the batched NMPC step solve.
 * TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): used by tests/ as a second,
 * stage-wise implementation next to the dense numpy oracle, and by bench.py's
 * cpu_baseline leg ("port": OpenMP over instances on the host cores).
 *
 * What it restates: one `AcadosOcpSolver.solve()` per instance
 * (src/force_model/controller.py:30-32, src/jerk_model/controller.py:31-33) for the
 * reference's LTI / LINEAR_LS / box-constrained OCPs (force_model/ocp.py:21-96,
 * jerk_model/ocp.py:20-95): SQP-GN == one QP, solved by a Mehrotra predictor-corrector
 * interior-point method whose Newton systems are solved by a backward Riccati recursion
 * over the N stages — the algorithm class of HPIPM's OCP-QP IPM [ext; HPIPM is not in
 * the tree]. It is the same algorithm, step for step, as the HIP kernel
 * (drone-attitude-control_amd/csrc/nmpc_kernels.hip), so its mean iteration count is
 * the n_ipm used for the roofline's algorithmic flop count.
 *
 * Problem per instance (stage k = 0..N, z_k = [x_k; u_k], z_N = x_N, x_0 = x0 pinned):
 *   min  sum_k 1/2 z_k' H z_k + (G yref_k)' z_k  +  1/2 x_N' He x_N + (Ge yref_N)' x_N
 *   s.t. x_{k+1} = A x_k + B u_k + c,   lb_k <= z_k <= ub_k  (|bound| >= 1e20: absent)
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define NZMAX 32
#define INFB 1e20

typedef struct {
    int nx, nu, N, ny, ny_e;
    const double *A, *B, *c;    /* row-major nx*nx, nx*nu, nx */
    const double *H, *G;        /* nz*nz, nz*ny (stage cost, already scaled) */
    const double *He, *Ge;      /* nx*nx, nx*ny_e */
    const double *lb0, *ub0;    /* nz (x part ignored) */
    const double *lb, *ub;      /* nz, stages 1..N-1 */
    const double *lbe, *ube;    /* nx, stage N */
    double tol_comp, tol_res, mu0;
    int max_iter;
    double polish_mu;           /* > 0: exact finish (active-set polish) once mu <= polish_mu */
    int polish_steps;           /* active-set Newton steps per finish attempt */
} ocp_ref_desc;

static int has(double b) { return fabs(b) < INFB; }

/* per-instance workspace sizes */
typedef struct {
    double *z, *ll, *lu, *dza, *dz, *gc, *gf, *gh, *re, *Pr, *Luu, *Lxu, *lu_vec, *sg;
    signed char *act;   /* finish: active bound per element (-1 lower, 1 upper, 0 none) */
} ws_t;

/* Relative weight of the exact finish's penalty on the identified active bounds: the
 * penalised solution sits lambda / rho from the bound and rho / |F| costs about eps * rho / |F|
 * in the Schur complements; the refinement step removes the first to first order, so a moderate
 * weight keeps the second small (1e5..1e7 give the same 1e-11 answers on the goldens, 1e8
 * starts to lose accepted solutions to rounding) */
#ifndef POLISH_RHO
#define POLISH_RHO 1e6
#endif
/* acceptance of the exact finish, relative to 1 + |bound|: an inactive bound may be violated by
 * POLISH_TOL (the result is clamped onto it); an active bound's multiplier rho * (bound - z)
 * must not fall below -rho * POLISH_TOL_ACTIVE (a few ulps: a wrongly fixed bound shows up as
 * a negative multiplier, i.e. z on the feasible side of the bound) */
#ifndef POLISH_TOL
#define POLISH_TOL 1e-9
#endif
#ifndef POLISH_TOL_ACTIVE
#define POLISH_TOL_ACTIVE 1e-15
#endif
/* largest refinement correction accepted, relative to 1 + |z| */
#define POLISH_TOL_REFINE 1e-3

static void interior(double *v, double l, double u)
{
    if (has(l) && has(u)) {
        double d = 0.01 * (u - l);
        if (*v < l + d) *v = l + d;
        if (*v > u - d) *v = u - d;
    } else if (has(l)) {
        double d = 0.01 * (fabs(l) > 1.0 ? fabs(l) : 1.0);
        if (*v < l + d) *v = l + d;
    } else if (has(u)) {
        double d = 0.01 * (fabs(u) > 1.0 ? fabs(u) : 1.0);
        if (*v > u - d) *v = u - d;
    }
}

/* bound accessors: stage k, component i */
static double LBk(const ocp_ref_desc *d, int k, int i)
{
    if (k == d->N) return d->lbe[i];
    if (k == 0) return i < d->nx ? -1e30 : d->lb0[i];
    return d->lb[i];
}
static double UBk(const ocp_ref_desc *d, int k, int i)
{
    if (k == d->N) return d->ube[i];
    if (k == 0) return i < d->nx ? 1e30 : d->ub0[i];
    return d->ub[i];
}

/* Backward Riccati factorisation of the Newton system with barrier / penalty Hessian diagonal
 * w->sg and gradient `gr` (stage-stacked, nz per stage): fills the per-stage records Pr, Luu,
 * Lxu, lu_vec used by the forward substitution. Returns 1 on a non-positive pivot. */
static int backward(const ocp_ref_desc *d, ws_t *w, const double *gr)
{
    const int nx = d->nx, nu = d->nu, N = d->N, nz = nx + nu;
    const double *A = d->A, *B = d->B;
    double P[NZMAX * NZMAX], M[NZMAX * NZMAX], F[NZMAX * NZMAX], p[NZMAX], v[NZMAX], h[NZMAX];
    int k, i, j, l;
    for (i = 0; i < nx; i++) {
        for (j = 0; j < nx; j++) P[i * nx + j] = d->He[i * nx + j];
        P[i * nx + i] += w->sg[N * nz + i];
        p[i] = gr[N * nz + i];
    }
    for (k = N - 1; k >= 0; k--) {
        double *Pr = &w->Pr[k * nx], *Luu = &w->Luu[k * nu * nu], *Lxu = &w->Lxu[k * nx * nu];
        double *luv = &w->lu_vec[k * nu];
        for (i = 0; i < nx; i++) {
            double s = 0.0;
            for (j = 0; j < nx; j++) s += P[i * nx + j] * w->re[k * nx + j];
            Pr[i] = s;
            v[i] = s + p[i];
        }
        /* M = P [A B]  (nx x nz) */
        for (i = 0; i < nx; i++)
            for (j = 0; j < nz; j++) {
                double s = 0.0;
                for (l = 0; l < nx; l++)
                    s += P[i * nx + l] * (j < nx ? A[l * nx + j] : B[l * nu + (j - nx)]);
                M[i * nz + j] = s;
            }
        /* F = [A B]' M + H + Sigma ; h = [A B]' v + gr */
        for (i = 0; i < nz; i++) {
            for (j = 0; j < nz; j++) {
                double s = d->H[i * nz + j];
                for (l = 0; l < nx; l++)
                    s += (i < nx ? A[l * nx + i] : B[l * nu + (i - nx)]) * M[l * nz + j];
                F[i * nz + j] = s;
            }
            double s = gr[k * nz + i];
            for (l = 0; l < nx; l++) s += (i < nx ? A[l * nx + i] : B[l * nu + (i - nx)]) * v[l];
            h[i] = s;
            F[i * nz + i] += w->sg[k * nz + i];
        }
        /* Luu = chol(F_uu) (row-major lower) */
        for (i = 0; i < nu; i++)
            for (j = 0; j <= i; j++) {
                double s = F[(nx + i) * nz + nx + j];
                for (l = 0; l < j; l++) s -= Luu[i * nu + l] * Luu[j * nu + l];
                if (i == j) {
                    if (!(s > 0.0)) return 1;
                    Luu[i * nu + i] = sqrt(s);
                } else {
                    Luu[i * nu + j] = s / Luu[j * nu + j];
                }
            }
        /* Lxu = F_xu Luu^-T  (row i: forward substitution) */
        for (i = 0; i < nx; i++)
            for (j = 0; j < nu; j++) {
                double s = F[i * nz + nx + j];
                for (l = 0; l < j; l++) s -= Lxu[i * nu + l] * Luu[j * nu + l];
                Lxu[i * nu + j] = s / Luu[j * nu + j];
            }
        /* l_u = Luu^-1 h_u */
        for (j = 0; j < nu; j++) {
            double s = h[nx + j];
            for (l = 0; l < j; l++) s -= Luu[j * nu + l] * luv[l];
            luv[j] = s / Luu[j * nu + j];
        }
        if (k > 0) {
            for (i = 0; i < nx; i++) {
                for (j = 0; j < nx; j++) {
                    double s = F[i * nz + j];
                    for (l = 0; l < nu; l++) s -= Lxu[i * nu + l] * Lxu[j * nu + l];
                    P[i * nx + j] = s;
                }
                double s = h[i];
                for (l = 0; l < nu; l++) s -= Lxu[i * nu + l] * luv[l];
                p[i] = s;
            }
        }
    }
    return 0;
}

/* Infeasibility certificate (interval reachability): X_0 = {x0}; X_{k+1} = hull([A B] (X_k x U_k)
 * + c) intersected with the state box of stage k+1, in midpoint / radius form. The hull
 * over-approximates the reachable set, so an empty X_{k+1} proves that no input sequence keeps the
 * states inside their boxes: the QP is infeasible (typically a closed-loop state pushed past a
 * position bound with the velocity still pointing out). Returns the first empty stage, 0 if none
 * (which proves nothing). Tolerance 1e-9 relative on the emptiness test. */
static int infeasible_stage(const ocp_ref_desc *d, const double *x0)
{
    const int nx = d->nx, nu = d->nu, N = d->N;
    double m[NZMAX], r[NZMAX], mn[NZMAX], rn[NZMAX], mu[NZMAX], ru[NZMAX];
    for (int j = 0; j < nu; j++) {
        const double l = d->lb0[nx + j], u = d->ub0[nx + j];   /* input boxes are stage-invariant */
        mu[j] = has(l) && has(u) ? 0.5 * (l + u) : 0.0;
        ru[j] = has(l) && has(u) ? 0.5 * (u - l) : INFINITY;
    }
    for (int i = 0; i < nx; i++) { m[i] = x0[i]; r[i] = 0.0; }
    for (int k = 0; k < N; k++) {
        for (int i = 0; i < nx; i++) {
            double s = d->c[i], t = 0.0;
            for (int j = 0; j < nx; j++) {
                const double a = d->A[i * nx + j];
                s += a * m[j];
                if (a != 0.0) t += fabs(a) * r[j];   /* (a zero entry times an unbounded radius adds 0) */
            }
            for (int j = 0; j < nu; j++) {
                const double b = d->B[i * nu + j];
                s += b * mu[j];
                if (b != 0.0) t += fabs(b) * ru[j];
            }
            mn[i] = s;
            rn[i] = t;
        }
        for (int i = 0; i < nx; i++) {
            const double lb = k + 1 == N ? d->lbe[i] : d->lb[i], ub = k + 1 == N ? d->ube[i] : d->ub[i];
            double lo = mn[i] - rn[i], hi = mn[i] + rn[i];
            if (has(lb) && lb > lo) lo = lb;
            if (has(ub) && ub < hi) hi = ub;
            if (lo > hi + 1e-9 * (1.0 + fabs(hi))) return k + 1;
            if (isfinite(lo) && isfinite(hi)) { m[i] = 0.5 * (lo + hi); r[i] = 0.5 * (hi - lo); }
            else { m[i] = mn[i]; r[i] = rn[i]; }
        }
    }
    return 0;
}

/* Acceptance test and active-set update of one exact-finish set step (step w->dz from w->z, active
 * flags w->act). Accepted (returns 1) when every active bound keeps a non-negative multiplier
 * rho (bound - z_new) (to POLISH_TOL_ACTIVE) and every inactive bound holds (to POLISH_TOL) — the
 * QP's KKT conditions. Otherwise the bounds with a negative multiplier leave the set and the violated
 * input bounds join; of the violated state bounds only each component's most violated one joins, and
 * only in the run's first step or in a step without removals. (Adding every violated state bound
 * together with the removals — the textbook PDAS update — cycles on a state bound active over a
 * stretch of stages, a velocity limit reached along the horizon: the multipliers of consecutive
 * stages alternate in sign and the set flips back and forth. On the 320 closed-loop QPs of the 16
 * longest quad13 bench chains (tools/dump_hard.py) this rule takes 2.7 Newton systems per solve
 * instead of 6.1, at most 9 instead of 36, with the same solutions; first-step QPs of the force,
 * jerk and quad13 benches are unchanged: 3.65, 1.07, 1.00.) w->dza is scratch here. */
static int pdas_update(const ocp_ref_desc *d, ws_t *w, int first)
{
    const int nx = d->nx, nu = d->nu, N = d->N, nz = nx + nu;
    double cv[NZMAX];
    int ck[NZMAX], nrem = 0, ok = 1;
    for (int i = 0; i < nz; i++) { cv[i] = 0.0; ck[i] = -1; }
    for (int k = 0; k <= N; k++) {
        const int n = k < N ? nz : nx;
        for (int i = (k == 0 ? nx : 0); i < n; i++) {
            const double zn = w->z[k * nz + i] + w->dz[k * nz + i], lbv = LBk(d, k, i), ubv = UBk(d, k, i);
            const signed char a = w->act[k * nz + i];
            double viol = 0.0;   /* add candidate: violation of an inactive bound (< 0: lower) */
            if (!isfinite(zn)) ok = 0;   /* a non-finite step is never accepted */
            if (a < 0) {
                if (zn > lbv + POLISH_TOL_ACTIVE * (1.0 + fabs(lbv))) { ok = 0; w->act[k * nz + i] = 0; nrem++; }
            } else if (a > 0) {
                if (zn < ubv - POLISH_TOL_ACTIVE * (1.0 + fabs(ubv))) { ok = 0; w->act[k * nz + i] = 0; nrem++; }
            } else if (has(lbv) && zn < lbv - POLISH_TOL * (1.0 + fabs(lbv))) {
                ok = 0; viol = zn - lbv;
            } else if (has(ubv) && zn > ubv + POLISH_TOL * (1.0 + fabs(ubv))) {
                ok = 0; viol = zn - ubv;
            }
            if (i >= nx && viol != 0.0) {   /* inputs join at once */
                w->act[k * nz + i] = viol < 0.0 ? -1 : 1;
                viol = 0.0;
            }
            w->dza[k * nz + i] = viol;
            if (fabs(viol) > cv[i]) { cv[i] = fabs(viol); ck[i] = k; }
        }
    }
    if (first || nrem == 0)
        for (int i = 0; i < nz; i++)
            if (ck[i] >= 0) w->act[ck[i] * nz + i] = w->dza[ck[i] * nz + i] < 0.0 ? -1 : 1;
    return ok;
}

static int solve_one(const ocp_ref_desc *d, const double *x0, const double *yref,
                     double *xo, double *uo, int *iters_out, ws_t *w)
{
    const int nx = d->nx, nu = d->nu, N = d->N, nz = nx + nu, ny = d->ny;
    const double *A = d->A, *B = d->B, *c = d->c;
    double p[NZMAX], v[NZMAX], h[NZMAX];
    int k, i, j, l, it, status = 2, m = 0;

    /* stage widths: stage k<N has nz comps, stage N has nx */
#define Z(k, i) w->z[(k) * nz + (i)]
#define LL(k, i) w->ll[(k) * nz + (i)]
#define LU(k, i) w->lu[(k) * nz + (i)]
    /* constant gradient part g_k = G yref_k */
    for (k = 0; k <= N; k++) {
        int n = k < N ? nz : nx;
        const double *Gm = k < N ? d->G : d->Ge;
        int nyk = k < N ? ny : d->ny_e;
        const double *y = yref + (size_t)k * ny;
        for (i = 0; i < n; i++) {
            double s = 0.0;
            for (j = 0; j < nyk; j++) s += Gm[i * nyk + j] * y[j];
            w->gc[k * nz + i] = s;
        }
    }
    /* initial point: states at the reference, inputs with a two-sided box at its midpoint (the
     * projected input reference of the force model sits next to the thrust bound and costs ~6
     * short-step iterations at the start), everything strictly inside the boxes, x0 pinned */
    for (k = 0; k <= N; k++) {
        int n = k < N ? nz : nx;
        const double *y = yref + (size_t)k * ny;
        for (i = 0; i < n; i++) {
            double val;   /* LINEAR_LS with Vx=[I;0], Vu=[0;I] layout: y = [x;u] */
            if (k < N ? (i < ny) : (i < d->ny_e)) val = y[i]; else val = 0.0;
            if (i >= nx && has(LBk(d, k, i)) && has(UBk(d, k, i))) val = 0.5 * (LBk(d, k, i) + UBk(d, k, i));
            interior(&val, LBk(d, k, i), UBk(d, k, i));
            Z(k, i) = val;
        }
        for (i = n; i < nz; i++) Z(k, i) = 0.0;
    }
    for (i = 0; i < nx; i++) Z(0, i) = x0[i];
    for (k = 0; k <= N; k++) {
        int n = k < N ? nz : nx;
        for (i = 0; i < nz; i++) { LL(k, i) = 0.0; LU(k, i) = 0.0; }
        for (i = 0; i < n; i++) {
            if (k == 0 && i < nx) continue;
            double lbv = LBk(d, k, i), ubv = UBk(d, k, i);
            if (has(lbv)) { LL(k, i) = d->mu0 / (Z(k, i) - lbv); m++; }
            if (has(ubv)) { LU(k, i) = d->mu0 / (ubv - Z(k, i)); m++; }
        }
    }
    /* gradient of the objective at z */
#define GRADF(k, out) do { \
        int n_ = (k) < N ? nz : nx; const double *Hm_ = (k) < N ? d->H : d->He; \
        for (int a_ = 0; a_ < n_; a_++) { double s_ = w->gc[(k) * nz + a_]; \
            for (int b_ = 0; b_ < n_; b_++) s_ += Hm_[a_ * n_ + b_] * Z(k, b_); (out)[a_] = s_; } \
    } while (0)
    /* initial residual scale r0 = max(|r_d|, |r_e|) with pi = 0 */
    double r0 = 0.0;
    for (k = 0; k <= N; k++) {
        double g[NZMAX];
        int n = k < N ? nz : nx;
        GRADF(k, g);
        for (i = (k == 0 ? nx : 0); i < n; i++) {
            double r = fabs(g[i] - LL(k, i) + LU(k, i));
            if (r > r0) r0 = r;
        }
    }
    for (k = 0; k < N; k++)
        for (i = 0; i < nx; i++) {
            double s = c[i] - Z(k + 1, i);
            for (j = 0; j < nx; j++) s += A[i * nx + j] * Z(k, j);
            for (j = 0; j < nu; j++) s += B[i * nu + j] * Z(k, nx + j);
            if (fabs(s) > r0) r0 = fabs(s);
        }
    double theta = 1.0;
    if (m == 0) m = 1;
    double polish_at = d->polish_mu > 0.0 ? d->polish_mu : -1.0, rho = 1.0;
    int fin_steps = 0;
    for (i = 0; i < nz * nz; i += nz + 1) rho = fmax(rho, fabs(d->H[i]));
    for (i = 0; i < nx * nx; i += nx + 1) rho = fmax(rho, fabs(d->He[i]));
    rho *= POLISH_RHO;
    it = 0;
    /* a certified-infeasible QP ends before the first iteration: status 4, the initial point */
    if (infeasible_stage(d, x0)) { status = 4; goto done; }

    /* ---- forward substitution: direction into out[] ---- */
#define FORWARD(out) do { \
        double dx_[NZMAX]; for (i = 0; i < nx; i++) dx_[i] = 0.0; \
        for (k = 0; k < N; k++) { \
            const double *Luu_ = &w->Luu[k * nu * nu], *Lxu_ = &w->Lxu[k * nx * nu], *lu_ = &w->lu_vec[k * nu]; \
            double t_[NZMAX]; \
            for (j = 0; j < nu; j++) { double s_ = lu_[j]; \
                for (i = 0; i < nx; i++) s_ += Lxu_[i * nu + j] * dx_[i]; t_[j] = s_; } \
            for (j = nu - 1; j >= 0; j--) { double s_ = t_[j]; \
                for (l = j + 1; l < nu; l++) s_ -= Luu_[l * nu + j] * t_[l]; t_[j] = s_ / Luu_[j * nu + j]; } \
            for (i = 0; i < nx; i++) (out)[k * nz + i] = dx_[i]; \
            for (j = 0; j < nu; j++) (out)[k * nz + nx + j] = -t_[j]; \
            for (i = 0; i < nx; i++) { double s_ = w->re[k * nx + i]; \
                for (j = 0; j < nx; j++) s_ += A[i * nx + j] * dx_[j]; \
                for (j = 0; j < nu; j++) s_ += B[i * nu + j] * (out)[k * nz + nx + j]; \
                t_[nu + i] = s_; } \
            for (i = 0; i < nx; i++) dx_[i] = t_[nu + i]; \
        } \
        for (i = 0; i < nx; i++) (out)[N * nz + i] = dx_[i]; \
    } while (0)
    for (it = 0; it < d->max_iter; it++) {
        /* complementarity measure */
        double mu = 0.0, zs = 0.0;
        for (k = 0; k <= N; k++) {
            int n = k < N ? nz : nx;
            for (i = 0; i < n; i++) {
                if (LL(k, i) > 0.0) mu += LL(k, i) * (Z(k, i) - LBk(d, k, i));
                if (LU(k, i) > 0.0) mu += LU(k, i) * (UBk(d, k, i) - Z(k, i));
                zs += Z(k, i) + LL(k, i) + LU(k, i);
            }
        }
        mu /= m;
        /* non-finite iterate (a multiplier of a NaN drops out of mu): QP failure */
        if (!isfinite(mu) || !isfinite(theta) || !isfinite(zs)) { status = 4; break; }
        if (mu <= d->tol_comp && theta * r0 <= d->tol_res) { status = 0; break; }

        /* objective gradient gf, dynamics residual re */
        for (k = 0; k <= N; k++) GRADF(k, &w->gf[k * nz]);
        for (k = 0; k < N; k++)
            for (i = 0; i < nx; i++) {
                double s = c[i] - Z(k + 1, i);
                for (j = 0; j < nx; j++) s += A[i * nx + j] * Z(k, j);
                for (j = 0; j < nu; j++) s += B[i * nu + j] * Z(k, nx + j);
                w->re[k * nx + i] = s;
            }
        if (mu <= polish_at) {
            /* exact finish, a primal-dual active-set (PDAS) run of at most polish_steps Newton
             * steps on the QP from the current iterate: the active bounds (first step: where the
             * IPM multiplier exceeds the slack) are held by a penalty of weight rho, the others
             * dropped; one Newton step lands on that active set's solution. Accepted when every
             * inactive bound holds and every active one keeps a non-negative multiplier
             * rho * (bound - z) — the QP's KKT conditions; otherwise the violated inactive bounds
             * join and the negative-multiplier ones leave the active set for the next step. If no
             * step is accepted the IPM iterate is untouched and the next run waits for mu to
             * drop 100-fold. */
            polish_at = (mu < polish_at ? mu : polish_at) * 1e-2;
            memset(w->act, 0, (size_t)(N + 1) * nz);
            for (k = 0; k <= N; k++) {
                int n = k < N ? nz : nx;
                for (i = 0; i < n; i++) {
                    signed char a = 0;
                    if (!(k == 0 && i < nx)) {
                        if (LL(k, i) > 0.0 && LL(k, i) > Z(k, i) - LBk(d, k, i)) a = -1;
                        else if (LU(k, i) > 0.0 && LU(k, i) > UBk(d, k, i) - Z(k, i)) a = 1;
                    }
                    w->act[k * nz + i] = a;
                }
            }
            int ok = 0;
            for (int step = 0; step < d->polish_steps && !ok; step++) {
                fin_steps++;
                for (k = 0; k <= N; k++) {
                    int n = k < N ? nz : nx;
                    for (i = 0; i < n; i++) {
                        const signed char a = w->act[k * nz + i];
                        double g = w->gf[k * nz + i];
                        if (a) g += rho * (Z(k, i) - (a < 0 ? LBk(d, k, i) : UBk(d, k, i)));
                        w->sg[k * nz + i] = a ? rho : 0.0;
                        w->gh[k * nz + i] = g;
                    }
                }
                if (backward(d, w, w->gh) != 0) break;
                FORWARD(w->dz);
                ok = pdas_update(d, w, step == 0);
            }
            int nact = 0;
            if (ok)
                for (k = 0; k <= N; k++)
                    for (i = 0; i < (k < N ? nz : nx); i++) nact += w->act[k * nz + i] != 0;
            if (ok && nact == 0) {
                /* no active bound: the step solved the unconstrained Newton system (no penalty),
                 * nothing to refine */
                for (k = 0; k <= N; k++) {
                    int n = k < N ? nz : nx;
                    for (i = (k == 0 ? nx : 0); i < n; i++) Z(k, i) += w->dz[k * nz + i];
                }
                status = 0;
                break;
            }
            if (ok) {
                /* refinement: the penalised solution z_a sits lambda / rho off its active bounds
                 * and carries the rounding of a rho-weighted solve; one more Newton step from z_a
                 * on the same active set with the bounds shifted by that offset (target
                 * 2 b - z_a, i.e. gradient H z_a + g_c + 2 rho (z_a - b)) removes both to first
                 * order. Accepted when the refined point holds every bound to POLISH_TOL, sits on
                 * its active bounds to POLISH_TOL and the correction stayed below POLISH_TOL_REFINE
                 * (a larger one means the rho-weighted solve was not accurate); otherwise the IPM
                 * goes on from its own iterate. */
                for (k = 0; k <= N; k++) {
                    int n = k < N ? nz : nx;
                    for (i = 0; i < n; i++) w->dza[k * nz + i] = Z(k, i) + (k == 0 && i < nx ? 0.0 : w->dz[k * nz + i]);
                }
                /* gradient at z_a (w->dza holds z_a); z_a satisfies the dynamics up to rounding, so the
                 * dynamics residual of the refinement's recursion is zero — the GPU kernel reuses the
                 * set step's factorisation and drops the P re term (same answers on every golden set
                 * and the dumped hard closed-loop QPs) */
                for (k = 0; k <= N; k++) {
                    const int n = k < N ? nz : nx;
                    const double *Hm = k < N ? d->H : d->He;
                    for (i = 0; i < n; i++) {
                        double g = w->gc[k * nz + i];
                        for (j = 0; j < n; j++) g += Hm[i * n + j] * w->dza[k * nz + j];
                        const signed char a = w->act[k * nz + i];
                        if (a) g += 2.0 * rho * (w->dza[k * nz + i] - (a < 0 ? LBk(d, k, i) : UBk(d, k, i)));
                        w->gh[k * nz + i] = g;
                    }
                }
                for (k = 0; k < N; k++)
                    for (i = 0; i < nx; i++) w->re[k * nx + i] = 0.0;
                fin_steps++;
                ok = backward(d, w, w->gh) == 0;
                if (ok) {
                    FORWARD(w->dz);
                    for (k = 0; k <= N && ok; k++) {
                        int n = k < N ? nz : nx;
                        for (i = (k == 0 ? nx : 0); i < n; i++) {
                            const double za = w->dza[k * nz + i], zr = za + w->dz[k * nz + i];
                            const double lbv = LBk(d, k, i), ubv = UBk(d, k, i);
                            const signed char a = w->act[k * nz + i];
                            const double tl = POLISH_TOL * (1.0 + fabs(lbv)), tu = POLISH_TOL * (1.0 + fabs(ubv));
                            if (!(fabs(w->dz[k * nz + i]) <= POLISH_TOL_REFINE * (1.0 + fabs(za))) ||
                                (a < 0 && fabs(zr - lbv) > tl) || (a > 0 && fabs(zr - ubv) > tu) ||
                                (!a && has(lbv) && zr < lbv - tl) || (!a && has(ubv) && zr > ubv + tu)) {
                                ok = 0;
                                break;
                            }
                        }
                    }
                }
                if (ok) {
                    for (k = 0; k <= N; k++) {
                        int n = k < N ? nz : nx;
                        for (i = (k == 0 ? nx : 0); i < n; i++) {
                            double zn = w->dza[k * nz + i] + w->dz[k * nz + i], lbv = LBk(d, k, i), ubv = UBk(d, k, i);
                            if (has(lbv) && zn < lbv) zn = lbv;
                            if (has(ubv) && zn > ubv) zn = ubv;
                            Z(k, i) = zn;
                        }
                    }
                    status = 0;
                    break;
                }
                /* the residual at the IPM iterate (overwritten above) for the iteration that follows */
                for (k = 0; k < N; k++)
                    for (i = 0; i < nx; i++) {
                        double s = c[i] - Z(k + 1, i);
                        for (j = 0; j < nx; j++) s += A[i * nx + j] * Z(k, j);
                        for (j = 0; j < nu; j++) s += B[i * nu + j] * Z(k, nx + j);
                        w->re[k * nx + i] = s;
                    }
            }
        }
        /* ---- backward factorisation (+ predictor vector) ---- */
        for (k = 0; k <= N; k++) {
            int n = k < N ? nz : nx;
            for (i = 0; i < n; i++) {
                double sgv = 0.0;
                if (!(k == 0 && i < nx)) {
                    if (LL(k, i) > 0.0) sgv += LL(k, i) / (Z(k, i) - LBk(d, k, i));
                    if (LU(k, i) > 0.0) sgv += LU(k, i) / (UBk(d, k, i) - Z(k, i));
                }
                w->sg[k * nz + i] = sgv;
            }
        }
        if (backward(d, w, w->gf)) { status = 4; goto done; }
        FORWARD(w->dza);

        /* affine step length and mu_aff */
        double a_aff = 1.0;
        for (k = 0; k <= N; k++) {
            int n = k < N ? nz : nx;
            for (i = (k == 0 ? nx : 0); i < n; i++) {
                double dz = w->dza[k * nz + i];
                if (LL(k, i) > 0.0) {
                    double t = Z(k, i) - LBk(d, k, i), dl = -LL(k, i) * (1.0 + dz / t);
                    if (dz < 0.0 && -t / dz < a_aff) a_aff = -t / dz;
                    if (dl < 0.0 && -LL(k, i) / dl < a_aff) a_aff = -LL(k, i) / dl;
                }
                if (LU(k, i) > 0.0) {
                    double t = UBk(d, k, i) - Z(k, i), dl = -LU(k, i) * (1.0 - dz / t);
                    if (dz > 0.0 && t / dz < a_aff) a_aff = t / dz;
                    if (dl < 0.0 && -LU(k, i) / dl < a_aff) a_aff = -LU(k, i) / dl;
                }
            }
        }
        double mu_aff = 0.0;
        for (k = 0; k <= N; k++) {
            int n = k < N ? nz : nx;
            for (i = (k == 0 ? nx : 0); i < n; i++) {
                double dz = w->dza[k * nz + i];
                if (LL(k, i) > 0.0) {
                    double t = Z(k, i) - LBk(d, k, i), dl = -LL(k, i) * (1.0 + dz / t);
                    mu_aff += (t + a_aff * dz) * (LL(k, i) + a_aff * dl);
                }
                if (LU(k, i) > 0.0) {
                    double t = UBk(d, k, i) - Z(k, i), dl = -LU(k, i) * (1.0 - dz / t);
                    mu_aff += (t - a_aff * dz) * (LU(k, i) + a_aff * dl);
                }
            }
        }
        mu_aff /= m;
        double sg = mu_aff / mu;
        double smu = sg * sg * sg * mu;
        /* corrector gradient gh */
        for (k = 0; k <= N; k++) {
            int n = k < N ? nz : nx;
            for (i = 0; i < n; i++) {
                double g = w->gf[k * nz + i], dz = w->dza[k * nz + i];
                if (!(k == 0 && i < nx)) {
                    if (LL(k, i) > 0.0) {
                        double t = Z(k, i) - LBk(d, k, i), dl = -LL(k, i) * (1.0 + dz / t);
                        g += (dl * dz - smu) / t;
                    }
                    if (LU(k, i) > 0.0) {
                        double t = UBk(d, k, i) - Z(k, i), dl = -LU(k, i) * (1.0 - dz / t);
                        g += (dl * dz + smu) / t;
                    }
                }
                w->gh[k * nz + i] = g;
            }
        }
        /* backward vector pass with gh */
        for (i = 0; i < nx; i++) p[i] = w->gh[N * nz + i];
        for (k = N - 1; k >= 0; k--) {
            const double *Pr = &w->Pr[k * nx], *Luu = &w->Luu[k * nu * nu], *Lxu = &w->Lxu[k * nx * nu];
            double *luv = &w->lu_vec[k * nu];
            for (i = 0; i < nx; i++) v[i] = Pr[i] + p[i];
            for (i = 0; i < nz; i++) {
                double s = w->gh[k * nz + i];
                for (l = 0; l < nx; l++) s += (i < nx ? A[l * nx + i] : B[l * nu + (i - nx)]) * v[l];
                h[i] = s;
            }
            for (j = 0; j < nu; j++) {
                double s = h[nx + j];
                for (l = 0; l < j; l++) s -= Luu[j * nu + l] * luv[l];
                luv[j] = s / Luu[j * nu + j];
            }
            if (k > 0)
                for (i = 0; i < nx; i++) {
                    double s = h[i];
                    for (l = 0; l < nu; l++) s -= Lxu[i * nu + l] * luv[l];
                    p[i] = s;
                }
        }
        FORWARD(w->dz);
        /* dual directions and step length */
        double alpha = 1.0;
        for (k = 0; k <= N; k++) {
            int n = k < N ? nz : nx;
            for (i = (k == 0 ? nx : 0); i < n; i++) {
                double dz = w->dz[k * nz + i], dza = w->dza[k * nz + i];
                if (LL(k, i) > 0.0) {
                    double t = Z(k, i) - LBk(d, k, i), dla = -LL(k, i) * (1.0 + dza / t);
                    double dl = (smu - LL(k, i) * t - dla * dza - LL(k, i) * dz) / t;
                    if (dz < 0.0 && -t / dz < alpha) alpha = -t / dz;
                    if (dl < 0.0 && -LL(k, i) / dl < alpha) alpha = -LL(k, i) / dl;
                }
                if (LU(k, i) > 0.0) {
                    double t = UBk(d, k, i) - Z(k, i), dla = -LU(k, i) * (1.0 - dza / t);
                    double dl = (smu - LU(k, i) * t + dla * dza + LU(k, i) * dz) / t;
                    if (dz > 0.0 && t / dz < alpha) alpha = t / dz;
                    if (dl < 0.0 && -LU(k, i) / dl < alpha) alpha = -LU(k, i) / dl;
                }
            }
        }
        alpha *= 0.995;
        if (alpha > 1.0) alpha = 1.0;
        {
            /* a non-finite direction ends the solve like a failed factorisation (iterate kept) */
            double nf = 0.0;
            for (k = 0; k <= N; k++)
                for (i = 0; i < (k < N ? nz : nx); i++) nf += w->dz[k * nz + i] * 0.0;
            if (!isfinite(alpha) || !isfinite(nf)) { status = 4; goto done; }
        }
        for (k = 0; k <= N; k++) {
            int n = k < N ? nz : nx;
            for (i = (k == 0 ? nx : 0); i < n; i++) {
                double dz = w->dz[k * nz + i], dza = w->dza[k * nz + i];
                if (LL(k, i) > 0.0) {
                    double t = Z(k, i) - LBk(d, k, i), dla = -LL(k, i) * (1.0 + dza / t);
                    LL(k, i) += alpha * (smu - LL(k, i) * t - dla * dza - LL(k, i) * dz) / t;
                }
                if (LU(k, i) > 0.0) {
                    double t = UBk(d, k, i) - Z(k, i), dla = -LU(k, i) * (1.0 - dza / t);
                    LU(k, i) += alpha * (smu - LU(k, i) * t + dla * dza + LU(k, i) * dz) / t;
                }
                Z(k, i) += alpha * dz;
            }
        }
        theta *= (1.0 - alpha);
    }
done:
    for (k = 0; k <= N; k++)
        for (i = 0; i < nx; i++) xo[k * nx + i] = Z(k, i);
    for (k = 0; k < N; k++)
        for (j = 0; j < nu; j++) uo[k * nu + j] = Z(k, nx + j);
    *iters_out = it + fin_steps;   /* Newton systems solved: IPM iterations + finish steps */
    return status;
#undef Z
#undef LL
#undef LU
#undef GRADF
#undef FORWARD
}

/* Solve `batch` independent instances. x0: batch*nx; yref: batch*(N*ny + ny_e);
 * xout: batch*(N+1)*nx; uout: batch*N*nu. nthreads <= 0: OpenMP default.
 * Returns the number of instances with status != 0. */
int riccati_ipm_solve_batch(const ocp_ref_desc *d, int batch, const double *x0, const double *yref,
                            double *xout, double *uout, int *status, int *iters, int nthreads)
{
    const int nx = d->nx, nu = d->nu, N = d->N, nz = nx + nu;
    if (nx + nu > NZMAX || nx < 1 || nu < 1 || N < 1 || d->ny != nz || d->ny_e != nx) return -1;
    const size_t ystride = (size_t)N * d->ny + d->ny_e;
    int nfail = 0;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads(); /* honours OMP_NUM_THREADS */
#else
    nthreads = 1;
#endif
#pragma omp parallel num_threads(nthreads) reduction(+ : nfail)
    {
        size_t S = (size_t)(N + 1) * nz;
        double *buf = (double *)malloc(sizeof(double) * (9 * S + (size_t)N * (2 * nx + nu * nu + nx * nu + nu)) + S);
        ws_t w;
        w.z = buf; w.ll = w.z + S; w.lu = w.ll + S; w.dza = w.lu + S; w.dz = w.dza + S;
        w.gc = w.dz + S; w.gf = w.gc + S; w.gh = w.gf + S;
        w.re = w.gh + S; w.Pr = w.re + (size_t)N * nx; w.Luu = w.Pr + (size_t)N * nx;
        w.Lxu = w.Luu + (size_t)N * nu * nu; w.lu_vec = w.Lxu + (size_t)N * nx * nu;
        w.sg = w.lu_vec + (size_t)N * nu;
        w.act = (signed char *)(w.sg + S);
#pragma omp for schedule(dynamic, 16)
        for (int b = 0; b < batch; b++) {
            int st = solve_one(d, x0 + (size_t)b * nx, yref + (size_t)b * ystride,
                               xout + (size_t)b * (N + 1) * nx, uout + (size_t)b * N * nu,
                               &iters[b], &w);
            status[b] = st;
            if (st != 0) nfail++;
        }
        free(buf);
    }
    return nfail;
}

int riccati_ipm_max_threads(void)
{
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
