// nmpc_api.cpp — C-ABI of the batched NMPC engine (declared in include/nmpc.h).
//
// Host side of the drop-in boundary: owns the device buffers of one batched solver handle,
// turns an acados-style OCP description (AcadosOcp: model / cost / constraints /
// solver_options, force_model/ocp.py:21-96) into the stage-wise QP data the kernels consume,
// and stages set/get traffic like acados's ocp_nlp_cost_model_set / ocp_nlp_out_get.
//
// "Sensitivity functions": the reference lets CasADi generate the integrator and its
// forward sensitivities for an affine model (force_model/dynamics.py:32-47 with IRK,
// jerk_model/dynamics.py:35-52 with ERK-1). For an affine ODE held over one step those
// sensitivities are constant, so they are computed here once, natively, from the Butcher
// tableau of the requested integrator (Gauss-Legendre collocation or explicit RK).

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/nmpc.h"
#include "nmpc_internal.h"

namespace {

thread_local std::string g_err;

constexpr double kInf = 1e30;

bool has_bound(double b) { return std::fabs(b) < 1e20; }

// ---------------------------------------------------------------- small dense linear algebra
// solve M X = R in place (M n x n, R n x m), partial pivoting; returns false if singular
bool gauss_solve(std::vector<double> &M, std::vector<double> &R, int n, int m)
{
    for (int col = 0; col < n; col++) {
        int piv = col;
        for (int r = col + 1; r < n; r++)
            if (std::fabs(M[r * n + col]) > std::fabs(M[piv * n + col])) piv = r;
        if (std::fabs(M[piv * n + col]) < 1e-300) return false;
        if (piv != col) {
            for (int j = 0; j < n; j++) std::swap(M[col * n + j], M[piv * n + j]);
            for (int j = 0; j < m; j++) std::swap(R[col * m + j], R[piv * m + j]);
        }
        for (int r = 0; r < n; r++) {
            if (r == col) continue;
            const double f = M[r * n + col] / M[col * n + col];
            if (f == 0.0) continue;
            for (int j = col; j < n; j++) M[r * n + j] -= f * M[col * n + j];
            for (int j = 0; j < m; j++) R[r * m + j] -= f * R[col * m + j];
        }
    }
    for (int r = 0; r < n; r++)
        for (int j = 0; j < m; j++) R[r * m + j] /= M[r * n + r];
    return true;
}

// Butcher tableau of the acados integrators used by the reference
bool butcher(int type, int s, std::vector<double> &a, std::vector<double> &b, std::vector<double> &c)
{
    a.assign(s * s, 0.0);
    b.assign(s, 0.0);
    c.assign(s, 0.0);
    if (type == NMPC_ERK) {
        if (s == 1) {
            b[0] = 1.0;
        } else if (s == 2) {  // explicit midpoint
            a[1 * 2 + 0] = 0.5;
            c[1] = 0.5;
            b[1] = 1.0;
        } else if (s == 4) {  // classic RK4
            a[1 * 4 + 0] = 0.5;
            a[2 * 4 + 1] = 0.5;
            a[3 * 4 + 2] = 1.0;
            c[1] = c[2] = 0.5;
            c[3] = 1.0;
            b[0] = b[3] = 1.0 / 6.0;
            b[1] = b[2] = 1.0 / 3.0;
        } else {
            return false;
        }
        return true;
    }
    if (type != NMPC_IRK || s < 1 || s > 9) return false;
    // Gauss-Legendre nodes: roots of P_s(2c-1), Newton on the Legendre recurrence
    for (int i = 0; i < s; i++) {
        double x = std::cos(M_PI * (i + 0.75) / (s + 0.5));
        for (int itn = 0; itn < 100; itn++) {
            double p0 = 1.0, p1 = x;
            for (int n = 2; n <= s; n++) {
                const double p2 = ((2.0 * n - 1.0) * x * p1 - (n - 1.0) * p0) / n;
                p0 = p1;
                p1 = p2;
            }
            const double pl = s == 1 ? x : p1;
            const double p_prev = s == 1 ? 1.0 : p0;
            const double dp = s * (x * pl - p_prev) / (x * x - 1.0);
            const double dx = pl / dp;
            x -= dx;
            if (std::fabs(dx) < 1e-16) break;
        }
        c[i] = 0.5 * (1.0 - x);
    }
    std::sort(c.begin(), c.end());
    // collocation conditions: sum_j a_ij c_j^(q-1) = c_i^q / q, sum_j b_j c_j^(q-1) = 1/q
    std::vector<double> V(s * s), R(s * (s + 1));
    for (int q = 0; q < s; q++)
        for (int j = 0; j < s; j++) V[q * s + j] = std::pow(c[j], q);
    for (int q = 0; q < s; q++) {
        for (int i = 0; i < s; i++) R[q * (s + 1) + i] = std::pow(c[i], q + 1) / (q + 1);
        R[q * (s + 1) + s] = 1.0 / (q + 1);
    }
    if (!gauss_solve(V, R, s, s + 1)) return false;
    for (int j = 0; j < s; j++) {
        for (int i = 0; i < s; i++) a[i * s + j] = R[j * (s + 1) + i];
        b[j] = R[j * (s + 1) + s];
    }
    return true;
}

// exact discrete map of x' = Ac x + Bc u + cc under one step of the RK scheme, composed
// over num_steps sub-steps of h/num_steps (forward sensitivities of the integrator)
bool discretize(int nx, int nu, const double *Ac, const double *Bc, const double *cc, int type, int stages,
                int steps, double h, std::vector<double> &A, std::vector<double> &B, std::vector<double> &c)
{
    std::vector<double> a, bw, cn;
    if (!butcher(type, stages, a, bw, cn) || steps < 1) return false;
    const double hs = h / steps;
    const int s = stages, n = s * nx, m = nx + nu + 1;
    std::vector<double> M(n * n, 0.0), Rh(n * m, 0.0);
    for (int i = 0; i < s; i++)
        for (int r = 0; r < nx; r++) {
            for (int j = 0; j < s; j++)
                for (int q = 0; q < nx; q++) M[(i * nx + r) * n + j * nx + q] = -hs * a[i * s + j] * Ac[r * nx + q];
            M[(i * nx + r) * n + i * nx + r] += 1.0;
            for (int q = 0; q < nx; q++) Rh[(i * nx + r) * m + q] = Ac[r * nx + q];
            for (int q = 0; q < nu; q++) Rh[(i * nx + r) * m + nx + q] = Bc[r * nu + q];
            Rh[(i * nx + r) * m + nx + nu] = cc[r];
        }
    if (!gauss_solve(M, Rh, n, m)) return false;
    // one-step map T = [Phi Gam gam]
    std::vector<double> T(nx * m, 0.0);
    for (int r = 0; r < nx; r++) {
        T[r * m + r] = 1.0;
        for (int i = 0; i < s; i++)
            for (int q = 0; q < m; q++) T[r * m + q] += hs * bw[i] * Rh[(i * nx + r) * m + q];
    }
    // compose: X_{j+1} = Phi X_j + [0 Gam gam]
    std::vector<double> Acur(nx * nx), Bcur(nx * nu), ccur(nx);
    for (int r = 0; r < nx; r++) {
        for (int q = 0; q < nx; q++) Acur[r * nx + q] = T[r * m + q];
        for (int q = 0; q < nu; q++) Bcur[r * nu + q] = T[r * m + nx + q];
        ccur[r] = T[r * m + nx + nu];
    }
    for (int st = 1; st < steps; st++) {
        std::vector<double> An(nx * nx, 0.0), Bn(nx * nu, 0.0), cn2(nx, 0.0);
        for (int r = 0; r < nx; r++) {
            for (int q = 0; q < nx; q++)
                for (int l = 0; l < nx; l++) An[r * nx + q] += T[r * m + l] * Acur[l * nx + q];
            for (int q = 0; q < nu; q++) {
                double v = T[r * m + nx + q];
                for (int l = 0; l < nx; l++) v += T[r * m + l] * Bcur[l * nu + q];
                Bn[r * nu + q] = v;
            }
            double v = T[r * m + nx + nu];
            for (int l = 0; l < nx; l++) v += T[r * m + l] * ccur[l];
            cn2[r] = v;
        }
        Acur.swap(An);
        Bcur.swap(Bn);
        ccur.swap(cn2);
    }
    A = Acur;
    B = Bcur;
    c = ccur;
    return true;
}

hipError_t upload_any(void *dst, const double *src, size_t n, bool f64, hipStream_t s, std::vector<float> &tmp)
{
    if (f64) return hipMemcpyAsync(dst, src, n * sizeof(double), hipMemcpyHostToDevice, s);
    tmp.resize(n);
    for (size_t i = 0; i < n; i++) tmp[i] = (float)src[i];
    return hipMemcpyAsync(dst, tmp.data(), n * sizeof(float), hipMemcpyHostToDevice, s);
}

}  // namespace

struct nmpc_solver {
    std::string name, err;
    int device = 0, precision = NMPC_FP64, batch = 0;
    int nx = 0, nu = 0, N = 0, ny = 0, ny_e = 0;
    int kidx = -1, ipw = 1, wpb = 1, lds = 0, yref_is_z = 0, g_diag = 0;
    int max_iter = 50;
    double tol_comp = 0, tol_res = 0, mu0 = 0, inv_m = 1, ts = 0, scale_e = 1;
    double polish_mu = 0, polish_rho = 0, polish_drop = 0.01;
    int polish_steps = 12, polish_first = 12;
    hipStream_t own_stream = nullptr, stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    float last_ms = 0.f;
    // host model (double)
    std::vector<double> A, B, c, W, Vx, Vu, W_e, Vx_e;
    std::vector<double> H, G, He, Ge, lbnd, ubnd;
    // host staging
    std::vector<double> h_x0, h_lbx0, h_ubx0, h_yref, h_x, h_u;
    std::vector<int32_t> h_status, h_iters;
    bool x0_dirty = true, yref_dirty = true, out_valid = false;
    // device
    void *d_model = nullptr, *d_x0 = nullptr, *d_yref = nullptr, *d_x = nullptr, *d_u = nullptr;
    void *d_scratch = nullptr;
    int *d_status = nullptr, *d_iters = nullptr;
    unsigned long long *d_cycles = nullptr;
    size_t off_AB = 0, off_ABt = 0, off_c = 0, off_H = 0, off_He = 0, off_G = 0, off_Ge = 0, off_lb = 0, off_ub = 0;
    size_t off_lqr = 0, off_lqrf = 0, off_lqrw = 0;   // unconstrained Riccati records (lqr_table, lqr_wmat)
    std::vector<double> lqr_host;                      // the lqr_table records (host copy)
    void *d_cltx = nullptr, *d_clv = nullptr;          // closed loop: explicit unconstrained solution (cl_explicit)
    // lean closed loop (nmpc_cl_fast.hip): slot tables, per-instance step / flags, park list
    bool clf = false;
    int clf_nslot = 0, clf_epl = 0, clf_x1slot = 0, clf_sid = 0;
    int clf_kidx = -1;                     // list-mode fallback kernel (lane per component)
    void *d_clf_scratch = nullptr;         // its scratch when the handle's own family is another
    unsigned *d_clf_check = nullptr;       // env NMPC_CLF_CHECK with a checked build: the failed index checks
    void *d_fsT = nullptr;                 // typed: s_lb, s_ub, s_tx, vb, uinit
    double *d_clw = nullptr;               // fp32 handles: the lean loop's W in fp64 (fp64 handles: the model's)
    // fp32 handles: the solve's exact finish (fin32_z0_kernel + fin32_kernel, nmpc_cl_fast.hip)
    bool fin32 = false;
    int fin_m16 = 0, fin_kp = 0, fin_nslot = 0, fin_nfree = 0, fin_resident = 0;
    float *d_fin_f = nullptr;              // s_lb, s_ub, uinit, M [m16][kp], vc [m16]
    size_t fino[5] = {0, 0, 0, 0, 0};
    int *d_fin_i = nullptr;                // s_e, s_free
    size_t fini[2] = {0, 0};
    float *d_z0 = nullptr;                 // [B][m16] unconstrained solutions of the batch
    size_t fso[5] = {0, 0, 0, 0, 0};
    int *d_fsI = nullptr;                  // s_e, s_src, eslot
    size_t fsi[4] = {0, 0, 0, 0};
    int clf_nfree = 0;
    // fp64 general solve on the shared factorisation (nmpc_solve_fast.hip sf_kernel + fin64_kernel; sf_setup)
    bool sfast = false, sf_pending = false;
    double *d_sf = nullptr;                // per-stage tables [N][ts], gradient diagonal [nz + nx]
    size_t sf_gd = 0;                      // offset of the gradient diagonal in d_sf
    double *d_f64 = nullptr;               // fin64 slot tables: s_lb, s_ub, uinit
    size_t f64o[3] = {0, 0, 0};
    int *d_f64i = nullptr;                 // s_e, s_free
    size_t f64i[2] = {0, 0};
    int f64_nslot = 0, f64_nfree = 0, f64_resident = 0;
    int *d_sfl = nullptr;                  // [0..4) two [listed, parked] counter pairs (solve i uses pair i & 1; its
                                           // fin64_kernel zeroes the other), [4..4+B) list, [4+B..4+2B) parked
    int sf_pair = 0;                       // the counter pair of the last fast solve
    int *h_sfpark = nullptr;               // pinned: the last fast solve's [listed, parked] counts (copied in
                                           // stream order behind its kernels; valid once the stream has drained)
    int sf_listed = 0, sf_parked = 0;      // ... as read at the last wait (nmpc_get_stats out[5], out[6])
    unsigned long long *d_sfcyc = nullptr; // timing builds (env NMPC_SF_CYCLES): sf_kernel's phase clocks
    size_t sfcyc_n = 0;
    int sf_kidx = -1;                      // lane-per-component kernel of the parked instances' full solves
    void *d_sf_scratch = nullptr;          // its scratch when the handle's own family is another
    hipEvent_t ev_fb = nullptr;            // start of the parked instances' full solve
    int *d_istep = nullptr, *d_park = nullptr;   // [B]; park count, work counter, park list [2 + B]
    signed char *d_flags = nullptr;        // [B][nslot]
    int clf_resident = 0;                  // workgroups of cl_fast_kernel the handle's device holds at once
    int *d_imap = nullptr;                 // the lean loop's position -> instance map (clf_xcd_map), or null
    int *d_gorder = nullptr;               // the device-wide claim's order (clf_order_launch), [B]
    int clf_kind = 0;                      // nmpc::CLF_FAST / CLF_LOCK (cl_lock_kernel) / CLF_WLDS (W in LDS) / CLF_ONE
    int clf_parked = 0, clf_rounds = 0;    // the last run: parked solves (list-mode full solves), fast launches
    size_t fnoise_cap = 0;                 // capacity of d_fnoise (doubles)
    std::vector<float> tmp_x0f, tmp_yf;
    // closed loop
    bool cl_ready = false;
    bool cl_traj_out = false, out_from_loop = false;   // the lean loop writes the last step's x / u trajectories (nmpc_closed_loop_set_outputs)
    nmpc_closed_loop_desc cl{};
    void *d_table = nullptr, *d_state = nullptr, *d_plant = nullptr, *d_wcl = nullptr;
    int *d_offsets = nullptr;
    double *d_acc = nullptr, *d_noise = nullptr;
    int cl_step = 0, cl_last_launches = 0, cl_last_steps = 0;
    double *d_fnoise = nullptr;   // fused closed loop: noise draws of a launch's steps [B][64]
    int *d_iter_log = nullptr;    // fused closed loop, env NMPC_ITER_LOG: per-step finish steps | IPM iterations << 8 | status << 16 [64][B]
    int iter_log_steps = 0;       // steps in the log (the last fused launch; the lean loop: the last run)
    size_t iter_log_cap = 0;      // capacity of d_iter_log (ints)
    int *h_park = nullptr;        // pinned host word: the lean loop's parked count per round
    int *h_parkr = nullptr;       // pinned: an asynchronous lean run's per-round counter pairs, CLF_ROUND_WORDS per chunk
    size_t parkr_cap = 0;         // ... capacity (ints)
    int clf_async_chunks = 0;     // chunks of the last asynchronous run whose counts h_parkr holds (0: none pending)
    std::vector<hipEvent_t> cl_events;
    double cl_last_ms = 0.0;
    double cost_s = 1.0;  // stage cost factor (time step or 1)
    // condensed family (nmpc_cond.hip): states eliminated on the host, MFMA Hessian GEMMs
    bool cond = false;
    int cond_wpb = 1;
    size_t cond_lds = 0;
    nmpc::CondHost ch;
    void *d_cond = nullptr;   // typed blob: Gx, H0, H0t, Fx, Fy, fc, Phx, dx, lox, hix, lou, hiu, Gall, Phall, dall
    int *d_cond_i = nullptr;  // xcols, rstart, ks
    size_t co[15] = {0};
    size_t ci[3] = {0};

    size_t ystride() const { return (size_t)N * ny + ny_e; }
    size_t esz() const { return precision == NMPC_FP64 ? sizeof(double) : sizeof(float); }
    int fail(int code, const std::string &msg)
    {
        err = msg;
        g_err = msg;
        return code;
    }
};

namespace {

// The Newton system of an exact-finish step whose active set is empty (no penalty, no barrier) is
// the unconstrained LQ problem: its Riccati factorisation is the same for every instance and step.
// Per stage k < N and lane r of the lane-per-component kernels, lqr_words(nx, nu) = nz + 1 words:
// x-lane r holds row r of P_{k+1} (nx words), column r of the gain K_k = -F_uu^{-1} F_ux (nu) and
// (P_{k+1} c)_r (1); u-lane u holds row u of F_uu^{-1} (nu words). P_N = He;
// F = [A B]' P_{k+1} [A B] + H; P_k = F_xx + F_xu K_k.
int lqr_words(int nx, int nu) { return nx + nu + 1; }
//
// The fast finish's rollout table (lqrf_words = 1 + 2 nu + nx words per stage and lane): x-lane r
// holds (P_{k+1} c)_r, column r of K_k, row r of B F_uu^{-1} and row r of the closed-loop matrix
// A + B K_k; u-lane u holds 0, nu zeros, row u of F_uu^{-1} and row u of K_k.
int lqrf_words(int nx, int nu) { return 1 + 2 * nu + nx; }
void lqr_table(int nx, int nu, int N, const std::vector<double> &A, const std::vector<double> &B,
               const std::vector<double> &c, const std::vector<double> &H, const std::vector<double> &He,
               std::vector<double> &tab, std::vector<double> &ftab)
{
    const int nz = nx + nu, W = lqr_words(nx, nu), WF = lqrf_words(nx, nu);
    tab.assign((size_t)N * nz * W, 0.0);
    ftab.assign((size_t)N * nz * WF, 0.0);
    std::vector<double> P(He), M((size_t)nx * nz), F((size_t)nz * nz), L((size_t)nu * nu), Fi((size_t)nu * nu),
        K((size_t)nu * nx);
    auto ab = [&](int l, int c) { return c < nx ? A[l * nx + c] : B[l * nu + (c - nx)]; };
    for (int k = N - 1; k >= 0; k--) {
        double *t = &tab[(size_t)k * nz * W];
        for (int i = 0; i < nx; i++)
            for (int j = 0; j < nz; j++) {
                double s_ = 0.0;
                for (int l = 0; l < nx; l++) s_ += P[i * nx + l] * ab(l, j);
                M[i * nz + j] = s_;
            }
        for (int r = 0; r < nx; r++) {
            double q = 0.0;
            for (int j = 0; j < nx; j++) {
                t[r * W + j] = P[r * nx + j];
                q += P[r * nx + j] * c[j];
            }
            t[r * W + nz] = q;
        }
        for (int i = 0; i < nz; i++)
            for (int j = 0; j < nz; j++) {
                double s_ = H[i * nz + j];
                for (int l = 0; l < nx; l++) s_ += ab(l, i) * M[l * nz + j];
                F[i * nz + j] = s_;
            }
        // F_uu^{-1} by Cholesky (F_uu is positive definite for the reference models' costs)
        for (int i = 0; i < nu; i++)
            for (int j = 0; j <= i; j++) {
                double s_ = F[(nx + i) * nz + nx + j];
                for (int l = 0; l < j; l++) s_ -= L[i * nu + l] * L[j * nu + l];
                L[i * nu + j] = i == j ? std::sqrt(std::max(s_, 1e-300)) : s_ / L[j * nu + j];
            }
        std::vector<double> y(nu);
        for (int c = 0; c < nu; c++) {   // column c of F_uu^{-1}: L L' x = e_c
            for (int i = 0; i < nu; i++) {
                double s_ = i == c ? 1.0 : 0.0;
                for (int l = 0; l < i; l++) s_ -= L[i * nu + l] * y[l];
                y[i] = s_ / L[i * nu + i];
            }
            for (int i = nu - 1; i >= 0; i--) {
                double s_ = y[i];
                for (int l = i + 1; l < nu; l++) s_ -= L[l * nu + i] * y[l];
                y[i] = s_ / L[i * nu + i];
            }
            for (int i = 0; i < nu; i++) Fi[i * nu + c] = y[i];
        }
        for (int i = 0; i < nu; i++)
            for (int j = 0; j < nx; j++) {
                double s_ = 0.0;
                for (int l = 0; l < nu; l++) s_ -= Fi[i * nu + l] * F[(nx + l) * nz + j];
                K[i * nx + j] = s_;
            }
        for (int r = 0; r < nx; r++)
            for (int i = 0; i < nu; i++) t[r * W + nx + i] = K[i * nx + r];
        for (int u = 0; u < nu; u++)
            for (int i = 0; i < nu; i++) t[(nx + u) * W + i] = Fi[u * nu + i];
        double *f = &ftab[(size_t)k * nz * WF];
        for (int r = 0; r < nx; r++) {
            f[r * WF] = t[r * W + nz];
            for (int i = 0; i < nu; i++) {
                f[r * WF + 1 + i] = K[i * nx + r];
                double s_ = 0.0;
                for (int l = 0; l < nu; l++) s_ += B[r * nu + l] * Fi[l * nu + i];
                f[r * WF + 1 + nu + i] = s_;
            }
            for (int j = 0; j < nx; j++) {
                double s_ = A[r * nx + j];
                for (int i = 0; i < nu; i++) s_ += B[r * nu + i] * K[i * nx + j];
                f[r * WF + 1 + 2 * nu + j] = s_;
            }
        }
        for (int u = 0; u < nu; u++) {
            for (int i = 0; i < nu; i++) f[(nx + u) * WF + 1 + nu + i] = Fi[u * nu + i];
            for (int j = 0; j < nx; j++) f[(nx + u) * WF + 1 + 2 * nu + j] = K[u * nx + j];
        }
        for (int i = 0; i < nx; i++)
            for (int j = 0; j < nx; j++) {
                double s_ = F[i * nz + j];
                for (int l = 0; l < nu; l++) s_ += F[i * nz + nx + l] * K[l * nx + j];
                P[i * nx + j] = s_;
            }
        for (int i = 0; i < nx; i++)
            for (int j = 0; j < i; j++) P[i * nx + j] = P[j * nx + i] = 0.5 * (P[i * nx + j] + P[j * nx + i]);
    }
}

// The projected inverse Hessian of the unconstrained LQ problem, ne = (N+1) nz elements e = k nz + r
// (x_0 pinned: its rows and columns are zero; stage N has no inputs): column e' is minus the
// solution of the homogeneous problem (x_0 = 0, c = 0) with a unit gradient at e', so the solution
// with the bounds of a set S held, z = z_0 + W[:, S] nu, W_SS nu = b_S - z_0,S, has the multipliers
// nu (the fast finish's active-set steps). Column-major, from the factorisation in tab.
void lqr_wmat(int nx, int nu, int N, const std::vector<double> &A, const std::vector<double> &B,
              const std::vector<double> &tab, std::vector<double> &w)
{
    const int nz = nx + nu, W = lqr_words(nx, nu), ne = (N + 1) * nz;
    w.assign((size_t)ne * ne, 0.0);
    auto ab = [&](int l, int c) { return c < nx ? A[l * nx + c] : B[l * nu + (c - nx)]; };
    std::vector<double> kff((size_t)N * nu), z((size_t)ne);
    for (int e1 = 0; e1 < ne; e1++) {
        const int k1 = e1 / nz, r1 = e1 % nz;
        if ((k1 == 0 && r1 < nx) || (k1 == N && r1 >= nx)) continue;
        std::vector<double> p(nx, 0.0), h(nz);
        if (k1 == N) p[r1] = 1.0;
        for (int k = N - 1; k >= 0; k--) {
            const double *t = &tab[(size_t)k * nz * W];
            for (int i = 0; i < nz; i++) {
                double s_ = (k == k1 && i == r1) ? 1.0 : 0.0;
                for (int l = 0; l < nx; l++) s_ += ab(l, i) * p[l];
                h[i] = s_;
            }
            for (int u = 0; u < nu; u++) {
                double s_ = 0.0;
                for (int i = 0; i < nu; i++) s_ -= t[(nx + u) * W + i] * h[nx + i];
                kff[(size_t)k * nu + u] = s_;
            }
            for (int j = 0; j < nx; j++) {
                double s_ = h[j];
                for (int i = 0; i < nu; i++) s_ += t[j * W + nx + i] * h[nx + i];
                p[j] = s_;
            }
        }
        std::vector<double> x(nx, 0.0), xn(nx);
        for (int k = 0; k < N; k++) {
            const double *t = &tab[(size_t)k * nz * W];
            std::vector<double> uu(nu);
            for (int u = 0; u < nu; u++) {
                double s_ = kff[(size_t)k * nu + u];
                for (int j = 0; j < nx; j++) s_ += t[j * W + nx + u] * x[j];
                uu[u] = s_;
            }
            for (int j = 0; j < nx; j++) z[(size_t)k * nz + j] = x[j];
            for (int u = 0; u < nu; u++) z[(size_t)k * nz + nx + u] = uu[u];
            for (int i = 0; i < nx; i++) {
                double s_ = 0.0;
                for (int j = 0; j < nx; j++) s_ += A[i * nx + j] * x[j];
                for (int u = 0; u < nu; u++) s_ += B[i * nu + u] * uu[u];
                xn[i] = s_;
            }
            x = xn;
        }
        for (int j = 0; j < nx; j++) z[(size_t)N * nz + j] = x[j];
        for (int j = 0; j < nu; j++) z[(size_t)N * nz + nx + j] = 0.0;
        for (int e = 0; e < ne; e++) w[(size_t)e1 * ne + e] = (e < nx) ? 0.0 : -z[e];
    }
}

// The unconstrained LQ solution from base 0 (the fast finish's first step, oracle-free host form of
// the kernel's recursion on the lqr_table records): gradient g (stage-stacked, nz per stage, stage N
// nx), initial state x0, affine term c on or off. z: (N+1) nz.
void lqr_solve(int nx, int nu, int N, const std::vector<double> &A, const std::vector<double> &B,
               const std::vector<double> &c, const std::vector<double> &tab, const double *g, const double *x0,
               bool use_c, double *z)
{
    const int nz = nx + nu, W = lqr_words(nx, nu);
    auto ab = [&](int l, int q) { return q < nx ? A[l * nx + q] : B[l * nu + (q - nx)]; };
    std::vector<double> p(g + (size_t)N * nz, g + (size_t)N * nz + nx), v(nx), h(nz), kff((size_t)N * nu);
    for (int k = N - 1; k >= 0; k--) {
        const double *t = &tab[(size_t)k * nz * W];
        for (int r = 0; r < nx; r++) v[r] = p[r] + (use_c ? t[r * W + nz] : 0.0);
        for (int i = 0; i < nz; i++) {
            double s_ = g[(size_t)k * nz + i];
            for (int l = 0; l < nx; l++) s_ += ab(l, i) * v[l];
            h[i] = s_;
        }
        for (int u = 0; u < nu; u++) {
            double s_ = 0.0;
            for (int i = 0; i < nu; i++) s_ -= t[(nx + u) * W + i] * h[nx + i];
            kff[(size_t)k * nu + u] = s_;
        }
        for (int j = 0; j < nx; j++) {
            double s_ = h[j];
            for (int i = 0; i < nu; i++) s_ += t[j * W + nx + i] * h[nx + i];
            p[j] = s_;
        }
    }
    std::vector<double> x(x0, x0 + nx), xn(nx), uu(nu);
    for (int k = 0; k < N; k++) {
        const double *t = &tab[(size_t)k * nz * W];
        for (int u = 0; u < nu; u++) {
            double s_ = kff[(size_t)k * nu + u];
            for (int j = 0; j < nx; j++) s_ += t[j * W + nx + u] * x[j];
            uu[u] = s_;
        }
        for (int j = 0; j < nx; j++) z[(size_t)k * nz + j] = x[j];
        for (int u = 0; u < nu; u++) z[(size_t)k * nz + nx + u] = uu[u];
        for (int i = 0; i < nx; i++) {
            double s_ = use_c ? c[i] : 0.0;
            for (int j = 0; j < nx; j++) s_ += A[i * nx + j] * x[j];
            for (int u = 0; u < nu; u++) s_ += B[i * nu + u] * uu[u];
            xn[i] = s_;
        }
        x = xn;
    }
    for (int j = 0; j < nx; j++) z[(size_t)N * nz + j] = x[j];
    for (int u = 0; u < nu; u++) z[(size_t)N * nz + nx + u] = 0.0;
}

int hip_fail(nmpc_solver *h, hipError_t e, const char *what)
{
    return h->fail(NMPC_EDEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

void free_all(nmpc_solver *h)
{
    hipSetDevice(h->device);
    for (void *p : {h->d_model, h->d_x0, h->d_yref, h->d_x, h->d_u, h->d_scratch, (void *)h->d_status,
                    (void *)h->d_iters, h->d_table, h->d_state, h->d_plant, h->d_wcl, (void *)h->d_offsets,
                    (void *)h->d_acc, (void *)h->d_noise, (void *)h->d_cycles, h->d_cond, (void *)h->d_cond_i,
                    (void *)h->d_fnoise, (void *)h->d_iter_log, h->d_cltx, h->d_clv, h->d_fsT, (void *)h->d_fsI,
                    (void *)h->d_istep, (void *)h->d_park, (void *)h->d_flags, h->d_clf_scratch, (void *)h->d_clw,
                    (void *)h->d_fin_f, (void *)h->d_fin_i, (void *)h->d_z0, (void *)h->d_sf, (void *)h->d_f64,
                    (void *)h->d_f64i, (void *)h->d_sfl, h->d_sf_scratch, (void *)h->d_sfcyc, (void *)h->d_clf_check, (void *)h->d_imap,
                    (void *)h->d_gorder})
        if (p) hipFree(p);
    if (h->h_sfpark) hipHostFree(h->h_sfpark);
    if (h->ev_fb) hipEventDestroy(h->ev_fb);
    for (hipEvent_t e : h->cl_events) hipEventDestroy(e);
    if (h->h_park) hipHostFree(h->h_park);
    if (h->h_parkr) hipHostFree(h->h_parkr);
    if (h->ev0) hipEventDestroy(h->ev0);
    if (h->ev1) hipEventDestroy(h->ev1);
    if (h->own_stream) hipStreamDestroy(h->own_stream);
}

template <typename T>
int launch_cond(nmpc_solver *h, hipEvent_t e0, hipEvent_t e1)
{
    nmpc::CondParams<T> p{};
    const nmpc::CondHost &c = h->ch;
    p.B = h->batch;
    p.N = h->N;
    p.nx = h->nx;
    p.nu = h->nu;
    p.n = c.n;
    p.nb = c.nb;
    p.mx = c.mx;
    p.ldg = c.ldg;
    p.nY = c.nY;
    p.ny = h->ny;
    p.yref_is_z = h->yref_is_z;
    p.max_iter = h->max_iter;
    p.wave_elems = (int)nmpc::cond_wave_elems<T>(c.nb, c.ldg);
    p.tol_comp = (T)h->tol_comp;
    p.tol_res = (T)h->tol_res;
    p.mu0 = (T)h->mu0;
    p.inv_m = (T)h->inv_m;
    const T *b = (const T *)h->d_cond;
    const T **f[15] = {&p.Gx, &p.H0, &p.H0t, &p.Fx, &p.Fy, &p.fc, &p.Phx, &p.dx, &p.lox, &p.hix,
                       &p.lou, &p.hiu, &p.Gall, &p.Phall, &p.dall};
    for (int i = 0; i < 15; i++) *f[i] = b + h->co[i];
    p.xcols = h->d_cond_i + h->ci[0];
    p.rstart = h->d_cond_i + h->ci[1];
    p.ks = h->d_cond_i + h->ci[2];
    p.x0 = (const T *)h->d_x0;
    p.yref = (const T *)h->d_yref;
    p.xout = (T *)h->d_x;
    p.uout = (T *)h->d_u;
    p.status = h->d_status;
    p.iters = h->d_iters;
    p.cycles = nullptr;
    static const bool cycles = std::getenv("NMPC_SWEEP_CYCLES") != nullptr;
    if (cycles) {
        if (!h->d_cycles && hipMalloc(&h->d_cycles, (size_t)h->batch * 9 * sizeof(unsigned long long)) != hipSuccess)
            h->d_cycles = nullptr;
        p.cycles = h->d_cycles;
    }
    hipEventRecord(e0 ? e0 : h->ev0, h->stream);
    hipError_t e = nmpc::cond_launch<T>(p, h->cond_wpb, h->cond_lds, h->stream);
    hipEventRecord(e1 ? e1 : h->ev1, h->stream);
    if (e != hipSuccess) return hip_fail(h, e, "condensed ipm kernel launch");
    if (cycles && h->d_cycles) {
        // tuning aid (NMPC_COND_TIMING builds): mean cycles per instance in each phase
        std::vector<unsigned long long> cy((size_t)h->batch * 9);
        hipStreamSynchronize(h->stream);
        hipMemcpy(cy.data(), h->d_cycles, cy.size() * sizeof(cy[0]), hipMemcpyDeviceToHost);
        double m[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int b = 0; b < h->batch; b++)
            for (int j = 0; j < 8; j++) m[j] += (double)cy[(size_t)b * 9 + j] / h->batch;
        std::fprintf(stderr, "[nmpc cond cycles] B=%d per instance: setup %.0f resid %.0f syrk %.0f chol %.0f pred %.0f"
                     " corr %.0f step %.0f out %.0f\n", h->batch, m[0], m[1], m[2], m[3], m[4], m[5], m[6], m[7]);
    }
    return 0;
}

template <typename T>
nmpc::ClParams<T> cl_params(nmpc_solver *h);

constexpr int CL_FUSED_CHUNK = 64;   // closed-loop steps per fused solve launch
constexpr int CLF_CHUNK = 64;        // closed-loop steps per lean-loop launch (bounded noise / log buffers)
// the lean loop's asynchronous runs (sync = 0): per round of a chunk its own [park count, claim counter] pair,
// after the park list in d_park
constexpr int CLF_ROUND_WORDS = 2 * (CLF_CHUNK + 1);
constexpr int CLF_NT_HOST = 24;      // timing builds: phase counters per instance (nmpc_cl_fast.hip CLF_NT)

int fin32_setup(nmpc_solver *h);
hipError_t fin32_enqueue(nmpc_solver *h);
int sf_setup(nmpc_solver *h);
int sf_resolve(nmpc_solver *h);

// list mode of the lane-per-component kernel: the lean closed loop's fallback (a full solve + plant step per
// listed instance, cl_steps = 1) or the fast general solve's (a cold full solve per listed instance, cl_steps = 0)
struct ListArgs {
    int count, step0, noise_ld;
    const int *list;
    int kidx;
    void *scratch;
    const int *count_dev = nullptr;   // the list's length on the device (count: the grid's capacity), or null
};

// cl_steps > 0: fused closed loop of that many steps (lane-per-component / wavefront kernels). fast: a plain
// solve of an fp64 handle may take the fast solve (sf_enqueue: complete in stream order, so the per-step closed
// loop's advance kernel can follow it on the stream with no host step between)
int sf_enqueue(nmpc_solver *h, hipEvent_t e0, hipEvent_t e1);

template <typename T>
int launch(nmpc_solver *h, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr, int cl_steps = 0, const ListArgs *la = nullptr,
           bool fast = true)
{
    if (h->cond) return launch_cond<T>(h, e0, e1);
    if (std::is_same<T, double>::value && fast && h->sfast && cl_steps == 0 && !la) return sf_enqueue(h, e0, e1);
    nmpc::IpmParams<T> p{};
    int kidx = h->kidx;
    void *scratch = h->d_scratch;
    p.cl_steps = cl_steps;
    if (la) {
        kidx = la->kidx;
        if (la->scratch) scratch = la->scratch;
        p.cl_list = la->list;
        p.cl_count = la->count;
        p.cl_count_dev = la->count_dev;
        p.cl_istep = h->d_istep;
        p.cl_noise_ld = la->noise_ld;
        p.cl_noise_step0 = la->step0;
        p.cl_flags = h->d_flags;
        p.cl_eslot = h->d_fsI + h->fsi[2];
        p.cl_nslot = h->clf_nslot;
    }
    if (cl_steps > 0) {
        p.cl = cl_params<T>(h);
        p.cl_noise = h->d_fnoise;
        // env NMPC_ITER_LOG: the fused launch's step record. The list mode (the lean loop's fallback)
        // neither writes nor resizes it: the lean loop's own log (clf_run) stays as that run left it
        static const bool iter_log = std::getenv("NMPC_ITER_LOG") != nullptr;
        if (iter_log && !la) {
            const size_t need = (size_t)h->batch * CL_FUSED_CHUNK;
            if (h->iter_log_cap < need) {   // the capacity is set only where the allocation happens
                if (h->d_iter_log) hipFree(h->d_iter_log);
                h->d_iter_log = nullptr;
                h->iter_log_cap = 0;
                if (hipMalloc((void **)&h->d_iter_log, need * sizeof(int)) == hipSuccess) h->iter_log_cap = need;
            }
            p.iter_log = h->d_iter_log;
            h->iter_log_steps = p.iter_log ? cl_steps : 0;
        }
        const bool no_expl = (std::getenv("NMPC_EXPLICIT") && std::getenv("NMPC_EXPLICIT")[0] == '0') ||
                             h->precision != NMPC_FP64;   // the fused loop's fast finish: fp64 handles
        p.cl_tx = no_expl ? nullptr : (const T *)h->d_cltx;
        p.cl_v = no_expl ? nullptr : (const T *)h->d_clv;
    }
    p.B = h->batch;
    p.N = h->N;
    p.ny = h->ny;
    p.ny_e = h->ny_e;
    p.yref_is_z = h->yref_is_z;
    p.g_diag = h->g_diag;
    p.max_iter = h->max_iter;
    p.tol_comp = (T)h->tol_comp;
    p.tol_res = (T)h->tol_res;
    p.mu0 = (T)h->mu0;
    p.inv_m = (T)h->inv_m;
    p.polish_mu = (T)h->polish_mu;
    p.polish_rho = (T)h->polish_rho;
    p.polish_steps = h->polish_steps;
    p.polish_first = h->polish_first;
    p.polish_drop = (T)h->polish_drop;
    const int warm_shift = std::getenv("NMPC_WARM_SHIFT") ? std::atoi(std::getenv("NMPC_WARM_SHIFT")) : 1;
    p.warm_shift = warm_shift;
    const int fast_mode = std::getenv("NMPC_FAST") ? std::atoi(std::getenv("NMPC_FAST")) : 1;
    p.fast_mode = fast_mode;
    const char *m = (const char *)h->d_model;
    p.AB = (const T *)(m + h->off_AB);
    p.ABt = (const T *)(m + h->off_ABt);
    p.c = (const T *)(m + h->off_c);
    p.H = (const T *)(m + h->off_H);
    p.He = (const T *)(m + h->off_He);
    p.G = (const T *)(m + h->off_G);
    p.Ge = (const T *)(m + h->off_Ge);
    p.lbnd = (const T *)(m + h->off_lb);
    p.ubnd = (const T *)(m + h->off_ub);
    // tuning / test switches, read per launch: NMPC_LQR=0 drops the shared factorisation (every finish
    // step factors), NMPC_FAST=0 / 2 the fast finish (2: not at a launch's first step),
    // NMPC_WARM_SHIFT=0 the warm-start shift
    const bool no_lqr = (std::getenv("NMPC_LQR") && std::getenv("NMPC_LQR")[0] == '0') || h->lqr_host.empty() ||
                        h->precision != NMPC_FP64;   // fp32 handles: no exact finish, the tables are the lean loop's
    p.lqr = no_lqr ? nullptr : (const T *)(m + h->off_lqr);
    p.lqrf = no_lqr ? nullptr : (const T *)(m + h->off_lqrf);
    const bool no_w = std::getenv("NMPC_WSET") && std::getenv("NMPC_WSET")[0] == '0';
    p.lqrw = (no_lqr || no_w) ? nullptr : (const T *)(m + h->off_lqrw);
    p.x0 = (const T *)h->d_x0;
    p.yref = (const T *)h->d_yref;
    p.xout = (T *)h->d_x;
    p.uout = (T *)h->d_u;
    p.status = h->d_status;
    p.iters = h->d_iters;
    p.scratch = (T *)scratch;
    p.ipw = h->ipw;
    p.lpi_stride = ((long long)h->batch + h->ipw - 1) / h->ipw * h->ipw;
    p.cycles = nullptr;
    static const bool sweep_cycles = std::getenv("NMPC_SWEEP_CYCLES") != nullptr;
    if (sweep_cycles) {
        if (!h->d_cycles && hipMalloc(&h->d_cycles, (size_t)h->batch * 9 * sizeof(unsigned long long)) != hipSuccess)
            h->d_cycles = nullptr;
        p.cycles = h->d_cycles;
    }
    hipError_t e = hipEventRecord(e0 ? e0 : h->ev0, h->stream);
    if (e == hipSuccess) e = nmpc::ipm_launch<T>(kidx, p, h->stream);
    // fp32 solves: the exact finish (inside the timed pair: it is part of the solve)
    if (e == hipSuccess && cl_steps == 0 && !la && h->fin32) e = fin32_enqueue(h);
    if (e == hipSuccess) e = hipEventRecord(e1 ? e1 : h->ev1, h->stream);
    if (e != hipSuccess) return hip_fail(h, e, "ipm kernel launch");
    if (sweep_cycles && h->d_cycles) {
        // tuning aid (experiment builds with NMPC_SWEEP_TIMING): mean clock cycles per instance
        // spent in each phase
        std::vector<unsigned long long> c((size_t)h->batch * 9);
        hipStreamSynchronize(h->stream);
        hipMemcpy(c.data(), h->d_cycles, c.size() * sizeof(c[0]), hipMemcpyDeviceToHost);
        double s[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int b = 0; b < h->batch; b++)
            for (int j = 0; j < 9; j++) s[j] += (double)c[(size_t)b * 9 + j] / h->batch;
        if (std::strcmp(std::getenv("NMPC_SWEEP_CYCLES"), "step") == 0)   // NMPC_STEP_TIMING builds
            std::fprintf(stderr, "[nmpc step cycles] B=%d steps=%d mean per instance: warm+fast %.0f cert+init %.0f finA %.0f"
                         " finB %.0f ipmA %.0f ipmBCD %.0f out %.0f adv %.0f total %.0f\n",
                         h->batch, cl_steps, s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7], s[8]);
        else
            std::fprintf(stderr, "[nmpc cycles] B=%d mean per instance: E_A %.0f A %.0f B %.0f E_B %.0f E_C %.0f C %.0f"
                         " D %.0f E_D %.0f total %.0f\n",
                         h->batch, s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7], s[8]);
    }
    return 0;
}

int field_is(const char *f, const char *name) { return f && std::strcmp(f, name) == 0; }

}  // namespace

extern "C" {

int nmpc_abi_version(void) { return NMPC_ABI_VERSION; }

int nmpc_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char *nmpc_last_error_global(void) { return g_err.c_str(); }

const char *nmpc_last_error(const nmpc_solver *h) { return h ? h->err.c_str() : g_err.c_str(); }

int nmpc_create(const nmpc_ocp_desc *d, int batch, int device, int precision, nmpc_solver **out)
{
    if (!out) return (g_err = "nmpc_create: out is NULL", NMPC_EINVAL);
    *out = nullptr;
    if (!d || d->abi_version != NMPC_ABI_VERSION) {
        g_err = "nmpc_create: missing descriptor or ABI version mismatch";
        return NMPC_EINVAL;
    }
    if (d->nx < 1 || d->nu < 1 || d->N < 1 || d->ny < 1 || d->ny_e < 0 || batch < 1) {
        g_err = "nmpc_create: invalid dimensions";
        return NMPC_EINVAL;
    }
    if (precision != NMPC_FP64 && precision != NMPC_FP32) {
        g_err = "nmpc_create: precision must be NMPC_FP64 or NMPC_FP32";
        return NMPC_EINVAL;
    }
    if (!d->A || !d->B || !d->c || !d->W || !d->Vx || !d->Vu || (d->ny_e > 0 && (!d->W_e || !d->Vx_e))) {
        g_err = "nmpc_create: dynamics / cost matrices missing";
        return NMPC_EINVAL;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
        g_err = "nmpc_create: no HIP device available (the engine has no CPU fallback)";
        return NMPC_EDEVICE;
    }
    if (device < 0 || device >= ndev) {
        g_err = "nmpc_create: device index out of range";
        return NMPC_EINVAL;
    }
    nmpc_solver *h = new nmpc_solver();
    h->name = d->name ? d->name : "nmpc";
    h->device = device;
    h->precision = precision;
    h->batch = batch;
    h->nx = d->nx;
    h->nu = d->nu;
    h->N = d->N;
    h->ny = d->ny;
    h->ny_e = d->ny_e;
    const int nx = d->nx, nu = d->nu, nz = nx + nu, N = d->N, ny = d->ny, ny_e = d->ny_e;

    int ipw_req = 0;
    if (const char *e = std::getenv("NMPC_IPW")) ipw_req = std::atoi(e);
    h->kidx = precision == NMPC_FP64 ? nmpc::ipm_find<double>(nx, nu, -1, batch, &h->ipw, &h->lds, &h->wpb)
                                     : nmpc::ipm_find<float>(nx, nu, -1, batch, &h->ipw, &h->lds, &h->wpb);
    {
        // kernel family: NMPC_KERNEL=cond forces the condensed MFMA kernels; they also take any
        // (nx, nu) without a compiled stage-wise kernel (dimension-generic at run time)
        const char *kf = std::getenv("NMPC_KERNEL");
        h->cond = (kf && (kf[0] == 'c' || kf[0] == 'C')) || h->kidx < 0;
    }
    // packing heuristic: keep >= 2 wavefronts per SIMD (1024 SIMDs on MI355X) if possible
    if (ipw_req <= 0 && !h->cond) {
        int cand[4] = {8, 4, 2, 1}, chosen = -1;
        for (int ipw : cand) {
            int ip, ld;
            const int idx = precision == NMPC_FP64 ? nmpc::ipm_find<double>(nx, nu, ipw, batch, &ip, &ld, nullptr)
                                                   : nmpc::ipm_find<float>(nx, nu, ipw, batch, &ip, &ld, nullptr);
            if (idx < 0) continue;
            if (chosen < 0) chosen = ipw;  // widest compiled
            if ((batch + ipw - 1) / ipw >= 2048) {
                chosen = ipw;
                break;
            }
            chosen = ipw;  // keep narrowing toward 1 while waves are scarce
        }
        ipw_req = chosen;
    }
    if (!h->cond) {
        const int idx = precision == NMPC_FP64 ? nmpc::ipm_find<double>(nx, nu, ipw_req, batch, &h->ipw, &h->lds, &h->wpb)
                                               : nmpc::ipm_find<float>(nx, nu, ipw_req, batch, &h->ipw, &h->lds, &h->wpb);
        if (idx >= 0) h->kidx = idx;
    }

    // ---- dynamics
    if (d->dyn_type == NMPC_DYN_DISCRETE_AFFINE) {
        h->A.assign(d->A, d->A + nx * nx);
        h->B.assign(d->B, d->B + nx * nu);
        h->c.assign(d->c, d->c + nx);
    } else if (d->dyn_type == NMPC_DYN_CONTINUOUS_AFFINE) {
        if (!(d->tf > 0.0)) {
            delete h;
            g_err = "nmpc_create: tf must be > 0 for continuous dynamics";
            return NMPC_EINVAL;
        }
        const int stages = d->num_stages > 0 ? d->num_stages : (d->integrator_type == NMPC_IRK ? 4 : 4);
        const int steps = d->num_steps > 0 ? d->num_steps : 1;
        if (!discretize(nx, nu, d->A, d->B, d->c, d->integrator_type, stages, steps, d->tf / N, h->A, h->B, h->c)) {
            delete h;
            g_err = "nmpc_create: unsupported integrator (IRK: 1..9 stages, ERK: 1, 2 or 4 stages)";
            return NMPC_EUNSUPPORTED;
        }
    } else {
        delete h;
        g_err = "nmpc_create: unknown dyn_type";
        return NMPC_EINVAL;
    }
    h->ts = d->tf > 0.0 ? d->tf / N : 1.0;
    // ---- LINEAR_LS cost -> stage QP data
    const double s = (d->cost_scaling == NMPC_COST_SCALING_TIME_STEPS) ? h->ts : 1.0;
    h->cost_s = s;
    h->W.assign(d->W, d->W + ny * ny);
    h->Vx.assign(d->Vx, d->Vx + ny * nx);
    h->Vu.assign(d->Vu, d->Vu + ny * nu);
    if (ny_e > 0) {
        h->W_e.assign(d->W_e, d->W_e + ny_e * ny_e);
        h->Vx_e.assign(d->Vx_e, d->Vx_e + ny_e * nx);
    }
    std::vector<double> V(ny * nz);
    for (int r = 0; r < ny; r++) {
        for (int q = 0; q < nx; q++) V[r * nz + q] = d->Vx[r * nx + q];
        for (int q = 0; q < nu; q++) V[r * nz + nx + q] = d->Vu[r * nu + q];
    }
    h->H.assign(nz * nz, 0.0);
    h->G.assign(nz * ny, 0.0);
    for (int i = 0; i < nz; i++)
        for (int j = 0; j < ny; j++) {
            double wv = 0.0;
            for (int r = 0; r < ny; r++) wv += V[r * nz + i] * d->W[r * ny + j];
            h->G[i * ny + j] = -s * wv;
        }
    for (int i = 0; i < nz; i++)
        for (int j = 0; j < nz; j++) {
            double acc = 0.0;
            for (int r = 0; r < ny; r++) acc += -h->G[i * ny + r] * V[r * nz + j];
            h->H[i * nz + j] = acc;
        }
    h->He.assign(nx * nx, 0.0);
    h->Ge.assign(nx * std::max(ny_e, 1), 0.0);
    for (int i = 0; i < nx; i++)
        for (int j = 0; j < ny_e; j++) {
            double wv = 0.0;
            for (int r = 0; r < ny_e; r++) wv += d->Vx_e[r * nx + i] * d->W_e[r * ny_e + j];
            h->Ge[i * ny_e + j] = -h->scale_e * wv;
        }
    for (int i = 0; i < nx; i++)
        for (int j = 0; j < nx; j++) {
            double acc = 0.0;
            for (int r = 0; r < ny_e; r++) acc += -h->Ge[i * ny_e + r] * d->Vx_e[r * nx + j];
            h->He[i * nx + j] = acc;
        }
    bool sel = (ny == nz) && (ny_e == nx);
    for (int r = 0; sel && r < ny; r++)
        for (int q = 0; sel && q < nz; q++)
            if (V[r * nz + q] != (r == q ? 1.0 : 0.0)) sel = false;
    for (int r = 0; sel && r < ny_e; r++)
        for (int q = 0; sel && q < nx; q++)
            if (d->Vx_e[r * nx + q] != (r == q ? 1.0 : 0.0)) sel = false;
    h->yref_is_z = sel ? 1 : 0;
    // diagonal gradient maps (diagonal W): the kernels form g_c = G_rr y_r
    bool gdiag = sel;
    for (int i = 0; gdiag && i < nz; i++)
        for (int j = 0; j < ny; j++)
            if (i != j && h->G[i * ny + j] != 0.0) gdiag = false;
    for (int i = 0; gdiag && i < nx; i++)
        for (int j = 0; j < ny_e; j++)
            if (i != j && h->Ge[i * ny_e + j] != 0.0) gdiag = false;
    h->g_diag = gdiag ? 1 : 0;
    // ---- bounds [3][nz]
    h->lbnd.assign(3 * nz, -kInf);
    h->ubnd.assign(3 * nz, kInf);
    int nlb_u = 0, nub_u = 0, nlb_x = 0, nub_x = 0, nlb_e = 0, nub_e = 0;
    for (int j = 0; j < d->nbu; j++) {
        const int i = d->idxbu[j];
        if (i < 0 || i >= nu) {
            delete h;
            g_err = "nmpc_create: idxbu out of range";
            return NMPC_EINVAL;
        }
        for (int t = 0; t < 2; t++) {
            h->lbnd[t * nz + nx + i] = d->lbu[j];
            h->ubnd[t * nz + nx + i] = d->ubu[j];
        }
        nlb_u += has_bound(d->lbu[j]);
        nub_u += has_bound(d->ubu[j]);
    }
    for (int j = 0; j < d->nbx; j++) {
        const int i = d->idxbx[j];
        if (i < 0 || i >= nx) {
            delete h;
            g_err = "nmpc_create: idxbx out of range";
            return NMPC_EINVAL;
        }
        h->lbnd[1 * nz + i] = d->lbx[j];
        h->ubnd[1 * nz + i] = d->ubx[j];
        nlb_x += has_bound(d->lbx[j]);
        nub_x += has_bound(d->ubx[j]);
    }
    for (int j = 0; j < d->nbx_e; j++) {
        const int i = d->idxbx_e[j];
        if (i < 0 || i >= nx) {
            delete h;
            g_err = "nmpc_create: idxbx_e out of range";
            return NMPC_EINVAL;
        }
        h->lbnd[2 * nz + i] = d->lbx_e[j];
        h->ubnd[2 * nz + i] = d->ubx_e[j];
        nlb_e += has_bound(d->lbx_e[j]);
        nub_e += has_bound(d->ubx_e[j]);
    }
    const long m = (long)N * (nlb_u + nub_u) + (long)(N - 1) * (nlb_x + nub_x) + (nlb_e + nub_e);
    h->inv_m = 1.0 / (double)std::max(1L, m);
    // ---- options
    const bool f64 = precision == NMPC_FP64;
    h->max_iter = d->qp_solver_iter_max > 0 ? d->qp_solver_iter_max : 50;
    // fp32 handles never ask for more than single precision can reach (1e-7 / 1e-5)
    h->tol_comp = d->qp_solver_tol_comp > 0 ? d->qp_solver_tol_comp : (f64 ? 1e-15 : 1e-7);
    h->tol_res = d->qp_solver_tol_res > 0 ? d->qp_solver_tol_res : (f64 ? 1e-12 : 1e-5);
    if (!f64) {
        h->tol_comp = std::max(h->tol_comp, 1e-7);
        h->tol_res = std::max(h->tol_res, 1e-5);
    }
    h->mu0 = d->qp_solver_mu0 > 0 ? d->qp_solver_mu0 : 1e-2;
    // exact finish: fp64 only (the penalised solve needs ~16 digits); the penalty is 1e6 x the
    // largest cost curvature, as in oracle/c/riccati_ipm.c (POLISH_RHO)
    h->polish_mu = !f64 || d->qp_solver_polish_mu < 0 ? 0.0 : (d->qp_solver_polish_mu > 0 ? d->qp_solver_polish_mu : 1.0);
    h->polish_steps = d->qp_solver_polish_steps > 0 ? d->qp_solver_polish_steps : 12;
    h->polish_first = h->polish_steps;
    // tuning overrides (experiments only): set steps of later / first finish runs, mu drop between runs
    if (const char *e = std::getenv("NMPC_POLISH_STEPS")) h->polish_steps = std::max(1, std::atoi(e));
    if (const char *e = std::getenv("NMPC_POLISH_FIRST")) h->polish_first = std::max(1, std::atoi(e));
    else h->polish_first = h->polish_steps;
    if (const char *e = std::getenv("NMPC_POLISH_DROP")) h->polish_drop = std::atof(e);
    {
        double hmax = 1.0;
        for (int i = 0; i < nz; i++) hmax = std::max(hmax, std::fabs(h->H[i * nz + i]));
        for (int i = 0; i < nx; i++) hmax = std::max(hmax, std::fabs(h->He[i * nx + i]));
        h->polish_rho = 1e6 * hmax;
    }
    // ---- host staging
    h->h_x0.assign((size_t)batch * nx, 0.0);
    if (d->x0)
        for (int b = 0; b < batch; b++) std::memcpy(&h->h_x0[(size_t)b * nx], d->x0, nx * sizeof(double));
    h->h_lbx0 = h->h_x0;
    h->h_ubx0 = h->h_x0;
    h->h_yref.assign((size_t)batch * h->ystride(), 0.0);
    if (d->yref || d->yref_e)
        for (int b = 0; b < batch; b++) {
            for (int k = 0; k < N && d->yref; k++)
                std::memcpy(&h->h_yref[b * h->ystride() + (size_t)k * ny], d->yref, ny * sizeof(double));
            if (d->yref_e && ny_e > 0)
                std::memcpy(&h->h_yref[b * h->ystride() + (size_t)N * ny], d->yref_e, ny_e * sizeof(double));
        }
    h->h_x.assign((size_t)batch * (N + 1) * nx, 0.0);
    h->h_u.assign((size_t)batch * N * nu, 0.0);
    h->h_status.assign(batch, 0);
    h->h_iters.assign(batch, 0);

    // ---- device
    hipError_t e;
    if ((e = hipSetDevice(device)) != hipSuccess) {
        int r = hip_fail(h, e, "hipSetDevice");
        delete h;
        return r;
    }
    if ((e = hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking)) != hipSuccess) {
        int r = hip_fail(h, e, "hipStreamCreate");
        delete h;
        return r;
    }
    h->stream = h->own_stream;
    hipEventCreate(&h->ev0);
    hipEventCreate(&h->ev1);
    const size_t es = h->esz();
    size_t off = 0;
    auto carve = [&](size_t n) {
        size_t o = off;
        off += ((n * es + 255) / 256) * 256;
        return o;
    };
    h->off_AB = carve((size_t)nx * nz);
    h->off_ABt = carve((size_t)nx * nz);
    h->off_c = carve(nx);
    h->off_H = carve((size_t)nz * nz);
    h->off_He = carve((size_t)nx * nx);
    h->off_G = carve((size_t)nz * ny);
    h->off_Ge = carve((size_t)nx * std::max(ny_e, 1));
    h->off_lb = carve(3 * nz);
    h->off_ub = carve(3 * nz);
    // the unconstrained factorisation's tables (lqr_table, lqr_wmat) serve the exact finish's shortcuts of
    // the stage-wise kernels and the fast solve (fp64 handles with the finish on: polish_mu > 0) and, from
    // the host copy, the lean closed loop's tables in both precisions. fp32 handles keep only the host copy:
    // their kernels never read the device tables (the lean loop and the fp32 finish use the fp64 W, d_clw)
    const bool lqr_on = !h->cond && (!f64 || h->polish_mu > 0);
    const bool lqr_dev = lqr_on && f64;
    h->off_lqr = carve(lqr_dev ? (size_t)N * nz * lqr_words(nx, nu) : 0);
    h->off_lqrf = carve(lqr_dev ? (size_t)N * nz * lqrf_words(nx, nu) : 0);
    h->off_lqrw = carve(lqr_dev ? (size_t)(N + 1) * nz * (N + 1) * nz : 0);
    const size_t model_bytes = off;
    if (h->cond) {
        if (!nmpc::cond_build(nx, nu, N, ny, ny_e, h->A, h->B, h->c, h->H, h->G, h->He, h->Ge, h->lbnd, h->ubnd, h->ch)) {
            delete h;
            g_err = "nmpc_create: no compiled kernel for nx=" + std::to_string(nx) + " nu=" + std::to_string(nu) +
                    " and the condensed kernels need N*nu <= 128 and N*nu + bounded x rows <= 512";
            return NMPC_EUNSUPPORTED;
        }
        // workgroup: the most wavefronts (<= 4) whose LDS (shared Gx + per-wave tiles/vectors) fits
        const size_t we = precision == NMPC_FP64 ? nmpc::cond_wave_elems<double>(h->ch.nb, h->ch.ldg)
                                                 : nmpc::cond_wave_elems<float>(h->ch.nb, h->ch.ldg);
        const size_t gx = (size_t)16 * h->ch.nb * h->ch.ldg + (((size_t)h->ch.n * h->ch.n + 3) & ~(size_t)3);
        h->cond_wpb = 0;
        for (int w = 4; w >= 1 && !h->cond_wpb; w--)
            if ((gx + w * we) * es <= 160 * 1024) h->cond_wpb = w;
        if (!h->cond_wpb) {
            delete h;
            g_err = "nmpc_create: the condensed kernel's LDS need exceeds 160 KB for this OCP";
            return NMPC_EUNSUPPORTED;
        }
        h->cond_lds = (gx + h->cond_wpb * we) * es;
        h->ipw = 1;
        h->wpb = h->cond_wpb;
        h->lds = (int)h->cond_lds;
    } else {
        // structure-specialised kernel when the model fits one (exact zeros of [A B], diagonal costs)
        std::vector<double> ABh((size_t)nx * nz);
        for (int r = 0; r < nx; r++) {
            for (int q = 0; q < nx; q++) ABh[r * nz + q] = h->A[r * nx + q];
            for (int q = 0; q < nu; q++) ABh[r * nz + nx + q] = h->B[r * nu + q];
        }
        h->kidx = precision == NMPC_FP64 ? nmpc::ipm_refine<double>(h->kidx, ABh.data(), h->H.data(), h->He.data())
                                         : nmpc::ipm_refine<float>(h->kidx, ABh.data(), h->H.data(), h->He.data());
    }
    const size_t scratch_bytes = h->cond ? 256
                                         : (precision == NMPC_FP64 ? nmpc::ipm_scratch_elems<double>(h->kidx, batch, N)
                                                                   : nmpc::ipm_scratch_elems<float>(h->kidx, batch, N)) * es;
    bool ok = hipMalloc(&h->d_model, model_bytes) == hipSuccess &&
              hipMalloc(&h->d_x0, (size_t)batch * nx * es) == hipSuccess &&
              hipMalloc(&h->d_yref, (size_t)batch * h->ystride() * es) == hipSuccess &&
              hipMalloc(&h->d_x, (size_t)batch * (N + 1) * nx * es) == hipSuccess &&
              hipMalloc(&h->d_u, (size_t)batch * N * nu * es) == hipSuccess &&
              hipMalloc((void **)&h->d_status, (size_t)batch * sizeof(int)) == hipSuccess &&
              hipMalloc((void **)&h->d_iters, (size_t)batch * sizeof(int)) == hipSuccess &&
              hipMalloc(&h->d_scratch, scratch_bytes) == hipSuccess;
    if (!ok) {
        h->fail(NMPC_ENOMEM, "nmpc_create: device allocation failed");
        free_all(h);
        delete h;
        return NMPC_ENOMEM;
    }
    // model upload
    std::vector<double> AB((size_t)nx * nz);
    for (int r = 0; r < nx; r++) {
        for (int q = 0; q < nx; q++) AB[r * nz + q] = h->A[r * nx + q];
        for (int q = 0; q < nu; q++) AB[r * nz + nx + q] = h->B[r * nu + q];
    }
    std::vector<double> ABt((size_t)nx * nz);
    for (int r = 0; r < nx; r++)
        for (int q = 0; q < nz; q++) ABt[q * nx + r] = AB[r * nz + q];
    char *dm = (char *)h->d_model;
    auto put_at = [&](char *base, size_t o, const std::vector<double> &v) {
        if (f64) {
            hipMemcpy(base + o, v.data(), v.size() * sizeof(double), hipMemcpyHostToDevice);
        } else {
            std::vector<float> t(v.begin(), v.end());
            hipMemcpy(base + o, t.data(), t.size() * sizeof(float), hipMemcpyHostToDevice);
        }
    };
    auto put = [&](size_t o, const std::vector<double> &v) { put_at(dm, o, v); };
    put(h->off_AB, AB);
    put(h->off_ABt, ABt);
    put(h->off_c, h->c);
    put(h->off_H, h->H);
    put(h->off_He, h->He);
    put(h->off_G, h->G);
    put(h->off_Ge, h->Ge);
    put(h->off_lb, h->lbnd);
    put(h->off_ub, h->ubnd);
    if (lqr_on) {
        std::vector<double> &lqr = h->lqr_host, lqrf;
        lqr_table(nx, nu, N, h->A, h->B, h->c, h->H, h->He, lqr, lqrf);
        if (lqr_dev) {
            put(h->off_lqr, lqr);
            put(h->off_lqrf, lqrf);
            std::vector<double> wm;
            lqr_wmat(nx, nu, N, h->A, h->B, lqr, wm);
            put(h->off_lqrw, wm);
        }
    }
    if (h->cond) {
        const nmpc::CondHost &c = h->ch;
        const std::vector<double> *parts[15] = {&c.Gx, &c.H0, &c.H0t, &c.Fx, &c.Fy, &c.fc, &c.Phx, &c.dx, &c.lox,
                                                &c.hix, &c.lou, &c.hiu, &c.Gall, &c.Phall, &c.dall};
        size_t tot = 0;
        for (int i = 0; i < 15; i++) {
            h->co[i] = tot;
            tot += (parts[i]->size() + 63) & ~(size_t)63;
        }
        const std::vector<int> *iparts[3] = {&c.xcols, &c.rstart, &c.ks};
        size_t itot = 0;
        for (int i = 0; i < 3; i++) {
            h->ci[i] = itot;
            itot += (iparts[i]->size() + 63) & ~(size_t)63;
        }
        if (hipMalloc(&h->d_cond, tot * es) != hipSuccess || hipMalloc((void **)&h->d_cond_i, itot * sizeof(int)) != hipSuccess) {
            h->fail(NMPC_ENOMEM, "nmpc_create: device allocation failed (condensed data)");
            free_all(h);
            delete h;
            return NMPC_ENOMEM;
        }
        char *cb = (char *)h->d_cond;
        for (int i = 0; i < 15; i++) put_at(cb, h->co[i] * es, *parts[i]);
        for (int i = 0; i < 3; i++)
            hipMemcpy(h->d_cond_i + h->ci[i], iparts[i]->data(), iparts[i]->size() * sizeof(int), hipMemcpyHostToDevice);
    }
    if ((e = hipDeviceSynchronize()) != hipSuccess) {
        int r = hip_fail(h, e, "model upload");
        free_all(h);
        delete h;
        return r;
    }
    {
        const int r = f64 ? sf_setup(h) : fin32_setup(h);
        if (r < 0) {
            g_err = h->err;
            free_all(h);
            delete h;
            return r;
        }
    }
    *out = h;
    return 0;
}

void nmpc_destroy(nmpc_solver *h)
{
    if (!h) return;
    free_all(h);
    delete h;
}

int nmpc_set_stream(nmpc_solver *h, void *s)
{
    if (!h) return NMPC_EINVAL;
    h->stream = s ? (hipStream_t)s : h->own_stream;
    return 0;
}

void *nmpc_get_stream(nmpc_solver *h) { return h ? (void *)h->stream : nullptr; }

int nmpc_get_model(const nmpc_solver *h, double *A, double *B, double *c)
{
    if (!h) return NMPC_EINVAL;
    if (A) std::memcpy(A, h->A.data(), h->A.size() * sizeof(double));
    if (B) std::memcpy(B, h->B.data(), h->B.size() * sizeof(double));
    if (c) std::memcpy(c, h->c.data(), h->c.size() * sizeof(double));
    return 0;
}

int nmpc_set(nmpc_solver *h, int inst, int stage, const char *field, const double *v, int n)
{
    if (!h || !field || !v) return NMPC_EINVAL;
    if (inst < -1 || inst >= h->batch) return h->fail(NMPC_EINVAL, "nmpc_set: instance out of range");
    const int b0 = inst < 0 ? 0 : inst, b1 = inst < 0 ? h->batch : inst + 1;
    if (field_is(field, "yref")) {
        if (stage < 0 || stage > h->N) return h->fail(NMPC_EINVAL, "nmpc_set: stage out of range");
        const int want = stage < h->N ? h->ny : h->ny_e;
        if (n != want)
            return h->fail(NMPC_EINVAL, "nmpc_set: yref at stage " + std::to_string(stage) + " needs " +
                                            std::to_string(want) + " values, got " + std::to_string(n));
        for (int b = b0; b < b1; b++)
            std::memcpy(&h->h_yref[b * h->ystride() + (size_t)stage * h->ny], v, n * sizeof(double));
        h->yref_dirty = true;
        return 0;
    }
    if (field_is(field, "lbx") || field_is(field, "ubx") || field_is(field, "x0")) {
        if (!field_is(field, "x0") && stage != 0)
            return h->fail(NMPC_EUNSUPPORTED,
                           "nmpc_set: state bounds can only be set at stage 0 (x0 pinning); stage " +
                               std::to_string(stage) + " bounds are part of the model");
        if (n != h->nx) return h->fail(NMPC_EINVAL, "nmpc_set: lbx/ubx/x0 need nx values");
        for (int b = b0; b < b1; b++) {
            if (!field_is(field, "ubx")) std::memcpy(&h->h_lbx0[(size_t)b * h->nx], v, n * sizeof(double));
            if (!field_is(field, "lbx")) std::memcpy(&h->h_ubx0[(size_t)b * h->nx], v, n * sizeof(double));
        }
        h->x0_dirty = true;
        return 0;
    }
    return h->fail(NMPC_EINVAL, std::string("nmpc_set: unknown field '") + field + "'");
}

int nmpc_get(nmpc_solver *h, int inst, int stage, const char *field, double *out, int n)
{
    if (!h || !field || !out) return NMPC_EINVAL;
    if (inst < 0 || inst >= h->batch) return h->fail(NMPC_EINVAL, "nmpc_get: instance out of range");
    if (!h->out_valid) return h->fail(NMPC_ESTATE, "nmpc_get: no solution available (call nmpc_solve first)");
    if (field_is(field, "x")) {
        if (stage < 0 || stage > h->N || n != h->nx) return h->fail(NMPC_EINVAL, "nmpc_get: bad stage/size for x");
        std::memcpy(out, &h->h_x[((size_t)inst * (h->N + 1) + stage) * h->nx], n * sizeof(double));
        return 0;
    }
    if (field_is(field, "u")) {
        if (stage < 0 || stage >= h->N || n != h->nu) return h->fail(NMPC_EINVAL, "nmpc_get: bad stage/size for u");
        std::memcpy(out, &h->h_u[((size_t)inst * h->N + stage) * h->nu], n * sizeof(double));
        return 0;
    }
    return h->fail(NMPC_EINVAL, std::string("nmpc_get: unknown field '") + field + "'");
}

int nmpc_set_batch(nmpc_solver *h, const char *field, const double *v, size_t count)
{
    if (!h || !field || !v) return NMPC_EINVAL;
    if (field_is(field, "x0")) {
        if (count != h->h_x0.size()) return h->fail(NMPC_EINVAL, "nmpc_set_batch: x0 needs batch*nx values");
        std::memcpy(h->h_lbx0.data(), v, count * sizeof(double));
        std::memcpy(h->h_ubx0.data(), v, count * sizeof(double));
        h->x0_dirty = true;
        return 0;
    }
    if (field_is(field, "yref")) {
        if (count != h->h_yref.size())
            return h->fail(NMPC_EINVAL, "nmpc_set_batch: yref needs batch*(N*ny+ny_e) values");
        std::memcpy(h->h_yref.data(), v, count * sizeof(double));
        h->yref_dirty = true;
        return 0;
    }
    return h->fail(NMPC_EINVAL, std::string("nmpc_set_batch: unknown field '") + field + "'");
}

int nmpc_get_batch(nmpc_solver *h, const char *field, double *out, size_t count)
{
    if (!h || !field || !out) return NMPC_EINVAL;
    if (!h->out_valid) return h->fail(NMPC_ESTATE, "nmpc_get_batch: no solution available");
    const std::vector<double> *src = field_is(field, "x") ? &h->h_x : field_is(field, "u") ? &h->h_u : nullptr;
    if (!src) return h->fail(NMPC_EINVAL, std::string("nmpc_get_batch: unknown field '") + field + "'");
    if (count != src->size()) return h->fail(NMPC_EINVAL, "nmpc_get_batch: size mismatch");
    std::memcpy(out, src->data(), count * sizeof(double));
    return 0;
}

int nmpc_get_batch_int(nmpc_solver *h, const char *field, int32_t *out, size_t count)
{
    if (!h || !field || !out) return NMPC_EINVAL;
    if (!h->out_valid) return h->fail(NMPC_ESTATE, "nmpc_get_batch_int: no solution available");
    const std::vector<int32_t> *src =
        field_is(field, "status") ? &h->h_status : field_is(field, "qp_iter") ? &h->h_iters : nullptr;
    if (!src) return h->fail(NMPC_EINVAL, std::string("nmpc_get_batch_int: unknown field '") + field + "'");
    if (count != src->size()) return h->fail(NMPC_EINVAL, "nmpc_get_batch_int: size mismatch");
    std::memcpy(out, src->data(), count * sizeof(int32_t));
    return 0;
}

int nmpc_device_ptr(nmpc_solver *h, const char *field, void **out)
{
    if (!h || !field || !out) return NMPC_EINVAL;
    if (field_is(field, "x0")) *out = h->d_x0;
    else if (field_is(field, "yref")) *out = h->d_yref;
    else if (field_is(field, "x")) *out = h->d_x;
    else if (field_is(field, "u")) *out = h->d_u;
    else if (field_is(field, "status")) *out = h->d_status;
    else if (field_is(field, "qp_iter")) *out = h->d_iters;
    else return h->fail(NMPC_EINVAL, std::string("nmpc_device_ptr: unknown field '") + field + "'");
    return 0;
}

int nmpc_solve_async(nmpc_solver *h)
{
    if (!h) return NMPC_EINVAL;
    hipSetDevice(h->device);
    h->out_valid = false;
    return h->precision == NMPC_FP64 ? launch<double>(h) : launch<float>(h);
}

// The host's wait for the handle's stream. hipStreamSynchronize parks the thread once its short active wait has
// passed and wakes ~10-20 µs after the work ends (the bench timeline, rocprofv3 API trace: 22 µs from the lean
// kernel's end to the return); a closed-loop controller waits on the critical path every step, so the wait
// polls the stream instead (hipStreamQuery until done: one core busy for the kernel's duration). Env
// NMPC_SPIN_WAIT=0: hipStreamSynchronize.
hipError_t stream_wait(hipStream_t s)
{
    static const bool spin = !(std::getenv("NMPC_SPIN_WAIT") && std::getenv("NMPC_SPIN_WAIT")[0] == '0');
    if (!spin) return hipStreamSynchronize(s);
    hipError_t e;
    while ((e = hipStreamQuery(s)) == hipErrorNotReady) {
    }
    (void)hipGetLastError();   // (the polls' not-ready status is not a launch error)
    return e;
}

int nmpc_synchronize(nmpc_solver *h)
{
    if (!h) return NMPC_EINVAL;
    hipError_t e = stream_wait(h->stream);
    if (e != hipSuccess) return hip_fail(h, e, "hipStreamSynchronize");
    const int r = sf_resolve(h);   // the last fast solve's listed / parked counts (its kernels are done)
    if (r < 0) return r;
    if ((e = hipEventElapsedTime(&h->last_ms, h->ev0, h->ev1)) != hipSuccess) return hip_fail(h, e, "solve timing events");
    return 0;
}

// the device trajectories, status and qp_iter of the last solve (or the lean closed loop's last step) to the
// host copies nmpc_get / nmpc_get_batch read; waits for the handle's stream
static int download_outputs(nmpc_solver *h)
{
    hipError_t e;
    const size_t nxo = h->h_x.size(), nuo = h->h_u.size();
    if (h->precision == NMPC_FP64) {
        hipMemcpyAsync(h->h_x.data(), h->d_x, nxo * sizeof(double), hipMemcpyDeviceToHost, h->stream);
        hipMemcpyAsync(h->h_u.data(), h->d_u, nuo * sizeof(double), hipMemcpyDeviceToHost, h->stream);
    }
    std::vector<float> fx, fu;
    if (h->precision == NMPC_FP32) {
        fx.resize(nxo);
        fu.resize(nuo);
        hipMemcpyAsync(fx.data(), h->d_x, nxo * sizeof(float), hipMemcpyDeviceToHost, h->stream);
        hipMemcpyAsync(fu.data(), h->d_u, nuo * sizeof(float), hipMemcpyDeviceToHost, h->stream);
    }
    hipMemcpyAsync(h->h_status.data(), h->d_status, h->batch * sizeof(int), hipMemcpyDeviceToHost, h->stream);
    hipMemcpyAsync(h->h_iters.data(), h->d_iters, h->batch * sizeof(int), hipMemcpyDeviceToHost, h->stream);
    if ((e = stream_wait(h->stream)) != hipSuccess) return hip_fail(h, e, "solve");
    if (h->precision == NMPC_FP32) {
        for (size_t i = 0; i < nxo; i++) h->h_x[i] = fx[i];
        for (size_t i = 0; i < nuo; i++) h->h_u[i] = fu[i];
    }
    h->out_valid = true;
    return 0;
}

int nmpc_solve(nmpc_solver *h)
{
    if (!h) return NMPC_EINVAL;
    hipSetDevice(h->device);
    hipError_t e;
    if (h->x0_dirty) {
        for (size_t i = 0; i < h->h_lbx0.size(); i++)
            if (h->h_lbx0[i] != h->h_ubx0[i])
                return h->fail(NMPC_EUNSUPPORTED,
                               "nmpc_solve: stage-0 lbx != ubx for instance " + std::to_string(i / h->nx) +
                                   " (the engine pins x0 = lbx = ubx, as the reference does)");
        h->h_x0 = h->h_lbx0;
        e = upload_any(h->d_x0, h->h_x0.data(), h->h_x0.size(), h->precision == NMPC_FP64, h->stream, h->tmp_x0f);
        if (e != hipSuccess) return hip_fail(h, e, "upload x0");
        h->x0_dirty = false;
    }
    if (h->yref_dirty) {
        e = upload_any(h->d_yref, h->h_yref.data(), h->h_yref.size(), h->precision == NMPC_FP64, h->stream,
                       h->tmp_yf);
        if (e != hipSuccess) return hip_fail(h, e, "upload yref");
        h->yref_dirty = false;
    }
    int r = h->precision == NMPC_FP64 ? launch<double>(h) : launch<float>(h);
    if (r < 0) return r;
    if ((r = download_outputs(h)) < 0) return r;   // waits for the stream
    if ((r = sf_resolve(h)) < 0) return r;         // fast solve: its listed / parked counts
    h->out_from_loop = false;
    if ((e = hipEventElapsedTime(&h->last_ms, h->ev0, h->ev1)) != hipSuccess) return hip_fail(h, e, "solve timing events");
    int st = 0;
    for (int b = 0; b < h->batch; b++) st = std::max(st, (int)h->h_status[b]);
    return st;
}

int nmpc_get_cost(nmpc_solver *h, int inst, double *cost)
{
    if (!h || !cost) return NMPC_EINVAL;
    if (inst < 0 || inst >= h->batch) return h->fail(NMPC_EINVAL, "nmpc_get_cost: instance out of range");
    if (!h->out_valid) return h->fail(NMPC_ESTATE, "nmpc_get_cost: no solution available");
    if (h->out_from_loop)   // the loop's windows come from its reference table, not from the host-staged yref
        return h->fail(NMPC_ESTATE, "nmpc_get_cost: the outputs are a closed-loop step's (nmpc_closed_loop_stats has its cost)");
    const int nx = h->nx, nu = h->nu, N = h->N, ny = h->ny, ny_e = h->ny_e;
    const double sc = h->cost_s;
    const double *X = &h->h_x[(size_t)inst * (N + 1) * nx];
    const double *U = &h->h_u[(size_t)inst * N * nu];
    const double *Y = &h->h_yref[(size_t)inst * h->ystride()];
    double total = 0.0;
    std::vector<double> r(std::max(ny, ny_e));
    for (int k = 0; k < N; k++) {
        for (int i = 0; i < ny; i++) {
            double y = -Y[(size_t)k * ny + i];
            for (int q = 0; q < nx; q++) y += h->Vx[i * nx + q] * X[k * nx + q];
            for (int q = 0; q < nu; q++) y += h->Vu[i * nu + q] * U[k * nu + q];
            r[i] = y;
        }
        double acc = 0.0;
        for (int i = 0; i < ny; i++)
            for (int j = 0; j < ny; j++) acc += r[i] * h->W[i * ny + j] * r[j];
        total += 0.5 * sc * acc;
    }
    if (ny_e > 0) {
        for (int i = 0; i < ny_e; i++) {
            double y = -Y[(size_t)N * ny + i];
            for (int q = 0; q < nx; q++) y += h->Vx_e[i * nx + q] * X[N * nx + q];
            r[i] = y;
        }
        double acc = 0.0;
        for (int i = 0; i < ny_e; i++)
            for (int j = 0; j < ny_e; j++) acc += r[i] * h->W_e[i * ny_e + j] * r[j];
        total += 0.5 * acc;
    }
    *cost = total;
    return 0;
}

int nmpc_get_stats(nmpc_solver *h, double *st, int n)
{
    if (!h || !st || n < 1) return NMPC_EINVAL;
    double mx = 0, mean = 0, nf = 0;
    for (int b = 0; b < h->batch; b++) {
        mx = std::max(mx, (double)h->h_iters[b]);
        mean += h->h_iters[b];
        nf += h->h_status[b] != 0;
    }
    const double v[7] = {mx, mean / h->batch, nf, (double)h->last_ms, 1.0, (double)h->sf_listed, (double)h->sf_parked};
    for (int i = 0; i < n && i < 7; i++) st[i] = v[i];
    return 0;
}

int nmpc_get_launch_info(const nmpc_solver *h, int *out, int n)
{
    if (!h || !out) return NMPC_EINVAL;
    const int waves = (h->batch + h->ipw - 1) / h->ipw;
    const bool f64 = h->precision == NMPC_FP64;
    const int kind = h->cond ? 2 : f64 ? nmpc::ipm_kind<double>(h->kidx) : nmpc::ipm_kind<float>(h->kidx);
    const int sid = h->cond ? 0 : f64 ? nmpc::ipm_structure<double>(h->kidx) : nmpc::ipm_structure<float>(h->kidx);
    const int v[9] = {h->ipw, (waves + h->wpb - 1) / h->wpb, 64 * h->wpb, h->lds, kind, sid, h->clf ? (h->clf_kind == nmpc::CLF_LOCK ? 2 : 1) : 0,
                      h->clf ? nmpc::cl_fast_wsmax(h->nx, h->nu) : 0, h->sfast ? 1 : 0};
    for (int i = 0; i < n && i < 9; i++) out[i] = v[i];
    return 0;
}

int nmpc_sim_plant(int device, int batch, int num_stages, double T, double mass, double g, const double *x_in,
                   const double *u, double *x_out)
{
    if (batch < 1 || !x_in || !u || !x_out || (num_stages != 1 && num_stages != 4)) {
        g_err = "nmpc_sim_plant: invalid arguments (num_stages must be 1 or 4)";
        return NMPC_EINVAL;
    }
    if (hipSetDevice(device) != hipSuccess) {
        g_err = "nmpc_sim_plant: no HIP device";
        return NMPC_EDEVICE;
    }
    double *d = nullptr;
    if (hipMalloc(&d, sizeof(double) * (size_t)batch * 10) != hipSuccess) {
        g_err = "nmpc_sim_plant: allocation failed";
        return NMPC_ENOMEM;
    }
    hipMemcpy(d, x_in, sizeof(double) * batch * 4, hipMemcpyHostToDevice);
    hipMemcpy(d + batch * 4, u, sizeof(double) * batch * 2, hipMemcpyHostToDevice);
    hipError_t e = nmpc::plant_step_launch(batch, num_stages, T, mass, g, d, d + batch * 4, d + batch * 6, 0);
    if (e == hipSuccess) e = hipMemcpy(x_out, d + batch * 6, sizeof(double) * batch * 4, hipMemcpyDeviceToHost);
    hipFree(d);
    if (e != hipSuccess) {
        g_err = std::string("nmpc_sim_plant: ") + hipGetErrorString(e);
        return NMPC_EDEVICE;
    }
    return 0;
}

}  // extern "C"

namespace {

template <typename T>
nmpc::ClParams<T> cl_params(nmpc_solver *h)
{
    // (declared above launch)
    nmpc::ClParams<T> p{};
    const nmpc_closed_loop_desc &d = h->cl;
    p.B = h->batch;
    p.N = h->N;
    p.ny = h->ny;
    p.ny_e = h->ny_e;
    p.nx = h->nx;
    p.nu = h->nu;
    p.plant = d.plant;
    p.period = d.ref_period;
    p.table_cols = d.ref_cols;
    p.step = h->cl_step;
    p.cost_stage = d.cost_stage;
    p.ncl = d.ncl;
    p.aed_dims = d.aed_dims;
    p.noise_dims = d.noise_dims;
    p.substeps = d.substeps;
    p.inst_base = d.instance_base;
    p.seed = d.seed;
    p.noise_std = d.noise_std;
    p.mass = d.mass;
    p.g = d.g;
    p.dt = d.dt;
    p.dt_conv = d.dt_conv;
    p.table = (const T *)h->d_table;
    p.offset = h->d_offsets;
    p.state = (T *)h->d_state;
    p.x0 = (T *)h->d_x0;
    p.yref = (T *)h->d_yref;
    p.xout = (const T *)h->d_x;
    p.uout = (const T *)h->d_u;
    p.status = h->d_status;
    const T *pm = (const T *)h->d_plant;
    p.A = pm;
    p.Bm = pm + h->nx * h->nx;
    p.c = pm + h->nx * h->nx + h->nx * h->nu;
    p.wcl = (const T *)h->d_wcl;
    p.noise_table = h->d_noise;
    p.noise_len = d.noise_len;
    p.acc = h->d_acc;
    return p;
}

// fused closed loop: the kernel families that run the steps inside the solve kernel
bool cl_fused(nmpc_solver *h)
{
    const char *env = std::getenv("NMPC_CL_FUSED");
    if (env && env[0] == '0') return false;
    if (h->cond) return false;
    const int kind = h->precision == NMPC_FP64 ? nmpc::ipm_kind<double>(h->kidx) : nmpc::ipm_kind<float>(h->kidx);
    return kind == 0 || kind == 1;
}

template <typename T>
int cl_fused_enqueue(nmpc_solver *h, int launch_idx, int n)
{
    nmpc::ClParams<T> p = cl_params<T>(h);
    hipError_t e = nmpc::cl_noise_launch<T>(p, h->cl_step, n, h->d_fnoise, h->stream);
    if (e != hipSuccess) return hip_fail(h, e, "closed-loop noise");
    const int r = launch<T>(h, h->cl_events[2 * launch_idx], h->cl_events[2 * launch_idx + 1], n);
    if (r < 0) return r;
    h->cl_step += n;
    return 0;
}

template <typename T>
int cl_step_enqueue(nmpc_solver *h, int launch_idx)
{
    nmpc::ClParams<T> p = cl_params<T>(h);
    hipError_t e = nmpc::cl_prepare_launch<T>(p, h->stream);
    if (e != hipSuccess) return hip_fail(h, e, "closed-loop prepare");
    const int r = launch<T>(h, h->cl_events[2 * launch_idx], h->cl_events[2 * launch_idx + 1]);
    if (r < 0) return r;
    e = nmpc::cl_advance_launch<T>(p, h->stream);
    if (e != hipSuccess) return hip_fail(h, e, "closed-loop advance");
    h->cl_step++;
    return 0;
}

hipError_t put_typed(void *dst, const double *src, size_t n, bool f64)
{
    if (f64) return hipMemcpy(dst, src, n * sizeof(double), hipMemcpyHostToDevice);
    std::vector<float> t(src, src + n);
    return hipMemcpy(dst, t.data(), n * sizeof(float), hipMemcpyHostToDevice);
}

// The lean loop's slot layout: the bounded elements of z in stage-major order (stage 0's inputs first; x_0
// and stage N's inputs are not elements of the QP's decision), their bounds, and the unbounded decision
// elements. false: a stage-0 input without both bounds (the failure output needs mid-box inputs).
bool slot_layout(const nmpc_solver *h, std::vector<int> &el, std::vector<int> &fr, std::vector<double> &lb,
                 std::vector<double> &ub, std::vector<double> &uinit)
{
    const int nx = h->nx, nu = h->nu, nz = nx + nu, N = h->N;
    el.clear();
    fr.clear();
    lb.clear();
    ub.clear();
    for (int k = 0; k <= N; k++)
        for (int r = 0; r < nz; r++) {
            if ((k == 0 && r < nx) || (k == N && r >= nx)) continue;
            const int ty = k == 0 ? 0 : (k == N ? 2 : 1);
            const double l = h->lbnd[ty * nz + r], u_ = h->ubnd[ty * nz + r];
            if (!has_bound(l) && !has_bound(u_)) {
                fr.push_back(k * nz + r);
                continue;
            }
            el.push_back(k * nz + r);
            lb.push_back(l);
            ub.push_back(u_);
        }
    uinit.assign(nu, 0.0);
    for (int i = 0; i < nu; i++) {
        if ((int)el.size() <= i || el[i] != nx + i) return false;
        const double l = h->lbnd[nx + i], u_ = h->ubnd[nx + i];
        if (!has_bound(l) || !has_bound(u_)) return false;
        uinit[i] = 0.5 * (l + u_);
    }
    return true;
}

// fp32 handles: the lean machinery's W in fp64 (an ill-conditioned set's multipliers amplify W's rounding
// by cond(W_SS), ~4e4 for force), shared by the solve finish and the lean closed loop
int ensure_w64(nmpc_solver *h)
{
    if (h->d_clw) return 0;
    std::vector<double> wm;
    lqr_wmat(h->nx, h->nu, h->N, h->A, h->B, h->lqr_host, wm);
    if (hipMalloc((void **)&h->d_clw, wm.size() * sizeof(double)) != hipSuccess)
        return h->fail(NMPC_ENOMEM, "fp64 W table");
    const hipError_t e = hipMemcpy(h->d_clw, wm.data(), wm.size() * sizeof(double), hipMemcpyHostToDevice);
    return e == hipSuccess ? 0 : hip_fail(h, e, "fp64 W table upload");
}

// The exact finish of fp32 solves (nmpc_cl_fast.hip fin32_*): for the lean loop's shapes with diagonal
// costs (env NMPC_FIN32=0: off). M = [T_x | V_y] and vc, the unconstrained solution's response to x0, to
// each reference component (stage-stacked as h_yref) and to c, by unconstrained Riccati solves on the host.
int fin32_setup(nmpc_solver *h)
{
    const char *env = std::getenv("NMPC_FIN32");
    const int nx = h->nx, nu = h->nu, nz = nx + nu, N = h->N, ne = (N + 1) * nz;
    if ((env && env[0] == '0') || h->cond || !h->g_diag || h->lqr_host.empty()) return 0;
    std::vector<int> el, fr;
    std::vector<double> lb, ub, uinit;
    if (!slot_layout(h, el, fr, lb, ub, uinit) || nmpc::fin32_resident(nx, nu, (int)el.size(), h->device) <= 0) return 0;
    const int ny = h->ny, nye = h->ny_e, ys = (int)h->ystride(), K = nx + ys;
    const int m16 = (ne + 15) / 16 * 16, kp = (K + 3) / 4 * 4;
    std::vector<double> M((size_t)m16 * kp, 0.0), vc(m16, 0.0), g(ne, 0.0), z(ne), e0(nx, 0.0);
    for (int j = 0; j < nx; j++) {   // T_x
        std::fill(e0.begin(), e0.end(), 0.0);
        e0[j] = 1.0;
        lqr_solve(nx, nu, N, h->A, h->B, h->c, h->lqr_host, g.data(), e0.data(), false, z.data());
        for (int e = 0; e < ne; e++) M[(size_t)e * kp + j] = z[e];
    }
    std::fill(e0.begin(), e0.end(), 0.0);
    for (int q = 0; q < ys; q++) {   // V_y: reference component q of the stage-stacked yref
        const int k = q < N * ny ? q / ny : N, c_ = q < N * ny ? q % ny : q - N * ny;
        const int n = k < N ? nz : nx, m = k < N ? ny : nye;
        const double *Gm = k < N ? h->G.data() : h->Ge.data();
        std::fill(g.begin(), g.end(), 0.0);
        for (int i = 0; i < n; i++) g[(size_t)k * nz + i] = Gm[i * m + c_];
        lqr_solve(nx, nu, N, h->A, h->B, h->c, h->lqr_host, g.data(), e0.data(), false, z.data());
        for (int e = 0; e < ne; e++) M[(size_t)e * kp + nx + q] = z[e];
    }
    std::fill(g.begin(), g.end(), 0.0);   // vc: the response to c
    lqr_solve(nx, nu, N, h->A, h->B, h->c, h->lqr_host, g.data(), e0.data(), true, z.data());
    for (int e = 0; e < ne; e++) vc[e] = z[e];
    const std::vector<double> *parts[5] = {&lb, &ub, &uinit, &M, &vc};
    size_t tot = 0;
    for (int i = 0; i < 5; i++) {
        h->fino[i] = tot;
        tot += (parts[i]->size() + 31) & ~(size_t)31;
    }
    const std::vector<int> *ip[2] = {&el, &fr};
    size_t itot = 0;
    for (int i = 0; i < 2; i++) {
        h->fini[i] = itot;
        itot += (ip[i]->size() + 63) & ~(size_t)63;
    }
    if (hipMalloc((void **)&h->d_fin_f, tot * sizeof(float)) != hipSuccess ||
        hipMalloc((void **)&h->d_fin_i, itot * sizeof(int)) != hipSuccess ||
        hipMalloc((void **)&h->d_z0, (size_t)h->batch * m16 * sizeof(float)) != hipSuccess)
        return h->fail(NMPC_ENOMEM, "nmpc_create: fp32 finish tables");
    hipError_t e = hipSuccess;
    for (int i = 0; i < 5 && e == hipSuccess; i++) e = put_typed(h->d_fin_f + h->fino[i], parts[i]->data(), parts[i]->size(), false);
    for (int i = 0; i < 2 && e == hipSuccess; i++)
        if (!ip[i]->empty()) e = hipMemcpy(h->d_fin_i + h->fini[i], ip[i]->data(), ip[i]->size() * sizeof(int), hipMemcpyHostToDevice);
    if (e != hipSuccess) return hip_fail(h, e, "nmpc_create: fp32 finish upload");
    const int r = ensure_w64(h);
    if (r < 0) return r;
    h->fin_resident = nmpc::fin32_resident(nx, nu, (int)el.size(), h->device);
    if (h->fin_resident <= 0) return 0;
    h->fin_m16 = m16;
    h->fin_kp = kp;
    h->fin_nslot = (int)el.size();
    h->fin_nfree = (int)fr.size();
    h->fin32 = true;
    return 0;
}

hipError_t fin32_enqueue(nmpc_solver *h)
{
    nmpc::Fin32Z0Params zp{};
    zp.B = h->batch;
    zp.nx = h->nx;
    zp.ystride = (int)h->ystride();
    zp.kp = h->fin_kp;
    zp.m16 = h->fin_m16;
    zp.M = h->d_fin_f + h->fino[3];
    zp.vc = h->d_fin_f + h->fino[4];
    zp.x0 = (const float *)h->d_x0;
    zp.yref = (const float *)h->d_yref;
    zp.z0 = h->d_z0;
    hipError_t e = nmpc::fin32_z0_launch(zp, h->stream);
    if (e != hipSuccess) return e;
    nmpc::ClFastParams<float> p{};
    const char *m = (const char *)h->d_model;
    p.B = h->batch;
    p.N = h->N;
    p.ne = (h->N + 1) * (h->nx + h->nu);
    p.nslot = h->fin_nslot;
    p.polish_steps = h->polish_steps;
    p.gi = 1;
    p.s_lb = h->d_fin_f + h->fino[0];
    p.s_ub = h->d_fin_f + h->fino[1];
    p.uinit = h->d_fin_f + h->fino[2];
    p.s_e = h->d_fin_i + h->fini[0];
    p.s_free = h->d_fin_i + h->fini[1];
    p.nfree = h->fin_nfree;
    p.W = h->d_clw;
    p.lbnd = (const float *)(m + h->off_lb);
    p.ubnd = (const float *)(m + h->off_ub);
    p.AB = (const float *)(m + h->off_AB);
    p.c = (const float *)(m + h->off_c);
    p.xout = (float *)h->d_x;
    p.uout = (float *)h->d_u;
    p.status = h->d_status;
    p.iters = h->d_iters;
    p.z0all = h->d_z0;
    p.z0_ld = h->fin_m16;
    p.x0in = (const float *)h->d_x0;
    if (!nmpc::fin32_launch(h->nx, h->nu, 0, p, h->fin_resident, h->stream)) return hipErrorInvalidValue;
    return hipGetLastError();
}

// The fp64 general solve on the shared factorisation (nmpc_solve_fast.hip sf_kernel, nmpc_cl_fast.hip
// fin64_kernel): for the compiled shapes with diagonal LINEAR_LS maps and the exact finish on (env
// NMPC_SOLVE_FAST=0: off, every solve runs the full IPM). Tables per stage k from the factorisation
// (lqr_table: K_k, F_uu,k^-1, P_{k+1}, P_{k+1} c): Acl_k' = (A + B K_k)', K_k', -F^-1 B', -F^-1, K_k,
// Acl_k' P_{k+1} c and -F^-1 B' P_{k+1} c, in sf::Tab's compact layout; the gradient diagonal; the slot tables
// of fin64_kernel (the lean loop's slot layout: bounded elements, bounds, unbounded elements, mid-box inputs).
int sf_setup(nmpc_solver *h)
{
    // (an explicit kernel family, env NMPC_KERNEL, selects that family's full solve as well)
    const char *env = std::getenv("NMPC_SOLVE_FAST");
    const int nx = h->nx, nu = h->nu, nz = nx + nu, N = h->N, W = lqr_words(nx, nu);
    const int ts = nmpc::sf_table_words(nx, nu);
    if ((env && env[0] == '0') || std::getenv("NMPC_KERNEL") || h->cond || !h->g_diag || h->lqr_host.empty() || ts <= 0 ||
        nmpc::sf_lds_bytes(nx, nu, N) > 160 * 1024)
        return 0;
    std::vector<int> el, fr;
    std::vector<double> lb, ub, uinit;
    if (!slot_layout(h, el, fr, lb, ub, uinit)) return 0;
    const int res = nmpc::fin64_resident(nx, nu, (int)el.size(), h->device);
    if (res <= 0) return 0;
    // the parked instances' full solves: the handle's kernel if it is of the lane-per-component family, else
    // that family's kernel with its own scratch
    int fk = h->kidx;
    if (nmpc::ipm_kind<double>(h->kidx) != 1) {
        fk = nmpc::ipm_find_family<double>(nx, nu, 1);
        if (fk < 0) return 0;
        std::vector<double> ABh((size_t)nx * nz);
        for (int r = 0; r < nx; r++) {
            for (int q = 0; q < nx; q++) ABh[r * nz + q] = h->A[r * nx + q];
            for (int q = 0; q < nu; q++) ABh[r * nz + nx + q] = h->B[r * nu + q];
        }
        fk = nmpc::ipm_refine<double>(fk, ABh.data(), h->H.data(), h->He.data());
    }
    const int bpg = nx <= 4 ? 1 : (nx <= 8 ? 2 : 4), R = 4 * bpg;
    const int o_aclt = 0, o_kt = o_aclt + bpg * R * 4, o_fibt = o_kt + R * 4, o_nfi = o_fibt + bpg * 16, o_kk = o_nfi + 16,
              o_cp = o_kk + bpg * 16, o_cf = o_cp + R;
    if (o_cf + 4 + 2 != ts) return h->fail(NMPC_EUNSUPPORTED, "sf_setup: table layout mismatch");   // + zero word, pad
    std::vector<double> tab((size_t)N * ts, 0.0), K((size_t)nu * nx), Fi((size_t)nu * nu), Pc(nx), Acl((size_t)nx * nx),
        FiBt((size_t)nu * nx);
    for (int k = 0; k < N; k++) {
        const double *t = &h->lqr_host[(size_t)k * nz * W];
        for (int r = 0; r < nx; r++) {
            for (int i = 0; i < nu; i++) K[i * nx + r] = t[r * W + nx + i];
            Pc[r] = t[r * W + nz];
        }
        for (int u = 0; u < nu; u++)
            for (int i = 0; i < nu; i++) Fi[u * nu + i] = t[(nx + u) * W + i];
        for (int i = 0; i < nx; i++)
            for (int j = 0; j < nx; j++) {
                double s_ = h->A[i * nx + j];
                for (int l = 0; l < nu; l++) s_ += h->B[i * nu + l] * K[l * nx + j];
                Acl[i * nx + j] = s_;
            }
        for (int i = 0; i < nu; i++)
            for (int j = 0; j < nx; j++) {
                double s_ = 0.0;
                for (int l = 0; l < nu; l++) s_ -= Fi[i * nu + l] * h->B[j * nu + l];
                FiBt[i * nx + j] = s_;
            }
        double *d = &tab[(size_t)k * ts];
        for (int kc = 0; kc < bpg; kc++)
            for (int row = 0; row < R; row++)
                for (int q = 0; q < 4; q++) {
                    const int col = 4 * kc + q;
                    d[o_aclt + (kc * R + row) * 4 + q] = (row < nx && col < nx) ? Acl[col * nx + row] : 0.0;
                }
        for (int row = 0; row < nx; row++)
            for (int q = 0; q < nu; q++) d[o_kt + row * 4 + q] = K[q * nx + row];
        for (int kc = 0; kc < bpg; kc++)
            for (int i = 0; i < nu; i++)
                for (int q = 0; q < 4; q++) {
                    const int col = 4 * kc + q;
                    if (col >= nx) continue;
                    d[o_fibt + (kc * 4 + i) * 4 + q] = FiBt[i * nx + col];
                    d[o_kk + (kc * 4 + i) * 4 + q] = K[i * nx + col];
                }
        for (int i = 0; i < nu; i++)
            for (int q = 0; q < nu; q++) d[o_nfi + i * 4 + q] = -Fi[i * nu + q];
        for (int row = 0; row < nx; row++) {
            double s_ = 0.0;
            for (int j = 0; j < nx; j++) s_ += Acl[j * nx + row] * Pc[j];
            d[o_cp + row] = s_;
        }
        for (int i = 0; i < nu; i++) {
            double s_ = 0.0;
            for (int j = 0; j < nx; j++) s_ += FiBt[i * nx + j] * Pc[j];
            d[o_cf + i] = s_;
        }
    }
    std::vector<double> gd(nz + nx, 0.0);
    for (int i = 0; i < nz; i++) gd[i] = h->G[i * h->ny + i];
    for (int i = 0; i < nx; i++) gd[nz + i] = h->Ge[i * h->ny_e + i];
    h->sf_gd = ((size_t)N * ts + 31) & ~(size_t)31;
    const std::vector<double> *fp[3] = {&lb, &ub, &uinit};
    size_t ftot = 0;
    for (int i = 0; i < 3; i++) {
        h->f64o[i] = ftot;
        ftot += (fp[i]->size() + 31) & ~(size_t)31;
    }
    const std::vector<int> *ipp[2] = {&el, &fr};
    size_t itot = 0;
    for (int i = 0; i < 2; i++) {
        h->f64i[i] = itot;
        itot += (ipp[i]->size() + 63) & ~(size_t)63;
    }
    const size_t sc = fk != h->kidx ? nmpc::ipm_scratch_elems<double>(fk, h->batch, N) * sizeof(double) : 0;
    if (hipMalloc((void **)&h->d_sf, (h->sf_gd + gd.size()) * sizeof(double)) != hipSuccess ||
        hipMalloc((void **)&h->d_f64, ftot * sizeof(double)) != hipSuccess ||
        hipMalloc((void **)&h->d_f64i, itot * sizeof(int)) != hipSuccess ||
        hipMalloc((void **)&h->d_sfl, (4 + 2 * (size_t)h->batch) * sizeof(int)) != hipSuccess ||
        (sc && hipMalloc(&h->d_sf_scratch, sc) != hipSuccess) ||
        hipHostMalloc((void **)&h->h_sfpark, 4 * sizeof(int), hipHostMallocDefault) != hipSuccess ||
        hipEventCreate(&h->ev_fb) != hipSuccess)
        return h->fail(NMPC_ENOMEM, "nmpc_create: fast-solve tables");
    hipError_t e = hipMemcpy(h->d_sf, tab.data(), tab.size() * sizeof(double), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(h->d_sf + h->sf_gd, gd.data(), gd.size() * sizeof(double), hipMemcpyHostToDevice);
    for (int i = 0; i < 3 && e == hipSuccess; i++)
        if (!fp[i]->empty()) e = hipMemcpy(h->d_f64 + h->f64o[i], fp[i]->data(), fp[i]->size() * sizeof(double), hipMemcpyHostToDevice);
    for (int i = 0; i < 2 && e == hipSuccess; i++)
        if (!ipp[i]->empty()) e = hipMemcpy(h->d_f64i + h->f64i[i], ipp[i]->data(), ipp[i]->size() * sizeof(int), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemset(h->d_sfl, 0, 4 * sizeof(int));
    if (e != hipSuccess) return hip_fail(h, e, "nmpc_create: fast-solve upload");
    h->h_sfpark[0] = h->h_sfpark[1] = 0;
    h->f64_nslot = (int)el.size();
    h->f64_nfree = (int)fr.size();
    h->f64_resident = res;
    h->sf_kidx = fk;
    h->sfast = true;
    return 0;
}

// one fast solve on the handle's stream, complete in stream order: sf_kernel (every instance's unconstrained
// solution; the violated ones listed), fin64_kernel (active-set steps for the listed), the full IPM in list mode
// for what the finish parked — no host step between them, so kernels the caller enqueues behind the solve read
// final outputs. Timed from e0 (or ev0) to e1 (or ev1); the listed / parked counts follow to the pinned host words
int sf_enqueue(nmpc_solver *h, hipEvent_t e0, hipEvent_t e1)
{
    const int nx = h->nx, nu = h->nu, nz = nx + nu;
    const char *m = (const char *)h->d_model;
    nmpc::SfParams sp{};
    sp.B = h->batch;
    sp.N = h->N;
    sp.ny = h->ny;
    sp.ystride = (int)h->ystride();
    sp.tab = h->d_sf;
    sp.gd = h->d_sf + h->sf_gd;
    sp.AB = (const double *)(m + h->off_AB);
    sp.c = (const double *)(m + h->off_c);
    sp.lbnd = (const double *)(m + h->off_lb);
    sp.ubnd = (const double *)(m + h->off_ub);
    sp.x0 = (const double *)h->d_x0;
    sp.yref = (const double *)h->d_yref;
    sp.xout = (double *)h->d_x;
    sp.uout = (double *)h->d_u;
    sp.status = h->d_status;
    sp.iters = h->d_iters;
    const int pair = h->sf_pair ^ 1;   // this solve's counter pair (zeroed by the last solve's sf_kernel)
    int *cnt = h->d_sfl + 2 * pair;
    sp.list_count = cnt;
    sp.list = h->d_sfl + 4;
    nmpc::ClFastParams<double> p{};
    p.B = h->batch;
    p.N = h->N;
    p.ne = (h->N + 1) * nz;
    p.nslot = h->f64_nslot;
    p.polish_steps = h->polish_steps;
    // env NMPC_CLF_NO_GI=1 (test knob): no dual fallback, so unsettled instances park and take the full solve
    const char *nogi = std::getenv("NMPC_CLF_NO_GI");
    p.gi = (nogi && nogi[0] == '1') ? 0 : 1;
    p.s_lb = h->d_f64 + h->f64o[0];
    p.s_ub = h->d_f64 + h->f64o[1];
    p.uinit = h->d_f64 + h->f64o[2];
    p.s_e = h->d_f64i + h->f64i[0];
    p.s_free = h->d_f64i + h->f64i[1];
    p.nfree = h->f64_nfree;
    p.W = (const double *)(m + h->off_lqrw);
    p.lbnd = sp.lbnd;
    p.ubnd = sp.ubnd;
    p.AB = sp.AB;
    p.c = sp.c;
    p.xout = sp.xout;
    p.uout = sp.uout;
    p.status = h->d_status;
    p.iters = h->d_iters;
    p.park_count = cnt + 1;
    p.park_list = h->d_sfl + 4 + h->batch;
    p.x0in = sp.x0;
    p.work_list = sp.list;
    p.work_count = cnt;
    p.z0_xu = 1;
    sp.next_counts = h->d_sfl + 2 * (pair ^ 1);
    // env NMPC_SF_CYCLES=<file> with a timing build (-DNMPC_SF_TIMING): per-wavefront phase clocks of this launch,
    // appended to <file> at the next sf_resolve ([waves][8] uint64, tools/sf_phases.py)
    static const char *sf_cyc = std::getenv("NMPC_SF_CYCLES");
    if (sf_cyc && !h->d_sfcyc) {
        h->sfcyc_n = (size_t)(h->batch + 3) / 4 * 8 * 2;   // >= wavefronts x 8 for every shape (<= 4 instances per wave)
        if (hipMalloc((void **)&h->d_sfcyc, h->sfcyc_n * sizeof(unsigned long long)) != hipSuccess) h->d_sfcyc = nullptr;
    }
    sp.cycles = h->d_sfcyc;
    hipError_t e = hipEventRecord(e0 ? e0 : h->ev0, h->stream);
    if (e == hipSuccess) e = nmpc::sf_launch(nx, nu, sp, h->stream);
    if (e != hipSuccess) return hip_fail(h, e, "fast solve launch (sf_kernel)");
    // sf_kernel ran: it zeroed the other pair for the next solve, whatever happens below
    h->sf_pair = pair;
    // the finish of the listed instances, always enqueued: the list's length is read on the device, so the solve
    // is complete in stream order (an empty list: every workgroup returns at once)
    if ((e = nmpc::fin64_launch(nx, nu, p, h->f64_resident, h->stream)) != hipSuccess)
        return hip_fail(h, e, "fast solve launch (fin64_kernel)");
    // the instances the finish parked: the cold full IPM + exact finish in list mode, the park count read on the
    // device (grid sized for the whole batch; workgroups past the count return before any setup), timed from ev_fb
    ListArgs la{h->batch, 0, 0, h->d_sfl + 4 + h->batch, h->sf_kidx, h->d_sf_scratch};
    la.count_dev = cnt + 1;
    const int r = launch<double>(h, h->ev_fb, e1 ? e1 : h->ev1, 0, &la);
    if (r < 0) return r;
    // the counts behind the kernels, for nmpc_get_stats (read at the next wait)
    if ((e = hipMemcpyAsync(h->h_sfpark, cnt, 2 * sizeof(int), hipMemcpyDeviceToHost, h->stream)) != hipSuccess)
        return hip_fail(h, e, "fast solve counts");
    h->sf_pending = true;
    return 0;
}

// after the stream has drained: the last fast solve's listed / parked counts; timing builds dump sf_kernel's clocks
int sf_resolve(nmpc_solver *h)
{
    if (!h->sf_pending) return 0;
    h->sf_pending = false;
    h->sf_listed = h->h_sfpark[0];
    h->sf_parked = h->h_sfpark[1];
    if (h->d_sfcyc) {
        static const char *sf_cyc = std::getenv("NMPC_SF_CYCLES");
        std::vector<unsigned long long> cy(h->sfcyc_n);
        const hipError_t e = hipMemcpy(cy.data(), h->d_sfcyc, cy.size() * sizeof(cy[0]), hipMemcpyDeviceToHost);
        if (e != hipSuccess) return hip_fail(h, e, "sf_kernel clocks");
        if (FILE *f = std::fopen(sf_cyc, "ab")) {
            std::fwrite(cy.data(), sizeof(cy[0]), cy.size(), f);
            std::fclose(f);
        }
    }
    return 0;
}

// The lean closed loop (nmpc_cl_fast.hip) for this handle: fp64 with the exact finish, or fp32 (the tables
// and the explicit form in fp32, the set solves and the acceptance in fp64), a compiled slot layout for
// (nx, nu) (quad13, jerk, force: on by default; NMPC_CL_FAST=0 off). Its fallback is the
// lane-per-component kernel's list mode: a handle of the wavefront family (small models at small
// batches) gets that family's kernel and scratch as well.
// Slots: the bounded elements of z in stage-major order (stage 0's inputs first), their bounds,
// T_x rows, v_t columns and warm-start sources (the element one stage later; stage N - 1's inputs
// keep their own flag, as the fused kernel's mirror of stage N).
int clf_xcd_map(nmpc_solver *h, const nmpc_closed_loop_desc &d, int sid, bool f64);

int clf_setup(nmpc_solver *h, const nmpc_closed_loop_desc &d, const std::vector<double> &tx, const std::vector<double> &vv)
{
    const int nx = h->nx, nu = h->nu, nz = nx + nu, N = h->N, ne = (N + 1) * nz, P_ = d.ref_period;
    const char *env = std::getenv("NMPC_CL_FAST");
    const bool want = !env || env[0] != '0';
    const int epl = nmpc::cl_fast_epl(nx, nu);
    const bool f64 = h->precision == NMPC_FP64;
    const std::string fenv = std::getenv("NMPC_CL_FAST32") ? std::getenv("NMPC_CL_FAST32") : "1";
    if (!want || (f64 && !(h->polish_mu > 0)) || (!f64 && fenv == "0") || !h->g_diag || h->cond || epl <= 0)
        return 0;
    int fk = h->kidx;
    const int kind = f64 ? nmpc::ipm_kind<double>(h->kidx) : nmpc::ipm_kind<float>(h->kidx);
    if (kind != 1) {
        fk = f64 ? nmpc::ipm_find_family<double>(nx, nu, 1) : nmpc::ipm_find_family<float>(nx, nu, 1);
        if (fk < 0) return 0;
        std::vector<double> ABh((size_t)nx * nz);
        for (int r = 0; r < nx; r++) {
            for (int q = 0; q < nx; q++) ABh[r * nz + q] = h->A[r * nx + q];
            for (int q = 0; q < nu; q++) ABh[r * nz + nx + q] = h->B[r * nu + q];
        }
        fk = f64 ? nmpc::ipm_refine<double>(fk, ABh.data(), h->H.data(), h->He.data())
                 : nmpc::ipm_refine<float>(fk, ABh.data(), h->H.data(), h->He.data());
    }
    const int fsid = f64 ? nmpc::ipm_structure<double>(fk) : nmpc::ipm_structure<float>(fk);
    const size_t es = h->esz();
    std::vector<int> el, fr;
    std::vector<double> lb, ub, uinit;
    // stage 0's inputs are slots 0..nu-1 (u0 broadcast), every input box two-sided (failure output)
    if (!slot_layout(h, el, fr, lb, ub, uinit)) return 0;
    const int nslot = (int)el.size(), NS = epl * 64;
    if (nslot > NS) return 0;
    std::vector<int> eslot(ne, -1);
    for (int s = 0; s < nslot; s++) eslot[el[s]] = s;
    int x1slot = 0;
    if (d.cost_stage != 0) {   // x_1's cost components on consecutive slots of j = 0
        if (d.cost_stage != 1) return 0;
        x1slot = eslot[nz];
        for (int i = 0; i < d.ncl; i++)
            if (x1slot < 0 || eslot[nz + i] != x1slot + i || x1slot + i >= 64) return 0;
    }
    // warm-start source code per slot (nmpc_cl_fast.hip run_instance): (source slot + 1) | (end partner + 1) << 12 |
    // kind << 24. Source: the slot of the same component one stage later (the shift). Kind 1 / 2: a state slot of
    // stage N - 1 / N - 2 and its partner the same component's slot of stage N - 2 / N - 1 — a bound active at
    // N - 1 but not at N - 2 stays at N - 1 (oracle/c/riccati_ipm.c, closed loop mode 1)
    std::vector<int> src(nslot, 0);
    for (int s = 0; s < nslot; s++) {
        const int k = el[s] / nz, r = el[s] % nz;
        int ks = k < N ? k + 1 : k;
        if (k == N - 1 && r >= nx) ks = k;   // inputs of stage N mirror N - 1
        src[s] = eslot[ks * nz + r] + 1;
        if (r < nx && N >= 3 && (k == N - 1 || k == N - 2)) {
            const int ps = eslot[(k == N - 1 ? N - 2 : N - 1) * nz + r];
            if (ps >= 0) src[s] |= (ps + 1) << 12 | (k == N - 1 ? 1 : 2) << 24;
        }
    }
    if (NS > 4095) return 0;   // (the code's slot fields)
    std::vector<double> stx((size_t)nslot * nx), vb((size_t)P_ * NS, 0.0);
    for (int s = 0; s < nslot; s++)
        for (int c = 0; c < nx; c++) stx[(size_t)s * nx + c] = tx[(size_t)el[s] * nx + c];
    for (int t = 0; t < P_; t++)
        for (int s = 0; s < nslot; s++) vb[(size_t)t * NS + s] = vv[(size_t)t * ne + el[s]];
    // device blobs
    const std::vector<double> *parts[5] = {&lb, &ub, &stx, &vb, &uinit};
    size_t tot = 0;
    for (int i = 0; i < 5; i++) {
        h->fso[i] = tot;
        tot += (parts[i]->size() + 31) & ~(size_t)31;
    }
    const std::vector<int> *ip[4] = {&el, &src, &eslot, &fr};
    size_t itot = 0;
    for (int i = 0; i < 4; i++) {
        h->fsi[i] = itot;
        itot += (ip[i]->size() + 63) & ~(size_t)63;
    }
    for (void **q : {&h->d_fsT, (void **)&h->d_fsI, (void **)&h->d_istep, (void **)&h->d_park, (void **)&h->d_flags,
                     &h->d_clf_scratch})
        if (*q) {
            hipFree(*q);
            *q = nullptr;
        }
    bool ok = hipMalloc(&h->d_fsT, tot * es) == hipSuccess &&
              hipMalloc((void **)&h->d_fsI, itot * sizeof(int)) == hipSuccess &&
              hipMalloc((void **)&h->d_istep, (size_t)h->batch * sizeof(int)) == hipSuccess &&
              hipMalloc((void **)&h->d_park, (size_t)(h->batch + 2 + CLF_ROUND_WORDS + 1) * sizeof(int)) == hipSuccess &&
              hipMalloc((void **)&h->d_flags, (size_t)h->batch * (nslot + 1)) == hipSuccess;   // + the order bytes
    if (ok && fk != h->kidx)
        ok = hipMalloc(&h->d_clf_scratch, (f64 ? nmpc::ipm_scratch_elems<double>(fk, h->batch, N)
                                                : nmpc::ipm_scratch_elems<float>(fk, h->batch, N)) * es) == hipSuccess;
    if (!ok) return h->fail(NMPC_ENOMEM, "nmpc_closed_loop_init: lean closed-loop tables");
    // the park count and claim counter, and the fast kernels' exit counter (after the asynchronous rounds'
    // counters): 0 between launches (each host-driven launch's last wavefront rezeroes them, report_exit)
    if (hipMemset(h->d_park, 0, 2 * sizeof(int)) != hipSuccess ||
        hipMemset(h->d_park + h->batch + 2 + CLF_ROUND_WORDS, 0, sizeof(int)) != hipSuccess)
        return h->fail(NMPC_EDEVICE, "nmpc_closed_loop_init: counters");
    if (!f64) {
        const int r = ensure_w64(h);
        if (r < 0) return r;
    }
    hipError_t e = hipSuccess;
    for (int i = 0; i < 5 && e == hipSuccess; i++)
        e = put_typed((char *)h->d_fsT + h->fso[i] * es, parts[i]->data(), parts[i]->size(), f64);
    for (int i = 0; i < 4 && e == hipSuccess; i++)
        if (!ip[i]->empty())
            e = hipMemcpy(h->d_fsI + h->fsi[i], ip[i]->data(), ip[i]->size() * sizeof(int), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemset(h->d_istep, 0, (size_t)h->batch * sizeof(int));
    if (e == hipSuccess) e = hipMemset(h->d_flags, 0, (size_t)h->batch * (nslot + 1));
    if (e != hipSuccess) return hip_fail(h, e, "nmpc_closed_loop_init lean tables");
    // the lockstep kernel for the shapes that have one, with the controller-model plant and the cost on x_0
    // (env NMPC_CLF_LOCK=0: the one-instance-per-wavefront kernel)
    const char *lenv = std::getenv("NMPC_CLF_LOCK");
    // (the controller-model plant, or the jerk shape with its converter plant; the cost on x_0 or x_1). The jerk
    // shape's lockstep variant is opt-in (NMPC_CLF_LOCK=1): its 20 tiles of z and v_t spill 130 VGPRs at 2 waves
    // per SIMD and it measured 200-202M against cl_fast_kernel's 253M steps/s (jerk B = 4096, tools/ab_check.sh lk4)
    const bool jerk = nx == 6 && nu == 2;
    // (the cost on x_1, cost_stage 1, is gathered from the MFMA tiles by the jerk variant only: other shapes with
    // cost_stage 1 run cl_fast_kernel)
    const bool lock = f64 && nmpc::cl_lock_shape(nx, nu) && (d.cost_stage == 0 || (jerk && d.cost_stage == 1)) &&
                      (d.plant == NMPC_PLANT_MODEL || (jerk && d.plant == NMPC_PLANT_CRAZYFLIE_JERK)) &&
                      (jerk ? (lenv && lenv[0] == '1') : !(lenv && lenv[0] == '0'));
    // W over the slots in LDS for the shapes that have the variant, env NMPC_CLF_WLDS=1 (tuning; off by default:
    // force B = 1024 17.9M vs 19.0M, B = 8192 57.0M vs 80.5M steps/s — one workgroup per CU, and the rare
    // path's steps are bound by their instruction chains, not by W's L2 latency; tools/ab_check.sh, wl1)
    const char *wenv = std::getenv("NMPC_CLF_WLDS");
    const bool wlds = nmpc::cl_wlds_shape(nx, nu) && wenv && wenv[0] == '1';
    // a batch no larger than the device's SIMD count runs one wavefront per SIMD anyway: the variant compiled
    // for that (its rare path unrolled further) where the shape has one (env NMPC_CLF_ONE=0: off)
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, h->device);
    const char *oenv = std::getenv("NMPC_CLF_ONE");
    const bool one = nmpc::cl_one_shape(nx, nu) && cus > 0 && h->batch <= 4 * cus && !(oenv && oenv[0] == '0');
    h->clf_kind = lock ? nmpc::CLF_LOCK : (wlds ? nmpc::CLF_WLDS : (one ? nmpc::CLF_ONE : nmpc::CLF_FAST));
    // resident workgroups on this handle's device (nmpc_closed_loop_init runs on it: hipSetDevice above)
    h->clf_resident = nmpc::cl_fast_resident(nx, nu, fsid, h->clf_kind, f64, h->device);
    // the lockstep kernel's per-workgroup queue holds at most 512 demoted instances
    if (lock && h->clf_resident > 0 && (h->batch + h->clf_resident - 1) / h->clf_resident > 512) {
        h->clf_kind = nmpc::CLF_FAST;
        h->clf_resident = nmpc::cl_fast_resident(nx, nu, fsid, h->clf_kind, f64, h->device);
    }
    if (h->clf_resident <= 0) return h->fail(NMPC_EDEVICE, "nmpc_closed_loop_init: lean closed-loop occupancy query");
    {
        const int r = clf_xcd_map(h, d, fsid, f64);
        if (r < 0) return r;
    }
    h->clf = true;
    h->clf_nslot = nslot;
    h->clf_nfree = (int)fr.size();
    h->clf_epl = epl;
    h->clf_x1slot = x1slot;
    h->clf_sid = fsid;
    h->clf_kidx = fk;
    return 0;
}

// XCD-aware instance placement for the lean loop's per-workgroup claim ranges. The hardware hands workgroup w to XCD
// w % 8, and each XCD has its own L2; an instance reads the v_t row of its reference-table row every step (offset +
// step, shared table). With instances in index order every XCD's L2 pulls the whole v_t table (period x slots: 1 MB
// quad13, 1.28 MB jerk) each launch. The map sorts the instances by start row and gives each XCD's workgroups one
// contiguous stretch of rows, so an XCD reads about an eighth of the table (+ the launch's steps). Results do not
// depend on it (instances are independent; every per-instance record stays indexed by the instance); env
// NMPC_CLF_XCD=0: index order. Not with the device-wide claim (the force shape): its positions go to any workgroup.
int clf_xcd_map(nmpc_solver *h, const nmpc_closed_loop_desc &d, int sid, bool f64)
{
    if (h->d_imap) {
        hipFree(h->d_imap);
        h->d_imap = nullptr;
    }
    const char *env = std::getenv("NMPC_CLF_XCD");
    if (env && env[0] == '0') return 0;
    const int B = h->batch, X = 8;
    const int G = nmpc::cl_fast_grid(h->nx, h->nu, sid, h->clf_kind, f64, B, h->clf_resident);
    if (G < 2 * X) return 0;
    const int per = (B + G - 1) / G;
    std::vector<int> order(B), map(B);
    for (int b = 0; b < B; b++) order[b] = b;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
        return d.offsets[a] % d.ref_period < d.offsets[b] % d.ref_period;
    });
    size_t next = 0;
    for (int x = 0; x < X; x++)
        for (int w = x; w < G; w += X)
            for (int q = w * per; q < std::min(B, (w + 1) * per); q++) map[q] = order[next++];
    if (hipMalloc((void **)&h->d_imap, (size_t)B * sizeof(int)) != hipSuccess)
        return h->fail(NMPC_ENOMEM, "nmpc_closed_loop_init: instance map");
    const hipError_t e = hipMemcpy(h->d_imap, map.data(), (size_t)B * sizeof(int), hipMemcpyHostToDevice);
    return e == hipSuccess ? 0 : hip_fail(h, e, "nmpc_closed_loop_init: instance map upload");
}

template <typename T>
nmpc::ClFastParams<T> clf_params(nmpc_solver *h, int target, int step0, int noise_ld)
{
    nmpc::ClFastParams<T> p{};
    const nmpc_closed_loop_desc &d = h->cl;
    const int nx = h->nx, nu = h->nu, nz = nx + nu;
    p.B = h->batch;
    p.N = h->N;
    p.ne = (h->N + 1) * nz;
    p.nslot = h->clf_nslot;
    p.period = d.ref_period;
    p.table_cols = d.ref_cols;
    p.cost_stage = d.cost_stage;
    p.ncl = d.ncl;
    p.aed_dims = d.aed_dims;
    p.noise_dims = d.noise_dims;
    p.plant = d.plant;
    p.substeps = d.substeps;
    p.ny = h->ny;
    p.ny_e = h->ny_e;
    p.mass = d.mass;
    p.g = d.g;
    p.dt = d.dt;
    p.dt_conv = d.dt_conv;
    p.target = target;
    p.traj_out = h->cl_traj_out ? 1 : 0;
    p.step0 = step0;
    p.noise_ld = noise_ld;
    p.polish_steps = h->polish_steps;
    p.x1_slot = h->clf_x1slot;
    p.table = (const T *)h->d_table;
    p.offset = h->d_offsets;
    p.state = (T *)h->d_state;
    p.acc = h->d_acc;
    p.istep = h->d_istep;
    p.flags = h->d_flags;
    p.noise = h->d_fnoise;
    const T *fT = (const T *)h->d_fsT;
    p.s_lb = fT + h->fso[0];
    p.s_ub = fT + h->fso[1];
    p.s_tx = fT + h->fso[2];
    p.vb = fT + h->fso[3];
    p.uinit = fT + h->fso[4];
    p.s_e = h->d_fsI + h->fsi[0];
    p.s_src = h->d_fsI + h->fsi[1];
    p.s_free = h->d_fsI + h->fsi[3];
    p.nfree = h->clf_nfree;
    p.vfull = (const T *)h->d_clv;
    p.txfull = (const T *)h->d_cltx;
    const char *m = (const char *)h->d_model;
    p.W = h->d_clw ? h->d_clw : (const double *)(m + h->off_lqrw);
    p.lbnd = (const T *)(m + h->off_lb);
    p.ubnd = (const T *)(m + h->off_ub);
    p.AB = (const T *)(m + h->off_AB);
    p.c = (const T *)(m + h->off_c);
    p.wcl = (const T *)h->d_wcl;
    p.xout = (T *)h->d_x;
    p.uout = (T *)h->d_u;
    p.status = h->d_status;
    p.iters = h->d_iters;
    p.park_count = h->d_park;
    p.park_list = h->d_park + 2;
    // env NMPC_CLF_NO_GI=1 (test knob): no dual active-set fallback, so every step whose PDAS run does
    // not settle parks and takes the list-mode full solve (tests/test_gpu_bench_parity.py forces parks)
    const char *nogi = std::getenv("NMPC_CLF_NO_GI");
    p.gi = (nogi && nogi[0] == '1') ? 0 : 1;
    const char *lw = std::getenv("NMPC_LOCK_WORKERS");
    // wavefronts per workgroup that start in phase 2 (drain demoted instances while the others still run
    // lockstep). Round 4: quad13 B = 8192 415M (0) -> 458-463M (1), 452-457M (2), 405-412M (3) steps/s
    // (tools/lock_ab.sh, ab1/ab2). Round 6, after the warm start at the horizon's end, the fallback's start and
    // the XCD map shortened the lockstep phase: 503-506M (0), 551-573M (1), 578-591M (2), 581-590M (3)
    // (profiles/r7/ab_lock_workers.jsonl, ab_lock_workers_run2_summary.txt), so two
    // (the jerk shape's lockstep variant, four wavefronts per workgroup and rarely a demotion: none)
    // (at most the variant's wavefronts per workgroup minus one, so some wavefront runs phase 1: quad13 8, jerk 4)
    const int lock_wpb = (h->nx == 6 && h->nu == 2) ? 4 : 8;
    p.lock_workers = lw ? std::max(0, std::min(lock_wpb - 1, std::atoi(lw))) : (h->nx == 6 && h->nu == 2 ? 0 : 2);
    const char *lp = std::getenv("NMPC_LOCK_PRIO");
    p.lock_prio = lp ? (lp[0] == '1') : 1;
    const char *ld = std::getenv("NMPC_LOCK_DIRECT");
    p.lock_direct = ld ? std::max(0, std::min(6, std::atoi(ld))) : 1;
    // the force shape claims its instances device-wide (env NMPC_CLF_GCLAIM=0 / 1 overrides)
    const char *gc = std::getenv("NMPC_CLF_GCLAIM");
    p.claim_global = gc ? (gc[0] == '1') : (h->nx == 4 && h->nu == 2);
    // the instances demoted (lockstep) or on the rare path (cl_fast_kernel) in the previous launch claimed first
    // (their chains start at the launch's beginning; env NMPC_CLF_ORDER=0: instance order)
    const char *lo = std::getenv("NMPC_CLF_ORDER");
    p.demoted = (lo && lo[0] == '0') ? nullptr : (unsigned char *)h->d_flags + (size_t)h->batch * h->clf_nslot;
    p.order_buckets = (lo && lo[0] == '2') ? 1 : 0;
    p.inst_map = p.claim_global ? nullptr : h->d_imap;
    // the rare path's W column cache in the workgroup's LDS (the shapes with sets of up to 16)
    const char *wce = std::getenv("NMPC_CLF_WCACHE");
    p.wcache = (wce && wce[0] == '0') ? 0 : 1;
    return p;
}

hipEvent_t cl_event(nmpc_solver *h, size_t i)
{
    while (h->cl_events.size() <= i) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        h->cl_events.push_back(e);
    }
    return h->cl_events[i];
}

// `steps` closed-loop steps on the lean loop, in chunks of at most CLF_CHUNK steps: per chunk the noise
// draws (by the first round's fast kernel itself, or the noise kernel), then rounds of (fast kernel over every
// instance up to the chunk's target step; the count of parked instances to the pinned host word — the one
// host wait per round; one full solve + plant step per parked instance, ipm_lpc_kernel in list mode) until
// none is parked. Returns the number of kernel
// launches (each bracketed by an event pair), or < 0. h->clf_parked / clf_rounds: the run's parked
// solves and fast launches.
// async (nmpc_closed_loop_run with sync = 0): no host wait at all — every chunk enqueues all its possible rounds
// (chunk length + 1), round r > 0's fast kernel guarded by round r - 1's park count on the device (0: every
// workgroup returns at entry) and each round's list-mode full solve sized by its own count on the device; the
// per-round counts follow to pinned host memory and nmpc_closed_loop_stats sums them.
template <typename T>
int clf_run(nmpc_solver *h, int steps, bool async)
{
    const size_t need = (size_t)h->batch * std::min(steps, CLF_CHUNK);
    if (h->fnoise_cap < need) {
        if (h->d_fnoise) hipFree(h->d_fnoise);
        h->d_fnoise = nullptr;
        h->fnoise_cap = 0;
        if (hipMalloc((void **)&h->d_fnoise, need * sizeof(double)) != hipSuccess)
            return h->fail(NMPC_EDEVICE, "nmpc_closed_loop_run: noise buffer");
        h->fnoise_cap = need;
    }
    // env NMPC_ITER_LOG: the per-step record of the run's last chunk (tuning aid, nmpc_closed_loop_iter_log);
    // filled with -1 first, so the rows of steps the list-mode fallback solved read as that marker
    static const bool iter_log = std::getenv("NMPC_ITER_LOG") != nullptr;
    static const bool dbg = std::getenv("NMPC_CLF_DEBUG") != nullptr;
    if (iter_log) {
        const size_t cap = need + 2 * (size_t)h->batch;   // + two rows: each instance's start and end
        if (h->iter_log_cap < cap) {
            if (h->d_iter_log) hipFree(h->d_iter_log);
            h->d_iter_log = nullptr;
            h->iter_log_cap = 0;
            if (hipMalloc((void **)&h->d_iter_log, cap * sizeof(int)) == hipSuccess) h->iter_log_cap = cap;
        }
    }
    // the parked count comes back through a pinned word (a pageable destination is a staged copy)
    if (!h->h_park && hipHostMalloc((void **)&h->h_park, 4 * sizeof(int), hipHostMallocDefault) != hipSuccess) {
        h->h_park = nullptr;
        return h->fail(NMPC_EDEVICE, "nmpc_closed_loop_run: pinned park word");
    }
    // env NMPC_CLF_CHECK with a checked build (-DNMPC_CLF_CHECK): the kernels' index checks report into a
    // device word, read after every round; a failed check fails the run
    static const bool check = std::getenv("NMPC_CLF_CHECK") != nullptr;
    if (check && !h->d_clf_check) {
        if (hipMalloc((void **)&h->d_clf_check, sizeof(unsigned)) != hipSuccess ||
            hipMemset(h->d_clf_check, 0, sizeof(unsigned)) != hipSuccess)
            return h->fail(NMPC_EDEVICE, "nmpc_closed_loop_run: check word");
    }
    int launches = 0;
    h->clf_parked = h->clf_rounds = 0;
    h->clf_async_chunks = 0;
    // (the diagnostic modes read the device after every round: host-driven rounds)
    if (iter_log || dbg || check || std::getenv("NMPC_CLF_CYCLES")) async = false;
    if (async) {
        const size_t need_r = (size_t)((steps + CLF_CHUNK - 1) / CLF_CHUNK) * CLF_ROUND_WORDS;
        if (h->parkr_cap < need_r) {
            hipError_t e = hipStreamSynchronize(h->stream);   // no copy into the old buffer is pending
            if (e != hipSuccess) return hip_fail(h, e, "nmpc_closed_loop_run");
            if (h->h_parkr) hipHostFree(h->h_parkr);
            h->h_parkr = nullptr;
            h->parkr_cap = 0;
            if ((e = hipHostMalloc((void **)&h->h_parkr, need_r * sizeof(int), hipHostMallocDefault)) != hipSuccess)
                return hip_fail(h, e, "nmpc_closed_loop_run: pinned round counters");
            h->parkr_cap = need_r;
        }
    }
    int *d_rc = h->d_park + 2 + h->batch;   // asynchronous runs: the rounds' [park count, claim counter] pairs
    // host-driven rounds: the fast kernel's last wavefront stores the park count into the pinned word (report_exit,
    // nmpc_cl_fast.hip), so the round's wait needs no copy behind the kernel (env NMPC_CLF_PARK_COPY=1: the copy)
    // (read per run: tests/test_gpu_bench_parity.py compares the paths in one process)
    const bool park_copy = std::getenv("NMPC_CLF_PARK_COPY") && std::getenv("NMPC_CLF_PARK_COPY")[0] == '1';
    const bool noise_kernel = std::getenv("NMPC_CLF_NOISE_KERNEL") && std::getenv("NMPC_CLF_NOISE_KERNEL")[0] == '1';
    volatile int *park_word = h->h_park;
    // env NMPC_CLF_CYCLES=<file> with a timing build (-DNMPC_CLF_TIMING): per-instance phase cycles of the
    // run, [B][CLF_NT_HOST] uint64, appended to <file> (tools/clf_phases.py)
    static const char *cyc_path = std::getenv("NMPC_CLF_CYCLES");
    unsigned long long *d_cyc = nullptr;
    if (cyc_path && hipMalloc((void **)&d_cyc, (size_t)h->batch * CLF_NT_HOST * sizeof(unsigned long long)) == hipSuccess)
        (void)hipMemsetAsync(d_cyc, 0, (size_t)h->batch * CLF_NT_HOST * sizeof(unsigned long long), h->stream);
    for (int done = 0; done < steps;) {
        const int n = std::min(CLF_CHUNK, steps - done), target = h->cl_step + n;
        nmpc::ClParams<T> cp = cl_params<T>(h);
        nmpc::ClFastParams<T> fp = clf_params<T>(h, target, h->cl_step, n);
        // host-driven rounds with per-workgroup claims: the first round's kernel draws the chunk's noise itself
        // (gen_noise) and the previous launch left the counters zero (report_exit); otherwise the noise kernel,
        // which also zeroes the park count and claim counter of the chunk's first round (env
        // NMPC_CLF_NOISE_KERNEL=1: always)
        const bool gen = !async && !park_copy && !noise_kernel && !fp.claim_global;
        hipError_t e = hipSuccess;
        if (!gen && (e = nmpc::cl_noise_launch<T>(cp, h->cl_step, n, h->d_fnoise, h->stream, h->d_park)) != hipSuccess)
            return hip_fail(h, e, "closed-loop noise");
        // the device-wide claim (the force shape): a batch-wide claim order from the previous launch's order bytes,
        // the longest chains first (env NMPC_CLF_GORDER=0: instance order)
        const char *go = std::getenv("NMPC_CLF_GORDER");
        // (not when every instance has a wavefront of its own: force B = 1024)
        if (fp.claim_global && fp.demoted && !(go && go[0] == '0') &&
            !nmpc::cl_fast_fits(h->nx, h->nu, h->clf_sid, h->clf_kind, std::is_same<T, double>::value, h->batch,
                                h->clf_resident)) {
            if (!h->d_gorder && hipMalloc((void **)&h->d_gorder, (size_t)h->batch * sizeof(int)) != hipSuccess) {
                h->d_gorder = nullptr;
                return h->fail(NMPC_ENOMEM, "nmpc_closed_loop_run: claim order");
            }
            if ((e = nmpc::clf_order_launch(fp.demoted, h->batch, h->d_gorder, h->stream)) != hipSuccess)
                return hip_fail(h, e, "claim order");
            fp.gorder = h->d_gorder;
        }
        fp.seed = cp.seed;
        fp.inst_base = cp.inst_base;
        fp.noise_std = cp.noise_std;
        fp.noise_table = cp.noise_table;
        fp.noise_len = cp.noise_len;
        fp.cycles = d_cyc;
        fp.check = h->d_clf_check;
        if (iter_log && h->d_iter_log) {
            const size_t rows = (size_t)(n + 2) * h->batch;
            if ((e = hipMemsetAsync(h->d_iter_log, 0xff, rows * sizeof(int), h->stream)) != hipSuccess)
                return hip_fail(h, e, "iter log reset");
            fp.iter_log = h->d_iter_log;
            h->iter_log_steps = n + 2;   // + the instance start / end rows
        }
        if (async && (e = hipMemsetAsync(d_rc, 0, (size_t)2 * (n + 1) * sizeof(int), h->stream)) != hipSuccess)
            return hip_fail(h, e, "round counters reset");
        for (int round = 0; round <= n; round++) {
            if (!async && round > 0 && (e = hipMemsetAsync(h->d_park, 0, 2 * sizeof(int), h->stream)) != hipSuccess)
                return hip_fail(h, e, "park reset");
            fp.park_count = async ? d_rc + 2 * round : h->d_park;
            fp.run_if = async && round > 0 ? d_rc + 2 * (round - 1) : nullptr;
            fp.park_host = async || park_copy ? nullptr : h->h_park;
            fp.noise_gen = gen && round == 0 ? h->d_fnoise : nullptr;
            fp.exit_count = (unsigned *)(h->d_park + h->batch + 2 + CLF_ROUND_WORDS);
            if (fp.park_host) park_word[0] = -1;   // (no copy into the word is pending: host-driven rounds wait)
            hipEvent_t ea = cl_event(h, 2 * launches), eb = cl_event(h, 2 * launches + 1);
            if (!ea || !eb) return h->fail(NMPC_EDEVICE, "nmpc_closed_loop_run: hipEventCreate");
            e = hipEventRecord(ea, h->stream);
            if (e == hipSuccess)
                e = nmpc::cl_fast_launch<T>(h->nx, h->nu, h->clf_sid, h->clf_kind, fp, h->batch, h->clf_resident, h->stream);
            if (e == hipSuccess) e = hipEventRecord(eb, h->stream);
            launches++;
            h->clf_rounds++;
            if (e != hipSuccess) return hip_fail(h, e, "lean closed-loop kernel launch");
            if (async) {   // this round's parked instances, their count read on the device
                ListArgs la{h->batch, h->cl_step, n, h->d_park + 2, h->clf_kidx, h->d_clf_scratch};
                la.count_dev = fp.park_count;
                const int r = launch<T>(h, cl_event(h, 2 * launches), cl_event(h, 2 * launches + 1), 1, &la);
                launches++;
                if (r < 0) return r;
                continue;
            }
            if (!fp.park_host) e = hipMemcpyAsync(h->h_park, h->d_park, sizeof(int), hipMemcpyDeviceToHost, h->stream);
            if (e == hipSuccess) e = stream_wait(h->stream);
            if (e != hipSuccess) return hip_fail(h, e, "lean closed loop (fast kernel)");
            const int parked = park_word[0];
            if (parked < 0) return h->fail(NMPC_EDEVICE, "lean closed loop: the fast kernel did not report its park count");
            if (h->d_clf_check) {
                unsigned bad = 0;
                if ((e = hipMemcpy(&bad, h->d_clf_check, sizeof(bad), hipMemcpyDeviceToHost)) != hipSuccess)
                    return hip_fail(h, e, "lean closed loop check word");
                if (bad)
                    return h->fail(NMPC_EDEVICE, "lean closed loop: index check failed, codes mask " + std::to_string(bad) +
                                                     " (nmpc_cl_fast.hip CLF_CHECK)");
            }
            if (dbg) std::fprintf(stderr, "[nmpc clf] steps %d..%d round %d: %d parked\n", h->cl_step, target, round, parked);
            if (parked <= 0) break;
            h->clf_parked += parked;
            // the fallback: one full solve + plant step for every parked instance
            const ListArgs la{parked, h->cl_step, n, h->d_park + 2, h->clf_kidx, h->d_clf_scratch};
            const int r = launch<T>(h, cl_event(h, 2 * launches), cl_event(h, 2 * launches + 1), 1, &la);
            launches++;
            if (r < 0) return r;
            if (dbg && (e = hipStreamSynchronize(h->stream)) != hipSuccess) return hip_fail(h, e, "lean closed loop (list-mode fallback)");
        }
        if (async) {   // the rounds' counts, summed by nmpc_closed_loop_stats
            e = hipMemcpyAsync(h->h_parkr + (size_t)h->clf_async_chunks * CLF_ROUND_WORDS, d_rc,
                               (size_t)2 * (n + 1) * sizeof(int), hipMemcpyDeviceToHost, h->stream);
            if (e != hipSuccess) return hip_fail(h, e, "round counters");
            if (n + 1 < CLF_CHUNK + 1)   // the rest of the chunk's slot: no rounds
                std::fill(h->h_parkr + (size_t)h->clf_async_chunks * CLF_ROUND_WORDS + 2 * (n + 1),
                          h->h_parkr + (size_t)(h->clf_async_chunks + 1) * CLF_ROUND_WORDS, 0);
            h->clf_async_chunks++;
        }
        h->cl_step = target;
        done += n;
    }
    if (d_cyc) {
        std::vector<unsigned long long> cy((size_t)h->batch * CLF_NT_HOST);
        if (hipStreamSynchronize(h->stream) == hipSuccess &&
            hipMemcpy(cy.data(), d_cyc, cy.size() * sizeof(cy[0]), hipMemcpyDeviceToHost) == hipSuccess) {
            if (FILE *f = std::fopen(cyc_path, "ab")) {
                std::fwrite(cy.data(), sizeof(cy[0]), cy.size(), f);
                std::fclose(f);
            }
        }
        (void)hipFree(d_cyc);
    }
    if (dbg && hipStreamSynchronize(h->stream) == hipSuccess)
        for (int i = 0; i < launches; i++) {
            float ms = 0.f, gap = 0.f;
            hipEventElapsedTime(&ms, cl_event(h, 2 * i), cl_event(h, 2 * i + 1));
            if (i + 1 < launches) hipEventElapsedTime(&gap, cl_event(h, 2 * i + 1), cl_event(h, 2 * i + 2));
            std::fprintf(stderr, "[nmpc clf] run of %d steps, launch %d: %.4f ms, then %.4f ms to the next\n", steps, i, ms, gap);
        }
    return launches;
}

// the lean loop keeps each instance's step and warm-start flags on the device (d_istep, d_flags); a run
// on another path (NMPC_CL_FUSED=0 / per-step launches) advances every instance to h->cl_step without
// them, so they are resynchronised after it: istep = cl_step for every instance, flags cleared (the
// warm start only steers the active-set path, the certified solutions do not depend on it)
int clf_resync(nmpc_solver *h)
{
    if (!h->clf) return 0;
    std::vector<int> st((size_t)h->batch, h->cl_step);
    hipError_t e = hipStreamSynchronize(h->stream);
    if (e == hipSuccess) e = hipMemcpy(h->d_istep, st.data(), st.size() * sizeof(int), hipMemcpyHostToDevice);
    // (the order bytes too: bit 7 promises a nonempty warm set, which the lockstep kernel routes to phase 2)
    if (e == hipSuccess) e = hipMemset(h->d_flags, 0, (size_t)h->batch * (h->clf_nslot + 1));
    return e == hipSuccess ? 0 : hip_fail(h, e, "lean closed loop resync");
}

}  // namespace

extern "C" {

int nmpc_closed_loop_init(nmpc_solver *h, const nmpc_closed_loop_desc *d)
{
    if (!h || !d) return NMPC_EINVAL;
    if (!d->ref_table || !d->offsets || !d->x_init || d->ref_rows < 1 || d->ref_period < 1)
        return h->fail(NMPC_EINVAL, "nmpc_closed_loop_init: table, offsets and x_init are required");
    if (d->ref_cols < std::max(h->ny, h->ny_e) || d->ref_cols < d->ncl || d->ref_cols < d->aed_dims)
        return h->fail(NMPC_EINVAL, "nmpc_closed_loop_init: ref_cols too small for ny / ny_e / ncl");
    if (d->ref_period - 1 + h->N >= d->ref_rows)
        return h->fail(NMPC_EINVAL, "nmpc_closed_loop_init: ref_rows must cover ref_period - 1 + N");
    if (d->plant < 0 || d->plant > 2) return h->fail(NMPC_EINVAL, "nmpc_closed_loop_init: unknown plant");
    if (d->plant == NMPC_PLANT_CRAZYFLIE_FORCE && (h->nx != 4 || h->nu != 2))
        return h->fail(NMPC_EINVAL, "force plant needs the force controller model (nx=4, nu=2)");
    if (d->plant == NMPC_PLANT_CRAZYFLIE_JERK && (h->nx != 6 || h->nu != 2))
        return h->fail(NMPC_EINVAL, "jerk plant needs the jerk controller model (nx=6, nu=2)");
    if (h->nx > 32) return h->fail(NMPC_EUNSUPPORTED, "closed loop supports nx <= 32");
    if (d->ncl > h->nx || d->aed_dims > h->nx || d->cost_stage < 0 || d->cost_stage > h->N)
        return h->fail(NMPC_EINVAL, "nmpc_closed_loop_init: ncl / aed_dims / cost_stage out of range");
    for (int b = 0; b < h->batch; b++)
        if (d->offsets[b] < 0) return h->fail(NMPC_EINVAL, "nmpc_closed_loop_init: negative offset");
    hipSetDevice(h->device);
    const bool f64 = h->precision == NMPC_FP64;
    const size_t es = h->esz();
    for (void **p : {&h->d_table, &h->d_state, &h->d_plant, &h->d_wcl, (void **)&h->d_offsets, (void **)&h->d_acc,
                     (void **)&h->d_noise})
        if (*p) {
            hipFree(*p);
            *p = nullptr;
        }
    const int nx = h->nx, nu = h->nu;
    bool ok = hipMalloc(&h->d_table, (size_t)d->ref_rows * d->ref_cols * es) == hipSuccess &&
              hipMalloc(&h->d_state, (size_t)h->batch * nx * es) == hipSuccess &&
              hipMalloc(&h->d_plant, (size_t)(nx * nx + nx * nu + nx) * es) == hipSuccess &&
              hipMalloc(&h->d_wcl, (size_t)std::max(d->ncl, 1) * es) == hipSuccess &&
              hipMalloc((void **)&h->d_offsets, (size_t)h->batch * sizeof(int)) == hipSuccess &&
              hipMalloc((void **)&h->d_acc, (size_t)h->batch * 4 * sizeof(double)) == hipSuccess;
    if (ok && d->noise_table && d->noise_len > 0)
        ok = hipMalloc((void **)&h->d_noise, (size_t)h->batch * d->noise_len * sizeof(double)) == hipSuccess;
    if (!ok) return h->fail(NMPC_ENOMEM, "nmpc_closed_loop_init: device allocation failed");
    std::vector<double> plant(h->A);
    plant.insert(plant.end(), h->B.begin(), h->B.end());
    plant.insert(plant.end(), h->c.begin(), h->c.end());
    std::vector<double> w(std::max(d->ncl, 1), 0.0);
    for (int i = 0; i < d->ncl; i++) w[i] = d->w_cl ? d->w_cl[i] : 1.0;
    hipError_t e = put_typed(h->d_table, d->ref_table, (size_t)d->ref_rows * d->ref_cols, f64);
    if (e == hipSuccess) e = put_typed(h->d_state, d->x_init, (size_t)h->batch * nx, f64);
    if (e == hipSuccess) e = put_typed(h->d_plant, plant.data(), plant.size(), f64);
    if (e == hipSuccess) e = put_typed(h->d_wcl, w.data(), w.size(), f64);
    if (e == hipSuccess) e = hipMemcpy(h->d_offsets, d->offsets, h->batch * sizeof(int), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemset(h->d_acc, 0, (size_t)h->batch * 4 * sizeof(double));
    if (e == hipSuccess && h->d_noise)
        e = hipMemcpy(h->d_noise, d->noise_table, (size_t)h->batch * d->noise_len * sizeof(double),
                      hipMemcpyHostToDevice);
    if (e != hipSuccess) return hip_fail(h, e, "nmpc_closed_loop_init upload");
    // explicit unconstrained solution for the fused closed loop's fast finish: z_0 = T_x x_0 + v_t, v_t
    // the response to the reference window starting at table row t (t < ref_period) and to c
    if (h->d_cltx) hipFree(h->d_cltx);
    if (h->d_clv) hipFree(h->d_clv);
    h->d_cltx = h->d_clv = nullptr;
    h->clf = false;
    if (!h->cond && !h->lqr_host.empty()) {
        const int N = h->N, nz = nx + nu, ne = (N + 1) * nz, ny = h->ny, nye = h->ny_e, P_ = d->ref_period;
        std::vector<double> tx((size_t)ne * nx), vv((size_t)P_ * ne), g((size_t)ne, 0.0), z((size_t)ne), e0(nx);
        for (int j = 0; j < nx; j++) {
            std::fill(e0.begin(), e0.end(), 0.0);
            e0[j] = 1.0;
            lqr_solve(nx, nu, N, h->A, h->B, h->c, h->lqr_host, g.data(), e0.data(), false, z.data());
            for (int e = 0; e < ne; e++) tx[(size_t)e * nx + j] = z[e];
        }
        std::fill(e0.begin(), e0.end(), 0.0);
        for (int t = 0; t < P_; t++) {
            std::fill(g.begin(), g.end(), 0.0);
            for (int k = 0; k <= N; k++) {
                const double *y = d->ref_table + (size_t)(t + k) * d->ref_cols;
                const int n = k < N ? nz : nx, m = k < N ? ny : nye;
                const double *Gm = k < N ? h->G.data() : h->Ge.data();
                for (int i = 0; i < n; i++) {
                    double s_ = 0.0;
                    for (int q = 0; q < m; q++) s_ += Gm[i * m + q] * y[q];
                    g[(size_t)k * nz + i] = s_;
                }
            }
            lqr_solve(nx, nu, N, h->A, h->B, h->c, h->lqr_host, g.data(), e0.data(), true, z.data());
            std::copy(z.begin(), z.end(), vv.begin() + (size_t)t * ne);
        }
        if (hipMalloc(&h->d_cltx, tx.size() * es) != hipSuccess || hipMalloc(&h->d_clv, vv.size() * es) != hipSuccess)
            return h->fail(NMPC_ENOMEM, "nmpc_closed_loop_init: explicit-solution tables");
        e = put_typed(h->d_cltx, tx.data(), tx.size(), f64);
        if (e == hipSuccess) e = put_typed(h->d_clv, vv.data(), vv.size(), f64);
        if (e != hipSuccess) return hip_fail(h, e, "nmpc_closed_loop_init explicit tables");
        const int r = clf_setup(h, *d, tx, vv);
        if (r < 0) return r;
    }
    h->cl = *d;
    h->cl.ref_table = nullptr;
    h->cl.offsets = nullptr;
    h->cl.x_init = nullptr;
    h->cl.noise_table = nullptr;
    h->cl.w_cl = nullptr;
    h->cl_step = 0;
    h->cl_ready = true;
    return 0;
}

int nmpc_closed_loop_run(nmpc_solver *h, int steps, int sync)
{
    if (!h) return NMPC_EINVAL;
    if (!h->cl_ready) return h->fail(NMPC_ESTATE, "nmpc_closed_loop_run: call nmpc_closed_loop_init first");
    if (steps < 0) return h->fail(NMPC_EINVAL, "nmpc_closed_loop_run: steps < 0");
    hipSetDevice(h->device);
    while ((int)h->cl_events.size() < 2 * steps) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return h->fail(NMPC_EDEVICE, "hipEventCreate");
        h->cl_events.push_back(e);
    }
    h->out_valid = false;
    h->iter_log_steps = 0;   // the log describes the last fused launch of this run only
    int launches = 0;
    const char *fused_env = std::getenv("NMPC_CL_FUSED");
    const bool lean = h->clf && !(fused_env && fused_env[0] == '0');
    h->clf_parked = h->clf_rounds = 0;
    if (lean) {
        launches = steps <= 0 ? 0 : (h->precision == NMPC_FP64 ? clf_run<double>(h, steps, !sync) : clf_run<float>(h, steps, !sync));
        if (launches < 0) return launches;
    } else if (cl_fused(h)) {
        if (h->fnoise_cap < (size_t)h->batch * CL_FUSED_CHUNK) {
            if (h->d_fnoise) hipFree(h->d_fnoise);
            h->d_fnoise = nullptr;
            if (hipMalloc((void **)&h->d_fnoise, (size_t)h->batch * CL_FUSED_CHUNK * sizeof(double)) != hipSuccess)
                return h->fail(NMPC_EDEVICE, "nmpc_closed_loop_run: noise buffer");
            h->fnoise_cap = (size_t)h->batch * CL_FUSED_CHUNK;
        }
        for (int s = 0; s < steps; s += CL_FUSED_CHUNK, launches++) {
            const int n = std::min(CL_FUSED_CHUNK, steps - s);
            const int r = h->precision == NMPC_FP64 ? cl_fused_enqueue<double>(h, launches, n)
                                                    : cl_fused_enqueue<float>(h, launches, n);
            if (r < 0) return r;
        }
    } else {
        for (int s = 0; s < steps; s++, launches++) {
            const int r = h->precision == NMPC_FP64 ? cl_step_enqueue<double>(h, s) : cl_step_enqueue<float>(h, s);
            if (r < 0) return r;
        }
    }
    if (!lean && steps > 0) {
        const int r = clf_resync(h);
        if (r < 0) return r;
    }
    h->cl_last_launches = launches;
    h->cl_last_steps = steps;
    if (lean && h->cl_traj_out && steps > 0) {   // the last step's solutions, readable through nmpc_get*
        const int r = download_outputs(h);
        if (r < 0) return r;
        h->out_from_loop = true;
    }
    // the loop rewrote the device x0 / yref: the next nmpc_solve re-uploads the host-staged inputs
    h->x0_dirty = h->yref_dirty = true;
    if (sync) {
        hipError_t e = hipStreamSynchronize(h->stream);
        if (e != hipSuccess) return hip_fail(h, e, "nmpc_closed_loop_run");
    }
    return 0;
}

int nmpc_closed_loop_stats(nmpc_solver *h, double *out, int n)
{
    if (!h || !out) return NMPC_EINVAL;
    if (!h->cl_ready) return h->fail(NMPC_ESTATE, "nmpc_closed_loop_stats: closed loop not initialised");
    hipSetDevice(h->device);
    hipError_t e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return hip_fail(h, e, "nmpc_closed_loop_stats");
    std::vector<double> acc((size_t)h->batch * 4);
    if ((e = hipMemcpy(acc.data(), h->d_acc, acc.size() * sizeof(double), hipMemcpyDeviceToHost)) != hipSuccess)
        return hip_fail(h, e, "nmpc_closed_loop_stats (accumulators)");
    double v[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int b = 0; b < h->batch; b++)
        for (int j = 0; j < 4; j++) v[j] += acc[(size_t)b * 4 + j];
    double ms = 0.0;
    for (int s = 0; s < h->cl_last_launches; s++) {
        // every launch of the run recorded its pair (launch / sf_enqueue / clf_run); a failed read is an error,
        // not a launch to leave out of the kernel time
        float t = 0.f;
        if ((e = hipEventElapsedTime(&t, h->cl_events[2 * s], h->cl_events[2 * s + 1])) != hipSuccess)
            return hip_fail(h, e, ("nmpc_closed_loop_stats: timing events of launch " + std::to_string(s)).c_str());
        ms += t;
    }
    v[4] = ms;
    v[5] = h->cl_last_launches;
    if (h->clf_async_chunks > 0) {   // an asynchronous lean run: its rounds' park counts (pinned, the stream has drained)
        h->clf_parked = 0;
        for (int c = 0; c < h->clf_async_chunks; c++)
            for (int r = 0; r <= CLF_CHUNK; r++) h->clf_parked += h->h_parkr[(size_t)c * CLF_ROUND_WORDS + 2 * r];
        h->clf_async_chunks = 0;
    }
    std::vector<int32_t> it(h->batch);
    if ((e = hipMemcpy(it.data(), h->d_iters, h->batch * sizeof(int32_t), hipMemcpyDeviceToHost)) != hipSuccess)
        return hip_fail(h, e, "nmpc_closed_loop_stats (qp_iter)");
    double mean = 0.0;
    for (int b = 0; b < h->batch; b++) mean += it[b];
    v[6] = mean / h->batch;
    v[7] = h->cl_last_steps;
    v[8] = h->clf_parked;
    v[9] = h->clf_rounds;
    for (int i = 0; i < n && i < 10; i++) out[i] = v[i];
    return 0;
}

int nmpc_closed_loop_iter_log(nmpc_solver *h, int32_t *out, size_t count)
{
    if (!h) return NMPC_EINVAL;
    if (!out) return h->d_iter_log ? h->iter_log_steps : 0;   // query: steps in the log
    if (!h->d_iter_log || h->iter_log_steps <= 0)
        return h->fail(NMPC_ESTATE, "nmpc_closed_loop_iter_log: no log (set NMPC_ITER_LOG and run a fused closed loop)");
    const size_t n = (size_t)h->iter_log_steps * h->batch;
    if (count != n) return h->fail(NMPC_EINVAL, "nmpc_closed_loop_iter_log: needs steps*batch values");
    hipSetDevice(h->device);
    hipError_t e = hipStreamSynchronize(h->stream);
    if (e == hipSuccess) e = hipMemcpy(out, h->d_iter_log, n * sizeof(int32_t), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return hip_fail(h, e, "nmpc_closed_loop_iter_log");
    return (int)h->iter_log_steps;
}

int nmpc_closed_loop_instance_stats(nmpc_solver *h, double *out, size_t count)
{
    if (!h || !out) return NMPC_EINVAL;
    if (!h->cl_ready) return h->fail(NMPC_ESTATE, "nmpc_closed_loop_instance_stats: closed loop not initialised");
    if (count != (size_t)h->batch * 4)
        return h->fail(NMPC_EINVAL, "nmpc_closed_loop_instance_stats: needs batch*4 values");
    hipSetDevice(h->device);
    hipError_t e = hipStreamSynchronize(h->stream);
    if (e == hipSuccess) e = hipMemcpy(out, h->d_acc, count * sizeof(double), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return hip_fail(h, e, "nmpc_closed_loop_instance_stats");
    return 0;
}

int nmpc_closed_loop_set_outputs(nmpc_solver *h, int on)
{
    if (!h) return NMPC_EINVAL;
    h->cl_traj_out = on != 0;
    return 0;
}

int nmpc_closed_loop_get_state(nmpc_solver *h, double *out, size_t count)
{
    if (!h || !out) return NMPC_EINVAL;
    if (!h->cl_ready) return h->fail(NMPC_ESTATE, "nmpc_closed_loop_get_state: closed loop not initialised");
    if (count != (size_t)h->batch * h->nx) return h->fail(NMPC_EINVAL, "nmpc_closed_loop_get_state: size mismatch");
    hipSetDevice(h->device);
    hipError_t e = hipStreamSynchronize(h->stream);
    if (e != hipSuccess) return hip_fail(h, e, "nmpc_closed_loop_get_state");
    if (h->precision == NMPC_FP64) {
        e = hipMemcpy(out, h->d_state, count * sizeof(double), hipMemcpyDeviceToHost);
    } else {
        std::vector<float> t(count);
        e = hipMemcpy(t.data(), h->d_state, count * sizeof(float), hipMemcpyDeviceToHost);
        for (size_t i = 0; i < count; i++) out[i] = t[i];
    }
    if (e != hipSuccess) return hip_fail(h, e, "nmpc_closed_loop_get_state");
    return 0;
}

}  // extern "C"
