// nmpc_cond.hip — condensed (dense-QP) interior-point solve of the batched LQ-OCP on gfx950,
// with the dense Hessian block-GEMMs on the matrix cores (MFMA).
//
// The same problem as nmpc_ipm.hip / nmpc_ipm_lpc.hip (one AcadosOcpSolver.solve() of
// src/force_model/controller.py:32 / src/jerk_model/controller.py:33: SQP-GN on an LTI /
// LINEAR_LS / box-constrained OCP == one QP), in the condensed form HPIPM's condensing
// produces (qp_solver PARTIAL_CONDENSING_HPIPM, src/force_model/ocp.py:83, with one block):
// the states are eliminated, x_k = Phi_k x0 + d_k + Gamma_k U (host, nmpc_cond_host.cpp), and
// every instance solves
//
//     min 1/2 U' H0 U + f' U     s.t.  lo <= U <= hi,   lx - xf <= Gx U <= hx - xf
//
// with U = [u_0; ...; u_{N-1}] (n = N nu), H0 / Gx shared by all instances and f, xf affine
// in (x0, yref). A Mehrotra predictor-corrector IPM with explicit slacks (infeasible start)
// runs per instance; each iteration factorises
//
//     K = H0 + diag(D_u) + Gx' diag(D_x) Gx        (D = lambda / t, the barrier Hessian)
//
// The Gx' D Gx product — the dense Hessian block-GEMM — and the trailing updates of the
// blocked Cholesky run as v_mfma_f64_16x16x4_f64 (fp32: v_mfma_f32_16x16x4_f32) on 16x16
// tiles; Gx is block lower triangular (x_k depends on u_0..u_{k-1}), so tile row-block I only
// accumulates the x rows of stages k with k nu > 16 I (host: ks[]).
//
// Mapping: one wavefront per instance. Gx (column-major, pitch ldg == 2 mod 32: conflict-free
// MFMA operand reads) is staged in LDS once per workgroup; each wavefront keeps its K tiles
// (lower triangle, 16x16 column-major tiles of pitch 17) and a few broadcast vectors in LDS, and
// its constraint rows (64 per register chunk: slacks, multipliers, steps) and the n-vectors
// (lanes = rows) in registers. Reductions over the wavefront are DPP row rotations + 4
// readlanes. Primal and dual steps have separate lengths. Termination: mu <= tol_comp and
// max |residual| <= tol_res (dual rd = H0 U + f - C' lambda, primal CU - lo - t_l, hi - CU - t_u,
// evaluated at every iterate); status codes and failure semantics follow the Riccati kernels:
// status 2 after max_iter, 4 on a non-positive pivot (the iterate of the start of that
// iteration is returned) or a non-finite mu.

#include <hip/hip_runtime.h>

#include "nmpc_internal.h"

namespace nmpc {
namespace cond {

#define CSYNC()                                                  \
    do {                                                         \
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   \
        __builtin_amdgcn_wave_barrier();                         \
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   \
    } while (0)

constexpr int TP = 17;        // tile column pitch (elements)
constexpr int TS = 16 * TP;   // tile stride

template <typename T>
struct Mf;
template <>
struct Mf<double> {
    typedef double v4 __attribute__((ext_vector_type(4)));
    __device__ static v4 mma(double a, double b, v4 c) { return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0); }
    // C/D layout of v_mfma_f64_16x16x4_f64: col = lane & 15, row = (lane >> 4) + 4 r
    __device__ static int row(int lane, int r) { return (lane >> 4) + 4 * r; }
};
template <>
struct Mf<float> {
    typedef float v4 __attribute__((ext_vector_type(4)));
    __device__ static v4 mma(float a, float b, v4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
    // C/D layout of v_mfma_f32_16x16x4_f32: col = lane & 15, row = 4 (lane >> 4) + r
    __device__ static int row(int lane, int r) { return 4 * (lane >> 4) + r; }
};

__device__ __forceinline__ double frsq(double x)
{
    double y = __builtin_amdgcn_rsq(x);
    const double h = 0.5 * x;
    y = fma(y, fma(-h, y * y, 0.5), y);
    return fma(y, fma(-h, y * y, 0.5), y);
}
__device__ __forceinline__ float frsq(float x)
{
    float y = __builtin_amdgcn_rsqf(x);
    return fmaf(y, fmaf(-0.5f * x, y * y, 0.5f), y);
}
__device__ __forceinline__ double frcp(double x)
{
    double r = __builtin_amdgcn_rcp(x);
    r = fma(fma(-x, r, 1.0), r, r);
    return fma(fma(-x, r, 1.0), r, r);
}
__device__ __forceinline__ float frcp(float x)
{
    float r = __builtin_amdgcn_rcpf(x);
    return fmaf(fmaf(-x, r, 1.0f), r, r);
}

// ---- cross-lane primitives (whole wavefront active)
template <int CTRL>
__device__ __forceinline__ float dpp(float v)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
template <int CTRL>
__device__ __forceinline__ double dpp(double v)
{
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xf, 0xf, false);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned)lo);
}
__device__ __forceinline__ float rl(float v, int l)
{
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
__device__ __forceinline__ double rl(double v, int l)
{
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_readlane((int)b, l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned)lo);
}
// wavefront reduction: quad butterflies, row rotations by 4 and 8 (every lane of a row then
// holds the row's result), then the four row results
template <typename T, typename Op>
__device__ __forceinline__ T wred(T v, Op op)
{
    v = op(v, dpp<0xB1>(v));    // quad_perm [1,0,3,2]
    v = op(v, dpp<0x4E>(v));    // quad_perm [2,3,0,1]
    v = op(v, dpp<0x124>(v));   // row_ror:4
    v = op(v, dpp<0x128>(v));   // row_ror:8
    return op(op(rl(v, 15), rl(v, 31)), op(rl(v, 47), rl(v, 63)));
}

// NMPC_COND_TIMING builds (tools): s_memtime per phase, accumulated per instance into p.cycles
#ifdef NMPC_COND_TIMING
#define CT_DECL unsigned long long ct_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, ct_last = __builtin_amdgcn_s_memtime();
#define CT(slot)                                                    \
    do {                                                            \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
        ct_acc[slot] += t_ - ct_last;                               \
        ct_last = t_;                                               \
    } while (0)
#else
#define CT_DECL
#define CT(slot) ((void)0)
#endif

template <typename T>
__device__ __forceinline__ bool has(T b)
{
    return fabs(b) < T(1e20);
}

template <typename T, int RC, int UC>
__global__ __launch_bounds__(256) void cond_ipm_kernel(CondParams<T> p)
{
    using M = Mf<T>;
    using v4 = typename M::v4;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    T *sh = (T *)smem_raw;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int n = p.n, nb = p.nb, np = 16 * nb, mx = p.mx, mc = n + mx, ldg = p.ldg, nx = p.nx, nu = p.nu;
    const int mxp = (mx + 3) & ~3;
    const int q = lane >> 4, c16 = lane & 15;

    // ---- shared: Gx column-major [np][ldg] (zero padded) and H0 column-major [n][n], once per
    //      workgroup
    CT_DECL
    T *G = sh;
    T *H0 = sh + (size_t)np * ldg;
    for (int e = threadIdx.x; e < np * ldg; e += blockDim.x) G[e] = p.Gx[e];
    for (int e = threadIdx.x; e < n * n; e += blockDim.x) H0[e] = p.H0[e];
    __syncthreads();
    const long long inst_l = (long long)blockIdx.x * (blockDim.x >> 6) + wave;
    if (inst_l >= p.B) return;
    const int inst = (int)inst_l;

    // ---- per-wavefront LDS
    T *Kt = H0 + (((size_t)n * n + 3) & ~(size_t)3) + (size_t)wave * p.wave_elems;
    const int ntiles = nb * (nb + 1) / 2;
    T *Uv = Kt + ntiles * TS;   // [np] iterate U (broadcast reads)
    T *Sv = Uv + np;            // [np] Newton step dU
    T *DU = Sv + np;            // [np] barrier Hessian of the u rows
    T *WX = DU + np;            // [ldg] weights of the x rows (C' w)
    T *DX = WX + ldg;           // [ldg] barrier Hessian of the x rows
    auto tile = [&](int I, int J) { return Kt + (I * (I + 1) / 2 + J) * TS; };

    const T *x0 = p.x0 + (size_t)inst * nx;
    const T *Y = p.yref + (size_t)inst * p.nY;

    // ---- gradient f = fc + Fx x0 + Fy yref (lanes = rows of U)
    T f[UC];
#pragma unroll
    for (int c = 0; c < UC; c++) {
        const int i = lane + 64 * c;
        T s0 = 0, s1 = 0, s2 = 0, s3 = 0;
        if (i < n) {
            s0 = p.fc[i];
            for (int a = 0; a < nx; a++) s1 = fma(p.Fx[(size_t)a * n + i], x0[a], s1);
            int b = 0;
            for (; b + 3 < p.nY; b += 4) {
                s0 = fma(p.Fy[(size_t)b * n + i], Y[b], s0);
                s1 = fma(p.Fy[(size_t)(b + 1) * n + i], Y[b + 1], s1);
                s2 = fma(p.Fy[(size_t)(b + 2) * n + i], Y[b + 2], s2);
                s3 = fma(p.Fy[(size_t)(b + 3) * n + i], Y[b + 3], s3);
            }
            for (; b < p.nY; b++) s0 = fma(p.Fy[(size_t)b * n + i], Y[b], s0);
        }
        f[c] = (s0 + s1) + (s2 + s3);
    }
    // ---- initial U: the u part of yref (LINEAR_LS with selection Vx/Vu) or 0, inside the bounds
#pragma unroll
    for (int c = 0; c < UC; c++) {
        const int i = lane + 64 * c;
        if (i < np) {
            T z = 0;
            if (i < n) {
                const int k = i / nu, iu = i - k * nu;
                z = p.yref_is_z ? Y[(size_t)k * p.ny + nx + iu] : T(0);
                const T lb = p.lou[i], ub = p.hiu[i];
                const bool hl = has(lb), hu = has(ub);
                if (hl && hu) {
                    const T d = T(0.01) * (ub - lb);
                    z = T(0.5) * (lb + ub);   // boxed inputs start mid-box (oracle/c/riccati_ipm.c)
                    z = fmin(fmax(z, lb + d), ub - d);
                } else if (hl) {
                    z = fmax(z, lb + T(0.01) * fmax(fabs(lb), T(1)));
                } else if (hu) {
                    z = fmin(z, ub - T(0.01) * fmax(fabs(ub), T(1)));
                }
            }
            Uv[i] = z;
            DU[i] = 0;
        }
    }
    for (int r = lane; r < ldg; r += 64) {
        WX[r] = 0;
        DX[r] = 0;
    }
    // ---- constraint rows rho = lane + 64 c: u rows (rho < n) and x rows (rho - n < mx)
    T lo[RC], hi[RC], tl[RC], tu[RC], ll[RC], lu[RC], cu[RC];
#pragma unroll
    for (int c = 0; c < RC; c++) {
        const int rho = lane + 64 * c;
        lo[c] = T(-1e30);
        hi[c] = T(1e30);
        if (rho < n) {
            lo[c] = p.lou[rho];
            hi[c] = p.hiu[rho];
        } else if (rho < mc) {
            const int r = rho - n;
            T xf = p.dx[r];
            for (int a = 0; a < nx; a++) xf = fma(p.Phx[(size_t)a * mx + r], x0[a], xf);
            const T lx = p.lox[r], hx = p.hix[r];
            lo[c] = has(lx) ? lx - xf : T(-1e30);
            hi[c] = has(hx) ? hx - xf : T(1e30);
        }
    }
    CSYNC();
    // C v for the broadcast vector v (LDS): u rows read v, x rows Gx(r, :) v over the nonzero
    // columns j < k nu of their stage (4 independent accumulators keep 8 LDS reads in flight)
    auto Cmul = [&](const T *v, T (&out)[RC]) {
#pragma unroll
        for (int c = 0; c < RC; c++) {
            const int rho = lane + 64 * c;
            T s0 = 0, s1 = 0, s2 = 0, s3 = 0;
            if (rho < n) {
                s0 = v[rho];
            } else if (rho < mc) {
                const int r = rho - n, nc = p.xcols[r];
                const T *g = G + r;
                int j = 0;
                for (; j + 3 < nc; j += 4) {
                    s0 = fma(g[j * ldg], v[j], s0);
                    s1 = fma(g[(j + 1) * ldg], v[j + 1], s1);
                    s2 = fma(g[(j + 2) * ldg], v[j + 2], s2);
                    s3 = fma(g[(j + 3) * ldg], v[j + 3], s3);
                }
                for (; j < nc; j++) s0 = fma(g[j * ldg], v[j], s0);
            }
            out[c] = (s0 + s1) + (s2 + s3);
        }
    };
    // C' w (lanes = rows of U): u part lane-local, x part Gx' w over the rows with nonzeros
    auto CTmul = [&](const T (&w)[RC], T (&out)[UC]) {
#pragma unroll
        for (int c = 0; c < RC; c++) {
            const int rho = lane + 64 * c;
            if (rho >= n && rho < mc) WX[rho - n] = w[c];
        }
        CSYNC();
#pragma unroll
        for (int c = 0; c < UC; c++) {
            const int i = lane + 64 * c;
            T s0 = 0, s1 = 0, s2 = 0, s3 = 0;
            if (i < n) {
                s0 = w[c];   // rho = i lives in the same lane and chunk (n <= 64 UC <= 64 RC)
                const T *g = G + i * ldg;
                int r = p.rstart[i];
                for (; r + 3 < mx; r += 4) {
                    s0 = fma(g[r], WX[r], s0);
                    s1 = fma(g[r + 1], WX[r + 1], s1);
                    s2 = fma(g[r + 2], WX[r + 2], s2);
                    s3 = fma(g[r + 3], WX[r + 3], s3);
                }
                for (; r < mx; r++) s0 = fma(g[r], WX[r], s0);
            }
            out[c] = (s0 + s1) + (s2 + s3);
        }
        CSYNC();
    };

    Cmul(Uv, cu);
    const T mu0 = p.mu0;
    bool hl[RC], hu[RC];
#pragma unroll
    for (int c = 0; c < RC; c++) {
        hl[c] = has(lo[c]);
        hu[c] = has(hi[c]);
        const T d = (hl[c] && hu[c]) ? T(0.01) * (hi[c] - lo[c]) : T(0.01) * fmax(fabs(hl[c] ? lo[c] : hi[c]), T(1));
        tl[c] = hl[c] ? fmax(cu[c] - lo[c], d) : T(1);
        tu[c] = hu[c] ? fmax(hi[c] - cu[c], d) : T(1);
        ll[c] = hl[c] ? mu0 * frcp(tl[c]) : T(0);
        lu[c] = hu[c] ? mu0 * frcp(tu[c]) : T(0);
    }
    auto sum = [](T a, T b) { return a + b; };
    auto vmin = [](T a, T b) { return fmin(a, b); };
    auto vmax = [](T a, T b) { return fmax(a, b); };
    T mu;
    {
        T s = 0;
#pragma unroll
        for (int c = 0; c < RC; c++) s += ll[c] * tl[c] + lu[c] * tu[c];
        mu = wred(s, sum) * p.inv_m;
    }

    T invd[UC];
#pragma unroll
    for (int c = 0; c < UC; c++) invd[c] = 0;
    T rres = 0;   // max |residual| (dual rd, primal rpl / rpu) at the current iterate
    int status = 2, iters = 0;
    const int ksteps = mxp >> 2;
    // element (chunk c) of a per-lane register array, chunk chosen by a wave-uniform index
    auto pick = [&](const T (&v)[UC], int c) {
        T x = v[0];
#pragma unroll
        for (int k = 1; k < UC; k++) x = (c == k) ? v[k] : x;
        return x;
    };

    // Newton solve for complementarity targets (rcl, rcu): dU -> Sv, C dU, dt, dlambda.
    // itl / itu: reciprocal slacks of the iterate
    T rd[UC], rpl[RC], rpu[RC], itl[RC], itu[RC];
    auto solve = [&](const T (&rcl)[RC], const T (&rcu)[RC], T (&cd)[RC], T (&dtl)[RC], T (&dtu)[RC], T (&dll)[RC],
                     T (&dlu)[RC]) {
        T w[RC], b[UC];
#pragma unroll
        for (int c = 0; c < RC; c++)
            w[c] = (hl[c] ? (rcl[c] + ll[c] * rpl[c]) * itl[c] : T(0)) - (hu[c] ? (rcu[c] + lu[c] * rpu[c]) * itu[c] : T(0));
        CTmul(w, b);
#pragma unroll
        for (int c = 0; c < UC; c++) b[c] = (lane + 64 * c < n) ? -(rd[c] + b[c]) : T(0);
        // forward substitution L y = b: per 16-column block the lanes' L entries are loaded
        // into registers at once, then column j is broadcast by readlane
        for (int J = 0; J < nb; J++) {
            T pn[UC][16];
#pragma unroll
            for (int c = 0; c < UC; c++) {
                const int i = lane + 64 * c;
                const bool own = i >= 16 * J && i < np;
                const int I = own ? i >> 4 : J;
                const T *src = tile(I, J) + (i & 15);
#pragma unroll
                for (int kk = 0; kk < 16; kk++) pn[c][kk] = own ? src[kk * TP] : T(0);
            }
#pragma unroll
            for (int jj = 0; jj < 16; jj++) {
                const int j = 16 * J + jj, cj = j >> 6;
                const T y = rl(pick(b, cj) * pick(invd, cj), j & 63);
#pragma unroll
                for (int c = 0; c < UC; c++) {
                    const int i = lane + 64 * c;
                    b[c] = (i == j) ? y : ((i > j) ? fma(-pn[c][jj], y, b[c]) : b[c]);
                }
            }
        }
        // backward substitution L' x = y: lane i needs L(j, i) of the block's rows j
        for (int J = nb - 1; J >= 0; J--) {
            T pr[UC][16];
#pragma unroll
            for (int c = 0; c < UC; c++) {
                const int i = lane + 64 * c;
                const bool own = (i >> 4) <= J;
                const T *src = tile(J, own ? i >> 4 : 0) + (i & 15) * TP;
#pragma unroll
                for (int kk = 0; kk < 16; kk++) pr[c][kk] = own ? src[kk] : T(0);
            }
#pragma unroll
            for (int jj = 15; jj >= 0; jj--) {
                const int j = 16 * J + jj, cj = j >> 6;
                const T x = rl(pick(b, cj) * pick(invd, cj), j & 63);
#pragma unroll
                for (int c = 0; c < UC; c++) {
                    const int i = lane + 64 * c;
                    b[c] = (i == j) ? x : ((i < j) ? fma(-pr[c][jj], x, b[c]) : b[c]);
                }
            }
        }
#pragma unroll
        for (int c = 0; c < UC; c++) {
            const int i = lane + 64 * c;
            if (i < np) Sv[i] = b[c];
        }
        CSYNC();
        Cmul(Sv, cd);
#pragma unroll
        for (int c = 0; c < RC; c++) {
            dtl[c] = hl[c] ? cd[c] + rpl[c] : T(0);
            dtu[c] = hu[c] ? -cd[c] + rpu[c] : T(0);
            dll[c] = hl[c] ? (-rcl[c] - ll[c] * dtl[c]) * itl[c] : T(0);
            dlu[c] = hu[c] ? (-rcu[c] - lu[c] * dtu[c]) * itu[c] : T(0);
        }
    };
    // largest primal (slacks) and dual (multipliers) steps that keep them non-negative
    auto max_step = [&](const T (&dtl)[RC], const T (&dtu)[RC], const T (&dll)[RC], const T (&dlu)[RC], T &ap, T &ad) {
        ap = 1;
        ad = 1;
#pragma unroll
        for (int c = 0; c < RC; c++) {
            if (hl[c] && dtl[c] < T(0)) ap = fmin(ap, -tl[c] * frcp(dtl[c]));
            if (hu[c] && dtu[c] < T(0)) ap = fmin(ap, -tu[c] * frcp(dtu[c]));
            if (hl[c] && dll[c] < T(0)) ad = fmin(ad, -ll[c] * frcp(dll[c]));
            if (hu[c] && dlu[c] < T(0)) ad = fmin(ad, -lu[c] * frcp(dlu[c]));
        }
        ap = wred(ap, vmin);
        ad = wred(ad, vmin);
    };

    CT(0);
    for (int it = 0;; it++) {
        // ---- residuals at the current iterate: rd = H0 U + f - C' (lambda_l - lambda_u), primal
        {
            T w[RC], ct[UC];
#pragma unroll
            for (int c = 0; c < RC; c++) w[c] = ll[c] - lu[c];
            CTmul(w, ct);
#pragma unroll
            for (int c = 0; c < UC; c++) {
                const int i = lane + 64 * c;
                T s0 = 0, s1 = 0, s2 = 0, s3 = 0;
                if (i < n) {
                    const T *h = H0 + i;
                    int j = 0;
                    for (; j + 3 < n; j += 4) {
                        s0 = fma(h[j * n], Uv[j], s0);
                        s1 = fma(h[(j + 1) * n], Uv[j + 1], s1);
                        s2 = fma(h[(j + 2) * n], Uv[j + 2], s2);
                        s3 = fma(h[(j + 3) * n], Uv[j + 3], s3);
                    }
                    for (; j < n; j++) s0 = fma(h[j * n], Uv[j], s0);
                    s0 = ((s0 + s1) + (s2 + s3)) + f[c] - ct[c];
                }
                rd[c] = s0;
            }
            T m = 0;
#pragma unroll
            for (int c = 0; c < UC; c++) m = fmax(m, fabs(rd[c]));
#pragma unroll
            for (int c = 0; c < RC; c++) {
                rpl[c] = hl[c] ? cu[c] - lo[c] - tl[c] : T(0);
                rpu[c] = hu[c] ? hi[c] - cu[c] - tu[c] : T(0);
                m = fmax(m, fmax(fabs(rpl[c]), fabs(rpu[c])));
            }
            rres = wred(m, vmax);
        }
        const bool conv = mu <= p.tol_comp && rres <= p.tol_res;
        if (conv || !isfinite(mu) || !isfinite(rres)) {
            status = conv ? 0 : 4;
            iters = it;
            break;
        }
        if (it >= p.max_iter) {
            status = 2;
            iters = it;
            break;
        }
        CT(1);
        // ---- barrier Hessian of the rows
#pragma unroll
        for (int c = 0; c < RC; c++) {
            const int rho = lane + 64 * c;
            itl[c] = hl[c] ? frcp(tl[c]) : T(0);
            itu[c] = hu[c] ? frcp(tu[c]) : T(0);
            const T d = ll[c] * itl[c] + lu[c] * itu[c];
            if (rho < n) DU[rho] = d;
            else if (rho < mc) DX[rho - n] = d;
        }
        CSYNC();
        // ---- K = H0 + diag(D_u) + Gx' diag(D_x) Gx: lower tiles, MFMA over the x rows (two
        //      independent accumulation chains)
        for (int I = 0; I < nb; I++) {
            const int k0 = p.ks[I];
            for (int J = 0; J <= I; J++) {
                const T *h0 = p.H0t + (size_t)(I * (I + 1) / 2 + J) * 256;
                v4 acc, acc2 = {0, 0, 0, 0};
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const int row = M::row(lane, r);
                    T v = h0[c16 * 16 + row];
                    if (I == J && row == c16) v += DU[16 * I + row];
                    acc[r] = v;
                }
                const T *ga = G + (16 * I + c16) * ldg + q;
                const T *gb = G + (16 * J + c16) * ldg + q;
                const T *dx = DX + q;
                int s2 = k0;
                for (; s2 + 1 < ksteps; s2 += 2) {
                    const T a0 = ga[4 * s2], b0 = dx[4 * s2] * gb[4 * s2];
                    const T a1 = ga[4 * s2 + 4], b1 = dx[4 * s2 + 4] * gb[4 * s2 + 4];
                    acc = M::mma(a0, b0, acc);
                    acc2 = M::mma(a1, b1, acc2);
                }
                if (s2 < ksteps) acc = M::mma(ga[4 * s2], dx[4 * s2] * gb[4 * s2], acc);
                T *t = tile(I, J);
#pragma unroll
                for (int r = 0; r < 4; r++) t[c16 * TP + M::row(lane, r)] = acc[r] + acc2[r];
            }
        }
        CSYNC();
        CT(2);
        // ---- blocked Cholesky K = L L' in place (tiles): each 16-column panel is factorised in
        //      registers (lane = row, pivots and column entries broadcast by readlane), then the
        //      trailing tiles are updated with MFMA
        bool fail = false;
        for (int J = 0; J < nb; J++) {
            const int j0 = 16 * J;
            T pn[UC][16];
#pragma unroll
            for (int c = 0; c < UC; c++) {
                const int i = lane + 64 * c;
                const bool own = i >= j0 && i < np;
                const int I = own ? i >> 4 : J;
                const T *src = tile(I, J) + (i & 15);
#pragma unroll
                for (int kk = 0; kk < 16; kk++) pn[c][kk] = own ? src[kk * TP] : T(0);
            }
#pragma unroll
            for (int jj = 0; jj < 16; jj++) {
                const int j = j0 + jj, cj = j >> 6;
                T dsel[UC];
#pragma unroll
                for (int c = 0; c < UC; c++) dsel[c] = pn[c][jj];
                const T d = rl(pick(dsel, cj), j & 63);
                const bool real = j < n;
                const bool pd = d > T(0) || !real;
                fail |= !pd;
                const T rj = real ? frsq(pd ? d : T(1)) : T(0);
                T li[UC];
#pragma unroll
                for (int c = 0; c < UC; c++) {
                    const int i = lane + 64 * c;
                    if (i == j) invd[c] = rj;
                    li[c] = (i > j) ? pn[c][jj] * rj : ((i == j) ? d * rj : pn[c][jj]);
                    pn[c][jj] = li[c];
                }
#pragma unroll
                for (int kk = jj + 1; kk < 16; kk++) {
                    const int k = j0 + kk;
                    const T lkj = rl(pick(li, k >> 6), k & 63);
#pragma unroll
                    for (int c = 0; c < UC; c++) {
                        const int i = lane + 64 * c;
                        pn[c][kk] = (i >= k) ? fma(-li[c], lkj, pn[c][kk]) : pn[c][kk];
                    }
                }
            }
#pragma unroll
            for (int c = 0; c < UC; c++) {
                const int i = lane + 64 * c;
                if (i >= j0 && i < np) {
                    T *dst = tile(i >> 4, J) + (i & 15);
#pragma unroll
                    for (int kk = 0; kk < 16; kk++) dst[kk * TP] = pn[c][kk];
                }
            }
            CSYNC();
            for (int I = J + 1; I < nb; I++) {
                const T *la = tile(I, J);
                for (int I2 = J + 1; I2 <= I; I2++) {
                    const T *lb = tile(I2, J);
                    T *t = tile(I, I2);
                    v4 acc;
#pragma unroll
                    for (int r = 0; r < 4; r++) acc[r] = t[c16 * TP + M::row(lane, r)];
#pragma unroll
                    for (int s = 0; s < 4; s++) acc = M::mma(-la[(4 * s + q) * TP + c16], lb[(4 * s + q) * TP + c16], acc);
#pragma unroll
                    for (int r = 0; r < 4; r++) t[c16 * TP + M::row(lane, r)] = acc[r];
                }
            }
            CSYNC();
        }
        if (fail) {   // non-positive pivot: keep the iterate of the start of this iteration
            status = 4;
            iters = it;
            break;
        }
        CT(3);
        // ---- predictor (affine)
        T rcl[RC], rcu[RC], cd[RC], atl[RC], atu[RC], all_[RC], alu[RC];
#pragma unroll
        for (int c = 0; c < RC; c++) {
            rcl[c] = ll[c] * tl[c];
            rcu[c] = lu[c] * tu[c];
        }
        solve(rcl, rcu, cd, atl, atu, all_, alu);
        T ap, ad;
        max_step(atl, atu, all_, alu, ap, ad);
        T mu_aff;
        {
            T s = 0;
#pragma unroll
            for (int c = 0; c < RC; c++)
                s += (tl[c] + ap * atl[c]) * (ll[c] + ad * all_[c]) + (tu[c] + ap * atu[c]) * (lu[c] + ad * alu[c]);
            mu_aff = wred(s, sum) * p.inv_m;
        }
        const T sg = mu > T(0) ? fmax(mu_aff, T(0)) * frcp(mu) : T(0);
        const T smu = sg * sg * sg * mu;
        CT(4);
        // ---- corrector (Mehrotra)
#pragma unroll
        for (int c = 0; c < RC; c++) {
            rcl[c] = hl[c] ? ll[c] * tl[c] + atl[c] * all_[c] - smu : T(0);
            rcu[c] = hu[c] ? lu[c] * tu[c] + atu[c] * alu[c] - smu : T(0);
        }
        T dtl[RC], dtu[RC], dll[RC], dlu[RC];
        solve(rcl, rcu, cd, dtl, dtu, dll, dlu);
        CT(5);
        max_step(dtl, dtu, dll, dlu, ap, ad);
        ap = fmin(T(1), T(0.995) * ap);
        ad = fmin(T(1), T(0.995) * ad);
        // ---- step: separate primal and dual lengths (one common length stalls on some
        //      instances: mu cycles while the primal residual converges)
#pragma unroll
        for (int c = 0; c < UC; c++) {
            const int i = lane + 64 * c;
            if (i < n) Uv[i] = fma(ap, Sv[i], Uv[i]);
        }
        T s = 0;
#pragma unroll
        for (int c = 0; c < RC; c++) {
            cu[c] = fma(ap, cd[c], cu[c]);
            tl[c] = hl[c] ? fma(ap, dtl[c], tl[c]) : T(1);
            tu[c] = hu[c] ? fma(ap, dtu[c], tu[c]) : T(1);
            ll[c] = hl[c] ? fma(ad, dll[c], ll[c]) : T(0);
            lu[c] = hu[c] ? fma(ad, dlu[c], lu[c]) : T(0);
            s += ll[c] * tl[c] + lu[c] * tu[c];
        }
        mu = wred(s, sum) * p.inv_m;
        CSYNC();
    }

    CT(6);
    // ---- outputs: U, X = Phi x0 + d + Gamma U (row 0 is x0 itself)
    const int nrow = (p.N + 1) * nx;
    T *xo = p.xout + (size_t)inst * nrow;
    for (int r = lane; r < nrow; r += 64) {
        T s;
        if (r < nx) {
            s = x0[r];
        } else {
            s = p.dall[r];
            for (int a2 = 0; a2 < nx; a2++) s = fma(p.Phall[(size_t)a2 * nrow + r], x0[a2], s);
            const int nc = (r / nx) * nu;   // x_k depends on u_0 .. u_{k-1}
            T s1 = 0;
            int j = 0;
            for (; j + 1 < nc; j += 2) {
                s = fma(p.Gall[(size_t)j * nrow + r], Uv[j], s);
                s1 = fma(p.Gall[(size_t)(j + 1) * nrow + r], Uv[j + 1], s1);
            }
            if (j < nc) s = fma(p.Gall[(size_t)j * nrow + r], Uv[j], s);
            s += s1;
        }
        xo[r] = s;
    }
    T *uo = p.uout + (size_t)inst * n;
    for (int i = lane; i < n; i += 64) uo[i] = Uv[i];
    CT(7);
    if (lane == 0) {
        p.status[inst] = status;
        p.iters[inst] = iters;
#ifdef NMPC_COND_TIMING
        if (p.cycles)
            for (int j = 0; j < 8; j++) p.cycles[(size_t)inst * 9 + j] = ct_acc[j];
#endif
    }
}

}  // namespace cond

template <typename T, int RC, int UC>
static hipError_t launch_cond_rcuc(const CondParams<T> &p, int wpb, size_t lds, hipStream_t s)
{
    const int blocks = (p.B + wpb - 1) / wpb;
    if (lds > 64 * 1024) {   // dynamic LDS beyond 64 KB must be enabled per kernel
        static hipError_t set = hipFuncSetAttribute((const void *)cond::cond_ipm_kernel<T, RC, UC>,
                                                    hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (set != hipSuccess) return set;
    }
    NMPC_LAUNCH((cond::cond_ipm_kernel<T, RC, UC>), dim3(blocks), dim3(64 * wpb), lds, s, p);
    return hipGetLastError();
}

template <typename T>
hipError_t cond_launch(const CondParams<T> &p, int wpb, size_t lds, hipStream_t s)
{
    const int mc = p.n + p.mx;
    if (p.n <= 64) {
        if (mc <= 128) return launch_cond_rcuc<T, 2, 1>(p, wpb, lds, s);
        if (mc <= 256) return launch_cond_rcuc<T, 4, 1>(p, wpb, lds, s);
        if (mc <= 512) return launch_cond_rcuc<T, 8, 1>(p, wpb, lds, s);
    } else if (p.n <= 128) {
        if (mc <= 256) return launch_cond_rcuc<T, 4, 2>(p, wpb, lds, s);
        if (mc <= 512) return launch_cond_rcuc<T, 8, 2>(p, wpb, lds, s);
    }
    return hipErrorInvalidValue;
}

// LDS elements of one wavefront (its K tiles and vectors); the shared part is
// 16 nb ldg + round4(n^2) (Gx and H0)
template <typename T>
size_t cond_wave_elems(int nb, int ldg)
{
    const size_t e = (size_t)nb * (nb + 1) / 2 * cond::TS + 3 * (size_t)(16 * nb) + 2 * (size_t)ldg;
    return (e + 3) & ~(size_t)3;
}

template hipError_t cond_launch<double>(const CondParams<double> &, int, size_t, hipStream_t);
template hipError_t cond_launch<float>(const CondParams<float> &, int, size_t, hipStream_t);
template size_t cond_wave_elems<double>(int, int);
template size_t cond_wave_elems<float>(int, int);

}  // namespace nmpc
