// nmpc_ipm_lpi.hip — batched box-constrained LQ-OCP solver, lane-per-instance layout (gfx950).
//
// Same problem and algorithm as nmpc_ipm_lpc.hip (one AcadosOcpSolver.solve() of
// src/force_model/controller.py:32 / src/jerk_model/controller.py:33: SQP-GN on an LTI /
// LINEAR_LS / box-constrained OCP == one QP, solved by a Mehrotra predictor-corrector IPM with
// a backward Riccati recursion per Newton system, four fused stage sweeps per iteration:
//   A  backward Riccati factorisation; applies the previous step lazily, forms Sigma,
//      g = H z + G yref, the dynamics residual and mu of the updated iterate on the fly;
//   B  forward predictor; ratio test and the closed-form mu_aff sums on the fly;
//   C  backward corrector vector; corrector right-hand side on the fly;
//   D  forward corrector; step length on the fly),
// mapped for small models (force nx=4 nu=2, jerk nx=6 nu=2): ONE LANE owns one instance and
// runs the whole stage recursion in its registers — no LDS exchange, no cross-lane reduction,
// nothing but the per-stage records in a wavefront-private scratch block (word w of stage k of
// lane l at (k NW + w) W + l: every access of a wavefront is one contiguous run).
// A small model's stage is a few hundred FMAs with plenty of independent work, so one lane's
// instruction stream is short; the host packs W = ceil(B / 1024) instances per wavefront (the
// other lanes idle) so that every SIMD of the GPU gets about one wavefront: the whole batch
// then takes about the time of ONE instance's stream, where the lane-per-component and
// wavefront-per-instance kernels pay an LDS round trip per stage sweep step.
// Model constants ([A B], H, He, bounds) are read from LDS with wave-uniform addresses; the
// model-structure template SP skips the structural zeros of [A B] (nmpc_lpc_geom.h).

#include <hip/hip_runtime.h>

#include "nmpc_internal.h"
#include "nmpc_lpc_geom.h"

#define NMPC_LPI_COMMA ,

namespace nmpc {
namespace lpi {

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
__device__ __forceinline__ double rcp_raw(double x) { return __builtin_amdgcn_rcp(x); }
__device__ __forceinline__ float rcp_raw(float x) { return __builtin_amdgcn_rcpf(x); }

template <typename T>
__device__ __forceinline__ bool has(T b)
{
    return fabs(b) < T(1e20);
}

__host__ __device__ constexpr int tri(int i, int j) { return i * (i + 1) / 2 + j; }

// scratch words per stage: elements z, lambda_l, lambda_u, G yref, dz_aff, dz (NZ each), then the
// stage record K (NU x NX), kff (NU), P re (NX), F_uu^{-1} (packed lower, NU(NU+1)/2)
template <int NX, int NU>
struct Words {
    static constexpr int NZ = NX + NU;
    static constexpr int Z = 0, LL = NZ, LU = 2 * NZ, GC = 3 * NZ, DZA = 4 * NZ, DZ = 5 * NZ;
    static constexpr int K = 6 * NZ, KFF = K + NU * NX, PR = KFF + NU, FI = PR + NX;
    static constexpr int NW = FI + NU * (NU + 1) / 2;
};

template <typename T, int NX, int NU, class SP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void ipm_lpi_kernel(IpmParams<T> p)
{
    constexpr int NZ = NX + NU, NUT = NU * (NU + 1) / 2;
    using Wd = Words<NX, NU>;
    constexpr int NW = Wd::NW;
    // ---- model constants in LDS (wave-uniform reads)
    __shared__ T sAB[NX * NZ], sH[NZ * NZ], sHe[NX * NX], sc[NX], slb[3 * NZ], sub[3 * NZ];
    for (int e = threadIdx.x; e < NX * NZ; e += blockDim.x) sAB[e] = p.AB[e];
    for (int e = threadIdx.x; e < NZ * NZ; e += blockDim.x) sH[e] = p.H[e];
    for (int e = threadIdx.x; e < NX * NX; e += blockDim.x) sHe[e] = p.He[e];
    for (int e = threadIdx.x; e < NX; e += blockDim.x) sc[e] = p.c[e];
    for (int e = threadIdx.x; e < 3 * NZ; e += blockDim.x) {
        slb[e] = p.lbnd[e];
        sub[e] = p.ubnd[e];
    }
    __syncthreads();
    const int W = p.ipw;   // instances per wavefront (lanes 0 .. W-1)
    const int lane = threadIdx.x & 63;
    const long long wave = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const long long slot = wave * W + lane;
    if (lane >= W || slot >= p.B) return;
    const int inst = (int)slot;
    const int N = p.N;
    // scratch: each wavefront owns one contiguous block of (N+1) NW W elements, stage-major, word
    // w of stage k of lane l at (k NW + w) W + l: a stage's words are a few dense cache lines that
    // stay in the XCD's L2 (instance-major interleaving over the whole batch put every lane's word
    // in a line shared with 15 other instances, most of them on other XCDs: 16x the L2 footprint).
    // The 32-bit offsets use W re-obscured per stage (fresh()): hoisting all NW offsets word * W
    // out of the stage loops made 70+ loop-invariant registers and spilled the stage state.
    int So = W;
    T *scr = p.scratch + (size_t)wave * (size_t)(N + 1) * NW * W + lane;
    auto ld = [&](int k, int w) { return scr[(unsigned)((k * NW + w) * So)]; };
    auto st = [&](int k, int w, T v) { scr[(unsigned)((k * NW + w) * So)] = v; };
    // the model constants are re-read from LDS at every stage: co is made opaque once per stage
    // (`fresh()`), so the compiler cannot hoist ~100 loop-invariant constants into registers
    // (that spilled the lane's stage state to scratch)
    int co = 0;
    auto fresh = [&]() {
        asm volatile("" : "+v"(co));
        asm volatile("" : "+v"(So));
    };
    auto LB = [&](int k, int i) { return slb[co + (k == 0 ? 0 : (k == N ? 2 : 1)) * NZ + i]; };
    auto UB = [&](int k, int i) { return sub[co + (k == 0 ? 0 : (k == N ? 2 : 1)) * NZ + i]; };
    auto ab = [&](int l, int c) { return sAB[co + l * NZ + c]; };
    const T *yref = p.yref + (size_t)inst * ((size_t)N * p.ny + p.ny_e);
    const T *x0 = p.x0 + (size_t)inst * NX;

    // g = H z + gc (stage k < N: NZ comps, k = N: NX comps)
    auto grad = [&](int k, const T (&z)[NZ], const T (&gc)[NZ], T (&g)[NZ]) {
        if (k < N) {
#pragma unroll
            for (int a = 0; a < NZ; a++) {
                T s = gc[a];
                if (SP::hdiag) {
                    s = fma(sH[co + a * NZ + a], z[a], s);
                } else {
#pragma unroll
                    for (int b = 0; b < NZ; b++) s = fma(sH[co + a * NZ + b], z[b], s);
                }
                g[a] = s;
            }
        } else {
#pragma unroll
            for (int a = 0; a < NX; a++) {
                T s = gc[a];
                if (SP::hdiag) {
                    s = fma(sHe[co + a * NX + a], z[a], s);
                } else {
#pragma unroll
                    for (int b = 0; b < NX; b++) s = fma(sHe[co + a * NX + b], z[b], s);
                }
                g[a] = s;
            }
#pragma unroll
            for (int a = NX; a < NZ; a++) g[a] = 0;
        }
    };
    // [A B] z + c (x_{k+1} predicted from stage k)
    auto dyn = [&](const T (&z)[NZ], T (&out)[NX]) {
#pragma unroll
        for (int i = 0; i < NX; i++) {
            T s = sc[co + i];
#pragma unroll
            for (int j = 0; j < NZ; j++)
                if (SP::ab(i, j)) s = fma(ab(i, j), z[j], s);
            out[i] = s;
        }
    };

    // ------------------------------------------------------------------ initial point
    T r0 = 0, mu = 0;
    {
        T xprev[NX];   // [A B] z_{k-1} + c
#pragma unroll
        for (int i = 0; i < NX; i++) xprev[i] = 0;
        #pragma unroll 1
        for (int k = 0; k <= N; k++) {
            fresh();
            const int ns = k < N ? NZ : NX;
            const T *yk = yref + (size_t)k * p.ny;
            T z[NZ], gc[NZ], l_[NZ], u_[NZ];
#pragma unroll
            for (int a = 0; a < NZ; a++) {
                T s = 0;
                if (a < ns) {
                    if (k < N) {
                        for (int j = 0; j < p.ny; j++) s = fma(p.G[a * p.ny + j], yk[j], s);
                    } else {
                        for (int j = 0; j < p.ny_e; j++) s = fma(p.Ge[a * p.ny_e + j], yk[j], s);
                    }
                }
                gc[a] = s;
                T v = 0, ll = 0, lu = 0;
                if (a < ns) {
                    if (k == 0 && a < NX) {
                        v = x0[a];
                    } else {
                        v = p.yref_is_z ? yk[a] : T(0);
                        const T lb = LB(k, a), ub = UB(k, a);
                        const bool hl = has(lb), hu = has(ub);
                        if (hl && hu) {
                            const T d = T(0.01) * (ub - lb);
                            v = a >= NX ? T(0.5) * (lb + ub) : v;   // boxed inputs start mid-box
                            v = fmin(fmax(v, lb + d), ub - d);
                        } else if (hl) {
                            v = fmax(v, lb + T(0.01) * fmax(fabs(lb), T(1)));
                        } else if (hu) {
                            v = fmin(v, ub - T(0.01) * fmax(fabs(ub), T(1)));
                        }
                        if (hl) ll = p.mu0 / (v - lb);
                        if (hu) lu = p.mu0 / (ub - v);
                    }
                }
                z[a] = v;
                l_[a] = ll;
                u_[a] = lu;
            }
            T g[NZ];
            grad(k, z, gc, g);
#pragma unroll
            for (int a = 0; a < NZ; a++) {
                if (a < ns && !(k == 0 && a < NX)) {
                    r0 = fmax(r0, fabs(g[a] - l_[a] + u_[a]));
                    if (l_[a] > T(0)) mu += l_[a] * (z[a] - LB(k, a));
                    if (u_[a] > T(0)) mu += u_[a] * (UB(k, a) - z[a]);
                }
                st(k, Wd::Z + a, z[a]);
                st(k, Wd::LL + a, l_[a]);
                st(k, Wd::LU + a, u_[a]);
                st(k, Wd::GC + a, gc[a]);
                st(k, Wd::DZ + a, T(0));
                st(k, Wd::DZA + a, T(0));
            }
            if (k > 0)
#pragma unroll
                for (int i = 0; i < NX; i++) r0 = fmax(r0, fabs(xprev[i] - z[i]));
            if (k < N) dyn(z, xprev);
        }
    }
    mu *= p.inv_m;
    const T m_bounds = T(1) / p.inv_m;
#ifdef NMPC_SWEEP_TIMING
    // experiment builds: clock cycles per sweep (A -> slot 1, B -> 2, C -> 5, D -> 6, total 8)
    unsigned long long tcy[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tmark = __builtin_amdgcn_s_memtime();
    const unsigned long long tstart = tmark;
    auto tick = [&](int slot) {
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        tcy[slot] += t - tmark;
        tmark = t;
    };
#define LPI_TICK(s) tick(s)
#else
#define LPI_TICK(s) ((void)0)
#endif

    T theta = 1, alpha = 0, smu = 0;
    bool pending = false, fail = false;
    int status = 2, iters = 0;

    // stage element state
    struct El {
        T z[NZ], ll[NZ], lu[NZ], gc[NZ], dz[NZ], dza[NZ];
    };
    auto load_el = [&](int k, El &e, bool steps) {
#pragma unroll
        for (int a = 0; a < NZ; a++) {
            e.z[a] = ld(k, Wd::Z + a);
            e.ll[a] = ld(k, Wd::LL + a);
            e.lu[a] = ld(k, Wd::LU + a);
            e.gc[a] = ld(k, Wd::GC + a);
            if (steps) {
                e.dz[a] = ld(k, Wd::DZ + a);
                e.dza[a] = ld(k, Wd::DZA + a);
            }
        }
    };

    for (int it = 0;; it++) {
        // ============================ A: lazy step + mu + backward Riccati factorisation
        T P[NX][NX], pv[NX], znext[NX];
        T musum = 0;
        {
            El e;
            load_el(N, e, true);
            // lazy application of the previous step to stage k's elements
            auto lazy = [&](int k, El &q) {
                const int ns = k < N ? NZ : NX;
#pragma unroll
                for (int a = 0; a < NZ; a++) {
                    if (a >= ns || (k == 0 && a < NX)) continue;
                    const T lb = LB(k, a), ub = UB(k, a);
                    if (pending) {
                        const T tl = q.z[a] - lb, tu = ub - q.z[a];
                        if (q.ll[a] > T(0)) {
                            const T itl = frcp(tl), dla = -q.ll[a] * (T(1) + q.dza[a] * itl);
                            q.ll[a] += alpha * ((smu - q.ll[a] * tl - dla * q.dza[a] - q.ll[a] * q.dz[a]) * itl);
                        }
                        if (q.lu[a] > T(0)) {
                            const T itu = frcp(tu), dla = -q.lu[a] * (T(1) - q.dza[a] * itu);
                            q.lu[a] += alpha * ((smu - q.lu[a] * tu + dla * q.dza[a] + q.lu[a] * q.dz[a]) * itu);
                        }
                        q.z[a] += alpha * q.dz[a];
                    }
                    if (q.ll[a] > T(0)) musum += q.ll[a] * (q.z[a] - lb);
                    if (q.lu[a] > T(0)) musum += q.lu[a] * (ub - q.z[a]);
                }
                if (pending) {
#pragma unroll
                    for (int a = 0; a < NZ; a++) {
                        st(k, Wd::Z + a, q.z[a]);
                        st(k, Wd::LL + a, q.ll[a]);
                        st(k, Wd::LU + a, q.lu[a]);
                    }
                }
            };
            auto sigma = [&](int k, const El &q, int a) {
                const T lb = LB(k, a), ub = UB(k, a);
                T s = 0;
                if (q.ll[a] > T(0)) s += q.ll[a] * frcp(q.z[a] - lb);
                if (q.lu[a] > T(0)) s += q.lu[a] * frcp(ub - q.z[a]);
                return s;
            };
            lazy(N, e);
            {
                T g[NZ];
                grad(N, e.z, e.gc, g);
#pragma unroll
                for (int i = 0; i < NX; i++) {
#pragma unroll
                    for (int j = 0; j < NX; j++) P[i][j] = sHe[co + i * NX + j];
                    P[i][i] += sigma(N, e, i);
                    pv[i] = g[i];
                    znext[i] = e.z[i];
                }
            }
            #pragma unroll 1
            for (int k = N - 1; k >= 0; k--) {
                fresh();
                El q;
                load_el(k, q, true);
                lazy(k, q);
                T g[NZ], re[NX];
                grad(k, q.z, q.gc, g);
                dyn(q.z, re);
#pragma unroll
                for (int i = 0; i < NX; i++) {
                    re[i] -= znext[i];
                    znext[i] = q.z[i];
                }
                // Pr = P re, v = Pr + p
                T pr[NX], v[NX];
#pragma unroll
                for (int i = 0; i < NX; i++) {
                    T s = 0;
#pragma unroll
                    for (int j = 0; j < NX; j++) s = fma(P[i][j], re[j], s);
                    pr[i] = s;
                    v[i] = s + pv[i];
                }
                // F = [A B]' P [A B] + H + Sigma (lower triangle), column by column: M(:, b) = P [A B](:, b)
                // is formed and consumed at once; h = [A B]' v + g
                T F[NZ][NZ], h[NZ];
#pragma unroll
                for (int b = 0; b < NZ; b++) {
                    T mcol[NX];
#pragma unroll
                    for (int i = 0; i < NX; i++) {
                        T s = 0;
#pragma unroll
                        for (int l = 0; l < NX; l++)
                            if (SP::ab(l, b)) s = fma(P[i][l], ab(l, b), s);
                        mcol[i] = s;
                    }
#pragma unroll
                    for (int a = b; a < NZ; a++) {
                        T s = SP::hdiag ? (a == b ? sH[co + a * NZ + a] : T(0)) : sH[co + a * NZ + b];
#pragma unroll
                        for (int l = 0; l < NX; l++)
                            if (SP::ab(l, a)) s = fma(ab(l, a), mcol[l], s);
                        F[a][b] = s;
                    }
                }
#pragma unroll
                for (int a = 0; a < NZ; a++) {
                    T s = g[a];
#pragma unroll
                    for (int l = 0; l < NX; l++)
                        if (SP::ab(l, a)) s = fma(ab(l, a), v[l], s);
                    h[a] = s;
                    if (!(k == 0 && a < NX)) F[a][a] += sigma(k, q, a);
                }
                // F_uu = L L' (packed, inverse diagonal)
                T lf[NUT];
#pragma unroll
                for (int i = 0; i < NU; i++)
#pragma unroll
                    for (int j = 0; j <= i; j++) {
                        T s_ = F[NX + i][NX + j];
#pragma unroll
                        for (int l = 0; l < j; l++) s_ = fma(-lf[tri(i, l)], lf[tri(j, l)], s_);
                        if (i == j) {
                            const bool pd = s_ > T(0);
                            fail |= !pd;
                            lf[tri(i, i)] = frsq(pd ? s_ : T(1));
                        } else {
                            lf[tri(i, j)] = s_ * lf[tri(j, j)];
                        }
                    }
                // F_uu^{-1} = L^{-T} L^{-1} (columns e_u), K = -F_uu^{-1} F_ux, kff = -F_uu^{-1} h_u
                T Fi[NU][NU];
#pragma unroll
                for (int cidx = 0; cidx < NU; cidx++) {
                    T y[NU], x[NU];
#pragma unroll
                    for (int i = 0; i < NU; i++) {
                        T s_ = (i == cidx) ? T(1) : T(0);
#pragma unroll
                        for (int l = 0; l < i; l++) s_ = fma(-lf[tri(i, l)], y[l], s_);
                        y[i] = s_ * lf[tri(i, i)];
                    }
#pragma unroll
                    for (int i = NU - 1; i >= 0; i--) {
                        T s_ = y[i];
#pragma unroll
                        for (int l = i + 1; l < NU; l++) s_ = fma(-lf[tri(l, i)], x[l], s_);
                        x[i] = s_ * lf[tri(i, i)];
                    }
#pragma unroll
                    for (int i = 0; i < NU; i++) Fi[i][cidx] = x[i];
                }
                T Kg[NU][NX], kff[NU];
#pragma unroll
                for (int u = 0; u < NU; u++) {
#pragma unroll
                    for (int j = 0; j < NX; j++) {
                        T s_ = 0;
#pragma unroll
                        for (int l = 0; l < NU; l++) s_ = fma(-Fi[u][l], F[NX + l][j], s_);
                        Kg[u][j] = s_;
                    }
                    T s_ = 0;
#pragma unroll
                    for (int l = 0; l < NU; l++) s_ = fma(-Fi[u][l], h[NX + l], s_);
                    kff[u] = s_;
                }
                // P <- F_xx + F_xu K (symmetric), p <- h_x + K' h_u
#pragma unroll
                for (int i = 0; i < NX; i++) {
#pragma unroll
                    for (int j = 0; j <= i; j++) {
                        T s_ = F[i][j];
#pragma unroll
                        for (int u = 0; u < NU; u++) s_ = fma(F[NX + u][i], Kg[u][j], s_);
                        P[i][j] = s_;
                        P[j][i] = s_;
                    }
                    T s_ = h[i];
#pragma unroll
                    for (int u = 0; u < NU; u++) s_ = fma(Kg[u][i], h[NX + u], s_);
                    pv[i] = s_;
                }
                // stage record
#pragma unroll
                for (int u = 0; u < NU; u++) {
#pragma unroll
                    for (int j = 0; j < NX; j++) st(k, Wd::K + u * NX + j, Kg[u][j]);
                    st(k, Wd::KFF + u, kff[u]);
                }
#pragma unroll
                for (int i = 0; i < NX; i++) st(k, Wd::PR + i, pr[i]);
#pragma unroll
                for (int i = 0; i < NU; i++)
#pragma unroll
                    for (int j = 0; j <= i; j++) st(k, Wd::FI + tri(i, j), Fi[i][j]);
            }
        }
        pending = false;
        mu = musum * p.inv_m;
        LPI_TICK(1);
        // ---- termination (the iterate is the one reached after `it` steps)
        const bool conv = mu <= p.tol_comp && theta * r0 <= p.tol_res;
        const bool bad = !isfinite(mu) || !isfinite(theta);
        if (conv || bad) {
            status = conv && !bad ? 0 : 4;
            iters = it;
            break;
        }
        if (fail) {   // non-positive pivot: the iterate of the start of this iteration is kept
            status = 4;
            iters = it;
            break;
        }
        if (it >= p.max_iter) {
            status = 2;
            iters = it;
            break;
        }

        // ============================ B / D: forward sweeps
        // corr = false: predictor dz_aff with the ratio test and mu_aff sums;
        // corr = true: corrector dz with the step length ratio test
        auto forward = [&](bool corr, T &s_min, T &s_a, T &s_b) {
            s_min = 1;
            s_a = s_b = 0;
            T dx[NX];
#pragma unroll
            for (int i = 0; i < NX; i++) dx[i] = 0;
            const int dst = corr ? Wd::DZ : Wd::DZA;
            auto stats = [&](int k, const T (&z)[NZ], const T (&lv)[NZ], const T (&uv)[NZ], const T (&dz)[NZ],
                             const T (&dza)[NZ]) {
                const int ns = k < N ? NZ : NX;
#pragma unroll
                for (int a = 0; a < NZ; a++) {
                    if (a >= ns || (k == 0 && a < NX)) continue;
                    const T lb = LB(k, a), ub = UB(k, a);
                    const bool vl = lv[a] > T(0), vu = uv[a] > T(0);
                    const T tl = z[a] - lb, tu = ub - z[a];
                    if (!corr) {
                        const T itl = rcp_raw(tl), itu = rcp_raw(tu);
                        const T al = dz[a] * itl, au = dz[a] * itu;
                        if (vl) s_min = fmax(s_min, fmax(-al, T(1) + al));
                        if (vu) s_min = fmax(s_min, fmax(au, T(1) - au));
                        s_a += (vl ? lv[a] * tl : T(0)) + (vu ? uv[a] * tu : T(0));
                        s_b += (vl ? lv[a] * dz[a] * (tl + dz[a]) * itl : T(0)) +
                               (vu ? uv[a] * dz[a] * (dz[a] - tu) * itu : T(0));
                    } else {
                        const T itl = frcp(tl), itu = frcp(tu);
                        const T dlal = -lv[a] * (T(1) + dza[a] * itl), dlau = -uv[a] * (T(1) - dza[a] * itu);
                        const T dll = (smu - lv[a] * tl - dlal * dza[a] - lv[a] * dz[a]) * itl;
                        const T dlu = (smu - uv[a] * tu + dlau * dza[a] + uv[a] * dz[a]) * itu;
                        if (vl && dz[a] < T(0)) s_min = fmin(s_min, -tl * rcp_raw(dz[a]));
                        if (vl && dll < T(0)) s_min = fmin(s_min, -lv[a] * rcp_raw(dll));
                        if (vu && dz[a] > T(0)) s_min = fmin(s_min, tu * rcp_raw(dz[a]));
                        if (vu && dlu < T(0)) s_min = fmin(s_min, -uv[a] * rcp_raw(dlu));
                    }
                }
            };
            #pragma unroll 1
            for (int k = 0; k < N; k++) {
                fresh();
                T z[NZ], lv[NZ], uv[NZ], dza[NZ], kf[NU], Kg[NU][NX], zn[NX];
#pragma unroll
                for (int a = 0; a < NZ; a++) {
                    z[a] = ld(k, Wd::Z + a);
                    lv[a] = ld(k, Wd::LL + a);
                    uv[a] = ld(k, Wd::LU + a);
                    dza[a] = corr ? ld(k, Wd::DZA + a) : T(0);
                }
#pragma unroll
                for (int u = 0; u < NU; u++) {
                    kf[u] = ld(k, Wd::KFF + u);
#pragma unroll
                    for (int j = 0; j < NX; j++) Kg[u][j] = ld(k, Wd::K + u * NX + j);
                }
#pragma unroll
                for (int i = 0; i < NX; i++) zn[i] = ld(k + 1, Wd::Z + i);
                T dz[NZ];
#pragma unroll
                for (int i = 0; i < NX; i++) dz[i] = dx[i];
#pragma unroll
                for (int u = 0; u < NU; u++) {
                    T s_ = kf[u];
#pragma unroll
                    for (int j = 0; j < NX; j++) s_ = fma(Kg[u][j], dx[j], s_);
                    dz[NX + u] = s_;
                }
#pragma unroll
                for (int a = 0; a < NZ; a++) st(k, dst + a, dz[a]);
                stats(k, z, lv, uv, dz, dza);
                // dx_{k+1} = [A B] (z_k + dz_k) + c - z_{k+1}  (residual folded in)
                T zz[NZ], xn[NX];
#pragma unroll
                for (int a = 0; a < NZ; a++) zz[a] = z[a] + dz[a];
                dyn(zz, xn);
#pragma unroll
                for (int i = 0; i < NX; i++) dx[i] = xn[i] - zn[i];
            }
            {
                T z[NZ], lv[NZ], uv[NZ], dza[NZ], dz[NZ];
#pragma unroll
                for (int a = 0; a < NZ; a++) {
                    z[a] = a < NX ? ld(N, Wd::Z + a) : T(0);
                    lv[a] = a < NX ? ld(N, Wd::LL + a) : T(0);
                    uv[a] = a < NX ? ld(N, Wd::LU + a) : T(0);
                    dza[a] = (corr && a < NX) ? ld(N, Wd::DZA + a) : T(0);
                    dz[a] = a < NX ? dx[a] : T(0);
                }
#pragma unroll
                for (int i = 0; i < NX; i++) st(N, dst + i, dx[i]);
                stats(N, z, lv, uv, dz, dza);
            }
        };

        // ============================ B: forward predictor
        T a_inv, S0, S2;
        forward(false, a_inv, S0, S2);
        const T a_aff = frcp(a_inv);
        const T mu_aff = ((T(1) - a_aff) * S0 - a_aff * a_aff * S2) * p.inv_m;
        const T sgm = mu > T(0) ? fmax(mu_aff, T(0)) * frcp(mu) : T(0);
        smu = sgm * sgm * sgm * mu;
        LPI_TICK(2);

        // ============================ C: backward corrector vector
        {
            auto ghat = [&](int k, int a, const T (&z)[NZ], const T (&lv)[NZ], const T (&uv)[NZ], const T (&dza)[NZ],
                            T g) {
                if (k == 0 && a < NX) return g;
                const T lb = LB(k, a), ub = UB(k, a);
                const T tl = z[a] - lb, tu = ub - z[a], itl = frcp(tl), itu = frcp(tu);
                const T dll = -lv[a] * (T(1) + dza[a] * itl), dlu = -uv[a] * (T(1) - dza[a] * itu);
                if (lv[a] > T(0)) g += (dll * dza[a] - smu) * itl;
                if (uv[a] > T(0)) g += (dlu * dza[a] + smu) * itu;
                return g;
            };
            auto load_c = [&](int k, T (&z)[NZ], T (&lv)[NZ], T (&uv)[NZ], T (&gc)[NZ], T (&dza)[NZ]) {
                const int ns = k < N ? NZ : NX;
#pragma unroll
                for (int a = 0; a < NZ; a++) {
                    const bool in = a < ns;
                    z[a] = in ? ld(k, Wd::Z + a) : T(0);
                    lv[a] = in ? ld(k, Wd::LL + a) : T(0);
                    uv[a] = in ? ld(k, Wd::LU + a) : T(0);
                    gc[a] = in ? ld(k, Wd::GC + a) : T(0);
                    dza[a] = in ? ld(k, Wd::DZA + a) : T(0);
                }
            };
            T z[NZ], lv[NZ], uv[NZ], gc[NZ], dza[NZ], g[NZ];
            load_c(N, z, lv, uv, gc, dza);
            grad(N, z, gc, g);
            T pvv[NX];
#pragma unroll
            for (int i = 0; i < NX; i++) pvv[i] = ghat(N, i, z, lv, uv, dza, g[i]);
            #pragma unroll 1
            for (int k = N - 1; k >= 0; k--) {
                fresh();
                load_c(k, z, lv, uv, gc, dza);
                T pr[NX], Kg[NU][NX], Fi[NU][NU];
#pragma unroll
                for (int i = 0; i < NX; i++) pr[i] = ld(k, Wd::PR + i);
#pragma unroll
                for (int u = 0; u < NU; u++)
#pragma unroll
                    for (int j = 0; j < NX; j++) Kg[u][j] = ld(k, Wd::K + u * NX + j);
#pragma unroll
                for (int i = 0; i < NU; i++)
#pragma unroll
                    for (int j = 0; j <= i; j++) Fi[i][j] = Fi[j][i] = ld(k, Wd::FI + tri(i, j));
                grad(k, z, gc, g);
                T v[NX], h[NZ];
#pragma unroll
                for (int i = 0; i < NX; i++) v[i] = pr[i] + pvv[i];
#pragma unroll
                for (int a = 0; a < NZ; a++) {
                    T s_ = ghat(k, a, z, lv, uv, dza, g[a]);
#pragma unroll
                    for (int l = 0; l < NX; l++)
                        if (SP::ab(l, a)) s_ = fma(ab(l, a), v[l], s_);
                    h[a] = s_;
                }
#pragma unroll
                for (int u = 0; u < NU; u++) {
                    T s_ = 0;
#pragma unroll
                    for (int l = 0; l < NU; l++) s_ = fma(-Fi[u][l], h[NX + l], s_);
                    st(k, Wd::KFF + u, s_);
                }
#pragma unroll
                for (int i = 0; i < NX; i++) {
                    T s_ = h[i];
#pragma unroll
                    for (int u = 0; u < NU; u++) s_ = fma(Kg[u][i], h[NX + u], s_);
                    pvv[i] = s_;
                }
            }
        }

        LPI_TICK(5);
        // ============================ D: forward corrector + step length
        T amax, dm1, dm2;
        forward(true, amax, dm1, dm2);
        alpha = fmin(T(1), T(0.995) * amax);
        pending = true;
        theta *= T(1) - alpha;
        (void)m_bounds;
        LPI_TICK(6);
    }

    // ------------------------------------------------------------------ outputs
    T *xo = p.xout + (size_t)inst * (N + 1) * NX;
    T *uo = p.uout + (size_t)inst * N * NU;
    #pragma unroll 1
    for (int k = 0; k <= N; k++) {
#pragma unroll
        for (int a = 0; a < NZ; a++) {
            if (k == N && a >= NX) continue;
            const T z = ld(k, Wd::Z + a);
            if (a < NX) xo[k * NX + a] = z;
            else uo[k * NU + a - NX] = z;
        }
    }
    p.status[inst] = status;
    p.iters[inst] = iters;
#ifdef NMPC_SWEEP_TIMING
    if (p.cycles) {
        unsigned long long *c = p.cycles + (size_t)inst * 9;
        for (int j = 0; j < 8; j++) c[j] = tcy[j];
        c[8] = __builtin_amdgcn_s_memtime() - tstart;
    }
#endif
}

}  // namespace lpi

template <typename T, int NX, int NU, class SP>
hipError_t launch_ipm_lpi(const IpmParams<T> &p, hipStream_t s)
{
    const int W = p.ipw > 0 ? p.ipw : 1;
    const long long waves = ((long long)p.B + W - 1) / W;
    const int wpb = 4;
    const int blocks = (int)((waves + wpb - 1) / wpb);
    NMPC_LAUNCH((lpi::ipm_lpi_kernel<T, NX, NU, SP>), dim3(blocks), dim3(64 * wpb), 0, s, p);
    return hipGetLastError();
}

template <int NX, int NU>
size_t lpi_words() { return (size_t)lpi::Words<NX, NU>::NW; }

#define NMPC_LPI_INST(NX, NU, SP)                                                                        \
    template hipError_t launch_ipm_lpi<double, NX, NU, SP>(const IpmParams<double> &, hipStream_t);      \
    template hipError_t launch_ipm_lpi<float, NX, NU, SP>(const IpmParams<float> &, hipStream_t);
NMPC_LPI_INST(4, 2, lpc::DenseStructure<4 NMPC_LPI_COMMA 2>)
NMPC_LPI_INST(6, 2, lpc::DenseStructure<6 NMPC_LPI_COMMA 2>)
NMPC_LPI_INST(4, 2, lpc::ForceStructure)
NMPC_LPI_INST(6, 2, lpc::JerkStructure)
#undef NMPC_LPI_INST
template size_t lpi_words<4, 2>();
template size_t lpi_words<6, 2>();

}  // namespace nmpc
