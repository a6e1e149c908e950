// nmpc_solve_fast.hip — the general batched solve's common path (gfx950): every instance's unconstrained
// solution by the Riccati recursion on the shared factorisation, on the f64 matrix cores, four instances
// per matrix-core block group.
//
// What it replaces: `AcadosOcpSolver.solve()` after `set(k, 'yref')` for every stage and the x0 pinning
// (src/force_model/ocp.py:117-122, src/force_model/controller.py:29-32): one box-constrained LQ-OCP per
// instance with its own reference window. Without active bounds its solution is the unconstrained LQ
// solution, which the Riccati factorisation of the unconstrained problem gives for any x0 and reference —
// the factorisation (K_k, F_uu^-1, P_{k+1}) is the same for every instance, built once per handle on the host
// (nmpc_api.cpp lqr_table). Per instance (the host form is lqr_solve, the oracle's
// riccati_ipm_solve_batch_fast):
//
//   backward  p_N = g_N,  p_k = g_x,k + K_k' g_u,k + Acl_k' p_{k+1} + Acl_k' P_{k+1} c     (Acl_k = A + B K_k)
//             kff_k = -F_uu,k^-1 g_u,k - F_uu,k^-1 B' p_{k+1} - F_uu,k^-1 B' P_{k+1} c
//   forward   u_k = kff_k + K_k x_k,  x_{k+1} = A x_k + B u_k + c                              (x_0 = x0)
//
// with the gradient g = G yref of a diagonal LINEAR_LS map (g_r = G_rr yref_r). Every product is a small
// dense matrix times a vector of four instances, so it runs on v_mfma_f64_4x4x4_4b_f64 (four 4x4x4 blocks):
// A[b][i][k] = lane 16k + 4b + i, B[b][k][n] = lane 16k + 4b + n, D[b][i][n] = lane 16i + 4b + n (the
// layouts cl_lock_kernel uses, pinned by tools/ubench/mfma_f64_layout.hip). A state of nx <= 4 BPG components
// spans BPG blocks: block b holds rows 4 (b % BPG) .. + 3 of instance group b / BPG, so a wavefront carries
// 16 / BPG instances (quad13: BPG 4, 4 instances; jerk: 2, 8; force: 1, 16). A matrix-vector product is BPG
// chained MFMAs (one per K chunk of 4 components); its D result goes back to the B layout by one lane permute
// per chunk. The per-stage matrices (Acl_k', K_k', -F^-1 B', -F^-1, K_k and the constant vectors) sit in the
// workgroup's LDS for the whole launch; kff_k of the backward sweep waits in LDS for the forward sweep.
//
// The forward sweep writes x and u (unclamped) and tests every bound (1e-13 relative, as the lean loop's fast
// path): an instance whose unconstrained solution meets them all is solved (status 0, one Newton system); the
// others are listed for fin64_kernel (nmpc_cl_fast.hip: primal-dual active-set steps on W from the written
// z_0, the dual fallback, KKT acceptance), which reads their z_0 from the outputs.

#include <hip/hip_runtime.h>

#include <cfloat>

#include "nmpc_internal.h"

namespace nmpc {
namespace sf {

// per-stage table layout (doubles), compact: only the rows / columns a lane can need
template <int BPG>
struct Tab {
    static constexpr int R = 4 * BPG;                        // padded state rows
    static constexpr int ACLT = 0;                           // [BPG chunks][R rows][4]: Acl_k'(row, 4 kc + k)
    static constexpr int KT = ACLT + BPG * R * 4;            // [R][4]: K_k'(row, input k)
    static constexpr int FIBT = KT + R * 4;                  // [BPG][4][4]: (-F^-1 B')(input i, 4 kc + k)
    static constexpr int NFI = FIBT + BPG * 16;              // [4][4]: -F^-1(i, k)
    static constexpr int KK = NFI + 16;                      // [BPG][4][4]: K_k(i, 4 kc + k)
    static constexpr int CP = KK + BPG * 16;                 // [R]: Acl_k' P_{k+1} c
    static constexpr int CF = CP + R;                        // [4]: -F^-1 B' P_{k+1} c
    static constexpr int TS = CF + 4;                        // per stage
};

__device__ __forceinline__ double mfma(double a, double b, double c)
{
    return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}

template <int NX, int NU, int WPB>
__global__ __launch_bounds__(64 * WPB) void sf_kernel(SfParams p)
{
    constexpr int BPG = NX <= 4 ? 1 : (NX <= 8 ? 2 : 4);
    constexpr int G = 4 / BPG, IPW = 4 * G, NZ = NX + NU;
    static_assert(NX <= 16 && NU <= 4, "four blocks of four rows; the inputs in one block");
    using TB = Tab<BPG>;
    constexpr int KW = 64 / BPG;   // kff entries per wavefront and stage (the lanes of the groups' first blocks)
    extern __shared__ double lds[];
    const int N = p.N;
    double *tab = lds;                                   // [N][TS]
    double *kffl = lds + (size_t)N * TB::TS;             // [WPB][N][KW]
    for (int e = threadIdx.x; e < N * TB::TS; e += 64 * WPB) tab[e] = p.tab[e];
    __syncthreads();

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int kk = lane >> 4, b = (lane >> 2) & 3, n = lane & 3;
    const int bb = b % BPG, g = b / BPG;
    const int ra = 4 * bb + n;      // this lane's A-operand row (A[b][i = n][k = kk])
    const int rd = 4 * bb + kk;     // this lane's D row (D[b][i = kk][n])
    const bool ub = bb == 0;        // the group's first block: the input rows
    const long long inst_ll = ((long long)blockIdx.x * WPB + wave) * IPW + 4 * g + n;
    const bool valid = inst_ll < p.B;
    const int inst = valid ? (int)inst_ll : 0;
    double *kffw = kffl + (size_t)wave * N * KW;
    const int kidx = kk * (16 / BPG) + g * 4 + n;      // this lane's kff entry (valid for ub lanes)
    const size_t ys = (size_t)p.ystride;
    const double *yr = p.yref + (size_t)inst * ys;

    // D -> B layout: chunk kc of a vector is row 4 kc + kk of block g BPG + kc, column n
    auto to_b = [&](double d, int kc) { return __shfl(d, (lane & 0x33) | ((g * BPG + kc) << 2)); };

    // ---- per-lane constants: gradient scalings, the plant's A / B operands, c, bound thresholds
    const double gx = rd < NX ? p.gd[rd] : 0.0;                    // D row rd (state)
    const double gu = kk < NU ? p.gd[NX + kk] : 0.0;               // B row kk (input)
    const double ge = rd < NX ? p.gd[NZ + rd] : 0.0;               // terminal
    double aop[BPG], bop;
#pragma unroll
    for (int kc = 0; kc < BPG; kc++) aop[kc] = (ra < NX && 4 * kc + kk < NX) ? p.AB[ra * NZ + 4 * kc + kk] : 0.0;
    bop = (ra < NX && kk < NU) ? p.AB[ra * NZ + NX + kk] : 0.0;
    const double cr = rd < NX ? p.c[rd] : 0.0;
    auto thr_lo = [](double l) { return fabs(l) < 1e20 ? l - 1e-13 * (1.0 + fabs(l)) : -DBL_MAX; };
    auto thr_hi = [](double u) { return fabs(u) < 1e20 ? u + 1e-13 * (1.0 + fabs(u)) : DBL_MAX; };
    const int rx = rd < NX ? rd : 0, ru = NX + (kk < NU ? kk : 0);
    const double xlo1 = thr_lo(p.lbnd[NZ + rx]), xhi1 = thr_hi(p.ubnd[NZ + rx]);
    const double xlo2 = thr_lo(p.lbnd[2 * NZ + rx]), xhi2 = thr_hi(p.ubnd[2 * NZ + rx]);
    const double ulo0 = thr_lo(p.lbnd[ru]), uhi0 = thr_hi(p.ubnd[ru]);
    const double ulo1 = thr_lo(p.lbnd[NZ + ru]), uhi1 = thr_hi(p.ubnd[NZ + ru]);
    const bool xrow = valid && rd < NX, urow = valid && ub && kk < NU;

    // ---- backward sweep: p (B layout, BPG chunks), kff to LDS
    double pb[BPG];
    {
        const double d = xrow ? ge * yr[(size_t)N * p.ny + rd] : 0.0;
#pragma unroll
        for (int kc = 0; kc < BPG; kc++) pb[kc] = to_b(d, kc);
    }
    // the stage's gradient loads one stage ahead
    double yx = 0.0, yu = 0.0;
    auto load_y = [&](int k) {
        yx = xrow ? yr[(size_t)k * p.ny + rd] : 0.0;
        yu = (valid && kk < NU) ? yr[(size_t)k * p.ny + NX + kk] : 0.0;
    };
    load_y(N - 1);
    for (int k = N - 1; k >= 0; k--) {
        const double gxk = gx * yx, guk = gu * yu;
        if (k > 0) load_y(k - 1);
        const double *t = tab + (size_t)k * TB::TS;
        double dp = (rd < NX ? t[TB::CP + rd] : 0.0) + gxk;
        double df = (ub && kk < NU) ? t[TB::CF + kk] : 0.0;
        dp = mfma(t[TB::KT + ra * 4 + kk], guk, dp);
        df = mfma(ub ? t[TB::NFI + n * 4 + kk] : 0.0, guk, df);
#pragma unroll
        for (int kc = 0; kc < BPG; kc++) {
            dp = mfma(t[TB::ACLT + (kc * TB::R + ra) * 4 + kk], pb[kc], dp);
            df = mfma(ub ? t[TB::FIBT + (kc * 4 + n) * 4 + kk] : 0.0, pb[kc], df);
        }
        if (ub) kffw[(size_t)k * KW + kidx] = df;
#pragma unroll
        for (int kc = 0; kc < BPG; kc++) pb[kc] = to_b(dp, kc);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // ---- forward sweep: x (B layout), outputs and the bound test
    double *xo = p.xout + (size_t)inst * (N + 1) * NX;
    double *uo = p.uout + (size_t)inst * N * NU;
    double xb[BPG];
#pragma unroll
    for (int kc = 0; kc < BPG; kc++) xb[kc] = (valid && 4 * kc + kk < NX) ? p.x0[(size_t)inst * NX + 4 * kc + kk] : 0.0;
    if (xrow) xo[rd] = p.x0[(size_t)inst * NX + rd];
    bool bad = false;
    for (int k = 0; k < N; k++) {
        const double *t = tab + (size_t)k * TB::TS;
        double du = ub ? kffw[(size_t)k * KW + kidx] : 0.0;
        double dx = cr;
#pragma unroll
        for (int kc = 0; kc < BPG; kc++) {
            du = mfma(ub ? t[TB::KK + (kc * 4 + n) * 4 + kk] : 0.0, xb[kc], du);
            dx = mfma(aop[kc], xb[kc], dx);
        }
        if (urow) {
            uo[(size_t)k * NU + kk] = du;
            bad |= !(du >= (k == 0 ? ulo0 : ulo1) && du <= (k == 0 ? uhi0 : uhi1));   // NaN: bad
        }
        dx = mfma(bop, __shfl(du, (lane & 0x33) | ((g * BPG) << 2)), dx);
        if (xrow) {
            xo[(size_t)(k + 1) * NX + rd] = dx;
            const bool last = k + 1 == N;
            bad |= !(dx >= (last ? xlo2 : xlo1) && dx <= (last ? xhi2 : xhi1));
        }
#pragma unroll
        for (int kc = 0; kc < BPG; kc++) xb[kc] = to_b(dx, kc);
    }

    // ---- per instance: solved, or listed for the active-set finish
    const unsigned long long bm = __ballot(bad);
    unsigned long long mine = 0;
#pragma unroll
    for (int q = 0; q < BPG; q++) mine |= 0x0001000100010001ull << (4 * (g * BPG + q) + n);
    if (valid && kk == 0 && bb == 0) {   // the instance's leader lane
        if (bm & mine) {
            const int pos = atomicAdd(p.list_count, 1);
            p.list[pos] = inst;
        } else {
            p.status[inst] = 0;
            p.iters[inst] = 1;
        }
    }
}

}  // namespace sf

// shapes compiled: quad13 (8 wavefronts per workgroup: 32 instances), jerk and force (2: 16 / 32)
template <class F>
static bool sf_dispatch(int nx, int nu, F &&f)
{
    if (nx == 13 && nu == 4) f(sf::sf_kernel<13, 4, 8>, 8, 4, sf::Tab<4>::TS, 16);
    else if (nx == 6 && nu == 2) f(sf::sf_kernel<6, 2, 2>, 2, 8, sf::Tab<2>::TS, 32);
    else if (nx == 4 && nu == 2) f(sf::sf_kernel<4, 2, 2>, 2, 16, sf::Tab<1>::TS, 64);
    else return false;
    return true;
}

int sf_table_words(int nx, int nu)
{
    int ts = 0;
    sf_dispatch(nx, nu, [&](auto, int, int, int t, int) { ts = t; });
    return ts;
}

size_t sf_lds_bytes(int nx, int nu, int N)
{
    size_t bytes = 0;
    sf_dispatch(nx, nu, [&](auto, int wpb, int, int ts, int kw) { bytes = ((size_t)N * ts + (size_t)wpb * N * kw) * sizeof(double); });
    return bytes;
}

hipError_t sf_launch(int nx, int nu, const SfParams &p, hipStream_t s)
{
    hipError_t e = hipErrorInvalidValue;
    sf_dispatch(nx, nu, [&](auto k, int wpb, int ipw, int ts, int kw) {
        const size_t lds = ((size_t)p.N * ts + (size_t)wpb * p.N * kw) * sizeof(double);
        if (lds > 160 * 1024 || p.B < 1) return;
        const int per_wg = wpb * ipw;
        hipLaunchKernelGGL(k, dim3((p.B + per_wg - 1) / per_wg), dim3(64 * wpb), lds, s, p);
        e = hipGetLastError();
    });
    return e;
}

}  // namespace nmpc
