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
#include <cstdlib>

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
    static constexpr int ZERO = CF + 4;                      // a zero word (the operand of lanes outside a table)
    static constexpr int TS = ZERO + 2;                      // per stage (even: 16-byte copies)
};

constexpr int SF_CHUNK = 4;   // stages per LDS ring slot of the runtime-horizon kernels

__device__ __forceinline__ double mfma(double a, double b, double c)
{
    return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}

// diagnostic build (-DNMPC_SF_TIMING, build.build_experiment; env NMPC_SF_CYCLES=<file>): per wavefront the
// wall-clock ticks (100 MHz) at its start, after the table copy, after the backward and after the forward sweep,
// and the shader cycles of the same phases, to p.cycles[wave][8] (tools/sf_phases.py)
#ifdef NMPC_SF_TIMING
#define SF_MARK(i)                                                      \
    do {                                                                \
        if (p.cycles && lane == 0) {                                    \
            p.cycles[wid * 8 + (i)] = (unsigned long long)wall_clock64(); \
            p.cycles[wid * 8 + 4 + (i)] = (unsigned long long)clock64(); \
        }                                                               \
    } while (0)
#else
#define SF_MARK(i) \
    do {           \
    } while (0)
#endif

// NT > 0: compiled for horizon N = NT — the sweeps unroll completely, so the memory-counter waits on the
// reference loads are exact (a runtime loop makes the compiler wait for each load one stage after it issues) and
// kff stays in registers; NT = 0: any N, kff in LDS.
// The stage tables stream through LDS in chunks of SCH stages: chunk c + 1's loads are issued when chunk c starts
// and stored (then a workgroup barrier) when it ends, into the other slot of a two-slot ring. The compiled horizons
// take the whole table as one chunk (SCH = NT, one slot): measured on quad13 B = 8192 (tools/sf_phases.py), the
// four-stage ring did not shorten the prologue (4.0 against 4.9 us: it waits for the instance loads, not the
// table) and lengthened the sweeps by its barriers and reloads (10.4 + 9.0 against 8.7 + 6.6 us).
template <int NX, int NU, int WPB, int NT, int SCH>
__global__ __launch_bounds__(64 * WPB) void sf_kernel(SfParams p)
{
    constexpr int BPG = NX <= 4 ? 1 : (NX <= 8 ? 2 : 4);
    constexpr int G = 4 / BPG, IPW = 4 * G, NZ = NX + NU;
    static_assert(NX <= 16 && NU <= 4, "four blocks of four rows; the inputs in one block");
    using TB = Tab<BPG>;
    typedef double dv2 __attribute__((ext_vector_type(2)));   // (HIP's double2 class defeats the register promotion)
    constexpr int KW = 64 / BPG;   // kff entries per wavefront and stage (the lanes of the groups' first blocks)
    constexpr int SC = SCH, CW = SC * TB::TS / 2, CPT = (CW + 64 * WPB - 1) / (64 * WPB);
    extern __shared__ double lds[];
    const int N = NT > 0 ? NT : p.N;
    const int NCH = (N + SC - 1) / SC;
    dv2 *ring = reinterpret_cast<dv2 *>(lds);            // [2][CW]
    double *kffl = lds + (SC >= N ? 1 : 2) * (size_t)CW * 2;   // [WPB][N][KW] (NT = 0)
    double kffr[NT > 0 ? NT : 1];                        // (NT > 0)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const size_t wid = (size_t)blockIdx.x * WPB + wave;
    (void)wid;
    SF_MARK(0);

    // ---- chunk c of a sweep: SC consecutive stages, the first (lowest) `chunk_lo`; backward from N - 1 down
    const dv2 *tsrc = reinterpret_cast<const dv2 *>(p.tab);
    const int wn = N * TB::TS / 2;
    dv2 cbuf[CPT];
    auto chunk_lo = [&](int c, bool fwd) { return fwd ? SC * c : (N - SC * (c + 1) > 0 ? N - SC * (c + 1) : 0); };
    auto chunk_load = [&](int c, bool fwd) {   // (unconditional loads at a clamped index)
        const int w0 = chunk_lo(c, fwd) * TB::TS / 2;
#pragma unroll
        for (int q = 0; q < CPT; q++) {
            const int e = (int)threadIdx.x + q * 64 * WPB, g_ = w0 + e;
            cbuf[q] = tsrc[(e < CW && g_ < wn) ? g_ : wn - 1];
        }
    };
    auto chunk_store = [&](int c) {
#pragma unroll
        for (int q = 0; q < CPT; q++) {
            const int e = (int)threadIdx.x + q * 64 * WPB;
            ring[(c & 1) * CW + (e < CW ? e : CW - 1)] = cbuf[q];   // (a clamped duplicate writes the same word)
        }
    };
    chunk_load(0, false);
    // the next solve's counters (the other pair of the double buffer; nothing reads them now) start at zero
    if (blockIdx.x == 0 && threadIdx.x < 2 && p.next_counts) p.next_counts[threadIdx.x] = 0;

    const int kk = lane >> 4, b = (lane >> 2) & 3, n = lane & 3;
    const int bb = b % BPG, g = b / BPG;
    const int ra = 4 * bb + n;      // this lane's A-operand row (A[b][i = n][k = kk])
    const int rd = 4 * bb + kk;     // this lane's D row (D[b][i = kk][n])
    const bool ub = bb == 0;        // the group's first block: the input rows
    const long long inst_ll = (long long)wid * IPW + 4 * g + n;
    const bool valid = inst_ll < p.B;
    const int inst = valid ? (int)inst_ll : 0;
    double *kffw = kffl + (size_t)wave * N * KW;
    const int kidx = kk * (16 / BPG) + g * 4 + n;      // this lane's kff entry (valid for ub lanes)
    const double *yr = p.yref + (size_t)inst * (size_t)p.ystride;
    const bool xrow = valid && rd < NX, urow = valid && ub && kk < NU;

    // D -> B layout: chunk kc of a vector is row 4 kc + kk of block g BPG + kc, column n
    auto to_b = [&](double d, int kc) { return __shfl(d, (lane & 0x33) | ((g * BPG + kc) << 2)); };

    // ---- the instance data, in flight together with the first chunk: the terminal reference, the first PD
    // stages' reference (a ring of registers PD stages deep), x0. Every load is unconditional at a clamped, valid
    // address and masked where it is used (a conditional load is a branch whose join drains the memory counter)
    const int rdc = rd < NX ? rd : 0, kuc = NX + (kk < NU ? kk : 0);
    const double yN = yr[(size_t)N * p.ny + rdc];
    constexpr int PD = 8;
    double ryx[PD], ryu[PD];
    auto load_y = [&](int k, double &vx, double &vu) {
        const size_t row = (size_t)(k > 0 ? k : 0) * p.ny;
        vx = yr[row + rdc];
        vu = yr[row + kuc];
    };
#pragma unroll
    for (int q = 0; q < PD; q++) load_y(N - 1 - q, ryx[q], ryu[q]);
    double xb[BPG];   // x0 for the forward sweep, B layout
#pragma unroll
    for (int kc = 0; kc < BPG; kc++) xb[kc] = p.x0[(size_t)inst * NX + (4 * kc + kk < NX ? 4 * kc + kk : 0)];
    const double x0d = p.x0[(size_t)inst * NX + rdc];

    // ---- per-lane constants: gradient scalings (zero on the lanes whose row / input does not exist, which
    // masks the reference loads), the plant's A / B operands, c, bound thresholds
    const double gx = rd < NX ? p.gd[rd] : 0.0;                    // D row rd (state)
    const double gu = kk < NU ? p.gd[NX + kk] : 0.0;               // B row kk (input)
    const double ge = rd < NX ? p.gd[NZ + rd] : 0.0;               // terminal
#pragma unroll
    for (int kc = 0; kc < BPG; kc++) xb[kc] = 4 * kc + kk < NX ? xb[kc] : 0.0;
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
    chunk_store(0);
    __syncthreads();
    SF_MARK(1);

    // ---- backward sweep: p (B layout, BPG chunks), kff. The stage's A operands and constants come from the
    // ring one stage ahead within a chunk (an LDS round trip per MFMA otherwise sits on the recursion's chain);
    // lanes outside the input rows read the stage's zero word, so every read is unconditional
    struct BOps {
        double cp, cf, kt, nfi, aclt[BPG], fibt[BPG];
    };
    const int i_cf = ub ? TB::CF + kk : TB::ZERO, i_nfi = ub ? TB::NFI + n * 4 + kk : TB::ZERO;
    auto stage_tab = [&](int k, int c, bool fwd) {
        return reinterpret_cast<const double *>(ring + (c & 1) * CW) + (size_t)(k - chunk_lo(c, fwd)) * TB::TS;
    };
    auto ld_b = [&](const double *t, BOps &o) {
        o.cp = t[TB::CP + rd];
        o.cf = t[i_cf];
        o.kt = t[TB::KT + ra * 4 + kk];
        o.nfi = t[i_nfi];
#pragma unroll
        for (int kc = 0; kc < BPG; kc++) {
            o.aclt[kc] = t[TB::ACLT + (kc * TB::R + ra) * 4 + kk];
            o.fibt[kc] = t[ub ? TB::FIBT + (kc * 4 + n) * 4 + kk : TB::ZERO];
        }
    };
    double pb[BPG];
#pragma unroll
    for (int kc = 0; kc < BPG; kc++) pb[kc] = to_b(ge * yN, kc);
#pragma unroll
    for (int c = 0; c < NCH; c++) {
        if (c + 1 < NCH) chunk_load(c + 1, false);
        const int khi = N - 1 - SC * c, klo = chunk_lo(c, false);
        BOps ob;
        ld_b(stage_tab(khi, c, false), ob);
#pragma unroll
        for (int q0 = 0; q0 < SC; q0++) {
            const int k = khi - q0;
            if (k >= klo) {   // wave-uniform (the last chunk may be short)
                const int q = (N - 1 - k) % PD;
                const double gxk = gx * ryx[q], guk = gu * ryu[q];
                load_y(k - PD, ryx[q], ryu[q]);
                BOps on;
                if (k > klo) ld_b(stage_tab(k - 1, c, false), on);
                double dp = ob.cp + gxk, df = ob.cf;
                dp = mfma(ob.kt, guk, dp);
                df = mfma(ob.nfi, guk, df);
#pragma unroll
                for (int kc = 0; kc < BPG; kc++) {
                    dp = mfma(ob.aclt[kc], pb[kc], dp);
                    df = mfma(ob.fibt[kc], pb[kc], df);
                }
                if constexpr (NT > 0) kffr[k] = df;
                else if (ub) kffw[(size_t)k * KW + kidx] = df;
#pragma unroll
                for (int kc = 0; kc < BPG; kc++) pb[kc] = to_b(dp, kc);
                if (k > klo) ob = on;
            }
        }
        if (c + 1 < NCH) {
            chunk_store(c + 1);   // (the other slot: its last readers passed the previous barrier)
            __syncthreads();
        }
    }
    SF_MARK(2);

    // ---- forward sweep: x (B layout), outputs and the bound test; kff and K_k one stage ahead
    __syncthreads();   // every wavefront is done with the backward chunks
    chunk_load(0, true);
    double *xo = p.xout + (size_t)inst * (N + 1) * NX;
    double *uo = p.uout + (size_t)inst * N * NU;
    if (xrow) xo[rd] = x0d;
    chunk_store(0);
    __syncthreads();
    struct FOps {
        double kff, kk_[BPG];
    };
    auto ld_f = [&](int k, int c, FOps &o) {
        const double *t = stage_tab(k, c, true);
        if constexpr (NT > 0) o.kff = kffr[k];
        else o.kff = kffw[(size_t)k * KW + (ub ? kidx : 0)];   // (masked at its use: rows outside the inputs add 0)
#pragma unroll
        for (int kc = 0; kc < BPG; kc++) o.kk_[kc] = t[ub ? TB::KK + (kc * 4 + n) * 4 + kk : TB::ZERO];
    };
    bool bad = false;
#pragma unroll
    for (int c = 0; c < NCH; c++) {
        if (c + 1 < NCH) chunk_load(c + 1, true);
        const int klo = SC * c, khi = SC * (c + 1) < N ? SC * (c + 1) - 1 : N - 1;
        FOps of;
        ld_f(klo, c, of);
#pragma unroll
        for (int q0 = 0; q0 < SC; q0++) {
            const int k = klo + q0;
            if (k <= khi) {
                FOps on;
                if (k < khi) ld_f(k + 1, c, on);
                double du = ub ? of.kff : 0.0;
                double dx = cr;
#pragma unroll
                for (int kc = 0; kc < BPG; kc++) {
                    du = mfma(of.kk_[kc], xb[kc], du);
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
                if (k < khi) of = on;
            }
        }
        if (c + 1 < NCH) {
            chunk_store(c + 1);
            __syncthreads();
        }
    }
    SF_MARK(3);

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

// shapes compiled: quad13 (8 wavefronts per workgroup: 32 instances), jerk and force (2: 16 / 32); horizons
// compiled in full: the shipped models' (quad13 20, force 20 / 30, jerk 30 / 40), other N on the runtime-N kernel.
// f(kernel, wavefronts per workgroup, instances per wavefront, table words per stage, kff LDS words per wave-stage)
template <class F>
static bool sf_dispatch(int nx, int nu, int N, F &&f)
{
    constexpr int C = sf::SF_CHUNK;
    if (nx == 13 && nu == 4) {
        if (N == 20) f(sf::sf_kernel<13, 4, 8, 20, 20>, 8, 4, sf::Tab<4>::TS, 0, 20);
        else f(sf::sf_kernel<13, 4, 8, 0, C>, 8, 4, sf::Tab<4>::TS, 16, C);
    } else if (nx == 6 && nu == 2) {
        if (N == 40) f(sf::sf_kernel<6, 2, 2, 40, 40>, 2, 8, sf::Tab<2>::TS, 0, 40);
        else if (N == 30) f(sf::sf_kernel<6, 2, 2, 30, 30>, 2, 8, sf::Tab<2>::TS, 0, 30);
        else f(sf::sf_kernel<6, 2, 2, 0, C>, 2, 8, sf::Tab<2>::TS, 32, C);
    } else if (nx == 4 && nu == 2) {
        if (N == 20) f(sf::sf_kernel<4, 2, 2, 20, 20>, 2, 16, sf::Tab<1>::TS, 0, 20);
        else if (N == 30) f(sf::sf_kernel<4, 2, 2, 30, 30>, 2, 16, sf::Tab<1>::TS, 0, 30);
        else f(sf::sf_kernel<4, 2, 2, 0, C>, 2, 16, sf::Tab<1>::TS, 64, C);
    } else {
        return false;
    }
    return true;
}

int sf_table_words(int nx, int nu)
{
    int ts = 0;
    sf_dispatch(nx, nu, 0, [&](auto, int, int, int t, int, int) { ts = t; });
    return ts;
}

// dynamic LDS: the table chunks (one slot when a chunk holds the whole horizon, else two), and kff for the
// runtime-horizon kernels
static size_t sf_lds(int N, int wpb, int ts, int kw, int sch)
{
    return ((size_t)(sch >= N ? 1 : 2) * sch * ts + (size_t)wpb * N * kw) * sizeof(double);
}

size_t sf_lds_bytes(int nx, int nu, int N)
{
    size_t bytes = 0;
    sf_dispatch(nx, nu, N, [&](auto, int wpb, int, int ts, int kw, int sch) { bytes = sf_lds(N, wpb, ts, kw, sch); });
    return bytes;
}

hipError_t sf_launch(int nx, int nu, const SfParams &p, hipStream_t s)
{
    hipError_t e = hipErrorInvalidValue;
    sf_dispatch(nx, nu, p.N, [&](auto k, int wpb, int ipw, int ts, int kw, int sch) {
        const size_t lds = sf_lds(p.N, wpb, ts, kw, sch);
        if (lds > 160 * 1024 || p.B < 1) return;
        const int per_wg = wpb * ipw;
        NMPC_LAUNCH(k, dim3((p.B + per_wg - 1) / per_wg), dim3(64 * wpb), lds, s, p);
        e = hipGetLastError();
    });
    return e;
}

}  // namespace nmpc
