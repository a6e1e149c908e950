// nmpc_ipm.hip — batched box-constrained LQ-OCP solver for CDNA4 (gfx950).
//
// Replaces, per trajectory instance, one `AcadosOcpSolver.solve()` of the reference
// (src/force_model/controller.py:32, src/jerk_model/controller.py:33): acados SQP-GN over
// an LTI model with LINEAR_LS cost and box constraints is exactly one QP, which acados
// hands to HPIPM's Riccati-based interior-point method (force_model/ocp.py:83). This file
// is a from-scratch interior-point solver of that QP laid out for the MI355X:
//
//   * one 64-lane wavefront owns IPW instances (G = 64/IPW lanes each; IPW = 1 for the
//     nx=13, nu=4 headline model: one wavefront per trajectory instance); WPB wavefronts
//     share a workgroup only to share the model constants in LDS;
//   * Mehrotra predictor-corrector IPM. Each iteration alternates lane-parallel elementwise
//     phases over all (N+1)*nz components of the instance with the three stage recursions
//     that actually couple stages:
//       E_A  lazily applied step of the previous iteration, barrier Hessian Sigma, objective
//            gradient g and dynamics residual re of every stage;
//       A    backward Riccati factorisation + predictor right-hand side;
//       B    forward predictor direction, then E_B: its ratio test and centring sums;
//       E_C  corrector right-hand side of every stage, then C: backward corrector vector;
//       D    forward corrector direction, then E_D: step length and the new complementarity
//            measure (closed form in alpha, so no extra sweep is needed).
//     The elementwise work runs on ~all 64 lanes instead of the nz lanes of one stage, and
//     the recursions' stage-to-stage dependency chains carry only the linear algebra;
//   * the stage matrices (P, M = P[A B] stored transposed, F = [A B]'M + H + Sigma) live in
//     LDS; the lanes form a (column c, row group rg) grid and each lane keeps its column of
//     [A B] in registers, so every LDS operand is a broadcast read;
//   * input-block gains in explicit form, K = -F_uu^{-1} F_ux and F_uu^{-1}: the forward
//     sweeps are then a matrix-vector product per stage, with no triangular solve on the
//     stage-to-stage dependency chain;
//   * per-stage iterates and gains stream through a per-instance scratch region (buffer
//     resource addressing); the recursions prefetch the next stage's data one stage ahead;
//   * lanes of one wavefront exchange LDS data without barriers: LDS operations of one
//     wavefront execute in issue order, so a wavefront-scope fence (compiler ordering only)
//     between writer and reader phases suffices. Global scratch hand-offs between lanes are
//     ordered by one workgroup-scope fence per phase.
//
// The algorithm is the one in oracle/c/riccati_ipm.c (the CPU baseline), step for step; its
// results are checked against the KKT-certified dense oracle (oracle/qp.py).

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>

#include "nmpc_cl_device.h"
#include "nmpc_internal.h"
#include "nmpc_lpc_geom.h"

// unroll factor of the row-round loops of the backward factorisation (M, F, P products)
#ifndef NMPC_UNROLL_A
#define NMPC_UNROLL_A 2
#endif
// stage records in flight ahead of the B/C/D recursions
#ifndef NMPC_STREAM_DEPTH
#define NMPC_STREAM_DEPTH 4
#endif
#define NMPC_STR2(x) #x
#define NMPC_STR(x) NMPC_STR2(x)

namespace nmpc {

#define WAVE_SYNC()                                              \
    do {                                                         \
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   \
        __builtin_amdgcn_wave_barrier();                         \
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   \
        asm volatile("" ::: "memory");                           \
    } while (0)

#define SWEEP_FENCE()                                            \
    do {                                                         \
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");   \
        __builtin_amdgcn_wave_barrier();                         \
    } while (0)

// LDS maximum of a non-negative value (its bit pattern orders like an unsigned integer)
__device__ __forceinline__ void lds_max(double *p, double v)
{
    atomicMax((unsigned long long *)p, (unsigned long long)__double_as_longlong(v));
}
__device__ __forceinline__ void lds_max(float *p, float v) { atomicMax((unsigned int *)p, __float_as_uint(v)); }

template <int G, typename T>
__device__ __forceinline__ T group_sum(T v)
{
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
template <int G, typename T>
__device__ __forceinline__ T group_min(T v)
{
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
    return v;
}
template <int G, typename T>
__device__ __forceinline__ T group_max(T v)
{
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}

// init + sum_l a(l) b(l) with two interleaved accumulators: halves the dependent-FMA
// chain of the stage products, which are latency- rather than throughput-bound
template <int N, typename T, typename FA, typename FB>
__device__ __forceinline__ T dot2(T init, FA a, FB b)
{
    T s0 = init, s1 = T(0);
#pragma unroll
    for (int l = 0; l + 1 < N; l += 2) {
        s0 = fma(a(l), b(l), s0);
        s1 = fma(a(l + 1), b(l + 1), s1);
    }
    if constexpr (N % 2) s0 = fma(a(N - 1), b(N - 1), s0);
    return s0 + s1;
}

// 1/sqrt(x) for x > 0: hardware estimate + two Newton steps (no IEEE sqrt scaling path)
__device__ __forceinline__ double frsq(double x)
{
    double y = __builtin_amdgcn_rsq(x);
    const double h = 0.5 * x;
    y = fma(y, fma(-h, y * y, 0.5), y);
    y = fma(y, fma(-h, y * y, 0.5), y);
    return y;
}
__device__ __forceinline__ float frsq(float x)
{
    float y = __builtin_amdgcn_rsqf(x);
    return fmaf(y, fmaf(-0.5f * x, y * y, 0.5f), y);
}

template <typename T>
__device__ __forceinline__ bool has_bound(T b)
{
    return fabs(b) < T(1e20);
}

// Per-wavefront scratch region addressed through a buffer resource: the base lives in SGPRs
// and every access is (32-bit lane offset VGPR) + (wave-uniform SGPR offset), so the stage
// loops carry no 64-bit per-array pointers in VGPRs.
template <typename T>
struct Scr {
    __amdgpu_buffer_rsrc_t r;
    unsigned go;   // byte offset of this lane group's instance (0 when IPW = 1)
    __device__ T ld(unsigned uni, unsigned lane) const
    {
        if constexpr (sizeof(T) == 8) {
            return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(r, go + lane * 8u, uni * 8u, 0));
        } else {
            return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(r, go + lane * 4u, uni * 4u, 0));
        }
    }
    __device__ void st(unsigned uni, unsigned lane, T v) const
    {
        if constexpr (sizeof(T) == 8) {
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(
                unsigned __attribute__((ext_vector_type(2))), v), r, go + lane * 8u, uni * 8u, 0);
        } else {
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, go + lane * 4u, uni * 4u, 0);
        }
    }
};

// reciprocal: hardware estimate + Newton refinement (fp64: two steps -> ~1 ulp)
__device__ __forceinline__ double frcp(double x)
{
    double r = __builtin_amdgcn_rcp(x);
    r = fma(fma(-x, r, 1.0), r, r);
    r = fma(fma(-x, r, 1.0), r, r);
    return r;
}
__device__ __forceinline__ float frcp(float x)
{
    float r = __builtin_amdgcn_rcpf(x);
    return fmaf(fmaf(-x, r, 1.0f), r, r);
}

// packed lower-triangular storage of the Cholesky factor of F_uu; diagonal holds 1/L_ii
__host__ __device__ constexpr int tri(int i, int j) { return i * (i + 1) / 2 + j; }

// x <- F_uu^{-1} x = L^{-T} L^{-1} x with L packed (inverse diagonal)
template <typename T, int NU>
__device__ __forceinline__ void chol_solve(const T (&lf)[NU * (NU + 1) / 2], T (&x)[NU])
{
#pragma unroll
    for (int i = 0; i < NU; i++) {
        T s = x[i];
#pragma unroll
        for (int l = 0; l < i; l++) s -= lf[tri(i, l)] * x[l];
        x[i] = s * lf[tri(i, i)];
    }
#pragma unroll
    for (int i = NU - 1; i >= 0; i--) {
        T s = x[i];
#pragma unroll
        for (int l = i + 1; l < NU; l++) s -= lf[tri(l, i)] * x[l];
        x[i] = s * lf[tri(i, i)];
    }
}


// per-instance scratch (elements of T)
// Stage records, each contiguous so that a recursion streams one stage with one load per lane
// and record slot (per G lanes):
//   frec[k] = [ K_k (nu x nx, row-major) | kff_k (nu) | re_k (nx) ]       forward sweeps B, D
//   crec[k] = [ F_uu^-1 factor (packed, inverse diagonal) | Pr_k (nx) | corrector rhs (nz) ]
//                                                                         backward sweep C
struct ScratchLayout {
    size_t z, ll, lu, gc, gf, sg, dza, dz, frec, crec, act, total;
    int rsf, rsc;   // record sizes (elements)
    __host__ __device__ ScratchLayout(int N, int nx, int nu)
    {
        const size_t nz = (size_t)nx + nu, S = (size_t)(N + 1) * nz;
        rsf = nu * nx + nu + nx;
        rsc = nu * (nu + 1) / 2 + nx + (int)nz;
        z = 0;
        ll = z + S;
        lu = ll + S;
        gc = lu + S;    // G yref (constant per solve)
        gf = gc + S;    // predictor rhs g = H z + gc (terminal stage: corrector rhs in C)
        sg = gf + S;    // barrier Hessian Sigma
        dza = sg + S;
        dz = dza + S;
        frec = dz + S;
        crec = frec + (size_t)N * rsf;
        act = crec + (size_t)N * rsc;   // the last solution's active flags (fused closed loop warm start)
        total = act + S;
        total = (total + 31) & ~size_t(31);
    }
};

size_t scratch_elems_per_instance(int N, int nx, int nu) { return ScratchLayout(N, nx, nu).total; }

template <typename T, int NX, int NU, int IPW, int WPB>
struct Geometry {
    static constexpr int NZ = NX + NU;
    static constexpr int G = 64 / IPW;
    static constexpr int R = G / NZ;
    static constexpr int RM = (NX + R - 1) / R;
    static constexpr int RF = (NZ + R - 1) / R;
    static constexpr int VW = 16 / (int)sizeof(T);                 // elements per 16 B
    static constexpr int LDZ = (NZ + VW - 1) / VW * VW;            // 16-B aligned rows
    static constexpr int LDX = (NX + VW - 1) / VW * VW;
    static constexpr int LDU = (NU + VW - 1) / VW * VW;
    // block-shared constants
    static constexpr int C_AB = 0, C_H = C_AB + NX * LDZ, C_HE = C_H + NZ * LDZ, C_C = C_HE + NX * LDX,
                         C_LB = C_C + LDX, C_UB = C_LB + 3 * LDZ, C_TOT = C_UB + 3 * LDZ;
    // per-instance work area; FP and MT are contiguous and double as the stage-z window of
    // the elementwise phase E_A (ZW elements)
    static constexpr int I_FP = 0, I_MT = I_FP + NZ * LDZ, I_RV = I_MT + NZ * LDX, I_SV = I_RV + LDX,
                         I_VV = I_SV + LDZ, I_HV = I_VV + LDX, I_PV = I_HV + LDZ, I_GV = I_PV + LDX,
                         I_DX = I_GV + LDZ, I_DU = I_DX + 2 * LDX, I_CM = I_DU + LDU, I_TOT = I_CM + 2 * LDX;
    // I_CM: exact finish, largest violation of each state component's add candidates (two buffers:
    // the previous set step's, read by this step's flags, and this step's)
    // symmetric stage matrices are computed as lower triangles: column c owns rows c..n-1 in
    // chunks of E consecutive rows, one chunk per lane, E the smallest that fits G lanes
    static constexpr int tri_lanes(int n, int E)
    {
        int s = 0;
        for (int c = 0; c < n; c++) s += (n - c + E - 1) / E;
        return s;
    }
    static constexpr int tri_chunk(int n)
    {
        int E = 1;
        while (tri_lanes(n, E) > G) E++;
        return E;
    }
    static constexpr int EF = tri_chunk(NZ), EP = tri_chunk(NX);
    static constexpr int ZW = NZ * LDZ + NZ * LDX;
    static constexpr int CH = ZW / NZ - 1;     // stages per E_A chunk (+1 stage of overlap)
    // stage-record ring of the B/C/D recursions: two buffers of (NSF + NSC) slots of G elements;
    // it shares the FP/MT area when that is large enough (E_A and A do not overlap B/C/D)
    static constexpr int NUT = NU * (NU + 1) / 2;
    static constexpr int RSF = NU * NX + NU + NX, RSC = NUT + NX + NZ;
    static constexpr int NSF = (RSF + G - 1) / G, NSC = (RSC + G - 1) / G;
    static constexpr int RB1 = (NSF + NSC) * G;
    static constexpr bool RB_ALIAS = 2 * RB1 <= ZW;
    static constexpr int I_RB = RB_ALIAS ? I_FP : I_TOT;
    static constexpr int I_ALL = RB_ALIAS ? I_TOT : I_TOT + 2 * RB1;
    static constexpr int LDS_ELEMS = C_TOT + WPB * IPW * I_ALL;
    static_assert(R >= 1, "lane group narrower than the stage width");
    static_assert(CH >= 1, "stage-z window too small");
};

// timing builds (tools/exp.sh): NMPC_SWEEP_TIMING = cycles per phase of the iteration;
// NMPC_PHASE_TIMING = cycles of the four phases of the Riccati stage loop (slots 0..3)
#if defined(NMPC_PHASE_TIMING)
#define NMPC_SWEEP_TIMING 1
#define NMPC_TICK(slot) ((void)0)
#define NMPC_PTICK(slot) tick(slot)
#elif defined(NMPC_SWEEP_TIMING)
#define NMPC_TICK(slot) tick(slot)
#define NMPC_PTICK(slot) ((void)0)
#else
#define NMPC_TICK(slot) ((void)0)
#define NMPC_PTICK(slot) ((void)0)
#endif

template <typename T, int NX, int NU, int IPW, int WPB, int MW>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(MW, 8))) void ipm_kernel(IpmParams<T> p)
{
    using Gm = Geometry<T, NX, NU, IPW, WPB>;
    constexpr int NZ = Gm::NZ, G = Gm::G, R = Gm::R, RM = Gm::RM, RF = Gm::RF;
    constexpr int LDZ = Gm::LDZ, LDX = Gm::LDX, NUT = Gm::NUT;
    constexpr int RSF = Gm::RSF, RSC = Gm::RSC, NSF = Gm::NSF, NSC = Gm::NSC, RB1 = Gm::RB1;
    constexpr int FK = 0, FKFF = NU * NX, FRE = NU * NX + NU;   // frec fields
    constexpr int CFI = 0, CPR = NUT, CGH = NUT + NX;           // crec fields
    constexpr int DF = NMPC_STREAM_DEPTH;                        // records in flight

    __shared__ __attribute__((aligned(16))) T lds[Gm::LDS_ELEMS];
    T *cab = lds + Gm::C_AB, *ch = lds + Gm::C_H, *che = lds + Gm::C_HE, *cc = lds + Gm::C_C;
    T *clb = lds + Gm::C_LB, *cub = lds + Gm::C_UB;

    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int grp = lane / G;
    const int ll = lane % G;
    const int inst_raw = (blockIdx.x * WPB + wave) * IPW + grp;
    const bool inst_ok = inst_raw < p.B;
    const int inst = inst_ok ? inst_raw : p.B - 1;
    const int col = ll % NZ;
    const int rg = ll / NZ;
    const bool gridl = rg < R;
    const int N = p.N;
    T *w = lds + Gm::C_TOT + (wave * IPW + grp) * Gm::I_ALL;
    T *fp = w + Gm::I_FP, *mt = w + Gm::I_MT, *hv = w + Gm::I_HV, *vv = w + Gm::I_VV, *pv = w + Gm::I_PV;
    T *rv = w + Gm::I_RV, *sv = w + Gm::I_SV, *gv = w + Gm::I_GV, *du_l = w + Gm::I_DU, *zw = w + Gm::I_FP;
    // this lane's lower-triangle chunk of F (column fc, rows fb0..fb0+fn-1) and of P (pj, pi0, pn)
    int fc = -1, fb0 = 0, fn = 0, pj = -1, pi0 = 0, pn = 0;
    {
        auto assign = [&](int n, int E, int &c_, int &r0, int &cnt) {
            int idx = ll;
#pragma unroll
            for (int c = 0; c < n; c++) {
                const int m = (n - c + E - 1) / E;
                if (c_ < 0 && idx < m) {
                    c_ = c;
                    r0 = c + idx * E;
                    cnt = min(E, n - r0);
                }
                idx -= m;
            }
        };
        assign(NZ, Gm::EF, fc, fb0, fn);
        assign(NX, Gm::EP, pj, pi0, pn);
    }

    // ---- model constants -> LDS (once per workgroup)
    for (int e = threadIdx.x; e < NX * NZ; e += 64 * WPB) cab[(e / NZ) * LDZ + e % NZ] = p.AB[e];
    for (int e = threadIdx.x; e < NZ * NZ; e += 64 * WPB) ch[(e / NZ) * LDZ + e % NZ] = p.H[e];
    for (int e = threadIdx.x; e < NX * NX; e += 64 * WPB) che[(e / NX) * LDX + e % NX] = p.He[e];
    for (int e = threadIdx.x; e < NX; e += 64 * WPB) cc[e] = p.c[e];
    for (int e = threadIdx.x; e < 3 * NZ; e += 64 * WPB) {
        clb[(e / NZ) * LDZ + e % NZ] = p.lbnd[e];
        cub[(e / NZ) * LDZ + e % NZ] = p.ubnd[e];
    }
    // column `col` of [A B]: re-read from LDS where it is used (a register copy kept across
    // all sweeps would cost 2*NX VGPRs at the kernel's register peak)
    auto load_abcol = [&](T (&ac)[NX]) {
#pragma unroll
        for (int l = 0; l < NX; l++) ac[l] = cab[l * LDZ + col];
    };
    __syncthreads();
    if (!__any(inst_ok)) return;   // tail wavefront of the last workgroup: nothing to solve

    const ScratchLayout L(N, NX, NU);
    // wave-uniform bases (SGPRs) + 32-bit lane offsets
    const unsigned wave_u = __builtin_amdgcn_readfirstlane(wave);
    const size_t inst0 = ((size_t)blockIdx.x * WPB + wave_u) * IPW;
    Scr<T> S;
    S.r = __builtin_amdgcn_make_buffer_rsrc(p.scratch + inst0 * L.total, 0,
                                            (int)(IPW * L.total * sizeof(T)), 0x00020000);
    S.go = (unsigned)grp * (unsigned)(L.total * sizeof(T));
    const unsigned Lz = L.z, Lll = L.ll, Llu = L.lu, Lgc = L.gc, Lgf = L.gf, Lsg = L.sg, Ldza = L.dza, Ldz = L.dz;
    const unsigned Lfrec = L.frec, Lcrec = L.crec, Lact = L.act;
    T *rb = w + Gm::I_RB;
    const int nel = (N + 1) * NZ;
    auto stype = [&](int k) { return k == 0 ? 0 : (k == N ? 2 : 1); };

    // one solve per closed-loop step; plain solves run one step (p.cl_steps = 0)
    const bool fused = p.cl_steps > 0;
    const int nsteps = fused ? p.cl_steps : 1;
    for (int cstep = 0; cstep < nsteps; cstep++) {
        // fused closed loop: the yref window straight from the reference table rows (offset + step) %
        // period (cl_prepare_kernel's gather), x0 from the closed-loop state
        const int t_ref = fused ? (p.cl.offset[inst] + p.cl.step + cstep) % p.cl.period : 0;
        const T *yref = fused ? p.cl.table + (size_t)t_ref * p.cl.table_cols
                              : p.yref + (size_t)inst * ((size_t)N * p.ny + p.ny_e);
        const int yrow = fused ? p.cl.table_cols : p.ny;
        const T *x0 = (fused ? p.cl.state : p.x0) + (size_t)inst * NX;
        // ------------------------------------------------------------------ infeasibility certificate
        // interval reachability (oracle/c/riccati_ipm.c infeasible_stage): lane ll < nx carries the
        // midpoint / radius of state ll of X_k, lanes nx.. the input box; an empty X_{k+1} (state
        // box of stage k+1 included) proves the QP infeasible
        bool infeas = false;
        {
            const int cl_ = ll < NZ ? ll : 0;
            T cm = ll < NX ? x0[cl_] : T(0), cr = 0;
            if (ll >= NX && ll < NZ) {
                const T l = clb[cl_], h = cub[cl_];   // stage-0 input bounds
                const bool bb = has_bound(l) && has_bound(h);
                cm = bb ? T(0.5) * (l + h) : T(0);
                cr = bb ? T(0.5) * (h - l) : T(INFINITY);
            }
            for (int k = 0; k < N; k++) {
                if (ll < NZ) {
                    sv[ll] = cm;
                    hv[ll] = cr;
                }
                WAVE_SYNC();
                T sm = cc[ll < NX ? ll : 0], sr = 0;
#pragma unroll
                for (int j = 0; j < NZ; j++) {
                    const T a = cab[(ll < NX ? ll : 0) * LDZ + j];
                    sm = fma(a, sv[j], sm);
                    sr = a != T(0) ? fma(fabs(a), hv[j], sr) : sr;   // 0 x unbounded radius adds 0
                }
                const T l = clb[stype(k + 1) * LDZ + cl_], h = cub[stype(k + 1) * LDZ + cl_];
                T lo = sm - sr, hi = sm + sr;
                lo = has_bound(l) ? fmax(lo, l) : lo;
                hi = has_bound(h) ? fmin(hi, h) : hi;
                infeas |= ll < NX && lo > hi + T(1e-9) * (T(1) + fabs(hi));
                const bool fin = isfinite(lo) && isfinite(hi);
                WAVE_SYNC();
                if (ll < NX) {
                    cm = fin ? T(0.5) * (lo + hi) : sm;
                    cr = fin ? T(0.5) * (hi - lo) : sr;
                }
            }
            infeas = group_max<G>(infeas ? T(1) : T(0)) > T(0);
        }
        // ------------------------------------------------------------------ initial point
        for (int e = ll; e < nel; e += G) {
            const int k = e / NZ, i = e % NZ;
            T z = 0, lam_l = 0, lam_u = 0, gc = 0;
            if (k < N || i < NX) {
                const T *yk = yref + (size_t)k * yrow;
                if (k < N) {
                    for (int j = 0; j < p.ny; j++) gc += p.G[i * p.ny + j] * yk[j];
                } else {
                    for (int j = 0; j < p.ny_e; j++) gc += p.Ge[i * p.ny_e + j] * yk[j];
                }
                if (k == 0 && i < NX) {
                    z = x0[i];
                } else {
                    z = p.yref_is_z ? yk[i] : T(0);
                    const T lb = clb[stype(k) * LDZ + i], ub = cub[stype(k) * LDZ + i];
                    const bool hl = has_bound(lb), hu = has_bound(ub);
                    if (hl && hu) {
                        const T d = T(0.01) * (ub - lb);
                        z = i >= NX ? T(0.5) * (lb + ub) : z;   // boxed inputs start mid-box (oracle/c/riccati_ipm.c)
                        z = fmin(fmax(z, lb + d), ub - d);
                    } else if (hl) {
                        z = fmax(z, lb + T(0.01) * fmax(fabs(lb), T(1)));
                    } else if (hu) {
                        z = fmin(z, ub - T(0.01) * fmax(fabs(ub), T(1)));
                    }
                    if (hl) lam_l = p.mu0 / (z - lb);
                    if (hu) lam_u = p.mu0 / (ub - z);
                }
            }
            S.st(Lz, e, z);
            S.st(Lll, e, lam_l);
            S.st(Llu, e, lam_u);
            S.st(Lgc, e, gc);
        }
        SWEEP_FENCE();
        T r0 = 0, mu = 0;
        for (int e = ll; e < nel; e += G) {
            const int k = e / NZ, i = e % NZ;
            if (k == N && i >= NX) continue;
            const unsigned k0 = (unsigned)(k * NZ);
            if (!(k == 0 && i < NX)) {
                T g = S.ld(Lgc, e);
                if (k < N) {
                    for (int b = 0; b < NZ; b++) g += ch[i * LDZ + b] * S.ld(Lz, k0 + b);
                } else {
                    for (int b = 0; b < NX; b++) g += che[i * LDX + b] * S.ld(Lz, k0 + b);
                }
                const T la = S.ld(Lll, e), lu_ = S.ld(Llu, e);
                r0 = fmax(r0, fabs(g - la + lu_));
                const T z = S.ld(Lz, e);
                if (la > T(0)) mu += la * (z - clb[stype(k) * LDZ + i]);
                if (lu_ > T(0)) mu += lu_ * (cub[stype(k) * LDZ + i] - z);
            }
            if (k < N && i < NX) {
                T r = cc[i] - S.ld(Lz, k0 + NZ + i);
                for (int j = 0; j < NZ; j++) r += cab[i * LDZ + j] * S.ld(Lz, k0 + j);
                r0 = fmax(r0, fabs(r));
            }
        }
        r0 = group_max<G>(r0);
        mu = group_sum<G>(mu) * p.inv_m;

        const T m_bounds = T(1) / p.inv_m;
        T theta = 1;
        bool active = inst_ok && !infeas;
        int status = infeas ? 4 : 2, iters = 0;   // certified infeasible: status 4, the initial point
        bool fail = false, pending = false;
        T alpha = 0, smu = 0;      // step and sigma*mu of the pending (lazily applied) update
        // exact finish (oracle/c/riccati_ipm.c "exact finish"; nmpc_ipm_lpc.hip): a primal-dual
        // active-set run of <= polish_steps penalised Newton steps + one refinement. polish_at: mu that
        // triggers the next run; pol: the group is in a run; fref: its next step is the refinement.
        // During a run dz holds the set step, dza the active flags (-1 lower, 1 upper, 0) and sg the
        // refinement's correction; a group the finish completes writes its outputs at once (status -1)
        T polish_at = p.polish_mu;
        int fin_steps = 0, fin_runs = 0;
        bool pol = false, fref = false, fs0 = false;
        // fused closed loop after its first step: the first finish run of a solve starts from the
        // previous step's active set shifted by one stage (act array; a warm start, the acceptance
        // tests are unchanged)
        const bool warm = fused && (cstep > 0 || p.cl.step > 0);
        bool fwarm = false;
        // PDAS update (oracle/c/riccati_ipm.c pdas_update): a violated inactive state bound is an add
        // candidate (flag +-(2 + violation)); it joins in the next step if it is its component's most
        // violated one (cmax buffer cmb) and the step that found it was the run's first or had no removals
        int cmb = 0;
        bool addok = false;
        // the solution's active flag of an element (z on a bound to 1e-7): the warm start's input
        auto act_flag = [&](T z, T lb, T ub) {
            const bool onl = has_bound(lb) && z <= lb + T(1e-7) * (T(1) + fabs(lb));
            const bool onu = has_bound(ub) && z >= ub - T(1e-7) * (T(1) + fabs(ub));
            return onl ? T(-1) : (onu ? T(1) : T(0));
        };

#ifdef NMPC_SWEEP_TIMING
        // experiment builds only (build_experiment(..., ["NMPC_SWEEP_TIMING"])): clock cycles per phase
        const bool timed = p.cycles != nullptr;
        unsigned long long tcy[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tmark = 0;
        auto tick = [&](int slot) {
            if (timed) {
                const unsigned long long t = __builtin_amdgcn_s_memtime();
                if (slot >= 0) tcy[slot] += t - tmark;
                tmark = t;
            }
        };
        const unsigned long long tstart = timed ? __builtin_amdgcn_s_memtime() : 0ull;
#endif

        // ---- stage-record streaming for the B/C/D recursions: records are loaded DF stages ahead
        // into registers and written to the LDS ring one stage before use
        auto rec_issue = [&](T (&r)[NSF + NSC], int k, bool with_c) {
            const unsigned kk = (unsigned)(k < 0 ? 0 : (k < N ? k : N - 1));
#pragma unroll
            for (int s_ = 0; s_ < NSF; s_++) r[s_] = S.ld(Lfrec + kk * RSF + s_ * G, ll);
            if (with_c) {
#pragma unroll
                for (int s_ = 0; s_ < NSC; s_++) r[NSF + s_] = S.ld(Lcrec + kk * RSC + s_ * G, ll);
            }
        };
        auto rec_put = [&](const T (&r)[NSF + NSC], int buf, bool with_c) {
            T *dstp = rb + buf * RB1;
#pragma unroll
            for (int s_ = 0; s_ < NSF; s_++) dstp[s_ * G + ll] = r[s_];
            if (with_c) {
#pragma unroll
                for (int s_ = 0; s_ < NSC; s_++) dstp[(NSF + s_) * G + ll] = r[NSF + s_];
            }
        };
        // The ring registers r[j] hold the records m = j (mod DF); the stage loops are unrolled by DF
        // so that every slot is a fixed register set (moving an in-flight load's destination would
        // force a wait on it).

        // ---- forward recursion shared by predictor (dst = dza) and corrector (dst = dz):
        // dx_0 = 0 (x0 pinned), du_k = kff_k + K_k dx_k, dx_{k+1} = [A B] [dx; du] + re_k
        auto forward = [&](unsigned dst, unsigned shift = 0) {   // shift: per-lane element offset of dst
            T *dxb = w + Gm::I_DX;
            if (ll < NX) dxb[ll] = T(0);
            T arow[NZ];   // row ll of [A B], register-resident for the whole sweep
#pragma unroll
            for (int j = 0; j < NZ; j++) arow[j] = cab[(ll < NX ? ll : 0) * LDZ + j];
            T r[DF][NSF + NSC];
#pragma unroll
            for (int j = 0; j < DF; j++) rec_issue(r[j], j, false);
            rec_put(r[0], 0, false);
            rec_issue(r[0], DF, false);
            WAVE_SYNC();
            int cur = 0;
            for (int kb = 0; kb < N; kb += DF)
#pragma unroll
            for (int j = 0; j < DF; j++) {
                const int k = kb + j;
                if (k >= N) break;
                const T *rec = rb + (k & 1) * RB1;
                const T *dxc = dxb + cur * LDX;
                T *dxn = dxb + (1 - cur) * LDX;
                if (ll < NU) {
                    du_l[ll] = dot2<NX>(rec[FKFF + ll], [&](int i) { return rec[FK + ll * NX + i]; },
                                        [&](int i) { return dxc[i]; });
                }
                WAVE_SYNC();
                if (ll < NX) {
                    dxn[ll] = dot2<NZ>(rec[FRE + ll], [&](int j) { return arow[j]; },
                                       [&](int j) { return j < NX ? dxc[j] : du_l[j - NX]; });
                }
                if (ll < NZ) S.st(dst + k * NZ, ll + shift, ll < NX ? dxc[ll] : du_l[ll - NX]);
                rec_put(r[(j + 1) % DF], (k + 1) & 1, false);
                rec_issue(r[(j + 1) % DF], k + 1 + DF, false);
                cur = 1 - cur;
                WAVE_SYNC();
            }
            if (ll < NX) S.st(dst + N * NZ, ll + shift, dxb[cur * LDX + ll]);
            SWEEP_FENCE();
        };

        int it = 0;
        bool pfail = false;
        for (;; it++) {
            const bool conv = mu <= p.tol_comp && theta * r0 <= p.tol_res;
            const bool bad = !isfinite(mu) || !isfinite(theta) || fail;
            if (active && (conv || bad)) {
                active = false;
                status = conv && !bad ? 0 : 4;
                iters = (fail ? it - 1 : it) + fin_steps;   // a failed factorisation ends the iteration it began
            }
            if (active && it >= p.max_iter) {
                active = false;
                status = 2;
                iters = it + fin_steps;
            }
            if (!__any(active)) break;
            NMPC_TICK(-1);

            // active flag of element e in a finish step: first step of a run where the multiplier
            // exceeds the slack, later steps from dza (x_0 never)
            auto fin_flag = [&](int k, int i, int e, T z, T lam_l, T lam_u, T lb, T ub) {
                if (k == 0 && i < NX) return T(0);
                if (fs0 && fwarm) {
                    const int ks = !p.warm_shift ? k : ((k < N - 1 || (k == N - 1 && i < NX)) ? k + 1 : k);
                    const T a = S.ld(Lact, (unsigned)(ks * NZ + i));
                    return (a < T(-0.5) && lam_l > T(0)) ? T(-1) : ((a > T(0.5) && lam_u > T(0)) ? T(1) : T(0));
                }
                if (!fs0) {
                    const T f = S.ld(Ldza, e);
                    if (!(fabs(f) > T(1.5))) return f;
                    const T *cmo = w + Gm::I_CM + cmb * Gm::LDX;
                    return (addok && fabs(f) - T(2) == cmo[i]) ? (f < T(0) ? T(-1) : T(1)) : T(0);
                }
                const bool al = lam_l > T(0) && lam_l > z - lb, au = !al && lam_u > T(0) && lam_u > ub - z;
                return al ? T(-1) : (au ? T(1) : T(0));
            };
            // E_A + A; the finish pass (finp, wave-uniform) forms the finish's penalty terms in place of
            // the barrier for the polishing groups
            auto factor = [&](bool finp) __attribute__((always_inline)) {
            // ============================ E_A: lazy step, Sigma, g = H z + gc, re = [A B] z_k + c - x_{k+1}
            // stage chunks whose z (plus one stage of overlap) fit the LDS window zw
            for (int k0 = 0; k0 <= N; k0 += Gm::CH) {
                const int k1 = min(k0 + Gm::CH, N + 1);       // stages owned by this chunk
                const int kz = min(k0 + Gm::CH + 1, N + 1);   // stages whose z the chunk reads
                for (int e = k0 * NZ + ll; e < kz * NZ; e += G) {
                    const int k = e / NZ, i = e - k * NZ;
                    T z = 0;
                    if (k < N || i < NX) {
                        z = S.ld(Lz, e);
                        T lam_l = S.ld(Lll, e), lam_u = S.ld(Llu, e);
                        const T lb = clb[stype(k) * LDZ + i], ub = cub[stype(k) * LDZ + i];
                        if (pending) {
                            const T dz = S.ld(Ldz, e), dza = S.ld(Ldza, e);
                            if (lam_l > T(0)) {
                                const T t = z - lb, it_ = frcp(t), dla = -lam_l * (T(1) + dza * it_);
                                lam_l += alpha * ((smu - lam_l * t - dla * dza - lam_l * dz) * it_);
                            }
                            if (lam_u > T(0)) {
                                const T t = ub - z, it_ = frcp(t), dla = -lam_u * (T(1) - dza * it_);
                                lam_u += alpha * ((smu - lam_u * t + dla * dza + lam_u * dz) * it_);
                            }
                            z += alpha * dz;
                        }
                        if (k < k1) {
                            if (pending) {
                                S.st(Lz, e, z);
                                S.st(Lll, e, lam_l);
                                S.st(Llu, e, lam_u);
                            }
                            T sig = 0;
                            if (lam_l > T(0)) sig += lam_l * frcp(z - lb);
                            if (lam_u > T(0)) sig += lam_u * frcp(ub - z);
                            if (finp && pol) sig = fin_flag(k, i, e, z, lam_l, lam_u, lb, ub) != T(0) ? p.polish_rho : T(0);
                            S.st(Lsg, e, sig);
                        }
                        if (finp && pol && fref) z += S.ld(Ldz, e);   // the refinement's base z_a = z + dz
                    }
                    zw[e - k0 * NZ] = z;
                }
                WAVE_SYNC();
                for (int e = k0 * NZ + ll; e < k1 * NZ; e += G) {
                    const int k = e / NZ, i = e - k * NZ;
                    const T *zk = zw + (k - k0) * NZ;
                    T gadd = 0;
                    if (finp && pol && (k < N || i < NX)) {
                        // the finish's penalty gradient rho (z - bound) (refinement: 2 rho (z_a - bound))
                        const T lb = clb[stype(k) * LDZ + i], ub = cub[stype(k) * LDZ + i];
                        const T a = fin_flag(k, i, e, zk[i], S.ld(Lll, e), S.ld(Llu, e), lb, ub);
                        gadd = a != T(0) ? (fref ? T(2) : T(1)) * p.polish_rho * (zk[i] - (a < T(0) ? lb : ub)) : T(0);
                    }
                    if (k < N) {
                        S.st(Lgf, e, dot2<NZ>(S.ld(Lgc, e) + gadd, [&](int b) { return ch[i * LDZ + b]; },
                                              [&](int b) { return zk[b]; }));
                    } else if (i < NX) {
                        S.st(Lgf, e, dot2<NX>(S.ld(Lgc, e) + gadd, [&](int b) { return che[i * LDX + b]; },
                                              [&](int b) { return zk[b]; }));
                    }
                }
                for (int e = k0 * NX + ll; e < min(k1, N) * NX; e += G) {
                    const int k = e / NX, i = e - k * NX;
                    const T *zk = zw + (k - k0) * NZ;
                    S.st(Lfrec + k * RSF + FRE, i, dot2<NZ>(cc[i] - zk[NZ + i], [&](int j) { return cab[i * LDZ + j]; },
                                                            [&](int j) { return zk[j]; }));
                }
                WAVE_SYNC();
            }
            pending = false;
            SWEEP_FENCE();
            NMPC_TICK(0);

            // ============================ A: backward Riccati factorisation + predictor vector
            {
                struct PreA {
                    T sg, g, re;
                };
                auto fetch_a = [&](int k, PreA &q) {
                    const unsigned kk = (unsigned)(k < 0 ? 0 : k);
                    q.sg = S.ld(Lsg + kk * NZ, ll);
                    q.g = S.ld(Lgf + kk * NZ, ll);
                    q.re = S.ld(Lfrec + (kk < (unsigned)N ? kk : N - 1) * RSF + FRE, ll);
                };
                // P_N = He + Sigma_N, p_N = g_N
                {
                    const T sgN = S.ld(Lsg + N * NZ, ll), gN = S.ld(Lgf + N * NZ, ll);
                    if (ll < NX) {
                        sv[ll] = sgN;
                        pv[ll] = gN;
                    }
                }
                PreA q{};
                fetch_a(N - 1, q);
                WAVE_SYNC();
                if (gridl && col < NX) {
#pragma unroll
                    for (int qq = 0; qq < RM; qq++) {
                        const int i = rg + R * qq;
                        if (i < NX) fp[i * LDZ + col] = che[i * LDX + col] + (i == col ? sv[col] : T(0));
                    }
                }
                WAVE_SYNC();
                if (ll < NX) rv[ll] = q.re;
                if (ll < NZ) sv[ll] = q.sg;
                WAVE_SYNC();
                for (int k = N - 1; k >= 0; k--) {
                    PreA qn{};
                    fetch_a(k - 1, qn);
                    NMPC_PTICK(-1);
                    // 1: Pr = P re, v = Pr + p, M^T = (P [A B])^T
                    T abcol[NX];
                    load_abcol(abcol);
                    if (ll < NX) {
                        const T s = dot2<NX>(T(0), [&](int l) { return fp[ll * LDZ + l]; }, [&](int l) { return rv[l]; });
                        S.st(Lcrec + k * RSC + CPR, ll, s);
                        vv[ll] = s + pv[ll];
                    }
                    if (ll < NZ) gv[ll] = q.g;
                    if (gridl) {
    _Pragma(NMPC_STR(unroll NMPC_UNROLL_A))
                        for (int qq = 0; qq < RM; qq++) {
                            const int i = rg + R * qq;
                            if (i < NX) {
                                mt[col * LDX + i] = dot2<NX>(T(0), [&](int l) { return fp[i * LDZ + l]; },
                                                             [&](int l) { return abcol[l]; });
                            }
                        }
                    }
                    WAVE_SYNC();
                    NMPC_PTICK(0);
                    // 2: F = [A B]' M + H + Sigma, lower triangle by column chunks, mirrored;
                    //    h = [A B]' v + g by the first chunk of each column
                    if (fc >= 0) {
                        T ac[NX];
#pragma unroll
                        for (int l = 0; l < NX; l++) ac[l] = cab[l * LDZ + fc];
#pragma unroll
                        for (int t = 0; t < Gm::EF; t++) {
                            const int bb = fb0 + t;
                            if (t < fn) {
                                T s_ = dot2<NX>(ch[fc * LDZ + bb], [&](int l) { return ac[l]; },
                                                [&](int l) { return mt[bb * LDX + l]; });
                                if (bb == fc) s_ += sv[fc];
                                fp[fc * LDZ + bb] = s_;
                                fp[bb * LDZ + fc] = s_;
                            }
                        }
                        if (fb0 == fc) hv[fc] = dot2<NX>(gv[fc], [&](int l) { return ac[l]; }, [&](int l) { return vv[l]; });
                    }
                    WAVE_SYNC();
                    NMPC_PTICK(1);
                    // 3: F_uu = L L' (wave-uniform), kff = -F_uu^-1 h_u; per P column j: K(:, j) =
                    //    -F_uu^-1 F_ux(:, j), p_j = h_j + K(:, j)' h_u, P(i, j) = F(i, j) + F_xu(i, :) K(:, j)
                    T lf[NUT];
#pragma unroll
                    for (int i = 0; i < NU; i++)
#pragma unroll
                        for (int j = 0; j <= i; j++) {
                            T s_ = fp[(NX + i) * LDZ + NX + j];
#pragma unroll
                            for (int l = 0; l < j; l++) s_ -= lf[tri(i, l)] * lf[tri(j, l)];
                            if (i == j) {
                                const bool pd = s_ > T(0);
                                if (finp) pfail |= pol & !pd;
                                else fail |= active & !pd;
                                lf[tri(i, i)] = frsq(pd ? s_ : T(1));
                            } else {
                                lf[tri(i, j)] = s_ * lf[tri(j, j)];
                            }
                        }
                    T hu[NU];
#pragma unroll
                    for (int j = 0; j < NU; j++) hu[j] = hv[NX + j];
                    {
                        T x[NU];
#pragma unroll
                        for (int j = 0; j < NU; j++) x[j] = hu[j];
                        chol_solve<T, NU>(lf, x);
                        T mine = 0, lmine = 0;
#pragma unroll
                        for (int j = 0; j < NU; j++) mine = (ll == j) ? -x[j] : mine;
#pragma unroll
                        for (int j = 0; j < NUT; j++) lmine = (ll == j) ? lf[j] : lmine;
                        if (ll < NU) S.st(Lfrec + k * RSF + FKFF, ll, mine);
                        if (ll < NUT) S.st(Lcrec + k * RSC + CFI, ll, lmine);
                    }
                    if (pj >= 0) {
                        T kc[NU];
#pragma unroll
                        for (int u = 0; u < NU; u++) kc[u] = fp[(NX + u) * LDZ + pj];
                        chol_solve<T, NU>(lf, kc);
#pragma unroll
                        for (int u = 0; u < NU; u++) kc[u] = -kc[u];
                        if (pi0 == pj) {
                            T s_ = hv[pj];
#pragma unroll
                            for (int u = 0; u < NU; u++) {
                                S.st(Lfrec + k * RSF + FK + u * NX, pj, kc[u]);
                                s_ += kc[u] * hu[u];
                            }
                            if (k > 0) pv[pj] = s_;
                        }
                        if (k > 0) {
#pragma unroll
                            for (int t = 0; t < Gm::EP; t++) {
                                const int i = pi0 + t;
                                if (t < pn) {
                                    T s_ = fp[i * LDZ + pj];
#pragma unroll
                                    for (int u = 0; u < NU; u++) s_ += fp[i * LDZ + NX + u] * kc[u];
                                    fp[i * LDZ + pj] = s_;
                                    fp[pj * LDZ + i] = s_;
                                }
                            }
                        }
                    }
                    // next stage's re and Sigma -> LDS (their last readers ran in phases 1 and 2)
                    if (k > 0) {
                        if (ll < NX) rv[ll] = qn.re;
                        if (ll < NZ) sv[ll] = qn.sg;
                    }
                    q = qn;
                    WAVE_SYNC();
                    NMPC_PTICK(3);
                }
            }
            SWEEP_FENCE();
            };

            // ============================ exact finish (groups with mu <= polish_at): a primal-dual
            // active-set run of penalised factorisations + forward sweeps (<= polish_steps set steps,
            // then the refinement); accepted groups write their outputs and are done, the others go on
            // with this iteration from their untouched IPM iterate
            pol = active && p.polish_mu > T(0) && mu <= polish_at;
            if (__any(pol)) {
                polish_at = pol ? fmin(polish_at, mu) * p.polish_drop : polish_at;
                const int plim = fin_runs == 0 ? p.polish_first : p.polish_steps;   // set steps of this run
                fin_runs += pol ? 1 : 0;
                fref = false;
                for (int fs = 0; fs <= (p.polish_first > p.polish_steps ? p.polish_first : p.polish_steps); fs++) {
                    fs0 = fs == 0;
                    fwarm = warm && fs0 && it == 0;
                    pfail = false;
                    factor(true);
                    // set steps -> dz, refinement corrections -> sg (dz and the flags in dza stay)
                    forward(Lsg, fref ? 0u : (unsigned)(Ldz - Lsg));
                    T nbad = 0, nact = 0, nrem = 0;
                    T *cmn = w + Gm::I_CM + (1 - cmb) * Gm::LDX;   // this step's candidate maxima
                    if (ll < NX) cmn[ll] = T(0);
                    WAVE_SYNC();
                    for (int e = ll; e < nel; e += G) {
                        const int k = e / NZ, i = e - k * NZ;
                        if ((k == N && i >= NX) || (k == 0 && i < NX)) continue;
                        const T lam_l = S.ld(Lll, e), lam_u = S.ld(Llu, e);
                        const T lb = clb[stype(k) * LDZ + i], ub = cub[stype(k) * LDZ + i];
                        T z = S.ld(Lz, e);
                        const T a = fin_flag(k, i, e, z, lam_l, lam_u, lb, ub);
                        const T dz = fref ? S.ld(Lsg, e) : S.ld(Ldz, e);
                        if (fref) z += S.ld(Ldz, e);
                        const T zn = z + dz;
                        const bool vl = lam_l > T(0), vu = lam_u > T(0);
                        const T tl = T(1e-9) * (T(1) + fabs(lb)), tu = T(1e-9) * (T(1) + fabs(ub));
                        const bool lo = vl && zn < lb - tl, hi = vu && zn > ub + tu;
                        bool bad = !isfinite(zn);   // a non-finite step is never accepted
                        T na = a;
                        if (fref) {
                            bad |= !(fabs(dz) <= T(1e-3) * (T(1) + fabs(z))) || (a < T(0) && fabs(zn - lb) > tl) ||
                                  (a > T(0) && fabs(zn - ub) > tu) || (a == T(0) && (lo || hi));
                        } else {
                            const bool rl = a < T(0) && zn > fma(T(1e-15), T(1) + fabs(lb), lb);
                            const bool ru = a > T(0) && zn < fma(T(-1e-15), T(1) + fabs(ub), ub);
                            const bool al = a == T(0) && lo, au = a == T(0) && !lo && hi;
                            bad |= rl || ru || al || au;
                            // inputs join at once, states as candidates +-(2 + violation)
                            const T cv = i < NX ? T(2) + (al ? lb - zn : zn - ub) : T(1);
                            na = (rl || ru) ? T(0) : (al ? -cv : (au ? cv : a));
                            if (i < NX && (al || au)) lds_max(&cmn[i], cv - T(2));
                            if (pol) S.st(Ldza, e, na);
                            nact += na != T(0) ? T(1) : T(0);
                            nrem += (rl || ru) ? T(1) : T(0);
                        }
                        nbad += bad ? T(1) : T(0);
                    }
                    nbad = group_sum<G>(nbad);
                    nact = group_sum<G>(nact);
                    nrem = group_sum<G>(nrem);
                    addok = fs0 || nrem == T(0);
                    cmb = 1 - cmb;
                    WAVE_SYNC();
                    bool done = false, done_ref = false;
                    if (pol) {
                        fin_steps++;
                        const bool okp = nbad == T(0) && !pfail;
                        if (fref) {
                            done = done_ref = okp;
                            pol = false;
                        } else if (okp && nact == T(0)) {
                            done = true;   // no active bound: an unpenalised Newton step, nothing to refine
                            pol = false;
                        } else if (okp) {
                            fref = true;
                        } else if (pfail || fs + 1 >= plim) {
                            pol = false;
                        }
                    }
                    if (done) {   // outputs: z + set step + refinement, clamped onto the bounds
                        active = false;
                        status = -1;
                        iters = it + fin_steps;
                        if (inst_ok) {
                            for (int e = ll; e < nel; e += G) {
                                const int k = e / NZ, i = e - k * NZ;
                                if (k == N && i >= NX) continue;
                                const T lb = clb[stype(k) * LDZ + i], ub = cub[stype(k) * LDZ + i];
                                T z = S.ld(Lz, e);
                                if (!(k == 0 && i < NX)) z += S.ld(Ldz, e) + (done_ref ? S.ld(Lsg, e) : T(0));
                                z = has_bound(lb) ? fmax(z, lb) : z;
                                z = has_bound(ub) ? fmin(z, ub) : z;
                                if (i < NX) p.xout[((size_t)inst * (N + 1) + k) * NX + i] = z;
                                else p.uout[((size_t)inst * N + k) * NU + (i - NX)] = z;
                                if (fused) S.st(Lact, e, act_flag(z, lb, ub));
                            }
                        }
                    }
                    SWEEP_FENCE();
                    if (!__any(pol)) break;
                }
                pol = fref = false;
                fwarm = false;
                if (!__any(active)) break;
            }
            factor(false);
            NMPC_TICK(1);

            // ============================ B: forward predictor; E_B: ratio test + centring sums
            forward(Ldza);
            NMPC_TICK(2);
            T a_aff = 1, S0 = 0, S2 = 0;
            for (int e = ll; e < nel; e += G) {
                const int k = e / NZ, i = e - k * NZ;
                if (k == N && i >= NX) continue;
                const T z = S.ld(Lz, e), lam_l = S.ld(Lll, e), lam_u = S.ld(Llu, e), dz = S.ld(Ldza, e);
                if (lam_l > T(0)) {
                    const T t = z - clb[stype(k) * LDZ + i], it_ = frcp(t);
                    const T dl = -lam_l * (T(1) + dz * it_);
                    if (dz < T(0)) a_aff = fmin(a_aff, -t * frcp(dz));
                    if (dl < T(0)) a_aff = fmin(a_aff, -lam_l * frcp(dl));
                    S0 += lam_l * t;
                    S2 += lam_l * dz * (t + dz) * it_;
                }
                if (lam_u > T(0)) {
                    const T t = cub[stype(k) * LDZ + i] - z, it_ = frcp(t);
                    const T dl = -lam_u * (T(1) - dz * it_);
                    if (dz > T(0)) a_aff = fmin(a_aff, t * frcp(dz));
                    if (dl < T(0)) a_aff = fmin(a_aff, -lam_u * frcp(dl));
                    S0 += lam_u * t;
                    S2 += lam_u * dz * (dz - t) * it_;
                }
            }
            a_aff = group_min<G>(a_aff);
            S0 = group_sum<G>(S0);
            S2 = group_sum<G>(S2);
            // mu_aff = [(1 - a) S0 - a^2 S2'] / m  with S2' = sum lam dz (t + dz) / t (closed form)
            const T mu_aff = ((T(1) - a_aff) * S0 - a_aff * a_aff * S2) * p.inv_m;
            const T sgm = mu > T(0) ? fmax(mu_aff, T(0)) * frcp(mu) : T(0);
            smu = sgm * sgm * sgm * mu;
            NMPC_TICK(3);

            // ============================ E_C: corrector rhs g^ = g + (dlam_a dz_a -/+ sigma mu) / t
            for (int e = ll; e < nel; e += G) {
                const int k = e / NZ, i = e - k * NZ;
                if (k == N && i >= NX) continue;
                const T z = S.ld(Lz, e), lam_l = S.ld(Lll, e), lam_u = S.ld(Llu, e), dza = S.ld(Ldza, e);
                T g = S.ld(Lgf, e);
                if (lam_l > T(0)) {
                    const T t = z - clb[stype(k) * LDZ + i], it_ = frcp(t), dl = -lam_l * (T(1) + dza * it_);
                    g += (dl * dza - smu) * it_;
                }
                if (lam_u > T(0)) {
                    const T t = cub[stype(k) * LDZ + i] - z, it_ = frcp(t), dl = -lam_u * (T(1) - dza * it_);
                    g += (dl * dza + smu) * it_;
                }
                if (k < N) S.st(Lcrec + k * RSC + CGH, i, g);
                else S.st(Lgf, e, g);
            }
            SWEEP_FENCE();
            NMPC_TICK(4);

            // ============================ C: backward corrector vector (kff, p)
            {
                {
                    const T gN = S.ld(Lgf + N * NZ, ll);
                    if (ll < NX) pv[ll] = gN;
                }
                T abcol[NX];   // column ll of [A B], register-resident for the whole sweep
                load_abcol(abcol);
                T r[DF][NSF + NSC];
#pragma unroll
                for (int j = 0; j < DF; j++) rec_issue(r[j], N - 1 - j, true);
                rec_put(r[0], 0, true);
                rec_issue(r[0], N - 1 - DF, true);
                WAVE_SYNC();
                for (int kb = N - 1; kb >= 0; kb -= DF)
#pragma unroll
                for (int j = 0; j < DF; j++) {
                    const int k = kb - j;
                    if (k < 0) break;
                    const T *fr = rb + ((N - 1 - k) & 1) * RB1, *cr = fr + NSF * G;
                    if (ll < NX) vv[ll] = cr[CPR + ll] + pv[ll];
                    WAVE_SYNC();
                    if (ll < NZ) hv[ll] = dot2<NX>(cr[CGH + ll], [&](int l) { return abcol[l]; }, [&](int l) { return vv[l]; });
                    WAVE_SYNC();
                    T lf[NUT], hu[NU], x[NU];
#pragma unroll
                    for (int j = 0; j < NUT; j++) lf[j] = cr[CFI + j];
#pragma unroll
                    for (int j = 0; j < NU; j++) x[j] = hu[j] = hv[NX + j];
                    chol_solve<T, NU>(lf, x);
                    T mine = 0;
#pragma unroll
                    for (int j = 0; j < NU; j++) mine = (ll == j) ? -x[j] : mine;
                    if (ll < NU) S.st(Lfrec + k * RSF + FKFF, ll, mine);
                    if (k > 0 && ll < NX) {
                        T s_ = hv[ll];
#pragma unroll
                        for (int u = 0; u < NU; u++) s_ += fr[FK + u * NX + ll] * hu[u];
                        pv[ll] = s_;
                    }
                    rec_put(r[(j + 1) % DF], (N - k) & 1, true);
                    rec_issue(r[(j + 1) % DF], k - 1 - DF, true);
                    WAVE_SYNC();
                }
            }
            SWEEP_FENCE();
            NMPC_TICK(5);

            // ============================ D: forward corrector; E_D: step length + new mu
            forward(Ldz);
            NMPC_TICK(6);
            T amax = 1, T0 = 0, C1 = 0, C2 = 0;
            for (int e = ll; e < nel; e += G) {
                const int k = e / NZ, i = e - k * NZ;
                if (k == N && i >= NX) continue;
                const T z = S.ld(Lz, e), lam_l = S.ld(Lll, e), lam_u = S.ld(Llu, e);
                const T dz = S.ld(Ldz, e), dza = S.ld(Ldza, e);
                C2 += dz * T(0);   // NaN for a non-finite direction (caught at the step below)
                if (lam_l > T(0)) {
                    const T t = z - clb[stype(k) * LDZ + i], it_ = frcp(t);
                    const T dla = -lam_l * (T(1) + dza * it_);
                    const T dl = (smu - lam_l * t - dla * dza - lam_l * dz) * it_;
                    if (dz < T(0)) amax = fmin(amax, -t * frcp(dz));
                    if (dl < T(0)) amax = fmin(amax, -lam_l * frcp(dl));
                    T0 += lam_l * t;
                    C1 += dla * dza;
                    C2 += dl * dz;
                }
                if (lam_u > T(0)) {
                    const T t = cub[stype(k) * LDZ + i] - z, it_ = frcp(t);
                    const T dla = -lam_u * (T(1) - dza * it_);
                    const T dl = (smu - lam_u * t + dla * dza + lam_u * dz) * it_;
                    if (dz > T(0)) amax = fmin(amax, t * frcp(dz));
                    if (dl < T(0)) amax = fmin(amax, -lam_u * frcp(dl));
                    T0 += lam_u * t;
                    C1 += -dla * dza;
                    C2 += -dl * dz;
                }
            }
            amax = group_min<G>(amax);
            T0 = group_sum<G>(T0);
            C1 = group_sum<G>(C1);
            C2 = group_sum<G>(C2);
            const T a = fmin(T(1), T(0.995) * amax);
            // a failed factorisation (F_uu not positive definite) leaves the iterate as it stood at the
            // start of this iteration, like the oracle's early exit (oracle/c/riccati_ipm.c:222)
            if (active && !fail) {
                // m mu_new = (1 - a) S0 + a (m smu - C1) + a^2 C2
                const T mu_new = ((T(1) - a) * T0 + a * (smu * m_bounds - C1) + a * a * C2) * p.inv_m;
                if (!isfinite(mu_new) || !isfinite(a)) {
                    fail = true;   // non-finite direction: ends like a failed factorisation (iterate kept)
                } else {
                    mu = mu_new;
                    theta *= (T(1) - a);
                    alpha = a;
                    pending = true;
                }
            }
            NMPC_TICK(7);
        }

        // ------------------------------------------------------------------ apply pending step, outputs
        if (inst_ok) {
            T *xo = p.xout + (size_t)inst * (N + 1) * NX;
            T *uo = p.uout + (size_t)inst * N * NU;
            for (int e = ll; e < nel; e += G) {
                const int k = e / NZ, i = e % NZ;
                if (k == N && i >= NX) continue;
                if (status < 0) break;   // completed by the finish, outputs already written
                T z = S.ld(Lz, e);
                if (pending) z += alpha * S.ld(Ldz, e);
                if (i < NX) xo[k * NX + i] = z;
                else uo[k * NU + (i - NX)] = z;
                if (fused) S.st(Lact, e, act_flag(z, clb[stype(k) * LDZ + i], cub[stype(k) * LDZ + i]));
            }
            if (ll == 0) {
                p.status[inst] = status < 0 ? 0 : status;
                p.iters[inst] = iters;
                if (fused && p.iter_log)   // finish steps | IPM iterations << 8 | status << 16
                    p.iter_log[(size_t)cstep * p.B + inst] = fin_steps | ((iters - fin_steps) << 8) | ((status < 0 ? 0 : status) << 16);
#ifdef NMPC_SWEEP_TIMING
                if (timed) {
                    unsigned long long *c = p.cycles + (size_t)inst * 9;
                    for (int j = 0; j < 8; j++) c[j] = tcy[j];
                    c[8] = __builtin_amdgcn_s_memtime() - tstart;
                }
#endif
            }
        }
        if (fused) {
            // closed-loop advance of this step by the instance's lanes (nmpc_cl_device.h), after the
            // outputs written above by this wavefront; the next step reads the new state
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            if (inst_ok)
                cl_advance_group<T, NX, NU>(p.cl, inst, p.cl.step + cstep, status < 0 ? 0 : status, ll,
                                            p.cl_noise[(size_t)inst * nsteps + cstep]);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        }
    }
}

// ---------------------------------------------------------------------- dispatch table
template <typename T, int NX, int NU, int IPW, int WPB, int MW>
static hipError_t launch_ipm(const IpmParams<T> &p, hipStream_t s)
{
    const int waves = (p.B + IPW - 1) / IPW;
    const int blocks = (waves + WPB - 1) / WPB;
    NMPC_LAUNCH((ipm_kernel<T, NX, NU, IPW, WPB, MW>), dim3(blocks), dim3(64 * WPB), 0, s, p);
    return hipGetLastError();
}

template <typename T>
struct IpmEntry {
    int kind;   // 0: one wavefront per IPW-instance lane block (ipm_kernel), 1: lane per component (ipm_lpc_kernel)
    int nx, nu, ipw, wpb, mw;
    hipError_t (*fn)(const IpmParams<T> &, hipStream_t);
    int lds_bytes;
    size_t (*scratch)(int B, int N);
    int sid;    // model structure the kernel is specialised for (0: dense, any model)
    bool (*fits)(const double *AB, const double *H, const double *He);
};

template <typename T, int NX, int NU, int IPW, int WPB>
static size_t wave_scratch_elems(int B, int N)
{
    const size_t per_wg = (size_t)IPW * WPB;
    return ((size_t)B + per_wg - 1) / per_wg * per_wg * ScratchLayout(N, NX, NU).total;
}

// MW: minimum wavefronts per SIMD requested from the register allocator (__launch_bounds__)
template <typename T, int NX, int NU, int IPW, int WPB, int MW = 1>
static constexpr IpmEntry<T> entry()
{
    return IpmEntry<T>{0, NX, NU, IPW, WPB, MW, &launch_ipm<T, NX, NU, IPW, WPB, MW>,
                       (int)(sizeof(T) * Geometry<T, NX, NU, IPW, WPB>::LDS_ELEMS),
                       &wave_scratch_elems<T, NX, NU, IPW, WPB>, 0, nullptr};
}

template <typename T, int NX, int NU, int WPB, int MW, class SP = lpc::DenseStructure<NX, NU>>
static constexpr IpmEntry<T> entry_lpc()
{
    return IpmEntry<T>{1, NX, NU, lpc::Geom<T, NX, NU, WPB>::IPW, WPB, MW, &launch_ipm_lpc<T, NX, NU, WPB, MW, SP>,
                       (int)(sizeof(T) * lpc::Geom<T, NX, NU, WPB>::LDS_ELEMS), &lpc::scratch_elems<T, NX, NU, WPB, SP::hdiag>,
                       SP::id, SP::id ? &lpc::structure_fits<SP, NX, NU> : nullptr};
}

// lane-per-instance kernels (nmpc_ipm_lpi.hip): W instances per wavefront, chosen so that the
// batch gives about one wavefront per SIMD (1024 on MI355X); env NMPC_LPI_W overrides
int lpi_instances_per_wave(int B)
{
    if (const char *e = getenv("NMPC_LPI_W")) {
        const int w = atoi(e);
        if (w >= 1 && w <= 64) return w;
    }
    const int w = (B + 1023) / 1024;
    return w < 1 ? 1 : (w > 64 ? 64 : w);
}

template <typename T, int NX, int NU>
static size_t lpi_scratch_elems(int B, int N)
{
    const int W = lpi_instances_per_wave(B);
    const size_t S = ((size_t)B + W - 1) / W * W;
    return (size_t)(N + 1) * lpi_words<NX, NU>() * S;
}

template <typename T, int NX, int NU, class SP = lpc::DenseStructure<NX, NU>>
static constexpr IpmEntry<T> entry_lpi()
{
    return IpmEntry<T>{3, NX, NU, 1, 4, 1, &launch_ipm_lpi<T, NX, NU, SP>, 0, &lpi_scratch_elems<T, NX, NU>, SP::id,
                       SP::id ? &lpc::structure_fits<SP, NX, NU> : nullptr};
}

template <typename T>
static const IpmEntry<T> *table(int *n)
{
    static const IpmEntry<T> t[] = {
        entry<T, 4, 2, 1, 4>(), entry<T, 4, 2, 2, 4>(), entry<T, 4, 2, 4, 4>(), entry<T, 4, 2, 8, 4>(),
        entry<T, 6, 2, 1, 4>(), entry<T, 6, 2, 2, 4>(), entry<T, 6, 2, 4, 4>(),
        // quad13: the first entry is the default (measured fastest, profiles/); the rest are
        // selectable with NMPC_VARIANT for tuning runs
        entry<T, 13, 4, 1, 1, 3>(), entry<T, 13, 4, 1, 4>(), entry<T, 13, 4, 1, 1, 2>(),
        entry<T, 13, 4, 1, 4, 3>(), entry<T, 13, 4, 1, 2, 4>(),
        // lane-per-component kernels (the default family); the first listed per (nx, nu) is
        // the default variant
        entry_lpc<T, 13, 4, 2, 2>(), entry_lpc<T, 13, 4, 4, 3>(), entry_lpc<T, 13, 4, 1, 3>(),
        entry_lpc<T, 4, 2, 4, 2>(), entry_lpc<T, 6, 2, 4, 2>(),
        // their structure-specialised twins (chosen by ipm_refine when the model fits)
        entry_lpc<T, 13, 4, 2, 2, lpc::Quad13Structure>(), entry_lpc<T, 13, 4, 4, 3, lpc::Quad13Structure>(),
        entry_lpc<T, 13, 4, 1, 3, lpc::Quad13Structure>(), entry_lpc<T, 4, 2, 4, 2, lpc::ForceStructure>(),
        entry_lpc<T, 6, 2, 4, 2, lpc::JerkStructure>(),
        // lane-per-instance kernels for the small models, dense and structure-specialised
        entry_lpi<T, 4, 2>(), entry_lpi<T, 6, 2>(),
        entry_lpi<T, 4, 2, lpc::ForceStructure>(), entry_lpi<T, 6, 2, lpc::JerkStructure>(),
    };
    *n = (int)(sizeof(t) / sizeof(t[0]));
    return t;
}

// kernel family: NMPC_KERNEL=lpc / =wave forces one; by default the lane-per-component
// kernels (ipm_lpc_kernel) run when the stage is wide (nx + nu >= 12: quad13) or the batch fills
// at least 384 of their wavefronts, else the wavefront-per-instance ones — for small models at
// small batches their per-instance latency floor is lower (tools/family_pairs.sh, fp64, lpc vs
// wave: force N=20 B=1024 1.09 vs 0.98 ms, B=4096 1.19 vs 1.31, B=8192 1.29 vs 1.88; jerk N=40
// B=2048 1.03 vs 0.91, B=4096 1.05 vs 1.16, B=8192 1.14 vs 1.79)
static int kernel_kind(int nx, int nu, int batch, bool f64)
{
    const char *k = getenv("NMPC_KERNEL");
    if (k && (k[0] == 'w' || k[0] == 'W')) return 0;
    if (k && (strcmp(k, "lpi") == 0 || strcmp(k, "LPI") == 0)) return 3;
    if (k && (k[0] == 'l' || k[0] == 'L')) return 1;
    const int nz = nx + nu;
    if (nz > 64) return 0;
    const long waves = ((long)batch + 64 / nz - 1) / (64 / nz);
    // round 2 (fast finish in the lane-per-component family, fp64 closed loops): jerk (nz = 8) runs it
    // faster from B = 1024 (7.3M vs 6.1M steps/s; B = 2048 12.8M vs 10.0M); force (nz = 6) does not —
    // its input-saturation sets exceed the fast finish's 8 bounds — so fp64 force stays on the
    // wavefront family up to B = 8192 (B = 1024 3.5M vs 2.0M, 4096 8.2M vs 6.2M, 8192 10.1M either);
    // fp32 (no finish) keeps the IPM-only crossover of 384 lane-per-component wavefronts
    if (nz >= 8) return 1;
    return waves >= (f64 ? 820 : 384) ? 1 : 0;
}

template <typename T>
int ipm_find(int nx, int nu, int ipw_req, int batch, int *ipw_out, int *lds_out, int *wpb_out)
{
    int n;
    const IpmEntry<T> *t = table<T>(&n);
    const int kind = kernel_kind(nx, nu, batch, sizeof(T) == 8);
    int best = -1;
    // NMPC_VARIANT=k picks the k-th compiled kernel of this (nx, nu) and family (tuning runs)
    const char *var = getenv("NMPC_VARIANT");
    if (var) {
        int want = atoi(var), seen = 0;
        for (int i = 0; i < n; i++) {
            if (t[i].nx != nx || t[i].nu != nu || t[i].kind != kind || t[i].sid) continue;
            if (seen++ == want) {
                *ipw_out = t[i].ipw;
                *lds_out = t[i].lds_bytes;
                if (wpb_out) *wpb_out = t[i].wpb;
                return i;
            }
        }
    }
    bool have = false;
    for (int i = 0; i < n; i++) have |= t[i].nx == nx && t[i].nu == nu && t[i].kind == kind && !t[i].sid;
    const int fam = have ? kind : (kind == 3 ? 1 : 1 - kind);   // no lane-per-instance twin: lane per component
    for (int i = 0; i < n; i++) {
        if (t[i].nx != nx || t[i].nu != nu || t[i].kind != fam || t[i].sid) continue;
        if (fam == 1) {   // lane-per-component: instances per wave fixed by nx + nu, first listed
            if (best < 0) best = i;
        } else if (fam == 3) {   // lane-per-instance: instances per wave from the batch
            if (best < 0) best = i;
        } else if (ipw_req > 0) {
            if (t[i].ipw == ipw_req && best < 0) best = i;   // first listed = preferred variant
        } else if (best < 0 || t[i].ipw > t[best].ipw) {
            best = i;
        }
    }
    if (best < 0) return -1;
    *ipw_out = t[best].kind == 3 ? lpi_instances_per_wave(batch) : t[best].ipw;
    *lds_out = t[best].lds_bytes;
    if (wpb_out) *wpb_out = t[best].wpb;
    return best;
}

// the first compiled dense entry of family `kind` for (nx, nu), or -1 (the lean closed loop's list-mode
// fallback runs the lane-per-component family whatever the handle's own family is)
template <typename T>
int ipm_find_family(int nx, int nu, int kind)
{
    int n;
    const IpmEntry<T> *t = table<T>(&n);
    for (int i = 0; i < n; i++)
        if (t[i].nx == nx && t[i].nu == nu && t[i].kind == kind && !t[i].sid) return i;
    return -1;
}

template int ipm_find_family<double>(int, int, int);
template int ipm_find_family<float>(int, int, int);

template <typename T>
hipError_t ipm_launch(int idx, const IpmParams<T> &p, hipStream_t s)
{
    int n;
    const IpmEntry<T> *t = table<T>(&n);
    return t[idx].fn(p, s);
}

template <typename T>
size_t ipm_scratch_elems(int idx, int B, int N)
{
    int n;
    const IpmEntry<T> *t = table<T>(&n);
    return t[idx].scratch(B, N);
}

// the structure-specialised twin of dense entry `idx` (same family, shape, workgroup and
// occupancy target) whose structure the model fits, else idx. NMPC_STRUCT=0 disables.
template <typename T>
int ipm_refine(int idx, const double *AB, const double *H, const double *He)
{
    int n;
    const IpmEntry<T> *t = table<T>(&n);
    const char *e = getenv("NMPC_STRUCT");
    if (e && e[0] == '0') return idx;
    const IpmEntry<T> &d = t[idx];
    for (int i = 0; i < n; i++) {
        const IpmEntry<T> &c = t[i];
        if (c.sid && c.kind == d.kind && c.nx == d.nx && c.nu == d.nu && c.wpb == d.wpb && c.mw == d.mw &&
            c.fits(AB, H, He))
            return i;
    }
    return idx;
}

template <typename T>
int ipm_structure(int idx)
{
    int n;
    const IpmEntry<T> *t = table<T>(&n);
    return t[idx].sid;
}

template int ipm_refine<double>(int, const double *, const double *, const double *);
template int ipm_refine<float>(int, const double *, const double *, const double *);
template int ipm_structure<double>(int);
template int ipm_structure<float>(int);

template <typename T>
int ipm_kind(int idx)
{
    int n;
    const IpmEntry<T> *t = table<T>(&n);
    return t[idx].kind;
}

template int ipm_kind<double>(int);
template int ipm_kind<float>(int);
template size_t ipm_scratch_elems<double>(int, int, int);
template size_t ipm_scratch_elems<float>(int, int, int);
template int ipm_find<double>(int, int, int, int, int *, int *, int *);
template int ipm_find<float>(int, int, int, int, int *, int *, int *);
template hipError_t ipm_launch<double>(int, const IpmParams<double> &, hipStream_t);
template hipError_t ipm_launch<float>(int, const IpmParams<float> &, hipStream_t);

}  // namespace nmpc
