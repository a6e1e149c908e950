// nmpc_ipm_lpc.hip — batched box-constrained LQ-OCP solver, lane-per-component layout (gfx950).
//
// Same problem and algorithm as nmpc_ipm.hip and oracle/c/riccati_ipm.c (one
// `AcadosOcpSolver.solve()` of src/force_model/controller.py:32 / src/jerk_model/controller.py:33:
// SQP-GN on an LTI / LINEAR_LS / box-constrained OCP == one QP, solved by a Mehrotra
// predictor-corrector interior-point method with a backward Riccati recursion per Newton
// system), mapped differently onto the CDNA4 wavefront:
//
//   * a lane group of NZ = nx + nu lanes owns one instance, IPW = 64 / NZ instances per
//     wavefront (quad13: 3 x 17 lanes); lane r owns component r of every stage z_k = [x_k; u_k]
//     (x-lanes r < nx, u-lanes r >= nx). All per-element iterates (z, lambda, steps) and every
//     per-stage record a lane reads back later were written by that same lane, so the HBM
//     scratch needs no cross-lane hand-off and no fences;
//   * the stage recursions keep their state in registers: x-lane i holds row i of P_{k+1}; the
//     stage products use the model matrix [A B] as a wave-uniform SGPR operand (constant
//     address space, s_load_dwordx16 streams), so the 13x17 products M = P [A B] (row i per
//     x-lane) and F = [A B]' M + H (column r per lane) are v_fma_f64 chains with 17
//     independent accumulators and no LDS operand traffic; M crosses lanes once through LDS
//     (transposed), F_uu / h_u / L^{-1} F_ux cross once each;
//   * the elementwise work of the IPM is fused into the four stage sweeps of an iteration:
//       A  backward Riccati factorisation; applies the previous step lazily, forms Sigma,
//          g = H z + G yref and the dynamics residual re of stage k on the fly;
//       B  forward predictor; ratio test and centring sums on the fly;
//       C  backward corrector vector; corrector right-hand side on the fly;
//       D  forward corrector; step length and the new complementarity measure (closed form
//          in alpha) on the fly;
//   * group reductions (min/sum over the NZ lanes of an instance) run on ds_bpermute.
//
// The diagonal barrier term Sigma of P (x part) is carried separately from the row of P
// (sdiag), so no lane ever indexes its registers with its own lane number.

#include <hip/hip_runtime.h>

#include "nmpc_cl_device.h"
#include "nmpc_internal.h"
#include "nmpc_lpc_geom.h"

#define NMPC_COMMA ,

// stage records in flight ahead of the vector sweeps B, C, D
#ifndef NMPC_LPC_PF
#define NMPC_LPC_PF 2
#endif
// Riccati / corrector-vector stages (experiment knob, off: measured 2-3 % slower on quad13): run
// the work the first LDS exchange does not need (dual part of the lazy step, Sigma, the corrector
// right-hand side) after that exchange instead of before it
#ifndef NMPC_LPC_EARLY_Z
#define NMPC_LPC_EARLY_Z 0
#endif
// structured Riccati stage: Sigma_x [A B](r, :) added to M^T by LDS atomics (1) or folded into
// the M accumulators from the dense LDS row (0)
#ifndef NMPC_LPC_ATOMIC_DIAG
#define NMPC_LPC_ATOMIC_DIAG 0
#endif
// forward sweeps: statistics of stage k-1 computed inside stage k's first LDS exchange
#ifndef NMPC_LPC_DEFER
#define NMPC_LPC_DEFER 1
#endif
// rows of Y = L^{-1} F_ux per LDS chunk in the P update of the Riccati stage
#ifndef NMPC_LPC_PCH
#define NMPC_LPC_PCH 2
#endif

namespace nmpc {
namespace lpc {

#define LPC_SYNC()                                               \
    do {                                                         \
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   \
        __builtin_amdgcn_wave_barrier();                         \
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   \
        asm volatile("" ::: "memory");                           \
    } while (0)

template <typename T>
using cptr = const T __attribute__((address_space(4))) *;

// Newton steps after the hardware fp64 rsq / rcp estimates (experiment builds may set 1)
#ifndef NMPC_LPC_NEWTON
#define NMPC_LPC_NEWTON 2
#endif
__device__ __forceinline__ double frsq(double x)
{
    double y = __builtin_amdgcn_rsq(x);
    const double h = 0.5 * x;
    y = fma(y, fma(-h, y * y, 0.5), y);
    if (NMPC_LPC_NEWTON > 1) y = fma(y, fma(-h, y * y, 0.5), y);
    return y;
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
    if (NMPC_LPC_NEWTON > 1) r = fma(fma(-x, r, 1.0), r, r);
    return r;
}
__device__ __forceinline__ float frcp(float x)
{
    float r = __builtin_amdgcn_rcpf(x);
    return fmaf(fmaf(-x, r, 1.0f), r, r);
}

// hardware reciprocal estimate without refinement (step-length heuristics only)
__device__ __forceinline__ double rcp_raw(double x) { return __builtin_amdgcn_rcp(x); }
__device__ __forceinline__ float rcp_raw(float x) { return __builtin_amdgcn_rcpf(x); }

__host__ __device__ constexpr int tri(int i, int j) { return i * (i + 1) / 2 + j; }

// x <- F_uu^{-1} x with the packed Cholesky factor (inverse diagonal)
template <typename T, int NU>
__device__ __forceinline__ void chol_solve(const T (&lf)[NU * (NU + 1) / 2], T (&x)[NU])
{
#pragma unroll
    for (int i = 0; i < NU; i++) {
        T s = x[i];
#pragma unroll
        for (int l = 0; l < i; l++) s = fma(-lf[tri(i, l)], x[l], s);
        x[i] = s * lf[tri(i, i)];
    }
#pragma unroll
    for (int i = NU - 1; i >= 0; i--) {
        T s = x[i];
#pragma unroll
        for (int l = i + 1; l < NU; l++) s = fma(-lf[tri(l, i)], x[l], s);
        x[i] = s * lf[tri(i, i)];
    }
}

// reductions over the NZ lanes of each lane group (tree on ds_bpermute, result broadcast)
template <int NZ, typename T, typename Op>
__device__ __forceinline__ T gred(T v, int lane, int r, Op op)
{
#pragma unroll
    for (int s = 1; s < NZ; s <<= 1) {
        const T o = __shfl(v, lane + s < 64 ? lane + s : 63, 64);
        if (r + s < NZ) v = op(v, o);
    }
    return __shfl(v, lane - r, 64);
}

// Stream the rows of a wave-uniform NR x NC matrix (constant address space) through SGPRs in
// chunks of RPC rows, one chunk ahead of its use: body(l, row) consumes row l while the next
// chunk is in flight. Only entries the structure SP allows are loaded (the rest read as 0 and
// the bodies skip them). The loads are inline-asm s_loads (not rematerialisable) followed by
// one explicit lgkmcnt(0) wait per chunk; the scheduling barriers keep the chunks in order.
template <int NR, int NC, int RPC, class SP, typename T, typename Body>
__device__ __forceinline__ void sgpr_rows(cptr<T> m, Body body)
{
    constexpr int NCH = (NR + RPC - 1) / RPC;
    T cur[RPC][NC], nxt[RPC][NC];
    auto load = [&](int ch, T (&dst)[RPC][NC]) {
#pragma unroll
        for (int rr = 0; rr < RPC; rr++) {
            const int l = ch * RPC + rr;
#pragma unroll
            for (int c = 0; c < NC; c++) {
                if (l < NR && SP::ab(l, c)) {
                    if constexpr (sizeof(T) == 8) {
                        asm volatile("s_load_dwordx2 %0, %1, %2" : "=s"(dst[rr][c]) : "s"(m), "i"((l * NC + c) * 8));
                    } else {
                        asm volatile("s_load_dword %0, %1, %2" : "=s"(dst[rr][c]) : "s"(m), "i"((l * NC + c) * 4));
                    }
                } else {
                    dst[rr][c] = T(0);
                }
            }
        }
    };
    load(0, cur);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int ch = 0; ch < NCH; ch++) {
        if (ch + 1 < NCH) load(ch + 1, nxt);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int rr = 0; rr < RPC; rr++)
            if (ch * RPC + rr < NR) body(ch * RPC + rr, cur[rr]);
        __builtin_amdgcn_sched_barrier(0);
        if (ch + 1 < NCH) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int rr = 0; rr < RPC; rr++)
#pragma unroll
                for (int c = 0; c < NC; c++) cur[rr][c] = nxt[rr][c];
        }
    }
}

// compact row / column of [A B] (structured kernels): values and byte offsets, loaded ahead of
// the LDS vector they are dotted with (s0 + sum_j v_j vec[o_j])
template <typename T, int NL>
struct SpL {
    T v[NL];
    int o[NL];
};
template <typename T, int NL>
__device__ __forceinline__ void sp_load(SpL<T, NL> &q, const T *vals, const int *offs, int base)
{
#pragma unroll
    for (int j = 0; j < NL; j++) {
        q.v[j] = vals[base + j];
        q.o[j] = offs[base + j];
    }
}
template <typename T, int NL>
__device__ __forceinline__ T sp_dot(const SpL<T, NL> &q, const T *vec, T s0)
{
    T s1 = 0;
#pragma unroll
    for (int j = 0; j < NL; j++) {
        const T x = *(const T *)((const char *)vec + q.o[j]);
        if (j & 1) s1 = fma(q.v[j], x, s1);
        else s0 = fma(q.v[j], x, s0);
    }
    return s0 + s1;
}

// compile-time pass selectors of the sweeps (forward: 0 predictor, 1 corrector, 2 finish;
// Riccati: 0 ordinary, 1 finish)
template <int V>
struct Pass {
    static constexpr int value = V;
};

template <typename T>
__device__ __forceinline__ bool has_bound(T b)
{
    return fabs(b) < T(1e20);
}

// Scratch accessor: buffer resource in SGPRs, per-lane 32-bit byte offset (VGPR), stage
// offset (wave-uniform). readfirstlane pins the stage offset to an SGPR: without it the
// compiler may keep it in a VGPR and wrap every access in a waterfall loop.
template <typename T>
struct Buf {
    __amdgpu_buffer_rsrc_t r;
    __device__ T ld(unsigned uni, unsigned lane) const
    {
        const unsigned so = __builtin_amdgcn_readfirstlane(uni * (unsigned)sizeof(T));
        if constexpr (sizeof(T) == 8)
            return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(r, lane * 8u, so, 0));
        else
            return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(r, lane * 4u, so, 0));
    }
    __device__ void st(unsigned uni, unsigned lane, T v) const
    {
        const unsigned so = __builtin_amdgcn_readfirstlane(uni * (unsigned)sizeof(T));
        if constexpr (sizeof(T) == 8)
            __builtin_amdgcn_raw_buffer_store_b64(
                __builtin_bit_cast(unsigned __attribute__((ext_vector_type(2))), v), r, lane * 8u, so, 0);
        else
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, lane * 4u, so, 0);
    }
};

template <typename T, int NX, int NU, int WPB, int MW, class SP>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(MW, 8))) void ipm_lpc_kernel(IpmParams<T> p)
{
    // rows of [A B] per SGPR chunk: ~16 loaded elements per chunk
#ifndef NMPC_LPC_RPC_SPARSE
#define NMPC_LPC_RPC_SPARSE 16
#endif
    // structured kernels: ~NMPC_LPC_RPC_SPARSE nonzeros per chunk (all of [A B] in one chunk when it
    // is that sparse); dense kernels: one 17-wide row per chunk
    constexpr int RPC = SP::id == 0 ? 1
                                    : (NMPC_LPC_RPC_SPARSE / SP::max_row_nnz < 1 ? 1
                                       : (NMPC_LPC_RPC_SPARSE / SP::max_row_nnz < NX ? NMPC_LPC_RPC_SPARSE / SP::max_row_nnz : NX));
    using Gm = Geom<T, NX, NU, WPB>;
    constexpr int NZ = Gm::NZ, IPW = Gm::IPW, VS = Gm::VS, LDZ = Gm::LDZ, LDX = Gm::LDX, LDU = Gm::LDU;
    constexpr int NUT = NU * (NU + 1) / 2;
    constexpr int PD = NMPC_LPC_PF;
    constexpr int XPR = Gm::XPR, UKFF = Gm::UKFF, UFI = Gm::UFI;

    __shared__ __attribute__((aligned(16))) T lds[Gm::LDS_ELEMS];
    T *abr = lds + Gm::C_ABR, *abt = lds + Gm::C_ABT, *hm = lds + Gm::C_H, *hem = lds + Gm::C_HE;

    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int grp = lane / NZ, r = lane - grp * NZ;
    const bool xl = r < NX, ul = !xl;
    const int u = ul ? r - NX : 0;
    const int N = p.N;
    const unsigned wave_u = __builtin_amdgcn_readfirstlane(wave);
    const size_t wg = (size_t)blockIdx.x * WPB + wave_u;
    const long long inst_raw = (long long)wg * IPW + grp;
    // list mode (the lean closed loop's fallback): lane group g solves instance cl_list[g]
    const bool lmode = p.cl_list != nullptr;
    // a list whose length is on the device (written by an earlier kernel of the stream): workgroups past it
    // leave before any setup (the grid is sized for the longest possible list)
    const long long lcount = lmode ? (p.cl_count_dev ? (long long)__builtin_amdgcn_readfirstlane(*p.cl_count_dev)
                                                     : (long long)p.cl_count)
                                   : 0;
    if (lmode && (long long)blockIdx.x * WPB * IPW >= lcount) return;
    const bool inst_ok = grp < IPW && inst_raw < (lmode ? lcount : (long long)p.B);
    const int inst = inst_ok ? (lmode ? p.cl_list[inst_raw] : (int)inst_raw) : 0;   // idle lanes read instance 0, never write outputs

    // ---- model constants -> LDS (once per workgroup)
    for (int e = threadIdx.x; e < NX * NZ; e += 64 * WPB) {
        const T v = p.AB[e];
        abr[(e / NZ) * LDZ + e % NZ] = v;
        abt[(e % NZ) * LDX + e / NZ] = v;
    }
    for (int e = threadIdx.x; e < NZ * NZ; e += 64 * WPB) hm[(e / NZ) * LDZ + e % NZ] = p.H[e];
    for (int e = threadIdx.x; e < NX * NX; e += 64 * WPB) hem[(e / NX) * LDX + e % NX] = p.He[e];
    for (int e = threadIdx.x; e < 3 * NZ; e += 64 * WPB) {
        lds[Gm::C_LB + (e / NZ) * LDZ + e % NZ] = p.lbnd[e];
        lds[Gm::C_UB + (e / NZ) * LDZ + e % NZ] = p.ubnd[e];
    }
    // structured kernels: row l and column c of [A B] as compact (value, byte offset) lists for
    // the per-lane dot products of the sweeps (dynamics residual / forward update: row r of the
    // x-lane; h = [A B]' v: column r) — quad13: <= 5 / <= 4 terms instead of 17 / 13; padding
    // entries are (0, 0)
#ifdef NMPC_LPC_DENSE_SWEEPS
    constexpr bool SPARSE = false;   // experiment builds: dense rows / columns in the sweeps
#else
    constexpr bool SPARSE = SP::id != 0;
#endif
    constexpr int RN = SPARSE ? SP::max_row_nnz : 1, CN = SPARSE ? SP::max_col_nnz : 1;
    __shared__ __attribute__((aligned(16))) T slv[NX * RN + NZ * CN];
    __shared__ __attribute__((aligned(16))) int sli[NX * RN + NZ * CN];
    if constexpr (SPARSE) {
        const int t = threadIdx.x;
        if (t < NX) {
            int n = 0;
#pragma unroll
            for (int c = 0; c < NZ; c++)
                if (SP::ab(t, c)) {
                    slv[t * RN + n] = p.AB[t * NZ + c];
                    sli[t * RN + n] = c * (int)sizeof(T);
                    n++;
                }
            for (; n < RN; n++) {
                slv[t * RN + n] = T(0);
                sli[t * RN + n] = 0;
            }
        } else if (t < NX + NZ) {
            const int c = t - NX, base = NX * RN + c * CN;
            int n = 0;
#pragma unroll
            for (int l = 0; l < NX; l++)
                if (SP::ab(l, c)) {
                    slv[base + n] = p.AB[l * NZ + c];
                    sli[base + n] = l * (int)sizeof(T);
                    n++;
                }
            for (; n < CN; n++) {
                slv[base + n] = T(0);
                sli[base + n] = 0;
            }
        }
    }
    __syncthreads();
    if (!__any(inst_ok)) return;

    T *gb = lds + Gm::C_TOT + Gm::group_area(wave, grp) * Gm::G_TOT;
    T *zb = gb + Gm::G_ZB, *rb = gb + Gm::G_RB, *vb = gb + Gm::G_VB, *hub = gb + Gm::G_HU, *fu = gb + Gm::G_FU;
    T *mt = gb + Gm::G_MT, *ylds = gb + Gm::G_MT;

    // per-lane constants: bounds of component r for stage types (0: k = 0, 1: 0 < k < N, 2: k = N)
    const T c_r = xl ? p.c[r] : T(0);
    const T *clb = lds + Gm::C_LB + r, *cub = lds + Gm::C_UB + r;
    auto LB = [&](int k) { return clb[(k == 0 ? 0 : (k == N ? 2 : 1)) * LDZ]; };
    auto UB = [&](int k) { return cub[(k == 0 ? 0 : (k == N ? 2 : 1)) * LDZ]; };

    // ---- scratch: VS instance slots per wavefront, lane-owned elements
    using L = Layout<NX, NU, SP::hdiag>;
    Buf<T> S;
    S.r = __builtin_amdgcn_make_buffer_rsrc(p.scratch + wg * L::wave_elems(N), 0, (int)(L::wave_elems(N) * sizeof(T)),
                                            0x00020000);
    // lane-interleaved: every word is one run of L::LW lanes; idle lanes point past the buffer
    const unsigned lo = lane < L::LW ? (unsigned)lane : 0x1000000u;
    auto off = [&](int k, int w) { return ((unsigned)k * L::NW + (unsigned)w) * (unsigned)L::LW; };
    auto ldE = [&](int arr, int k) { return S.ld(off(k, arr), lo); };
    auto stE = [&](int arr, int k, T v) { S.st(off(k, arr), lo, v); };
    auto ldX = [&](int k, int w) { return S.ld(off(k, L::REC + w), lo); };
    auto stX = [&](int k, int w, T v) { S.st(off(k, L::REC + w), lo, v); };
    auto ldU = [&](int k, int w) { return S.ld(off(k, L::REC + w), lo); };
    auto stU = [&](int k, int w, T v) { S.st(off(k, L::REC + w), lo, v); };

    auto gmin = [&](T v) { return gred<NZ>(v, lane, r, [](T a, T b) { return fmin(a, b); }); };
    auto gmax = [&](T v) { return gred<NZ>(v, lane, r, [](T a, T b) { return fmax(a, b); }); };
    auto gsum = [&](T v) { return gred<NZ>(v, lane, r, [](T a, T b) { return a + b; }); };

    const int row_base = (xl ? r : 0) * RN, col_base = NX * RN + r * CN;

    // one solve per closed-loop step; plain solves run one step (p.cl_steps = 0)
    const bool fused = p.cl_steps > 0;
    const int nsteps = fused ? p.cl_steps : 1;
    // fused closed loop: the active flags of the last solution (the warm start) as a per-lane bit
    // mask, 2 bits per stage (1 lower, 2 upper; N <= 31), kept in registers for the whole launch and
    // in the scratch ACT words between launches — instead of one scratch word per stage and step
    const bool amask = fused && N <= 31;
    auto mflag = [](unsigned long long m, int k) {
        const unsigned b = (unsigned)(m >> (2 * k)) & 3u;
        return b == 1u ? T(-1) : (b == 2u ? T(1) : T(0));
    };
    auto mset = [](unsigned long long &m, int k, T f) {
        m = (m & ~(3ull << (2 * k))) | (f < T(0) ? (1ull << (2 * k)) : (f > T(0) ? (2ull << (2 * k)) : 0ull));
    };
    unsigned long long actm = 0;
    // the closed-loop step of this launch's first step: the handle's, or (list mode) the instance's own
    // (idle lanes of list mode sit at the noise table's first column: every address they form stays valid)
    const int cl_base = fused ? (lmode ? (inst_ok ? p.cl_istep[inst] : p.cl_noise_step0) : p.cl.step) : 0;
    if (amask && p.cl.step > 0 && !lmode)
        for (int k = 0; k <= N; k++) mset(actm, k, ldE(L::ACT, k));
    // fused closed loop with the controller-model plant (quad13), fp64, cost at x_0: the state stays in
    // the group's LDS for the whole launch (G_CL: state, this step's output z_0, yref row 0, sums),
    // the plant step is one LDS exchange and a row of the solver's own [A B] (the same data
    // nmpc_closed_loop_init uploads as the plant), and the cost / AED / failure sums of
    // cl_advance_group are accumulated in LDS and added to the global sums once at the end
    const bool fastpl = sizeof(T) == 8 && fused && p.cl.plant == 0 && p.cl.cost_stage == 0;
    T *const clx = lds + Gm::C_TOT + Gm::group_area(wave, grp) * Gm::G_TOT + Gm::G_CL, *const clz = clx + LDZ,
            *const cly = clz + LDZ, *const cls = cly + LDZ;
    if (fastpl) {
        clx[r] = (xl && inst_ok) ? p.cl.state[(size_t)inst * NX + r] : T(0);
        if (r < 4) cls[r] = T(0);
    }
#ifdef NMPC_STEP_TIMING
    // experiment builds only (build_experiment(..., ["NMPC_STEP_TIMING"]), env NMPC_SWEEP_CYCLES): clock
    // cycles of each phase of a closed-loop step, summed over the launch's steps: 0 certificate, 1
    // initial point, 2 finish Riccati, 3 finish forward, 4 IPM Riccati, 5 IPM B/C/D, 6 outputs, 7 advance
    // (slot 0: the warm-flag copy and the fast finish; slot 1: certificate + initial point)
    unsigned long long st_cy[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
    for (int cstep = 0; cstep < nsteps; cstep++) {
#ifdef NMPC_STEP_TIMING
        unsigned long long st_mark = __builtin_amdgcn_s_memtime();
        auto stick = [&](int slot) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            st_cy[slot] += t - st_mark;
            st_mark = t;
        };
#define LPC_STICK(slot) stick(slot)
#else
#define LPC_STICK(slot) ((void)0)
#endif
        // fused closed loop: the yref window straight from the reference table rows (offset + step) %
        // period (cl_prepare_kernel's gather), x0 from the closed-loop state
        const int t_ref = fused ? (p.cl.offset[inst] + cl_base + cstep) % p.cl.period : 0;
        const T *yref = fused ? p.cl.table + (size_t)t_ref * p.cl.table_cols
                              : p.yref + (size_t)inst * ((size_t)N * p.ny + p.ny_e);
        const int yrow = fused ? p.cl.table_cols : p.ny;
        const T *x0 = (fused ? p.cl.state : p.x0) + (size_t)inst * NX;
        const T x0r = fastpl ? clx[r] : (xl ? x0[r] : T(0));
        T *const xo = p.xout + (size_t)inst * (N + 1) * NX, *const uo = p.uout + (size_t)inst * N * NU;
        // the bounds of element (k, r) are read once per stage, ahead of their use (B)
        struct Bd {
            T lb, ub;
        };
        auto bnd = [&](int k) { return Bd{LB(k), UB(k)}; };
        // outputs of a finish step, written by its forward sweep (status -1 skips the output pass):
        // z_new clamped onto the bounds and, in the fused closed loop, its active flags (the next
        // step's warm start; u-lanes also write stage N, a mirror of N - 1). A step that is not
        // accepted is overwritten by a later one or by the output pass of an IPM-ended solve.
        auto fin_out = [&](int k, T z, const Bd &b) {
            z = has_bound(b.lb) ? fmax(z, b.lb) : z;
            z = has_bound(b.ub) ? fmin(z, b.ub) : z;
            if (xl) xo[k * NX + r] = z;
            else uo[k * NU + u] = z;
            if (fastpl && k == 0) clz[r] = z;
            if (fused) {
                const bool onl = has_bound(b.lb) && z <= b.lb + T(1e-7) * (T(1) + fabs(b.lb));
                const bool onu = has_bound(b.ub) && z >= b.ub - T(1e-7) * (T(1) + fabs(b.ub));
                const T f = onl ? T(-1) : (onu ? T(1) : T(0));
                if (amask) {
                    mset(actm, k, f);
                    if (ul && k == N - 1) mset(actm, N, f);
                } else {
                    stE(L::ACT, k, f);
                    if (ul && k == N - 1) stE(L::ACT, N, f);
                }
            }
        };
        // row r of [A B] as a compact list (structured kernels): certificate, initial point, plant step
        SpL<T, RN> arl0;
        if constexpr (SPARSE) sp_load(arl0, slv, sli, row_base);
    // fused closed loop after its first step: the first finish run of a solve starts from the
    // previous step's active set shifted by one stage (ACT word; warm start, the acceptance tests
    // are unchanged), read into the dza slots, which the first iteration does not use otherwise
    // (list mode: a cold solve — the lean loop parks an instance its fast path could not finish)
    const bool warm = fused && !lmode && (cstep > 0 || p.cl.step > 0);
    bool fwarm = false;   // wave-uniform: the current finish pass reads the warm flags
    // the warm-start set: the previous solution's flags (ACT), shifted by one stage, copied into the
    // DZA words the first finish step reads its flags from (so ACT is free for this solve's outputs),
    // and counted (an empty set takes the fast finish / lqr_back)
    T warm_act = 0;
    unsigned long long wm = 0;   // mask mode: the fast finish's working set (DZA only for a full solve)
    if (warm && amask) {
        for (int k = 0; k <= N; k++) {
            const bool valid = !(k == 0 && xl) && (k < N || xl);
            if (valid) mset(wm, k, mflag(actm, (p.warm_shift && k < N) ? k + 1 : k));
        }
        warm_act = gsum(T(__popcll(wm)));
    } else if (warm) {
        constexpr int AC = 4;
        for (int kc = 0; kc <= N; kc += AC) {
            T a_[AC];
#pragma unroll
            for (int j = 0; j < AC; j++) {
                const int k = kc + j <= N ? kc + j : N;
                a_[j] = ldE(L::ACT, (p.warm_shift && k < N) ? k + 1 : k);
            }
#pragma unroll
            for (int j = 0; j < AC; j++) {
                const int k = kc + j;
                const bool valid = k <= N && !(k == 0 && xl) && (k < N || xl);
                warm_act += (valid && a_[j] != T(0)) ? T(1) : T(0);
                if (k <= N) stE(L::DZA, k, valid ? a_[j] : T(0));
            }
        }
        warm_act = gsum(warm_act);
    }
#ifdef NMPC_STEP_SPLIT
    LPC_STICK(4);   // experiment builds: the warm-flag copy
#endif


        // ------------------------------------------------------------------ fast exact finish
        // (fused closed loop, structured kernels with diagonal gradient maps): when the warm-start set
        // is empty, the first finish step is the unconstrained LQ solution, taken here from the base
        // point z = 0 (a Newton step on the QP lands on the same point from any base): backward
        // p_N = g_N, v = p_{k+1} + P_{k+1} c, h = g_k + [A B]' v, kff_k = -F_uu^{-1} h_u,
        // p_k = h_x + K_k' h_u with g = G yref (one LDS exchange per stage, the factorisation from
        // p.lqr), then the forward rollout x_0 = x0, u_k = kff_k + K_k x_k, x_{k+1} = [A B] z_k + c.
        // If every bound holds (the finish's acceptance test for an empty set) the solve is complete
        // (status 0, one Newton system) and the group skips the certificate, the initial point and
        // the IPM; otherwise it runs the full solve below.
        bool fast_ok = false;
        int fin_ws = 0;   // active-set steps on the shared factorisation (counted in qp_iter)
        {
            // rollout records (p.lqrf, lqr_table): x-lane [q_r | K(:, r) | (B F_uu^{-1})(r, :) |
            // (A + B K)(r, :)], u-lane [0 | 0 | F_uu^{-1}(u, :) | K(u, :)]
            constexpr int WF = 1 + 2 * NU + NX, OM = 1, OW = 1 + NU, OR = 1 + 2 * NU;
            constexpr double FAST_TOL = 1e-13;
            const bool try_fast = SP::hdiag && p.lqrf != nullptr && p.g_diag && p.polish_mu > T(0) && warm && inst_ok &&
                                  p.fast_mode != 0 && (p.fast_mode == 1 || cstep > 0) &&
                                  (warm_act == T(0) || p.lqrw != nullptr);
            const bool empty0 = warm_act == T(0);   // the unconstrained solution is the first set step
            if (__any(try_fast)) {
                const T gdr = p.G[r * p.ny + r], gde = xl ? p.Ge[r * p.ny_e + r] : T(0);
                T gdu[NU];
#pragma unroll
                for (int i = 0; i < NU; i++) gdu[i] = p.G[(NX + i) * p.ny + NX + i];
                SpL<T, CN> acl;
                if constexpr (SPARSE) sp_load(acl, slv, sli, col_base);
                const T *acol = abt + r * LDX;
                auto frow = [&](int k, int lane) { return p.lqrf + ((size_t)k * NZ + lane) * WF; };
                // backward, one LDS exchange per stage: v = p_{k+1} + q_k; every lane forms h_u; u-lanes
                // kff_k = -F_uu^{-1} h_u, x-lanes d_k = B kff_k = -(B F_uu^{-1}) h_u (their rollout
                // offset), both into the lane's DZ word; x-lanes p_k = h_x + K_k' h_u
                struct Bk {
                    T y, yu[NU], m[NU], w[NU], q;
                };
                auto bload = [&](int k, Bk &b) {
                    const T *yk = yref + (size_t)k * yrow, *t_ = frow(k, r);
                    b.y = yk[r];
                    b.q = t_[0];
#pragma unroll
                    for (int i = 0; i < NU; i++) {
                        b.yu[i] = yk[NX + i];
                        b.m[i] = t_[OM + i];
                        b.w[i] = t_[OW + i];
                    }
                };
                // the bound test of the unconstrained solution at element (k, r), its z_0 word, the
                // tentative outputs and the first set of the active-set steps (violated inputs, each
                // state's most violated stage)
                T nbad = 0;
                T wcv = 0, wcs = 0;
                int wck = -1;
                auto fcheck = [&](int k, T z, const Bd &bk) {
                    // stricter than the finish's 1e-9: a bound violated inside that band goes through the
                    // full solve, whose rounding decides it exactly as without the fast path
                    const T tl = T(FAST_TOL) * (T(1) + fabs(bk.lb)), tu = T(FAST_TOL) * (T(1) + fabs(bk.ub));
                    const bool lo_ = has_bound(bk.lb) && z < bk.lb - tl, hi_ = has_bound(bk.ub) && z > bk.ub + tu;
                    nbad += (!isfinite(z) || lo_ || hi_) ? T(1) : T(0);
                    stE(L::Z, k, z);   // z_0 of the active-set steps below
                    if (try_fast && empty0) {
                        fin_out(k, z, bk);
                        const T v_ = lo_ ? bk.lb - z : (hi_ ? z - bk.ub : T(0));
                        if (ul) {
                            if (amask) mset(wm, k, lo_ ? T(-1) : (hi_ ? T(1) : T(0)));
                            else stE(L::DZA, k, lo_ ? T(-1) : (hi_ ? T(1) : T(0)));
                        }
                        wck = v_ > wcv ? k : wck;
                        wcs = v_ > wcv ? (lo_ ? T(-1) : T(1)) : wcs;
                        wcv = fmax(wcv, v_);
                    }
                };
                if (p.cl_tx != nullptr) {
                    // explicit form (nmpc_closed_loop_init): the unconstrained solution is linear in x_0
                    // and the reference window, z_0 = T_x x_0 + v_t with v_t per reference row t (the
                    // closed loop's yref windows are rows of its table), so each lane forms its elements
                    // directly — one LDS exchange (x_0) per step, no recursion
                    T *xb = gb + Gm::G_MT;
                    if (xl) xb[r] = x0r;
                    LPC_SYNC();
                    T x0v[NX];
#pragma unroll
                    for (int j = 0; j < NX; j++) x0v[j] = xb[j];
                    const int ne = (N + 1) * NZ;
                    const T *vt = p.cl_v + (size_t)t_ref * ne;
                    const Bd b0 = bnd(0), bm = bnd(1), bN = bnd(N);
#ifndef NMPC_FAST_EC
#define NMPC_FAST_EC 2
#endif
                    constexpr int EC = NMPC_FAST_EC;   // stages whose table rows are in flight together (A/B on one box, quad13 B=8192: 1 0.110-0.112 ms, 2 0.106-0.107, 3 0.108, 4 0.121, 7 0.19)
                    for (int kc = 0; kc <= N; kc += EC) {
                        T zc[EC];
#pragma unroll
                        for (int j = 0; j < EC; j++) {
                            const int k = kc + j <= N ? kc + j : N, e = k * NZ + r;
                            const T *tx = p.cl_tx + (size_t)e * NX;
                            T s0 = vt[e], s1 = 0;
#pragma unroll
                            for (int jj = 0; jj + 1 < NX; jj += 2) {
                                s0 = fma(tx[jj], x0v[jj], s0);
                                s1 = fma(tx[jj + 1], x0v[jj + 1], s1);
                            }
                            if (NX % 2) s0 = fma(tx[NX - 1], x0v[NX - 1], s0);
                            zc[j] = s0 + s1;
                        }
#pragma unroll
                        for (int j = 0; j < EC; j++) {
                            const int k = kc + j;
                            if (k > N) break;
                            if (k == N && ul) continue;
                            fcheck(k, (k == 0 && xl) ? x0r : zc[j], k == 0 ? b0 : (k == N ? bN : bm));
                        }
                    }
                    LPC_SYNC();
                } else {
                T pv = gde * yref[(size_t)N * yrow + (xl ? r : 0)];   // p_N = g_N (x-lanes)
                Bk bc;
                bload(N - 1, bc);
                for (int k = N - 1; k >= 0; k--) {
                    Bk bn;
                    bload(k > 0 ? k - 1 : 0, bn);   // next stage's inputs, in flight during this stage
                    if (xl) vb[r] = pv + bc.q;
                    LPC_SYNC();
                    T hu[NU];
#pragma unroll
                    for (int i = 0; i < NU; i++) {
                        const T gu = gdu[i] * bc.yu[i];
                        if constexpr (SPARSE) {
                            SpL<T, CN> bcl;
                            sp_load(bcl, slv, sli, NX * RN + (NX + i) * CN);
                            hu[i] = sp_dot(bcl, vb, gu);
                        } else {
                            T s0 = gu;
#pragma unroll
                            for (int l = 0; l < NX; l++) s0 = fma(abt[(NX + i) * LDX + l], vb[l], s0);
                            hu[i] = s0;
                        }
                    }
                    T dk = 0;   // u-lane: kff_k(u); x-lane: (B kff_k)(r)
#pragma unroll
                    for (int j = 0; j < NU; j++) dk = fma(-bc.w[j], hu[j], dk);
                    T h;
                    if constexpr (SPARSE) {
                        h = sp_dot(acl, vb, gdr * bc.y);
                    } else {
                        T h0 = gdr * bc.y, h1 = 0;
#pragma unroll
                        for (int i = 0; i + 1 < NX; i += 2) {
                            h0 = fma(acol[i], vb[i], h0);
                            h1 = fma(acol[i + 1], vb[i + 1], h1);
                        }
                        if (NX % 2) h0 = fma(acol[NX - 1], vb[NX - 1], h0);
                        h = h0 + h1;
                    }
#pragma unroll
                    for (int i = 0; i < NU; i++) h = fma(bc.m[i], hu[i], h);
                    pv = h;
                    stE(L::DZ, k, dk);
                    bc = bn;
                }
                // forward rollout, one LDS exchange per stage (x_k, two alternating buffers):
                // x_{k+1} = (A + B K_k) x_k + B kff_k + c, u_k = kff_k + K_k x_k; bound test, outputs
                T xk = x0r;
                T fr[NX], frn[NX], dd = ldE(L::DZ, 0), ddn;
                {
                    const T *t_ = frow(0, r);
#pragma unroll
                    for (int j = 0; j < NX; j++) fr[j] = t_[OR + j];
                }
                const Bd b0 = bnd(0), bm = bnd(1);
                for (int k = 0; k < N; k++) {
                    const int kn = k + 1 < N ? k + 1 : k;
                    {
                        const T *t_ = frow(kn, r);
#pragma unroll
                        for (int j = 0; j < NX; j++) frn[j] = t_[OR + j];
                        ddn = ldE(L::DZ, kn);
                    }
                    T *xb = gb + Gm::G_MT + (k & 1) * LDZ;
                    if (xl) xb[r] = xk;
                    LPC_SYNC();
                    T s0 = dd, s1 = 0;
#pragma unroll
                    for (int j = 0; j + 1 < NX; j += 2) {
                        s0 = fma(fr[j], xb[j], s0);
                        s1 = fma(fr[j + 1], xb[j + 1], s1);
                    }
                    if (NX % 2) s0 = fma(fr[NX - 1], xb[NX - 1], s0);
                    const T z = xl ? xk : s0 + s1;   // u-lane: u_k = kff + K(u, :) x_k
                    fcheck(k, z, k == 0 ? b0 : bm);
                    xk = xl ? s0 + s1 + c_r : xk;   // x-lane: x_{k+1} = (A + B K) x_k + d_k + c
#pragma unroll
                    for (int j = 0; j < NX; j++) fr[j] = frn[j];
                    dd = ddn;
                }
                if (xl) fcheck(N, xk, bnd(N));
                }
                if (try_fast && empty0 && xl && wck >= 0) {
                    if (amask) mset(wm, wck, wcs);
                    else stE(L::DZA, wck, wcs);
                }
                nbad = gsum(nbad);
                fast_ok = try_fast && empty0 && nbad == T(0);
#ifdef NMPC_STEP_SPLIT
                LPC_STICK(0);   // experiment builds: the unconstrained solve (slot 5: the active-set steps)
#endif
                // ---- active-set steps on the shared factorisation (p.lqrw): S = the flagged bounds
                // (DZA: the warm-start set, or the first set from the unconstrained solution's
                // violations), z = z_0 + W[:, S] nu with W_SS nu = b_S - z_0,S — the exact solution with S
                // held, its multipliers nu. Accepted when every other bound holds and every multiplier has
                // its sign (the finish's KKT test, no penalty and no refinement); otherwise the PDAS update
                // of the finish. At most polish_steps steps and sets of at most WSMAX bounds; a group that
                // ends unaccepted runs the full solve below from the set it reached.
                fin_ws = 0;
                bool wrun = try_fast && !fast_ok && p.lqrw != nullptr;
                for (int ws = 0; ws < p.polish_steps && __any(wrun); ws++) {
#ifndef NMPC_WSMAX
#define NMPC_WSMAX 8
#endif
                    constexpr int WSMAX = NMPC_WSMAX;   // largest active set of the fast finish's steps
                    const int ne = (N + 1) * NZ;
                    // the set: per-lane count, group prefix, entries in LDS (element, sign, b - z_0)
                    T *le = gb + Gm::G_MT;                       // [WSMAX] element index
                    T *ls = le + WSMAX, *lt = ls + WSMAX;        // [WSMAX] sign, [WSMAX] target step
                    int nmine = 0;
                    if (amask) nmine = __popcll(wm);
                    else
                        for (int k = 0; k <= N; k++) nmine += (k < N || xl) && !(k == 0 && xl) && ldE(L::DZA, k) != T(0);
                    int pre = nmine;
#pragma unroll
                    for (int sh = 1; sh < NZ; sh <<= 1) {
                        const int o = __shfl(pre, lane - sh >= 0 ? lane - sh : 0, 64);
                        pre += r >= sh ? o : 0;
                    }
                    const int m = (int)gsum(r == NZ - 1 ? T(pre) : T(0));   // the last lane's prefix = |S|
                    pre -= nmine;   // exclusive prefix
                    // restart: a group whose set is empty (every held bound left) is at the unconstrained
                    // solution z_0 — accepted if every bound holds (1e-13), else its set becomes the
                    // violated inputs and each state component's most violated stage (this round takes
                    // no active-set step; oracle/c/riccati_ipm.c fast_finish)
                    const bool rst = wrun && m == 0;
                    if (__any(rst)) {
                        T nb = 0, cv3 = 0, cs3 = 0;
                        int ck3 = -1;
                        for (int k = 0; rst && k <= N; k++) {
                            if ((k == N && ul) || (k == 0 && xl)) continue;
                            const T z = ldE(L::Z, k);
                            const Bd b_ = bnd(k);
                            const T tl = T(1e-13) * (T(1) + fabs(b_.lb)), tu = T(1e-13) * (T(1) + fabs(b_.ub));
                            const bool lo_ = has_bound(b_.lb) && z < b_.lb - tl, hi_ = has_bound(b_.ub) && z > b_.ub + tu;
                            nb += (lo_ || hi_ || !isfinite(z)) ? T(1) : T(0);
                            const T v_ = lo_ ? b_.lb - z : (hi_ ? z - b_.ub : T(0));
                            if (ul && (lo_ || hi_)) {
                                if (amask) mset(wm, k, lo_ ? T(-1) : T(1));
                                else stE(L::DZA, k, lo_ ? T(-1) : T(1));
                            }
                            ck3 = v_ > cv3 ? k : ck3;
                            cs3 = v_ > cv3 ? (lo_ ? T(-1) : T(1)) : cs3;
                            cv3 = fmax(cv3, v_);
                            fin_out(k, z, b_);   // tentative outputs (z_0 accepted)
                        }
                        if (rst && xl && ck3 >= 0) {
                            if (amask) mset(wm, ck3, cs3);
                            else stE(L::DZA, ck3, cs3);
                        }
                        nb = gsum(nb);
                        const bool acc0 = rst && nb == T(0);
                        fast_ok = fast_ok || acc0;
                        wrun = wrun && !acc0;
                    }
                    // the groups that take an active-set step this round (a set larger than WSMAX ends
                    // the group's fast finish: it runs the full solve)
                    bool wact = wrun && !rst && m <= WSMAX;
                    wrun = wrun && (rst || m <= WSMAX);
                    LPC_SYNC();
                    if (wact) {
                        int q_ = pre;
                        for (int k = 0; k <= N; k++) {
                            const T f = ((k < N || xl) && !(k == 0 && xl)) ? (amask ? mflag(wm, k) : ldE(L::DZA, k)) : T(0);
                            if (f != T(0)) {
                                const Bd b_ = bnd(k);
                                le[q_] = T(k * NZ + r);
                                ls[q_] = f;
                                lt[q_] = (f < T(0) ? b_.lb : b_.ub) - ldE(L::Z, k);
                                q_++;
                            }
                        }
                    }
                    LPC_SYNC();
                    // nu = W_SS^{-1} (b - z_0)_S by Cholesky, every lane (m <= WSMAX)
                    T L_[WSMAX][WSMAX], nu_[WSMAX], wd_[WSMAX];
                    int ei[WSMAX];
#pragma unroll
                    for (int i = 0; i < WSMAX; i++) {
                        ei[i] = (wact && i < m) ? (int)le[i] : 0;
                        nu_[i] = (wact && i < m) ? lt[i] : T(0);
                    }
                    bool pdf = true;
#pragma unroll
                    for (int i = 0; i < WSMAX; i++)
#pragma unroll
                        for (int j = 0; j <= i; j++) {
                            T s_ = (i < m && j < m) ? p.lqrw[(size_t)ei[j] * ne + ei[i]] : (i == j ? T(1) : T(0));
                            if (i == j) wd_[i] = s_;
#pragma unroll
                            for (int l = 0; l < j; l++) s_ = fma(-L_[i][l], L_[j][l], s_);
                            if (i == j) {
                                pdf = pdf && s_ > T(0);
                                L_[i][i] = s_ > T(0) ? sqrt(s_) : T(1);
                            } else {
                                L_[i][j] = s_ / L_[j][j];
                            }
                        }
#pragma unroll
                    for (int i = 0; i < WSMAX; i++) {
                        T s_ = nu_[i];
#pragma unroll
                        for (int l = 0; l < i; l++) s_ = fma(-L_[i][l], nu_[l], s_);
                        nu_[i] = s_ / L_[i][i];
                    }
#pragma unroll
                    for (int i = WSMAX - 1; i >= 0; i--) {
                        T s_ = nu_[i];
#pragma unroll
                        for (int l = i + 1; l < WSMAX; l++) s_ = fma(-L_[l][i], nu_[l], s_);
                        nu_[i] = s_ / L_[i][i];
                    }
                    wrun = wrun && (!wact || pdf);   // W_SS not positive definite: the full solve
                    wact = wact && pdf;
                    // multiplier signs (lower: nu >= 0, upper: nu <= 0), measured as the displacement
                    // nu_i W_ii the multiplier causes at its own element: a wrong-sign multiplier of
                    // displacement d moves the solution by about d, so the tolerance is a z-scale one,
                    // 1e-10 (1 + |b - z_0|), above the rounding of the W_SS solve (oracle/c/riccati_ipm.c
                    // fast_finish; a gradient-scale tolerance let quad13's low-curvature angular
                    // accelerations and the force inputs keep wrong-sign bounds worth 1e-6..1e-5)
                    int nrem = 0;
                    bool remk[WSMAX];
#pragma unroll
                    for (int i = 0; i < WSMAX; i++) {
                        const T f = (i < m) ? ls[i] : T(0);
                        const T tol_ = T(1e-10) * (T(1) + fabs(lt[i])), dsp = nu_[i] * wd_[i];
                        remk[i] = i < m && ((f < T(0) && dsp < -tol_) || (f > T(0) && dsp > tol_) || !isfinite(nu_[i]));
                        nrem += remk[i] ? 1 : 0;
                    }
                    // z = z_0 + W[:, S] nu at the lane's elements: bounds, the next set, tentative outputs
                    T wbad = T(nrem), cv2 = 0, cs2 = 0;
                    int ck2 = -1;
                    const bool addok = ws == 0 || nrem == 0;
                    for (int k = 0; k <= N; k++) {
                        if (k == N && ul) break;
                        const int e = k * NZ + r;
                        T z = ldE(L::Z, k);
#pragma unroll
                        for (int i = 0; i < WSMAX; i++)
                            if (i < m) z = fma(p.lqrw[(size_t)ei[i] * ne + e], nu_[i], z);
                        const Bd b_ = bnd(k);
                        const T f = amask ? mflag(wm, k) : ldE(L::DZA, k);
                        T nf = f;
                        if (f != T(0)) {
                            // held: z_0 + W[:, S] nu lands on the bound up to the solve's rounding (1e-9, the
                            // refinement's test); then exactly on it
                            const T bb = f < T(0) ? b_.lb : b_.ub;
                            wbad += (!(fabs(z - bb) <= T(1e-9) * (T(1) + fabs(bb)))) ? T(1) : T(0);
                            z = bb;
#pragma unroll
                            for (int i = 0; i < WSMAX; i++)
                                if (remk[i] && ei[i] == e) nf = T(0);
                        } else if (!(k == 0 && xl)) {
                            const T tl = T(1e-13) * (T(1) + fabs(b_.lb)), tu = T(1e-13) * (T(1) + fabs(b_.ub));
                            const bool lo_ = has_bound(b_.lb) && z < b_.lb - tl, hi_ = has_bound(b_.ub) && z > b_.ub + tu;
                            wbad += (lo_ || hi_ || !isfinite(z)) ? T(1) : T(0);
                            const T v_ = lo_ ? b_.lb - z : (hi_ ? z - b_.ub : T(0));
                            if (ul && (lo_ || hi_)) nf = lo_ ? T(-1) : T(1);   // inputs join at once
                            ck2 = v_ > cv2 ? k : ck2;
                            cs2 = v_ > cv2 ? (lo_ ? T(-1) : T(1)) : cs2;
                            cv2 = fmax(cv2, v_);
                        }
                        if (wact) {
                            if (nf != f) {
                                if (amask) mset(wm, k, nf);
                                else stE(L::DZA, k, nf);
                            }
                            fin_out(k, z, b_);
                        }
                    }
                    if (wact && xl && addok && ck2 >= 0) {
                        if (amask) mset(wm, ck2, cs2);
                        else stE(L::DZA, ck2, cs2);
                    }
                    wbad = gsum(wbad);
                    fin_ws += wact ? 1 : 0;
                    const bool acc = wact && wbad == T(0);
                    fast_ok = fast_ok || acc;
                    wrun = wrun && !acc;
                    LPC_SYNC();
                }
                // a group that took active-set steps left its last set in DZA: the full solve's first
                // finish step starts from it (never as an empty set)
                if (fin_ws > 0) warm_act = T(1);
#ifdef NMPC_STEP_SPLIT
                LPC_STICK(5);
#endif
                if (fastpl) cly[r] = yref[xl || r < p.ny ? r : 0];   // yref row 0 (cost / AED reference)
            }
        }
        const bool need_full = __any(inst_ok && !fast_ok);
        if (amask && warm && need_full && inst_ok && !fast_ok)   // the full solve reads its warm set from DZA
            for (int k = 0; k <= N; k++) stE(L::DZA, k, mflag(wm, k));
        LPC_STICK(0);
        // ------------------------------------------------------------------ infeasibility certificate
        // interval reachability (oracle/c/riccati_ipm.c infeasible_stage): x-lane r carries the
        // midpoint / radius of state r of X_k, u-lanes the input box; X_{k+1} = hull([A B] X_k x U
        // + c) meets the state box of stage k+1, an empty intersection proves the QP infeasible
        bool infeas = false;
        // row r of [A B] as a compact list (structured kernels) for the certificate and the residual
        // of the initial point
        if (need_full) {
            T cm = xl ? x0r : T(0), cr = 0;
            if (ul) {
                const T l = LB(0), h = UB(0);
                const bool bb = has_bound(l) && has_bound(h);
                cm = bb ? T(0.5) * (l + h) : T(0);
                cr = bb ? T(0.5) * (h - l) : T(INFINITY);
            }
            const Bd bm = bnd(1);
            // one LDS exchange per stage: midpoints and radii alternate between two buffers
            for (int k = 0; k < N; k++) {
                T *cmb = gb + Gm::G_MT + (k & 1) * 2 * LDZ, *rad = cmb + LDZ;
                cmb[r] = cm;
                rad[r] = cr;
                LPC_SYNC();
                T sm = c_r, sr = 0;
                if constexpr (SPARSE) {
#pragma unroll
                    for (int j = 0; j < RN; j++) {
                        const T a = arl0.v[j];
                        sm = fma(a, *(const T *)((const char *)cmb + arl0.o[j]), sm);
                        // 0 x unbounded radius adds 0 (padding entries are (0, 0))
                        sr = a != T(0) ? fma(fabs(a), *(const T *)((const char *)rad + arl0.o[j]), sr) : sr;
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < NZ; j++) {
                        const T a = abr[(xl ? r : 0) * LDZ + j];
                        sm = fma(a, cmb[j], sm);
                        sr = a != T(0) ? fma(fabs(a), rad[j], sr) : sr;
                    }
                }
                const Bd b1 = k + 1 == N ? bnd(N) : bm;
                T lo = sm - sr, hi = sm + sr;
                lo = has_bound(b1.lb) ? fmax(lo, b1.lb) : lo;
                hi = has_bound(b1.ub) ? fmin(hi, b1.ub) : hi;
                infeas |= xl && lo > hi + T(1e-9) * (T(1) + fabs(hi));
                const bool fin = isfinite(lo) && isfinite(hi);
                if (xl) {
                    cm = fin ? T(0.5) * (lo + hi) : sm;
                    cr = fin ? T(0.5) * (hi - lo) : sr;
                }
            }
            infeas = gmax(infeas ? T(1) : T(0)) > T(0);
        }
        LPC_STICK(1);
        // ------------------------------------------------------------------ initial point
        // y = z with diagonal W (p.g_diag, every reference model): g_c = G_rr y_r from the lane's own
        // y component; stage rows are loaded YC stages at a time (one memory latency per chunk)
        constexpr int YC = 4;
        const bool gd = p.g_diag != 0;
        const T gdr = gd ? p.G[r * p.ny + r] : T(0), gde = (gd && xl) ? p.Ge[r * p.ny_e + r] : T(0);
        const T hrr0 = SP::hdiag ? hm[r * LDZ + r] : T(0), hre0 = SP::hdiag ? hem[(xl ? r : 0) * LDX + (xl ? r : 0)] : T(0);
        T r0 = 0, mu = 0, abz = 0;
        T cold_act = 0;   // bounds the finish's first-set rule marks at the initial point (lqr_back)
        const Bd b0i = bnd(0), bmi = bnd(1);
        LPC_SYNC();   // the certificate's last exchange buffers are read before they are rewritten
        for (int kc = 0; need_full && kc <= N; kc += YC) {
            T ych[YC];
#pragma unroll
            for (int j = 0; j < YC; j++) {
                const int k = kc + j <= N ? kc + j : N;
                const bool yv = k < N ? r < p.ny : r < p.ny_e;   // row N holds ny_e entries
                ych[j] = yref[(size_t)k * yrow + (yv ? r : 0)];
                ych[j] = yv ? ych[j] : T(0);
            }
#pragma unroll
            for (int j = 0; j < YC; j++) {
                const int k = kc + j;
                if (k > N) break;
                const bool ex = k < N || xl;
                const T yr = ych[j];
                if (fastpl && k == 0) cly[r] = yr;
                T z = 0, lam_l = 0, lam_u = 0, gc = 0;
                const Bd bk = k == 0 ? b0i : (k == N ? bnd(N) : bmi);
                const T lb = bk.lb, ub = bk.ub;
                if (ex) {
                    if (gd) {
                        gc = (k < N ? gdr : gde) * yr;
                    } else {
                        const T *yk = yref + (size_t)k * yrow;
                        if (k < N) {
                            for (int jj = 0; jj < p.ny; jj++) gc += p.G[r * p.ny + jj] * yk[jj];
                        } else {
                            for (int jj = 0; jj < p.ny_e; jj++) gc += p.Ge[r * p.ny_e + jj] * yk[jj];
                        }
                    }
                    if (k == 0 && xl) {
                        z = x0r;
                    } else {
                        z = p.yref_is_z ? yr : T(0);
                        const bool hl = has_bound(lb), hu = has_bound(ub);
                        if (hl && hu) {
                            const T d = T(0.01) * (ub - lb);
                            z = ul ? T(0.5) * (lb + ub) : z;   // boxed inputs start mid-box (oracle/c/riccati_ipm.c)
                            z = fmin(fmax(z, lb + d), ub - d);
                        } else if (hl) {
                            z = fmax(z, lb + T(0.01) * fmax(fabs(lb), T(1)));
                        } else if (hu) {
                            z = fmin(z, ub - T(0.01) * fmax(fabs(ub), T(1)));
                        }
                        if (hl) lam_l = p.mu0 / (z - lb);
                        if (hu) lam_u = p.mu0 / (ub - z);
                        cold_act += ((hl && lam_l > z - lb) || (hu && lam_u > ub - z)) ? T(1) : T(0);
                    }
                }
                stE(L::Z, k, z);
                stE(L::LL, k, lam_l);
                stE(L::LU, k, lam_u);
                stE(L::GC, k, gc);
                // one LDS exchange per stage (two alternating buffers)
                T *zx = gb + Gm::G_MT + (k & 1) * LDZ;
                zx[r] = z;
                LPC_SYNC();
                if (ex) {
                    T g = gc;
                    if (SP::hdiag) {
                        g = fma(k < N ? hrr0 : hre0, z, g);
                    } else if (k < N) {
#pragma unroll
                        for (int b = 0; b < NZ; b++) g = fma(hm[r * LDZ + b], zx[b], g);
                    } else {
#pragma unroll
                        for (int b = 0; b < NX; b++) g = fma(hem[r * LDX + b], zx[b], g);
                    }
                    if (!(k == 0 && xl)) {
                        r0 = fmax(r0, fabs(g - lam_l + lam_u));
                        if (lam_l > T(0)) mu += lam_l * (z - lb);
                        if (lam_u > T(0)) mu += lam_u * (ub - z);
                    }
                    if (xl && k > 0) r0 = fmax(r0, fabs(abz - z));
                    if (xl && k < N) {
                        if constexpr (SPARSE) {
                            abz = sp_dot(arl0, zx, c_r);
                        } else {
                            T s_ = c_r;
#pragma unroll
                            for (int jj = 0; jj < NZ; jj++) s_ = fma(abr[r * LDZ + jj], zx[jj], s_);
                            abz = s_;
                        }
                    }
                }
            }
        }
        r0 = gmax(r0);
        mu = gsum(mu) * p.inv_m;
        cold_act = gsum(cold_act);
        LPC_STICK(1);

        const T m_bounds = T(1) / p.inv_m;
        T theta = 1;
        bool active = inst_ok && !infeas && !fast_ok;
        // certified infeasible: status 4, the initial point; completed by the fast finish: status -1
        int status = fast_ok ? -1 : (infeas ? 4 : 2), iters = fast_ok ? 1 + fin_ws : 0;
        bool fail = false, pending = false;
        T alpha = 0, smu = 0;
        // exact finish (oracle/c/riccati_ipm.c "exact finish"): a primal-dual active-set run of at
        // most polish_steps penalised Newton steps from the IPM iterate, then one refinement step.
        // polish_at: mu that triggers the next run; pol: the group is in a run; fref: its next step
        // is the refinement; fin_steps: finish steps taken (counted in qp_iter). During a run DZ holds
        // the step and DZA the active flags (-1 lower, 1 upper, 0); after the refinement DZA holds
        // its correction. status -1: completed by the finish, outputs = Z + DZ + DZA (B and D skip
        // the group's DZA / DZ)
        T polish_at = p.polish_mu;
        int fin_steps = fast_ok ? 1 + fin_ws : 0, fin_runs = 0;
        bool pol = false, fref = false;
        bool fs0 = false;   // wave-uniform: the current finish pass is the first step of its runs

        // elementwise state of element (k, r) fetched one stage ahead in the sweeps
        struct El {
            T z, ll, lu, dz, dza, g;
        };
        // lazily apply the pending step of the previous iteration to element (k, r)
        // lazily apply the pending step of the previous iteration to element (k, r); the arithmetic
        // is branch-free (selects), the write-back a write-only divergent block
        auto lazy = [&](int k, El &q, const Bd &b) {
            const bool upd = pending && (k < N || xl);
            const T lb = b.lb, ub = b.ub;
            const bool vl = q.ll > T(0), vu = q.lu > T(0);
            const T tl = q.z - lb, tu = ub - q.z, itl = frcp(tl), itu = frcp(tu);
            const T dlal = -q.ll * (T(1) + q.dza * itl), dlau = -q.lu * (T(1) - q.dza * itu);
            const T nl = q.ll + alpha * ((smu - q.ll * tl - dlal * q.dza - q.ll * q.dz) * itl);
            const T nu_ = q.lu + alpha * ((smu - q.lu * tu + dlau * q.dza + q.lu * q.dz) * itu);
            q.ll = (upd && vl) ? nl : q.ll;
            q.lu = (upd && vu) ? nu_ : q.lu;
            q.z = upd ? q.z + alpha * q.dz : q.z;
            if (upd) {
                stE(L::Z, k, q.z);
                stE(L::LL, k, q.ll);
                stE(L::LU, k, q.lu);
            }
        };
        auto sigma = [&](const El &q, const Bd &b) {
            const T sl = q.ll * frcp(q.z - b.lb), su = q.lu * frcp(b.ub - q.z);
            return (q.ll > T(0) ? sl : T(0)) + (q.lu > T(0) ? su : T(0));
        };
        // exact finish, first active set: a bound is active where its multiplier exceeds its slack
        auto finish_rule = [&](const El &q, const Bd &b) {
            const bool al = q.ll > T(0) && q.ll > q.z - b.lb;
            const bool au = !al && q.lu > T(0) && q.lu > b.ub - q.z;
            return al ? T(-1) : (au ? T(1) : T(0));
        };
        // finish terms of element (k, r): active bounds held by the penalty rho (Hessian rho,
        // gradient rho (z - bound); the refinement: 2 rho (z_a - bound) at z_a = z + dz), the others
        // dropped. fs0: first step of the run (active set from the multipliers, else from DZA).
        // Branch-free; q.z becomes the step's base point.
        // active flag of a finish step from the dza slot (flags of the run, or the warm-start flags,
        // kept to bounds the element has), or from the multipliers at the first step of a cold run
        // an add candidate (flag +-2, a violated inactive state bound of the previous set step) joins
        // only if it is its component's most violated stage (addk) — see the PDAS update in forward()
        int addk = -1;
        auto fin_flag = [&](const El &q, const Bd &b, bool first, int k) {
            if (first && !fwarm) return finish_rule(q, b);
            const bool cand = fabs(q.dza) > T(1.5);
            const T f = cand && k != addk ? T(0) : q.dza;
            return (f < T(-0.5) && q.ll > T(0)) ? T(-1) : ((f > T(0.5) && q.lu > T(0)) ? T(1) : T(0));
        };
        auto finish_terms = [&](El &q, const Bd &b, bool fs0, int k, T &sg, T &gadd) {
            const T a = fin_flag(q, b, fs0, k);
            q.z = fref ? q.z + q.dz : q.z;
            const T rho = p.polish_rho;
            sg = a != T(0) ? rho : T(0);
            gadd = a != T(0) ? (fref ? T(2) : T(1)) * rho * (q.z - (a < T(0) ? b.lb : b.ub)) : T(0);
        };
        // acceptance tests of a finish step at element (k, r) (the oracle's POLISH_TOL_*): q.z is the
        // step's base, dz the step, a the active flag it used. A set step: active bounds keep a
        // non-negative multiplier rho (bound - z_new) (to a few ulps), inactive ones hold (to 1e-9);
        // the next active set (na) drops the first kind (rem) and marks the second as add candidates
        // (flag +-2, violation viol). The refinement: the correction stays below 1e-3 (1 + |z|) and
        // the refined point sits on its active bounds and inside the others to 1e-9. Returns 1 for a
        // violated test.
        auto finish_check = [&](T dz, const El &q, const Bd &b, T a, T &na, T &viol, bool &rem) {
            const bool vl = q.ll > T(0), vu = q.lu > T(0);
            const T zn = q.z + dz;
            const T tl = T(1e-9) * (T(1) + fabs(b.lb)), tu = T(1e-9) * (T(1) + fabs(b.ub));
            const bool lo = vl && zn < b.lb - tl, hi = vu && zn > b.ub + tu;
            bool bad = !isfinite(zn);   // a non-finite step is never accepted
            if (fref) {
                bad |= !(fabs(dz) <= T(1e-3) * (T(1) + fabs(q.z))) || (a < T(0) && fabs(zn - b.lb) > tl) ||
                      (a > T(0) && fabs(zn - b.ub) > tu) || (a == T(0) && (lo || hi));
                na = a;
                viol = 0;
                rem = false;
            } else {
                const bool rl = a < T(0) && zn > fma(T(1e-15), T(1) + fabs(b.lb), b.lb);
                const bool ru = a > T(0) && zn < fma(T(-1e-15), T(1) + fabs(b.ub), b.ub);
                const bool al = a == T(0) && lo, au = a == T(0) && !lo && hi;
                bad |= rl || ru || al || au;
                // inputs join at once, states as candidates (+-2, PDAS update in forward())
                const T add = xl ? T(2) : T(1);
                na = (rl || ru) ? T(0) : (al ? -add : (au ? add : a));
                viol = !xl ? T(0) : (al ? b.lb - zn : (au ? zn - b.ub : T(0)));
                rem = rl || ru;
            }
            return bad ? T(1) : T(0);
        };
        // the same lazy step split in two for the Riccati stages k < N: the primal update first (it
        // is all the stage's first LDS exchange needs), the dual update after that exchange, where
        // it fills the latency of the residual's LDS reads; the write-back is unconditional (a
        // frozen group rewrites its unchanged words), so the stage stays one scheduling region
        auto lazy_z = [&](El &q) {
            const T zo = q.z;
            q.z = pending ? q.z + alpha * q.dz : q.z;
            return zo;
        };
        auto lazy_duals = [&](int k, El &q, T zo, const Bd &b) {
            const bool vl = q.ll > T(0), vu = q.lu > T(0);
            const T tl = zo - b.lb, tu = b.ub - zo, itl = frcp(tl), itu = frcp(tu);
            const T dlal = -q.ll * (T(1) + q.dza * itl), dlau = -q.lu * (T(1) - q.dza * itu);
            const T nl = q.ll + alpha * ((smu - q.ll * tl - dlal * q.dza - q.ll * q.dz) * itl);
            const T nu_ = q.lu + alpha * ((smu - q.lu * tu + dlau * q.dza + q.lu * q.dz) * itu);
            q.ll = (pending && vl) ? nl : q.ll;
            q.lu = (pending && vu) ? nu_ : q.lu;
            stE(L::Z, k, q.z);
            stE(L::LL, k, q.ll);
            stE(L::LU, k, q.lu);
        };

        // ---- forward recursion (B: predictor into dza with ratio test / centring sums;
        //      D: corrector into dz with step length / new-mu sums):
        //      dx_0 = 0, du_k = kff_k + K_k dx_k, dx_{k+1} = [A B] [dx_k; du_k] + re_k
#if (defined(NMPC_PHASE_TIMING) || defined(NMPC_FWD_TIMING)) && !defined(NMPC_SWEEP_TIMING)
#define NMPC_SWEEP_TIMING 1
#endif
#ifdef NMPC_SWEEP_TIMING
        // experiment builds only (build_experiment(..., ["NMPC_SWEEP_TIMING"])): clock cycles per
        // sweep, reported through the E_A/A/B/../D slots of nmpc_api.cpp (A -> 1, B -> 2, C -> 5, D -> 6)
        const bool timed = p.cycles != nullptr;
        unsigned long long tcy[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tmark = timed ? __builtin_amdgcn_s_memtime() : 0ull;
        const unsigned long long tstart = tmark;
        auto tick = [&](int slot) {
            if (timed) {
                const unsigned long long t = __builtin_amdgcn_s_memtime();
                if (slot >= 0) tcy[slot] += t - tmark;
                tmark = t;
            }
        };
#define LPC_TICK(slot) tick(slot)
#else
#define LPC_TICK(slot) ((void)0)
#endif
    // NMPC_PHASE_TIMING: also split the Riccati stage into pre (lazy step, g, re) -> slot 0,
    // M -> 3, F -> 4, Cholesky / gains / P update -> 7
#ifdef NMPC_PHASE_TIMING
#define LPC_PTICK(slot) tick(slot)
#else
#define LPC_PTICK(slot) ((void)0)
#endif
    // NMPC_FWD_TIMING: split the predictor sweep B into x writes (slot 0), u sums (3), x update (4),
    // statistics / store (7); the sweep remainder stays in slot 2
#ifdef NMPC_FWD_TIMING
#define LPC_FTICK(slot) do { if (!corr) tick(slot); } while (0)
#else
#define LPC_FTICK(slot) ((void)0)
#endif

        auto forward = [&](auto PASS, T &s_min, T &s_a, T &s_b, T &s_c) __attribute__((always_inline)) {
            constexpr bool corr = decltype(PASS)::value == 1, fin = decltype(PASS)::value == 2;
            const T *arow = abr + (xl ? r : 0) * LDZ;   // row r of [A B] (LDS, read per stage)
            s_min = 1;
            s_a = s_b = s_c = 0;
            // ratio tests and closed-form mu sums of element (k, r), branch-free (selects instead of
            // divergent arms). The predictor's quantities only steer the step length (safety factor
            // 0.995) and sigma, so they use the raw hardware reciprocal; the corrector's dual step
            // feeds mu_new (termination) and keeps the refined one.
            auto stats = [&](T dz, const El &q, const Bd &b) {
                const T lb = b.lb, ub = b.ub;
                const bool vl = q.ll > T(0), vu = q.lu > T(0);
                const T tl = q.z - lb, tu = ub - q.z;
                T c = 1;
                if constexpr (fin) {
                    // the finish: acceptance count (finish_check, at the stage store)
                } else if constexpr (!corr) {
                    // predictor: the largest inverse step ratio, division-free — primal -dz/t_l and
                    // dual -dlam_l/lam_l = 1 + dz/t_l (the affine dual step is -lam (1 + dz/t)), and
                    // the mirrored pair for the upper bound; alpha_aff = 1 / max(1, ...) per group
                    const T itl = rcp_raw(tl), itu = rcp_raw(tu);
                    const T al = dz * itl, au = dz * itu;
                    c = vl ? fmax(c, fmax(-al, T(1) + al)) : c;
                    c = vu ? fmax(c, fmax(au, T(1) - au)) : c;
                    s_a += (vl ? q.ll * tl : T(0)) + (vu ? q.lu * tu : T(0));
                    s_b += (vl ? q.ll * dz * (tl + dz) * itl : T(0)) + (vu ? q.lu * dz * (dz - tu) * itu : T(0));
                } else {
                    const T rdz = rcp_raw(dz);
                    const T dza = q.dza;
                    const T itl = frcp(tl), itu = frcp(tu);
                    const T dlal = -q.ll * (T(1) + dza * itl), dlau = -q.lu * (T(1) - dza * itu);
                    const T dll = (smu - q.ll * tl - dlal * dza - q.ll * dz) * itl;
                    const T dlu = (smu - q.lu * tu + dlau * dza + q.lu * dz) * itu;
                    c = (vl && dz < T(0)) ? fmin(c, -tl * rdz) : c;
                    c = (vl && dll < T(0)) ? fmin(c, -q.ll * rcp_raw(dll)) : c;
                    c = (vu && dz > T(0)) ? fmin(c, tu * rdz) : c;
                    c = (vu && dlu < T(0)) ? fmin(c, -q.lu * rcp_raw(dlu)) : c;
                    s_a += (vl ? q.ll * tl : T(0)) + (vu ? q.lu * tu : T(0));
                    s_b += (vl ? dlal * dza : T(0)) - (vu ? dlau * dza : T(0));
                    // + dz * 0: NaN for a non-finite direction (caught at the step below)
                    s_c += (vl ? dll * dz : T(0)) - (vu ? dlu * dz : T(0)) + dz * T(0);
                }
                s_min = corr ? fmin(s_min, c) : fmax(s_min, c);
            };
            struct Rec {
                El e;
                T c0, kq[NU];   // x-lane: K_k(:, r); u-lane: kff_k(u)
            };
            auto fetch = [&](int k, Rec &q) {
                k = k < N ? k : N;
                const int kk = k < N ? k : N - 1;
                q.e.z = ldE(L::Z, k);
                q.e.ll = ldE(L::LL, k);
                q.e.lu = ldE(L::LU, k);
                if (corr || fin) q.e.dza = ldE(L::DZA, k);   // warm flags: copied into DZA at the step start
                if constexpr (fin) {   // finish: the step's base point (refinement: z_a = z + dz)
                    const T dzp = ldE(L::DZ, k);
                    q.e.z = fref ? q.e.z + dzp : q.e.z;
                }
                // every lane loads the same record words (x: K(:, r); u: word 0 = kff) — loads in
                // divergent arms get merged with a divergent offset (waterfall + private array)
#pragma unroll
                for (int i = 0; i < NU; i++) q.kq[i] = ldX(kk, i);
                q.c0 = q.kq[UKFF];
            };
            const int dst = (corr || fin) ? L::DZ : L::DZA;   // the finish's step goes to DZ
            T cviol = 0;   // finish: this lane's most violated add candidate and its stage
            int ck = -1;
            T *part = gb + Gm::G_MT;   // [NX][LDU] partial products K(u, j) dx_j
            // dx_{k+1}(r) = c_r + [A B](r, :) (z_k + dz_k) - z_{k+1}(r): the dynamics residual is
            // folded in, so the sweep carries xt = dx_{k+1} + z_{k+1} and subtracts z_{k+1} when
            // stage k+1's iterate has arrived
            T xt = 0;
            // stage records in flight PD stages ahead (ring slot j holds stage k = j mod PD; the
            // stage loop is unrolled by PD so every slot is a fixed register set)
            Rec ring[PD];
#pragma unroll
            for (int j = 0; j < PD; j++) fetch(j, ring[j]);
            SpL<T, RN> arl;
            if constexpr (SPARSE) sp_load(arl, slv, sli, row_base);
            const Bd b0 = bnd(0), bm = bnd(1);   // stage 0 and interior bounds (sweep constants)
#if NMPC_LPC_DEFER
            // statistics pending from the previous stage (neutral before stage 0: no bound active)
            T pm = 0;
            El pe{};
            Bd pb = b0;
#endif
            for (int kb = 0; kb < N; kb += PD) {
#pragma unroll
                for (int j = 0; j < PD; j++) {
                    const int k = kb + j;
                    if (k >= N) break;
                    LPC_FTICK(2);
                    // the slot is read in place and refilled after its last use: copying it out
                    // first makes the compiler move the refill's registers at the loop back edge,
                    // which waits for those loads and exposes their whole latency
                    Rec &q = ring[j];
                    const Bd bk = k == 0 ? b0 : bm;
                    const T dx = (k == 0 || !xl) ? T(0) : xt - q.e.z;   // x-lanes: dx_k (x_0 pinned)
#if NMPC_LPC_DEFER
                    // branch-free stage (one scheduling region per LDS exchange): u-lanes write their
                    // partial-product row into the spare row NX, which nobody reads
                    {
                        const int pr_ = xl ? r : NX;
#pragma unroll
                        for (int i = 0; i < NU; i++) part[pr_ * LDU + i] = q.kq[i] * dx;
                    }
                    LPC_SYNC();
                    LPC_FTICK(0);
                    // the statistics of stage k-1 run here, between issuing the partial-sum reads
                    // and their first use, instead of at the end of stage k-1 on its critical path
                    stats(pm, pe, pb);
                    T du;
                    {
                        const int uu = ul ? u : 0;
                        T s0 = q.c0, s1 = 0;
#pragma unroll
                        for (int jj = 0; jj + 1 < NX; jj += 2) {
                            s0 += part[jj * LDU + uu];
                            s1 += part[(jj + 1) * LDU + uu];
                        }
                        if (NX % 2) s0 += part[(NX - 1) * LDU + uu];
                        du = ul ? s0 + s1 : T(0);
                    }
                    const T my = xl ? dx : du;
                    zb[r] = q.e.z + my;
                    LPC_SYNC();
                    LPC_FTICK(3);
#else
                    if (xl) {   // write-only divergent block
#pragma unroll
                        for (int i = 0; i < NU; i++) part[r * LDU + i] = q.kq[i] * dx;
                        zb[r] = q.e.z + dx;
                    }
                    LPC_SYNC();
                    LPC_FTICK(0);
                    // u-lanes: du_u = kff_u + sum_j K(u, j) dx_j; every lane runs the same straight-line
                    // code (x-lanes sum column 0 and discard it)
                    T du;
                    {
                        const int uu = ul ? u : 0;
                        T s0 = q.c0, s1 = 0;
#pragma unroll
                        for (int jj = 0; jj + 1 < NX; jj += 2) {
                            s0 += part[jj * LDU + uu];
                            s1 += part[(jj + 1) * LDU + uu];
                        }
                        if (NX % 2) s0 += part[(NX - 1) * LDU + uu];
                        du = ul ? s0 + s1 : T(0);
                    }
                    if (ul) zb[r] = q.e.z + du;
                    LPC_SYNC();
                    LPC_FTICK(3);
                    const T my = xl ? dx : du;
#endif
                    if constexpr (SPARSE) {
                        const T s = sp_dot(arl, zb, c_r);
                        xt = xl ? s : xt;
                    } else {
                        T s0 = c_r, s1 = 0;
#pragma unroll
                        for (int jj = 0; jj + 1 < NZ; jj += 2) {
                            s0 = fma(arow[jj], zb[jj], s0);
                            s1 = fma(arow[jj + 1], zb[jj + 1], s1);
                        }
                        if (NZ % 2) s0 = fma(arow[NZ - 1], zb[NZ - 1], s0);
                        xt = xl ? s0 + s1 : xt;
                    }
                    LPC_FTICK(4);
                    if constexpr (fin) {
                        // finish: acceptance tests, next active set; polishing groups only store (a
                        // finished group's DZ / DZA are its result)
                        T na, viol;
                        bool rem;
                        const T a = fin_flag(q.e, bk, fs0, k);
                        s_c += finish_check(my, q.e, bk, a, na, viol, rem);
                        s_a += na != T(0) ? T(1) : T(0);   // active bounds of the next set
                        s_b += rem ? T(1) : T(0);           // removals
                        ck = viol > cviol ? k : ck;
                        cviol = fmax(cviol, viol);
                        if (pol) fin_out(k, q.e.z + my, bk);
                        if (pol) {
                            if (fref) {
                                stE(L::DZA, k, my);
                            } else {
                                stE(L::DZ, k, my);
                                stE(L::DZA, k, na);
                            }
                        }
                    } else if (status >= 0) {
                        stE(dst, k, my);   // groups the finish completed keep their DZ / DZA
                    }
#if NMPC_LPC_DEFER
                    pm = my;
                    pe = q.e;
                    pb = bk;
#else
                    stats(my, q.e, bk);
#endif
                    fetch(k + PD, ring[j]);
                    LPC_SYNC();
                    LPC_FTICK(7);
                }
            }
#if NMPC_LPC_DEFER
            stats(pm, pe, pb);
#endif
            if (xl) {
                El e;
                e.z = ldE(L::Z, N);
                e.ll = ldE(L::LL, N);
                e.lu = ldE(L::LU, N);
                if (corr || fin) e.dza = ldE(L::DZA, N);
                if constexpr (fin) {
                    const T dzp = ldE(L::DZ, N);
                    e.z = fref ? e.z + dzp : e.z;
                }
                const T dx = xt - e.z;
                if constexpr (fin) {
                    T na, viol;
                    bool rem;
                    const T a = fin_flag(e, bnd(N), fs0, N);
                    s_c += finish_check(dx, e, bnd(N), a, na, viol, rem);
                    s_a += na != T(0) ? T(1) : T(0);
                    s_b += rem ? T(1) : T(0);
                    ck = viol > cviol ? N : ck;
                    cviol = fmax(cviol, viol);
                    if (pol) fin_out(N, e.z + dx, bnd(N));
                    if (pol) {
                        if (fref) {
                            stE(L::DZA, N, dx);
                        } else {
                            stE(L::DZ, N, dx);
                            stE(L::DZA, N, na);
                        }
                    }
                } else if (status >= 0) {
                    stE(dst, N, dx);
                }
                stats(dx, e, bnd(N));
            }
            s_min = corr ? gmin(s_min) : frcp(gmax(s_min));
            s_a = gsum(s_a);
            s_b = gsum(s_b);
            s_c = gsum(s_c);
            if constexpr (fin) {
                // PDAS update (oracle/c/riccati_ipm.c pdas_update): bounds with a negative multiplier
                // leave the set, violated input bounds join; of the violated state bounds only each
                // component's most violated one joins, and only in the run's first step or a step
                // without removals
                addk = (fs0 || s_b == T(0)) ? ck : -1;
            }
        };

        cptr<T> abs_ = (cptr<T>)p.AB;   // [NX][NZ] row-major, wave-uniform SGPR operand


        for (int it = 0;; it++) {
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
            LPC_TICK(-1);

            // ============================ A: backward Riccati factorisation (+ lazy step, Sigma, g, re);
            // the finish pass factors with the finish's penalty terms instead of the barrier
            bool pfail = false;
            auto riccati = [&](auto PASS) __attribute__((always_inline)) {
                constexpr bool FIN = decltype(PASS)::value == 1;
                T prow[NX], sdiag, pv;
                T znext;
                El q, qn;
                auto fetchA = [&](int k, El &e) {
                    e.z = ldE(L::Z, k);
                    e.ll = ldE(L::LL, k);
                    e.lu = ldE(L::LU, k);
                    e.g = ldE(L::GC, k);
                    e.dz = ldE(L::DZ, k);     // unconditional: a divergent load arm costs more than
                    // the bytes (first iteration: unused stale words; warm finish: the shifted flags)
                    e.dza = ldE(L::DZA, k);   // (warm flags: copied into DZA at the step start)
                };
                // terminal stage: P_N = He + Sigma_N, p_N = g_N
                fetchA(N, q);
                fetchA(N - 1, qn);
                lazy(N, q, bnd(N));
                {
                    T sg = xl ? sigma(q, bnd(N)) : T(0), gadd = 0;
                    if constexpr (FIN) {
                        finish_terms(q, bnd(N), fs0, N, sg, gadd);
                        sg = xl ? sg : T(0);
                    }
                    zb[r] = xl ? q.z : T(0);
                    LPC_SYNC();
                    T g = q.g + gadd;
                    const int rx = xl ? r : 0;
                    if (SP::hdiag) {
                        g = fma(hem[rx * LDX + rx], q.z, g);
                    } else {
#pragma unroll
                        for (int b = 0; b < NX; b++) g = fma(hem[rx * LDX + b], zb[b], g);
                    }
                    if (xl && !SP::hdiag) stE(L::GF, N, g);   // diagonal costs: C recomputes g
#pragma unroll
                    for (int i = 0; i < NX; i++) prow[i] = SP::hdiag ? T(0) : hem[rx * LDX + i];
                    sdiag = sg + (SP::hdiag ? hem[rx * LDX + rx] : T(0));
                    pv = g;
                    znext = q.z;
                    LPC_SYNC();
                }
                for (int k = N - 1; k >= 0; k--) {
                    LPC_PTICK(1);
                    q = qn;
                    if (k > 0) fetchA(k - 1, qn);
                    SpL<T, RN> arl;
                    SpL<T, CN> acl;
                    if constexpr (SPARSE) {
                        sp_load(arl, slv, sli, row_base);
                        sp_load(acl, slv, sli, col_base);
                    }
                    const Bd bk = bnd(k);
                    const T hrr = SP::hdiag ? hm[r * LDZ + r] : T(0);   // read once per stage
#if NMPC_LPC_EARLY_Z
                    const T zo = lazy_z(q);
                    zb[r] = q.z;
                    LPC_SYNC();
                    lazy_duals(k, q, zo, bk);
                    T sg = sigma(q, bk), gadd = 0;
                    if constexpr (FIN) finish_terms(q, bk, fs0, k, sg, gadd);
#else
                    lazy(k, q, bk);
                    T sg = sigma(q, bk), gadd = 0;
                    if constexpr (FIN) finish_terms(q, bk, fs0, k, sg, gadd);
                    zb[r] = q.z;
                    LPC_SYNC();
#endif
                    // g = H z + G yref (+ the finish's penalty gradient), re = [A B] z_k + c - x_{k+1}
                    T g = q.g + gadd, re = 0;
                    if (SP::hdiag) {
                        g = fma(hrr, q.z, g);
                    } else {
                        T g1 = 0;
#pragma unroll
                        for (int b = 0; b + 1 < NZ; b += 2) {
                            g = fma(hm[r * LDZ + b], zb[b], g);
                            g1 = fma(hm[r * LDZ + b + 1], zb[b + 1], g1);
                        }
                        if (NZ % 2) g = fma(hm[r * LDZ + NZ - 1], zb[NZ - 1], g);
                        g += g1;
                    }
                    if (!SP::hdiag) stE(L::GF, k, g);
                    if constexpr (SPARSE) {
                        re = sp_dot(arl, zb, c_r - znext);
                        if (xl) rb[r] = re;
                    } else if (xl) {
                        T s0 = c_r - znext, s1 = 0;
#pragma unroll
                        for (int j = 0; j + 1 < NZ; j += 2) {
                            s0 = fma(abr[r * LDZ + j], zb[j], s0);
                            s1 = fma(abr[r * LDZ + j + 1], zb[j + 1], s1);
                        }
                        if (NZ % 2) s0 = fma(abr[r * LDZ + NZ - 1], zb[NZ - 1], s0);
                        re = s0 + s1;
                        rb[r] = re;
                    }
                    znext = q.z;
                    LPC_SYNC();
                    LPC_PTICK(0);
                    // M = P [A B] (row r per x-lane; [A B] from SGPRs), Pr = P re, v = Pr + p
                    cptr<T> ab = abs_;
                    asm volatile("" : "+s"(ab));
                    if (xl) {
                        T pr0 = sdiag * re, pr1 = 0;
#pragma unroll
                        for (int l = 0; l + 1 < NX; l += 2) {
                            pr0 = fma(prow[l], rb[l], pr0);
                            pr1 = fma(prow[l + 1], rb[l + 1], pr1);
                        }
                        if (NX % 2) pr0 = fma(prow[NX - 1], rb[NX - 1], pr0);
                        const T pr = pr0 + pr1;
                        stX(k, XPR, pr);
                        vb[r] = pr + pv;
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    if (xl) {
                        // structured kernels: the diagonal part Sigma_x [A B](r, :) of M's row r
                        // touches only the <= RN structural nonzeros of row r; it is added to M^T in
                        // LDS (atomic adds after the plain stores, in order within the wavefront)
                        // instead of scaling the dense LDS row of [A B] into all NZ accumulators
                        constexpr bool ADIAG = SPARSE && NMPC_LPC_ATOMIC_DIAG;
                        SpL<T, RN> arm;
                        if constexpr (ADIAG) sp_load(arm, slv, sli, row_base);
                        T mrow[NZ];
#pragma unroll
                        for (int c = 0; c < NZ; c++) mrow[c] = ADIAG ? T(0) : sdiag * abr[r * LDZ + c];
                        sgpr_rows<NX, NZ, RPC, SP, T>(ab, [&](int l, const T (&row)[NZ]) {
#pragma unroll
                            for (int c = 0; c < NZ; c++)
                                if (SP::ab(l, c)) mrow[c] = fma(prow[l], row[c], mrow[c]);
                        });
#pragma unroll
                        for (int c = 0; c < NZ; c++) mt[c * LDX + r] = mrow[c];
                        if constexpr (ADIAG) {
#pragma unroll
                            for (int j = 0; j < RN; j++)
                                __hip_atomic_fetch_add((T *)((char *)mt + arm.o[j] * LDX) + r, sdiag * arm.v[j],
                                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                        }
                    }
                    LPC_SYNC();
                    LPC_PTICK(3);
                    // F = [A B]' M + H (column r per lane; + Sigma on the diagonal, applied by the
                    // readers), h = [A B]' v + g
                    T fcol[NZ], h;
                    if constexpr (SPARSE) {
                        h = sp_dot(acl, vb, g);
                    } else {
                        T h0 = g, h1 = 0;
#pragma unroll
                        for (int i = 0; i + 1 < NX; i += 2) {
                            h0 = fma(abt[r * LDX + i], vb[i], h0);
                            h1 = fma(abt[r * LDX + i + 1], vb[i + 1], h1);
                        }
                        if (NX % 2) h0 = fma(abt[r * LDX + NX - 1], vb[NX - 1], h0);
                        h = h0 + h1;
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    {
                        T mc[NX];
#pragma unroll
                        for (int i = 0; i < NX; i++) mc[i] = mt[r * LDX + i];
#pragma unroll
                        for (int a = 0; a < NZ; a++) fcol[a] = SP::hdiag ? T(0) : hm[r * LDZ + a];
                        asm volatile("" : "+s"(ab));
                        sgpr_rows<NX, NZ, RPC, SP, T>(ab, [&](int i, const T (&row)[NZ]) {
#pragma unroll
                            for (int a = 0; a < NZ; a++)
                                if (SP::ab(i, a)) fcol[a] = fma(row[a], mc[i], fcol[a]);
                        });
                        // materialise F here (IR sinking would otherwise defer the x part to the P
                        // update and keep every streamed row of [A B] alive in SGPRs until then)
#pragma unroll
                        for (int a = 0; a < NZ; a++) asm volatile("" : "+v"(fcol[a]));
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    if (ul) {
                        T fd = fcol[NX];
#pragma unroll
                        for (int a = 0; a < NU; a++) {
                            fu[a * NU + u] = fcol[NX + a];
                            fd = (u == a) ? fcol[NX + a] : fd;
                        }
                        fu[u * NU + u] = fd + sg + hrr;
                        hub[u] = h;
                    }
                    LPC_SYNC();
                    LPC_PTICK(4);
                    // F_uu = L L' (every lane), kff = -F_uu^{-1} h_u
                    T lf[NUT], hu[NU];
#pragma unroll
                    for (int i = 0; i < NU; i++) hu[i] = hub[i];
#pragma unroll
                    for (int i = 0; i < NU; i++)
#pragma unroll
                        for (int j = 0; j <= i; j++) {
                            T s_ = fu[i * NU + j];
#pragma unroll
                            for (int l = 0; l < j; l++) s_ = fma(-lf[tri(i, l)], lf[tri(j, l)], s_);
                            if (i == j) {
                                const bool pd = s_ > T(0);
                                if constexpr (FIN) pfail |= pol & !pd;
                                else fail |= active & !pd;
                                lf[tri(i, i)] = frsq(pd ? s_ : T(1));
                            } else {
                                lf[tri(i, j)] = s_ * lf[tri(j, j)];
                            }
                        }
                    // x-lane r: Y(:, r) = L^{-1} F_ux(:, r), K(:, r) = -L^{-T} Y(:, r), p_r = h_r + K(:, r)' h_u;
                    // u-lane u: F_uu^{-1}(u, :) = L^{-T} L^{-1} e_u, kff_u = -F_uu^{-1}(u, :) h_u — the same
                    // two triangular solves on different right-hand sides, run by every lane at once
                    T y[NU], xs[NU], pnew;
                    {
                        T f[NU];
#pragma unroll
                        for (int i = 0; i < NU; i++) f[i] = xl ? fcol[NX + i] : ((u == i) ? T(1) : T(0));
#pragma unroll
                        for (int i = 0; i < NU; i++) {
                            T s_ = f[i];
#pragma unroll
                            for (int l = 0; l < i; l++) s_ = fma(-lf[tri(i, l)], y[l], s_);
                            y[i] = s_ * lf[tri(i, i)];
                        }
#pragma unroll
                        for (int i = NU - 1; i >= 0; i--) {
                            T s_ = y[i];
#pragma unroll
                            for (int l = i + 1; l < NU; l++) s_ = fma(-lf[tri(l, i)], xs[l], s_);
                            xs[i] = s_ * lf[tri(i, i)];
                        }
                        T d = 0;
#pragma unroll
                        for (int i = 0; i < NU; i++) d = fma(xs[i], hu[i], d);
                        pnew = (xl ? h : T(0)) - d;   // x: p_r; u: kff_u
                    }
                    // stage record words 0..NU: x-lane r: K(:, r) = -xs (Pr_r sits in word NU, stored
                    // above); u-lane u: kff_u, F_uu^{-1}(u, :) = xs
                    if (xl) {   // write-only divergent block
#pragma unroll
                        for (int i = 0; i < NU; i++) ylds[r * LDU + i] = y[i];
                    }
                    stX(k, 0, xl ? -xs[0] : pnew);
#pragma unroll
                    for (int i = 1; i < NU; i++) stX(k, i, xl ? -xs[i] : xs[i - 1]);
                    if (ul) stU(k, NU, xs[NU - 1]);
                    LPC_SYNC();
                    // P(r, :) = F(r, 0:nx) - Y(:, r)' Y  (+ Sigma_x of stage k on the diagonal); u-lanes
                    // compute a dummy row (keeps the loop-carried registers dead between stages)
                    // The rows of Y stream from LDS in chunks of PCH rows, one chunk in flight while
                    // the previous one is consumed: left to itself the scheduler reused one register
                    // quad for all 26 reads, i.e. 26 serialised LDS round trips per stage.
#if NMPC_LPC_PCH == 0
#pragma unroll
                    for (int i = 0; i < NX; i++) {
                        T s_ = fcol[i];
#pragma unroll
                        for (int a = 0; a < NU; a++) s_ = fma(-ylds[i * LDU + a], y[a], s_);
                        prow[i] = s_;
                    }
#else
                    {
                        constexpr int PCH = NMPC_LPC_PCH, NPC = (NX + PCH - 1) / PCH;
                        T yb[2][PCH][NU];
                        auto yload = [&](int ch, T (&dst)[PCH][NU]) {
#pragma unroll
                            for (int ii = 0; ii < PCH; ii++) {
                                const int i = ch * PCH + ii;
#pragma unroll
                                for (int a = 0; a < NU; a++) dst[ii][a] = i < NX ? ylds[i * LDU + a] : T(0);
                            }
                        };
                        yload(0, yb[0]);
#pragma unroll
                        for (int ch = 0; ch < NPC; ch++) {
                            if (ch + 1 < NPC) yload(ch + 1, yb[(ch + 1) & 1]);
                            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                            for (int ii = 0; ii < PCH; ii++) {
                                const int i = ch * PCH + ii;
                                if (i < NX) {
                                    T s_ = fcol[i];
#pragma unroll
                                    for (int a = 0; a < NU; a++) s_ = fma(-yb[ch & 1][ii][a], y[a], s_);
                                    prow[i] = s_;
                                }
                            }
                            __builtin_amdgcn_sched_barrier(0);
                        }
                    }
#endif
                    sdiag = sg + hrr;   // F(r, r) = F_col(r) + H_rr + Sigma
                    pv = pnew;
                    LPC_SYNC();
                    LPC_PTICK(7);
                }
            };

            // ============================ exact finish step on an empty active set (structured kernels):
            // no penalty and no barrier, so the Newton system is the unconstrained LQ problem, whose
            // Riccati factorisation is the same for every instance (p.lqr, computed once per handle on
            // the host: P_{k+1}, K_k, F_uu^{-1}). What remains per instance is the vector recursion
            // p_k = h_x + K' h_u, h = g_k + [A B]' (P_{k+1} re_k + p_{k+1}), kff = -F_uu^{-1} h_u with
            // g = H z + G yref and re the dynamics residual at z; K and kff go to the stage records for
            // the forward sweep, as the full factorisation would write them
            auto lqr_back = [&]() __attribute__((always_inline)) {
                // three LDS exchanges per stage: [z_k; g_k], the residual re_k, v = p_{k+1} + P_{k+1} re_k;
                // every lane forms h_u = g_u + B' v itself (no fourth exchange), x-lanes h_x = g_x + A' v
                constexpr int OK = NX;
                const T hrr = hm[r * LDZ + r], hre = hem[(xl ? r : 0) * LDX + (xl ? r : 0)];
                T *const zk = gb + Gm::G_MT, *const gk = zk + LDZ;
                T rowc[NZ];
                auto rowld = [&](int k, T (&d_)[NZ]) {
                    const T *t_ = p.lqr + ((size_t)(k < 0 ? 0 : k) * NZ + r) * (NZ + 1);   // lqr_table rows
#pragma unroll
                    for (int j = 0; j < NZ; j++) d_[j] = t_[j];
                };
                SpL<T, RN> arl;
                SpL<T, CN> acl;
                if constexpr (SPARSE) {
                    sp_load(arl, slv, sli, row_base);
                    sp_load(acl, slv, sli, col_base);
                }
                const T *arow = abr + (xl ? r : 0) * LDZ, *acol = abt + r * LDX;
                T znext = ldE(L::Z, N), pv = fma(hre, znext, ldE(L::GC, N));   // p_N = g_N (x-lanes)
                for (int k = N - 1; k >= 0; k--) {
                    const T z = ldE(L::Z, k), gc = ldE(L::GC, k);
                    rowld(k, rowc);   // the table row (L2-resident), in flight during the first exchanges
                    zk[r] = z;
                    gk[r] = fma(hrr, z, gc);
                    LPC_SYNC();
                    T re;
                    if constexpr (SPARSE) {
                        re = sp_dot(arl, zk, c_r) - znext;
                    } else {
                        T s0 = c_r, s1 = 0;
#pragma unroll
                        for (int jj = 0; jj + 1 < NZ; jj += 2) {
                            s0 = fma(arow[jj], zk[jj], s0);
                            s1 = fma(arow[jj + 1], zk[jj + 1], s1);
                        }
                        if (NZ % 2) s0 = fma(arow[NZ - 1], zk[NZ - 1], s0);
                        re = s0 + s1 - znext;
                    }
                    if (xl) rb[r] = re;
                    LPC_SYNC();
                    T v0 = pv, v1 = 0;
#pragma unroll
                    for (int j = 0; j + 1 < NX; j += 2) {
                        v0 = fma(rowc[j], rb[j], v0);
                        v1 = fma(rowc[j + 1], rb[j + 1], v1);
                    }
                    if (NX % 2) v0 = fma(rowc[NX - 1], rb[NX - 1], v0);
                    if (xl) vb[r] = v0 + v1;
                    LPC_SYNC();
                    T hu[NU];
#pragma unroll
                    for (int i = 0; i < NU; i++) {
                        if constexpr (SPARSE) {
                            SpL<T, CN> bc;
                            sp_load(bc, slv, sli, NX * RN + (NX + i) * CN);
                            hu[i] = sp_dot(bc, vb, gk[NX + i]);
                        } else {
                            T s0 = gk[NX + i];
#pragma unroll
                            for (int l = 0; l < NX; l++) s0 = fma(abt[(NX + i) * LDX + l], vb[l], s0);
                            hu[i] = s0;
                        }
                    }
                    if (ul) {
                        T kf = 0;
#pragma unroll
                        for (int i = 0; i < NU; i++) kf = fma(-rowc[i], hu[i], kf);
                        stU(k, UKFF, kf);
                    } else {
                        T h;
                        if constexpr (SPARSE) {
                            h = sp_dot(acl, vb, gk[r]);
                        } else {
                            T h0 = gk[r], h1 = 0;
#pragma unroll
                            for (int i = 0; i + 1 < NX; i += 2) {
                                h0 = fma(acol[i], vb[i], h0);
                                h1 = fma(acol[i + 1], vb[i + 1], h1);
                            }
                            if (NX % 2) h0 = fma(acol[NX - 1], vb[NX - 1], h0);
                            h = h0 + h1;
                        }
#pragma unroll
                        for (int i = 0; i < NU; i++) {
                            h = fma(rowc[OK + i], hu[i], h);
                            stX(k, i, rowc[OK + i]);
                        }
                        pv = h;
                    }
                    znext = z;
                }
            };

            // ============================ refinement of the exact finish, vector pass (structured kernels):
            // the refinement solves the set step's Newton system again — same active set, same penalty,
            // so the same factorisation, whose records (K, F_uu^{-1}) are still in scratch — with the
            // gradient H z_a + G yref + 2 rho (z_a - bound) at z_a = z + dz. z_a satisfies the dynamics
            // up to rounding, so the residual term P re of the recursion is dropped (oracle/c/
            // riccati_ipm.c does the same). A backward vector recursion like sweep C writes the new kff.
            auto refine_back = [&]() __attribute__((always_inline)) {
                const T hrr = hm[r * LDZ + r], hre = hem[(xl ? r : 0) * LDX + (xl ? r : 0)];
                const Bd b0 = bnd(0), bm = bnd(1);
                struct RecR {
                    El e;
                    T kq[NU];
                };
                auto fetchR = [&](int k, RecR &q) {
                    k = k < 0 ? 0 : k;
                    q.e.z = ldE(L::Z, k);
                    q.e.dz = ldE(L::DZ, k);
                    q.e.dza = ldE(L::DZA, k);
                    q.e.ll = ldE(L::LL, k);
                    q.e.lu = ldE(L::LU, k);
                    q.e.g = ldE(L::GC, k);
                    const int kk = k < N ? k : N - 1;
                    T w_[NU + 1];
#pragma unroll
                    for (int i = 0; i <= NU; i++) w_[i] = ldX(kk, i);
#pragma unroll
                    for (int i = 0; i < NU; i++) q.kq[i] = xl ? w_[i] : w_[UFI + i];
                };
                auto gref = [&](int k, RecR &q) {
                    const Bd b = k == N ? bnd(N) : (k == 0 ? b0 : bm);
                    T sg, gadd;
                    finish_terms(q.e, b, false, k, sg, gadd);   // q.e.z becomes z_a
                    return fma(k < N ? hrr : hre, q.e.z, q.e.g + gadd);
                };
                RecR qN;
                fetchR(N, qN);
                T pv = gref(N, qN);
                RecR ring[PD];
#pragma unroll
                for (int j = 0; j < PD; j++) fetchR(N - 1 - j, ring[j]);
                SpL<T, CN> acl;
                if constexpr (SPARSE) sp_load(acl, slv, sli, col_base);
                const T *acol = abt + r * LDX;
                for (int kb = 0; kb < N; kb += PD) {
#pragma unroll
                    for (int j = 0; j < PD; j++) {
                        const int k = N - 1 - kb - j;
                        if (k < 0) break;
                        RecR &q = ring[j];
                        const T gh = gref(k, q);
                        if (xl) vb[r] = pv;
                        LPC_SYNC();
                        T h;
                        if constexpr (SPARSE) {
                            h = sp_dot(acl, vb, gh);
                        } else {
                            T h0 = gh, h1 = 0;
#pragma unroll
                            for (int i = 0; i + 1 < NX; i += 2) {
                                h0 = fma(acol[i], vb[i], h0);
                                h1 = fma(acol[i + 1], vb[i + 1], h1);
                            }
                            if (NX % 2) h0 = fma(acol[NX - 1], vb[NX - 1], h0);
                            h = h0 + h1;
                        }
                        if (ul) hub[u] = h;
                        LPC_SYNC();
                        T hu[NU];
#pragma unroll
                        for (int i = 0; i < NU; i++) hu[i] = hub[i];
                        if (ul) {
                            T kf = 0;
#pragma unroll
                            for (int i = 0; i < NU; i++) kf = fma(-q.kq[i], hu[i], kf);
                            stU(k, UKFF, kf);
                        } else {
                            T s_ = h;
#pragma unroll
                            for (int i = 0; i < NU; i++) s_ = fma(q.kq[i], hu[i], s_);
                            pv = s_;
                        }
                        fetchR(k - PD, ring[j]);
                        LPC_SYNC();
                    }
                }
            };

            // ============================ exact finish (groups with mu <= polish_at): a primal-dual
            // active-set run of penalised factorisations + forward sweeps (<= polish_steps set steps,
            // then the refinement) for the polishing groups; accepted groups are done, the others go
            // on with this iteration from their untouched IPM iterate
            pol = active && p.polish_mu > T(0) && mu <= polish_at;
            if (__any(pol)) {
                polish_at = pol ? fmin(polish_at, mu) * p.polish_drop : polish_at;
                const int plim = fin_runs == 0 ? p.polish_first : p.polish_steps;   // set steps of this run
                fin_runs += pol ? 1 : 0;
                fref = false;
                for (int fs = 0; fs <= (p.polish_first > p.polish_steps ? p.polish_first : p.polish_steps); fs++) {
                    fs0 = fs == 0;
                    fwarm = warm && fs0 && it == 0;   // first run of the solve: pending is false
                    pfail = false;
                    // the refinement reuses the set step's factorisation when every polishing group of
                    // the wavefront is refining (structured kernels: diagonal costs)
                    // and an empty first set (warm: the previous solution had no active bound; cold: the
                    // first-set rule marks none) runs lqr_back
                    const bool sempty = fs0 && it == 0 && (fwarm ? warm_act == T(0) : cold_act == T(0));
                    if (SP::hdiag && __all(!pol || fref)) refine_back();
                    else if (SP::hdiag && p.lqr && __all(!pol || sempty)) lqr_back();
                    else riccati(Pass<1>{});
                    LPC_STICK(2);
                    pending = false;
                    T d0, nact, d2, nbad;
                    forward(Pass<2>{}, d0, nact, d2, nbad);
                    LPC_STICK(3);
                    if (pol) {
                        fin_steps++;
                        const bool okp = nbad == T(0) && !pfail;
                        if (fref) {
                            if (okp) {
                                active = false;
                                status = -1;
                                iters = it + fin_steps;
                            }
                            pol = false;
                        } else if (okp && nact == T(0)) {
                            // no active bound: an unpenalised Newton step, nothing to refine
                            // (DZA holds the all-zero flags, the output adds nothing)
                            active = false;
                            status = -1;
                            iters = it + fin_steps;
                            pol = false;
                        } else if (okp) {
                            fref = true;
                        } else if (pfail || fs + 1 >= plim) {
                            pol = false;
                        }
                    }
                    if (!__any(pol)) break;
                }
                pol = fref = false;
                fwarm = false;
                if (!__any(active)) break;
            }
            riccati(Pass<0>{});
            LPC_STICK(4);

            LPC_TICK(1);
            pending = false;   // the previous step is applied (converged groups stay frozen from here)

            // ============================ B: forward predictor + ratio test / centring sums
            T a_aff, S0, S2, dummy;
            forward(Pass<0>{}, a_aff, S0, S2, dummy);
            LPC_TICK(2);
            // mu_aff = [(1 - a) S0 - a^2 S2'] / m with S2' = sum lam dz (t + dz) / t (closed form)
            const T mu_aff = ((T(1) - a_aff) * S0 - a_aff * a_aff * S2) * p.inv_m;
            const T sgm = mu > T(0) ? fmax(mu_aff, T(0)) * frcp(mu) : T(0);
            smu = sgm * sgm * sgm * mu;

            // ============================ C: backward corrector vector
            {
                // sweep constants: H_rr, interior and stage-0 bounds
                const T hrr = SP::hdiag ? hm[r * LDZ + r] : T(0);
                const Bd b0 = bnd(0), bm = bnd(1);
                auto ghat = [&](int k, const El &e) {
                    T g = e.g;
                    if (SP::hdiag) g = fma(k < N ? hrr : hem[(xl ? r : 0) * LDX + (xl ? r : 0)], e.z, g);
                    const Bd b = k == N ? bnd(N) : (k == 0 ? b0 : bm);
                    const T tl = e.z - b.lb, tu = b.ub - e.z, itl = frcp(tl), itu = frcp(tu);
                    const T dll = -e.ll * (T(1) + e.dza * itl), dlu = -e.lu * (T(1) - e.dza * itu);
                    const T cl = (dll * e.dza - smu) * itl, cu = (dlu * e.dza + smu) * itu;
                    return g + (e.ll > T(0) ? cl : T(0)) + (e.lu > T(0) ? cu : T(0));
                };
                struct RecC {
                    El e;
                    T pr, kq[NU];
                };
                auto fetchC = [&](int k, RecC &q) {
                    k = k < 0 ? 0 : k;
                    q.e.z = ldE(L::Z, k);
                    q.e.ll = ldE(L::LL, k);
                    q.e.lu = ldE(L::LU, k);
                    q.e.dza = ldE(L::DZA, k);
                    q.e.g = ldE(SP::hdiag ? L::GC : L::GF, k);   // diagonal costs: g = G yref + H_rr z below
                    const int kk = k < N ? k : N - 1;
                    // same words for every lane (see fetch of the forward sweeps): x-lane K(:, r) and
                    // Pr_r in words 0..NU, u-lane F_uu^{-1}(u, :) in words 1..NU
                    T w[NU + 1];
#pragma unroll
                    for (int i = 0; i <= NU; i++) w[i] = ldX(kk, i);
                    q.pr = w[XPR];
#pragma unroll
                    for (int i = 0; i < NU; i++) q.kq[i] = xl ? w[i] : w[UFI + i];
                };
                const T *acol = abt + r * LDX;   // column r of [A B] (LDS, read per stage)
                RecC qN;
                fetchC(N, qN);
                T pv = ghat(N, qN.e);
                RecC ring[PD];
#pragma unroll
                for (int j = 0; j < PD; j++) fetchC(N - 1 - j, ring[j]);
                SpL<T, CN> acl;
                if constexpr (SPARSE) sp_load(acl, slv, sli, col_base);
                for (int kb = 0; kb < N; kb += PD) {
#pragma unroll
                    for (int j = 0; j < PD; j++) {
                        const int k = N - 1 - kb - j;
                        if (k < 0) break;
                        RecC &q = ring[j];   // read in place, refilled after its last use (see forward)
#if NMPC_LPC_EARLY_Z
                        // v first: the corrector right-hand side is only needed after the exchange
                        if (xl) vb[r] = q.pr + pv;
                        LPC_SYNC();
                        const T gh = ghat(k, q.e);
#else
                        const T gh = ghat(k, q.e);
                        if (xl) vb[r] = q.pr + pv;
                        LPC_SYNC();
#endif
                        T h;
                        if constexpr (SPARSE) {
                            h = sp_dot(acl, vb, gh);
                        } else {
                            T h0 = gh, h1 = 0;
#pragma unroll
                            for (int i = 0; i + 1 < NX; i += 2) {
                                h0 = fma(acol[i], vb[i], h0);
                                h1 = fma(acol[i + 1], vb[i + 1], h1);
                            }
                            if (NX % 2) h0 = fma(acol[NX - 1], vb[NX - 1], h0);
                            h = h0 + h1;
                        }
                        if (ul) hub[u] = h;
                        LPC_SYNC();
                        T hu[NU];
#pragma unroll
                        for (int i = 0; i < NU; i++) hu[i] = hub[i];
                        if (ul) {
                            T kf = 0;
#pragma unroll
                            for (int i = 0; i < NU; i++) kf = fma(-q.kq[i], hu[i], kf);
                            stU(k, UKFF, kf);
                        } else {
                            T s_ = h;
#pragma unroll
                            for (int i = 0; i < NU; i++) s_ = fma(q.kq[i], hu[i], s_);
                            pv = s_;
                        }
                        fetchC(k - PD, ring[j]);
                        LPC_SYNC();
                    }
                }
            }

            LPC_TICK(5);
            // ============================ D: forward corrector + step length / new mu
            T amax, T0, C1, C2;
            forward(Pass<1>{}, amax, T0, C1, C2);
            LPC_TICK(6);
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
            LPC_STICK(5);
        }

        // ------------------------------------------------------------------ apply pending step, outputs
        // (groups the finish completed, status -1, wrote their outputs in the accepted step's sweep)
        if (inst_ok && status >= 0) {
            T fprev = 0;
            // the iterate words of OC stages are loaded together (one memory latency per chunk)
            constexpr int OC = 4;
            for (int kc = 0; kc <= N; kc += OC) {
                T zc[OC], dc[OC];
#pragma unroll
                for (int j = 0; j < OC; j++) {
                    const int k = kc + j <= N ? kc + j : N;
                    zc[j] = ldE(L::Z, k);
                    dc[j] = ldE(L::DZ, k);
                }
#pragma unroll
                for (int j = 0; j < OC; j++) {
                    const int k = kc + j;
                    if (k > N) break;
                    if (k == N && ul) {   // u-lanes: stage N mirrors N - 1 for the shift
                        if (amask) mset(actm, N, fprev);
                        else if (fused) stE(L::ACT, N, fprev);
                        continue;
                    }
                    const Bd bk = bnd(k);
                    T z = zc[j];
                    if (pending) z += alpha * dc[j];
                    if (fastpl && k == 0) clz[r] = z;
                    if (xl) xo[k * NX + r] = z;
                    else uo[k * NU + u] = z;
                    if (fused) {   // the solution's active flags, the next step's warm start
                        const bool onl = has_bound(bk.lb) && z <= bk.lb + T(1e-7) * (T(1) + fabs(bk.lb));
                        const bool onu = has_bound(bk.ub) && z >= bk.ub - T(1e-7) * (T(1) + fabs(bk.ub));
                        fprev = onl ? T(-1) : (onu ? T(1) : T(0));
                        if (amask) mset(actm, k, fprev);
                        else stE(L::ACT, k, fprev);
                    }
                }
            }
        }
        if (inst_ok) {
            if (r == 0) {
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
        LPC_STICK(6);
        if (fused) {
            // closed-loop advance of this step by the instance's lanes (its outputs were written by
            // the lanes of this wavefront just above); the next step's x0 is read by the whole group
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            if (fastpl) {
                // cl_advance_group for the controller-model plant: cost sum_i w_i (x_0 - xref)_i^2 and
                // AED numerator sum_i |xref - x|_i at the current state (x_0 is pinned to it; xref =
                // yref row 0), then x <- [A B] [x; u_0] + c + noise
                const int nc = p.cl.ncl, na_ = p.cl.aed_dims;
                const T xs = clx[r];
                const double e_ = (double)xs - (double)cly[r];
                double ce = (xl && r < nc) ? (double)p.cl.wcl[r] * e_ * e_ : 0.0;
                double ae = (xl && r < na_) ? fabs(e_) : 0.0;
                ce = gsum(ce);
                ae = gsum(ae);
                T *zx = gb + Gm::G_MT;
                zx[r] = xl ? xs : clz[r];
                LPC_SYNC();
                T sx;
                if constexpr (SPARSE) {
                    sx = sp_dot(arl0, zx, c_r);
                } else {
                    T s0 = c_r, s1 = 0;
#pragma unroll
                    for (int jj = 0; jj + 1 < NZ; jj += 2) {
                        s0 = fma(abr[(xl ? r : 0) * LDZ + jj], zx[jj], s0);
                        s1 = fma(abr[(xl ? r : 0) * LDZ + jj + 1], zx[jj + 1], s1);
                    }
                    if (NZ % 2) s0 = fma(abr[(xl ? r : 0) * LDZ + NZ - 1], zx[NZ - 1], s0);
                    sx = s0 + s1;
                }
                const double w_ = lmode ? p.cl_noise[(size_t)inst * p.cl_noise_ld + (cl_base + cstep - p.cl_noise_step0)]
                                        : p.cl_noise[(size_t)inst * nsteps + cstep];
                if (xl) clx[r] = (T)((double)sx + (r < p.cl.noise_dims ? w_ : 0.0));
                if (r == 0) {
                    cls[0] += (T)ce;
                    cls[1] += (T)ae;
                    cls[2] += (status > 0) ? T(1) : T(0);
                    cls[3] += T(1);
                }
            } else if (inst_ok) {
                cl_advance_group<T, NX, NU>(p.cl, inst, cl_base + cstep, status < 0 ? 0 : status, r,
                                            lmode ? p.cl_noise[(size_t)inst * p.cl_noise_ld + (cl_base + cstep - p.cl_noise_step0)]
                                                  : p.cl_noise[(size_t)inst * nsteps + cstep]);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        }
        LPC_STICK(7);
    }
    if (lmode && fused) {
        // the lean loop's state of the instance: its solution's active flags by slot, the next step
        // (the fast general solve's list mode, cl_steps = 0, is a plain cold solve per listed instance)
        if (inst_ok) {
            for (int k = 0; k <= N; k++) {
                if ((k == N && ul) || (k == 0 && xl)) continue;
                const int sl = p.cl_eslot[k * NZ + r];
                if (sl >= 0) {
                    const T f = amask ? mflag(actm, k) : ldE(L::ACT, k);
                    p.cl_flags[(size_t)inst * p.cl_nslot + sl] = f < T(0) ? -1 : (f > T(0) ? 1 : 0);
                }
            }
            if (r == 0) p.cl_istep[inst] = cl_base + nsteps;
        }
    } else if (amask) {   // the warm start of the next launch
        for (int k = 0; k <= N; k++) stE(L::ACT, k, mflag(actm, k));
    }
    if (fastpl && inst_ok) {   // the launch's final state and its closed-loop sums
        if (xl) p.cl.state[(size_t)inst * NX + r] = clx[r];
        if (r < 4) p.cl.acc[(size_t)inst * 4 + r] += (double)cls[r];
    }
#ifdef NMPC_STEP_TIMING
    if (p.cycles && inst_ok && r == 0) {
        unsigned long long *c = p.cycles + (size_t)inst * 9, tot = 0;
        for (int j = 0; j < 8; j++) {
            c[j] = st_cy[j];
            tot += st_cy[j];
        }
        c[8] = tot;
    }
#endif
#undef LPC_STICK
}

}  // namespace lpc

// ---------------------------------------------------------------------- launch glue
template <typename T, int NX, int NU, int WPB, int MW, class SP>
hipError_t launch_ipm_lpc(const IpmParams<T> &p, hipStream_t s)
{
    using Gm = lpc::Geom<T, NX, NU, WPB>;
    const int waves = ((p.cl_list ? p.cl_count : p.B) + Gm::IPW - 1) / Gm::IPW;
    const int blocks = (waves + WPB - 1) / WPB;
    if (blocks < 1) return hipSuccess;
    NMPC_LAUNCH((lpc::ipm_lpc_kernel<T, NX, NU, WPB, MW, SP>), dim3(blocks), dim3(64 * WPB), 0, s, p);
    return hipGetLastError();
}

// explicit instantiations (the dispatch table in nmpc_ipm.hip binds them)
#define NMPC_LPC_INST(NX, NU, WPB, MW, SP)                                                              \
    template hipError_t launch_ipm_lpc<double, NX, NU, WPB, MW, SP>(const IpmParams<double> &, hipStream_t); \
    template hipError_t launch_ipm_lpc<float, NX, NU, WPB, MW, SP>(const IpmParams<float> &, hipStream_t);
NMPC_LPC_INST(13, 4, 4, 3, lpc::DenseStructure<13 NMPC_COMMA 4>)
NMPC_LPC_INST(13, 4, 1, 3, lpc::DenseStructure<13 NMPC_COMMA 4>)
NMPC_LPC_INST(13, 4, 2, 2, lpc::DenseStructure<13 NMPC_COMMA 4>)
NMPC_LPC_INST(4, 2, 4, 2, lpc::DenseStructure<4 NMPC_COMMA 2>)
NMPC_LPC_INST(6, 2, 4, 2, lpc::DenseStructure<6 NMPC_COMMA 2>)
NMPC_LPC_INST(13, 4, 4, 3, lpc::Quad13Structure)
NMPC_LPC_INST(13, 4, 1, 3, lpc::Quad13Structure)
NMPC_LPC_INST(13, 4, 2, 2, lpc::Quad13Structure)
NMPC_LPC_INST(4, 2, 4, 2, lpc::ForceStructure)
NMPC_LPC_INST(6, 2, 4, 2, lpc::JerkStructure)
#undef NMPC_LPC_INST

}  // namespace nmpc
