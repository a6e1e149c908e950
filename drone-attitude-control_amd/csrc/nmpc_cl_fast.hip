// nmpc_cl_fast.hip — the lean fused closed loop (gfx950): the exact finish's fast path as its own
// kernel, one wavefront per instance at a time.
//
// Each closed-loop step of the reference (src/force_model/controller.py:25-54: yref window from the
// reference table (force_model/ocp.py:117-122), x0 pinned to the state, solve(), u0 to the plant,
// cost (controller.py:40-41) and AED (store_results.py:233-236)) solves one box-constrained LQ-OCP.
// Its exact solution is almost always reached without any factorisation (the fast
// finish of the lane-per-component kernel, oracle/c/riccati_ipm.c fast_finish):
//
//   * explicit unconstrained solution: z_0 = T_x x0 + v_t, linear in the state and in the reference
//     row t the window starts at (tables built at nmpc_closed_loop_init);
//   * if the previous solution touched no bound and z_0 satisfies every bound (1e-13), it is the
//     solution; otherwise primal-dual active-set steps on the projected inverse Hessian W of the
//     unconstrained problem (z = z_0 + W[:, S] nu, W_SS nu = b_S - z_0,S, sets of <= WSM bounds,
//     KKT acceptance with the multiplier signs measured as displacements nu_i W_ii);
//   * a QP the interval certificate proves infeasible returns status 4 with the initial point's
//     inputs (the lane-per-component kernel's failure output);
//   * anything else is parked: the instance stops, and the host runs one full solve (IPM + exact
//     finish, ipm_lpc_kernel in list mode) for every parked instance before the next round.
//
// Layout: only the bounded elements of z matter for the test (quad13: 251 of 357), so the wavefront's
// 64 lanes own them in "slots" s = j * 64 + lane (j < EPL, stage-major order: stage 0's inputs are
// slots 0..nu-1, stage 1's bounded elements follow). The slots' T_x rows, bounds and test thresholds
// sit in the workgroup's LDS (shared by its wavefronts). The closed-loop state is lane-distributed:
// lane i < nx holds x_i, so the plant step is one dense row per lane ([A B] row from LDS, x from a
// broadcast LDS copy, u0 by readlane) and the cost / AED terms are per-lane partial sums reduced once,
// when the instance's launch ends. A step costs one coalesced load of the window's v_t slots (one step
// ahead), EPL x nx FMAs per lane, one wave vote, the plant row and the per-lane sums. No per-step
// stores: the solution's active flags stay in a register mask, the trajectory outputs are written once,
// at the instance's last step.

#include <hip/hip_runtime.h>

#include <cfloat>
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "nmpc_cl_device.h"
#include "nmpc_internal.h"
#include "nmpc_lpc_geom.h"

namespace nmpc {
namespace clf {


constexpr int PDAS_ROUNDS = 6;   // rounds of the first PDAS run before the fallback (oracle: fast_finish's cap)

// diagnostic build (-DNMPC_CLF_TIMING, build.build_experiment; env NMPC_CLF_CYCLES): shader cycles per
// phase, summed per instance in the wavefront's LDS record and added to p.cycles[inst][CLF_NT] at its
// write-back. Phases: 0 step prologue (loads, warm-start shift), 1 explicit form + bound test, 2 PDAS
// runs (wsteps_run), 3 of which the set solves, 4 of which the W[:, S] nu combinations, 5 the dual
// fallback (gi_set), 6 certificate, 7 outputs, 8 plant + cost, 9 instance record load / write-back;
// counts: 10 PDAS rounds, 11 GI iterations, 12 slow steps, 13 steps; GI parts: 14 entering-bound choice,
// 15 a = W[S, p] loads + r = H a + theta + ratio test, 16 dz combination, 17 H update; PDAS parts: 18 set
// load, 19 bound tests / additions after the combination, of which 20 the state additions (add_states);
// 21 the multiplier signs after the set solve, 22 the round's set count at its top, 23 the z checks alone
constexpr int CLF_NT = 24;   // (nmpc_api.cpp CLF_NT_HOST)
#ifdef NMPC_CLF_TIMING
#define CLF_T(v) const long long v = clock64()
#define CLF_TADD(L, i, v)                              \
    do {                                               \
        if (lane == 0) (L).tacc[i] += clock64() - (v); \
    } while (0)
#define CLF_TCNT(L, i, n)                 \
    do {                                  \
        if (lane == 0) (L).tacc[i] += (n); \
    } while (0)
#else
#define CLF_T(v) \
    do {         \
    } while (0)
#define CLF_TADD(L, i, v) \
    do {                  \
    } while (0)
#define CLF_TCNT(L, i, n) \
    do {                  \
    } while (0)
#endif

// Checked builds (-DNMPC_CLF_CHECK, build.build_experiment("clfcheck", ["NMPC_CLF_CHECK"])): every index the
// lean loops form from run-time data is tested before its access; a failed test sets bit `code` of p.check
// (a global vector atomic), prints its first occurrence, and the host fails the run (nmpc_api.cpp clf_run).
// Codes: 1 claim-order position, 2 claimed instance, 3 v_t row, 4 phase-2 queue position, 5 noise column,
// 6 reference row, 7 run_instance's instance, 8 run_instance's step below the launch's first, 9 phase-2
// instance, 10 output element
#ifdef NMPC_CLF_CHECK
template <typename P>
__device__ __noinline__ void clf_violation(const P &p, int code, long long v, int line)
{
    if (p.check && atomicOr(p.check, 1u << code) == 0u) printf("[clf check] code %d value %lld (line %d)\n", code, v, line);
}
#define CLF_CHECK(ok, code, v)                                                 \
    do {                                                                       \
        if (!(ok)) clf_violation(p, (code), (long long)(v), __LINE__);         \
    } while (0)
#else
#define CLF_CHECK(ok, code, v) \
    do {                       \
    } while (0)
#endif

// decision thresholds by storage precision, relative to 1 + |b|: viol — a bound counts as violated beyond
// it (fast-path acceptance, PDAS additions, the dual fallback's entering bound); onb — the solution's
// warm-start flags (z within it of a bound). fp32 handles hold z_0 = v_t + T_x x to a few fp32 ulps of the
// terms' magnitude (|T_x x| ~ 1-10: ~1e-6 absolute), so their thresholds sit above that noise; the held-bound
// check (1e-9) and the multiplier signs (1e-10) are taken on fp64 quantities in both precisions (W is
// fp64 for both — an ill-conditioned set's multipliers would amplify its fp32 rounding by cond(W_SS) — the
// W[:, S] nu combinations accumulate in fp64, the set solves run in fp64), DESIGN.md §6
template <typename T>
struct ClfTol {
    static constexpr double viol = 1e-13, onb = 1e-7;
};
template <>
struct ClfTol<float> {
    static constexpr double viol = 2e-6, onb = 1e-5;
};

template <typename T>
__device__ __forceinline__ bool has_b(T b)
{
    return fabs(b) < T(1e20);
}

// wave-uniform double from lane l
__device__ __forceinline__ double bcast(double v, int l)
{
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}

// 1 / d: v_rcp_f64 refined by two Newton steps (to the last bit or one off; a division is ~10 dependent
// instructions on the sweep's critical path)
__device__ __forceinline__ double rcp_nr(double d)
{
    double f = __builtin_amdgcn_rcp(d);
    f = fma(fma(-d, f, 1.0), f, f);
    return fma(fma(-d, f, 1.0), f, f);
}

// sum / max / min over the wavefront's lanes (butterfly)
__device__ __forceinline__ double wave_sum(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ double wave_max(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ double wave_min(double v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
    return v;
}

// per-wavefront LDS: active flags by slot (the warm-start shift), the set of an active-set step
// (element, sign, target b - z_0, multiplier), the explicit inverse H = W_SS^-1 of the set's block of W
// (hm, rows by set position; the dual fallback's incremental updates, the sweep of sets > 16), two
// broadcast vectors, the per-component argmax of the violated states, the certificate's stage exchange
// and the state copy
template <int WSM>
struct HGeom {
    static constexpr int CPL = WSM * WSM / 64;   // H columns per lane: lane = row i + WSM * column group g
    static constexpr int HP = WSM + 2;           // row pitch (even: 16-byte aligned column groups)
};
// SW2: the symmetric sweep with its pivots unrolled per column group (the one-wavefront-per-SIMD variant, which
// has the register room; sweep_inverse)
template <int NSLOT, int NZ, int WSM, bool SW2 = false>
struct Lds {
    static constexpr bool sweep2 = SW2;
    alignas(16) double xs[32];   // x (lane i writes x_i; x_nx.. stay 0): explicit form, plant rows, rare paths
    signed char fl[NSLOT];       // the warm-start shift buffer
    alignas(16) double hm[WSM][HGeom<WSM>::HP];
    alignas(16) double vb1[WSM], vb2[WSM];
    double se_t[WSM], se_nu[WSM], wdg[WSM];
    int se_e[WSM], se_s[WSM], gi_slot[WSM], se_ord[WSM];
    int cl_e[WSM], cl_s[WSM];    // compacted element / slot list of the active positions (w_combo_slots)
    double cl_c[WSM];            // ... and their coefficients
    unsigned long long vmax[NZ];
    int vslot[NZ];
    double cm[32], cr[32];       // certificate exchange
#ifdef NMPC_CLF_TIMING
    long long tacc[CLF_NT];
#endif
};

// the workgroup's slot constants (LDS), seen from one lane: slot j of this lane is j * 64 + lane.
// lo / hi: violation thresholds of the fast path (z < lo or z > hi: a bound violated beyond 1e-13
// relative to 1 + |b|; -/+DBL_MAX without a bound); onl / onu: on-bound thresholds of the warm-start
// flags (z <= onl: on the lower bound to 1e-7, z >= onu: on the upper)
template <int EPL>
struct SlotView {
    const double *lb_, *ub_, *lo_, *hi_, *onl_, *onu_;
    const int *e_, *src_;   // src_: the warm-start source codes (nmpc_api.cpp clf_setup; 0: none)
    int lane;
    // wl_: W over the slots in the workgroup's LDS (lower triangle, row s: wt_[s (s + 1) / 2 + s'], s' <= s);
    // else W from the global table by element. W is symmetric. (A flag, not a null test: the compiler cannot
    // null-test a generic pointer into LDS.)
    const double *wt_ = nullptr;
    bool wl_ = false;
    // wc_: this wavefront holds the workgroup's W column cache (WCache; quad13 / jerk shapes): W[ea][eb] is column
    // colof[sa] of the cache at slot sb — the caller made that column resident (wc_fill) before the access
    const double *wcol_ = nullptr;
    const short *wcolof_ = nullptr;
    int wcld_ = 0;
    bool wc_ = false;
    // W[e(sa)][e(sb)] from the cache (column of slot sa resident)
    __device__ double wcv(int sa, int sb) const
    {
        const int c = wcolof_[sa];
        return wcol_[(c < 0 ? 0 : c) * wcld_ + sb];
    }
    template <typename T>
    __device__ double w(const ClFastParams<T> &p, int ea, int sa, int eb, int sb) const
    {
        if (wl_) {   // (24-bit multiply: full rate, the 32-bit one is quarter rate)
            const int hi = sa > sb ? sa : sb, lo = sa > sb ? sb : sa;
            return wt_[(int)(__umul24((unsigned)hi, (unsigned)(hi + 1)) >> 1) + lo];
        }
        return p.W[(size_t)ea * p.ne + eb];
    }
    __device__ double lb(int j) const { return lb_[j * 64 + lane]; }
    __device__ double ub(int j) const { return ub_[j * 64 + lane]; }
    __device__ double lo(int j) const { return lo_[j * 64 + lane]; }
    __device__ double hi(int j) const { return hi_[j * 64 + lane]; }
    __device__ double onl(int j) const { return onl_[j * 64 + lane]; }
    __device__ double onu(int j) const { return onu_[j * 64 + lane]; }
    __device__ int e(int j) const { return e_[j * 64 + lane]; }
    __device__ int src(int j) const { return src_[j * 64 + lane]; }
};

#define CLF_SYNC()                                               \
    do {                                                         \
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   \
        __builtin_amdgcn_wave_barrier();                         \
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   \
    } while (0)

// The workgroup's cache of W columns over the slots (quad13 / jerk shapes; LDS): column c holds W[e][s] for the
// element e of slot ce[c] and every slot s of the layout; colof[s] = the column of slot s's element, or -1. W is one
// matrix for every instance and step, so a resident column stays valid across steps, instances and wavefronts; one
// wavefront at a time owns the cache (owner, taken per rare step in slow_step), the others read W from L2. An
// active-set round then reads W_SS and W[:, S] from LDS; only the set's new columns are loaded (the set of the
// next round, step, or the next instance riding the same bound mostly repeats). WC = the largest set + 1 (the dual
// fallback's entering bound beside a full set)
template <int WC, int NSLOT>
struct WCache {
    double col[WC][NSLOT];
    short colof[NSLOT];
    short ce[WC];
    int owner;   // the owning wavefront, or -1
    int next;    // the round-robin eviction start
};

// the empty cache (every thread of the workgroup, before the workgroup's first barrier)
template <int WC, int NSLOT>
__device__ void wc_init(WCache<WC, NSLOT> &C)
{
    for (int s = threadIdx.x; s < NSLOT; s += blockDim.x) C.colof[s] = -1;
    for (int c = threadIdx.x; c < WC; c += blockDim.x) C.ce[c] = -1;
    if (threadIdx.x == 0) {
        C.owner = -1;
        C.next = 0;
    }
}

// make the columns of the slots of lanes 0..n-1 (slot_i on lane i; wave-uniform n, n + popcount(keep) <= WC)
// resident, evicting only columns outside that list and outside `keep` (a column bit mask). Each lane loads its
// slots' entries of a missing column, WCB columns in flight at a time
#ifndef NMPC_WCB
#define NMPC_WCB 2
#endif
#ifndef NMPC_WCACHE
#define NMPC_WCACHE 0   // experiment builds: -DNMPC_WCACHE=1 compiles the cache into the lean kernels
#endif
constexpr int WCB = NMPC_WCB;
template <typename T, int EPL, int WC, int NSLOT>
__device__ __noinline__ void wc_fill(const ClFastParams<T> &p, WCache<WC, NSLOT> &C, const SlotView<EPL> &sv, int slot_i, int n,
                        unsigned keep, int lane)
{
    if constexpr (WC > 32) return;   // (no cache for sets beyond 16: the force shape's kernels never pass one)
    const int si = lane < n ? slot_i : 0;
    const int ci = lane < n ? (int)C.colof[si] : -1;
    const unsigned long long miss = __ballot(lane < n && ci < 0);
    if (!miss) return;
    unsigned used = keep | (ci >= 0 ? 1u << ci : 0u);
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) used |= (unsigned)__shfl_xor((int)used, o);
    int nxt = C.next;
    int e[EPL];
#pragma unroll
    for (int j = 0; j < EPL; j++) e[j] = sv.e(j);
    for (unsigned long long mm = miss; mm;) {
        int cs[WCB], ss[WCB], nb = 0;
        double w[WCB][EPL];
#pragma unroll
        for (int q = 0; q < WCB; q++) {
            cs[q] = -1;
            ss[q] = 0;
            if (mm) {
                const int i = (int)__builtin_ctzll(mm);
                mm &= mm - 1;
                int c = nxt;
                for (int t = 0; t < WC && ((used >> c) & 1u); t++) c = c + 1 == WC ? 0 : c + 1;
                used |= 1u << c;
                nxt = c + 1 == WC ? 0 : c + 1;
                cs[q] = c;
                ss[q] = __builtin_amdgcn_readfirstlane(__shfl(si, i));
                nb = q + 1;
            }
        }
#pragma unroll
        for (int q = 0; q < WCB; q++) {
            const int ea = q < nb ? sv.e_[ss[q]] : 0;
#pragma unroll
            for (int j = 0; j < EPL; j++)
                w[q][j] = (q < nb && e[j] >= 0) ? p.W[(size_t)ea * p.ne + e[j]] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < WCB; q++) {
            if (q >= nb) continue;
#pragma unroll
            for (int j = 0; j < EPL; j++) C.col[cs[q]][j * 64 + lane] = w[q][j];
            if (lane == 0) {
                const int old = C.ce[cs[q]];
                if (old >= 0) C.colof[old] = -1;
                C.ce[cs[q]] = (short)ss[q];
                C.colof[ss[q]] = (short)cs[q];
            }
        }
        CLF_SYNC();
    }
    if (lane == 0) C.next = nxt;
    CLF_SYNC();
}

// The rare path's W gathers as unconditional loads (a clamped index outside the set, the value masked after the
// load; a load under a branch makes the join wait for every load in flight) and the dual fallback's W[p, :] row
// issued with its a = W[S, p]: for the force shape (two slots per lane). Same-box A/B (profiles/
// r6r_gather_ab.jsonl, r6s_mix_ab.jsonl): force B = 1024 and 8192 +7..10 %; quad13 and jerk -6 %, so they keep the
// branches
template <int EPL>
constexpr bool UNCOND_GATHER = EPL <= 2;

// 2-bit flags of a per-lane mask (bit 2j lower, 2j+1 upper) <-> -1 / 0 / 1
__device__ __forceinline__ signed char flag_of(unsigned m, int j)
{
    const unsigned b = (m >> (2 * j)) & 3u;
    return b == 1u ? (signed char)-1 : (b == 2u ? (signed char)1 : (signed char)0);
}
__device__ __forceinline__ unsigned bits_of(signed char f) { return f < 0 ? 1u : (f > 0 ? 2u : 0u); }

// the solver's initial point at element (k, r) (the lane-per-component kernel's failure output):
// x_0 pinned, states at the reference projected 1 % inside their box, inputs mid-box
template <typename T>
__device__ T init_point(const ClFastParams<T> &p, int nx, int nz, int k, int r, int t, T x0r)
{
    const int ty = k == 0 ? 0 : (k == p.N ? 2 : 1);
    const T lb = p.lbnd[ty * nz + r], ub = p.ubnd[ty * nz + r];
    if (k == 0 && r < nx) return x0r;
    const bool yv = k < p.N ? r < p.ny : r < p.ny_e;
    T v = yv ? p.table[(size_t)(t + k) * p.table_cols + r] : T(0);
    const bool hl = has_b(lb), hu = has_b(ub);
    if (r >= nx && hl && hu) v = T(0.5) * (lb + ub);
    if (hl && hu) {
        const T d = T(0.01) * (ub - lb);
        v = fmax(v, lb + d);
        v = fmin(v, ub - d);
    } else if (hl) {
        v = fmax(v, lb + T(0.01) * fmax(fabs(lb), T(1)));
    } else if (hu) {
        v = fmin(v, ub - T(0.01) * fmax(fabs(ub), T(1)));
    }
    return v;
}

// W_SS nu = t for the m elements in L.se_e by Gauss-Jordan elimination in registers: lane i holds row i
// of W_SS (gathered with all its loads in flight) and t_i; pivot c's row reaches the other lanes by
// readlane, every other row eliminates column c, so at the end nu_i = t_i / (row i's pivot). Pivots get
// fast_finish's regularisation (below 1e-9 of W_ii: + 1e-6 W_ii), i.e. the same regularised system the
// oracle's Cholesky solves. The diagonal W_ii goes to L.wdg (the multiplier test). pd: every W_ii > 0.
template <typename T, int WSM, int EPL, class LdsT>
__device__ double solve_set_gj(const ClFastParams<T> &p, LdsT &L, const SlotView<EPL> &sv, int m, int lane, double t, bool &pd)
{
    double row[WSM];
    const int ei = lane < m ? L.se_e[lane] : 0, si = lane < m ? L.gi_slot[lane] : 0;
    if (NMPC_WCACHE && sv.wc_) {   // W_SS from the cached columns
#pragma unroll
        for (int j = 0; j < WSM; j++) row[j] = (j < m && lane < m) ? sv.wcv(L.gi_slot[j], si) : 0.0;
    } else {
#pragma unroll
    for (int j = 0; j < WSM; j++) {
        if constexpr (UNCOND_GATHER<EPL>) {   // clamped index, value masked after the load (no branch per load)
            const int jj = j < m ? j : 0;
            const double w = sv.w(p, L.se_e[jj], L.gi_slot[jj], ei, si);
            row[j] = (j < m && lane < m) ? w : 0.0;
        } else {
            row[j] = (j < m && lane < m) ? sv.w(p, L.se_e[j], L.gi_slot[j], ei, si) : 0.0;
        }
    }
    }
    double wii = 1.0;
#pragma unroll
    for (int j = 0; j < WSM; j++)
        if (j == lane) wii = row[j];
    if (lane < m) L.wdg[lane] = wii;
    pd = true;
    // every pivot unrolled: row[c] / row[j] and the readlane source are compile-time (a runtime pivot loop
    // indexes the register row dynamically: s_set_gpr_idx moves on every access). Columns j >= m are zero in
    // every row, so their updates leave them zero and need no guard
#pragma clang loop unroll(full)
    for (int c = 0; c < WSM; c++) {
        if (c < m) {
            const double d0 = bcast(row[c], c), wcc = bcast(wii, c), tc = bcast(t, c);
            pd = pd && wcc > 0.0;
            const double d = d0 > 1e-9 * wcc ? d0 : fmax(d0, 0.0) + 1e-6 * wcc;
            const double f = lane != c ? row[c] * rcp_nr(d) : 0.0;
#pragma clang loop unroll(full)
            for (int j = c + 1; j < WSM; j++) row[j] = fma(-f, bcast(row[j], c), row[j]);
            t = fma(-f, tc, t);
            if (lane == c) row[c] = d;
        }
    }
    double dd = 1.0;
#pragma unroll
    for (int j = 0; j < WSM; j++)
        if (j == lane) dd = row[j];
    return lane < m ? t / dd : 0.0;
}

// The symmetric sweep (in-place Gauss-Jordan inversion) of W_SS for the m set elements in L.se_e
// (positions 0..m-1): lane = row i + WSM * column group g holds CPL entries of its row in registers; pivot
// k's column reaches every lane through one LDS all-gather (each row's holder of column k writes it, every
// lane reads its row's entry, the pivot and its column group's entries), then the rank-1 update
// a_ij -= a_ik a_kj / d, row and column k scaled by 1 / d, a_kk = -1 / d. After m pivots a = -W_SS^-1.
// The pivot d (the Schur complement of the leading block, i.e. the Cholesky pivot squared) gets
// fast_finish's regularisation: below 1e-9 W_kk it becomes max(d, 0) + 1e-6 W_kk, so the result is the
// inverse of the same regularised system the Cholesky / Gauss-Jordan paths solve. H = W_SS^-1 goes to
// L.hm (zero outside the m x m block), W_ii to L.wdg. false: a non-positive W_ii.
// The sweep's gather and result (the lane's register row a[CPL]: lane = row i + WSM * column group g)
template <typename T, int WSM, int EPL, class LdsT>
__device__ __forceinline__ void sweep_gather(const ClFastParams<T> &p, LdsT &L, const SlotView<EPL> &sv, int m, int i, int g,
                                             double (&a)[HGeom<WSM>::CPL])
{
    constexpr int CPL = HGeom<WSM>::CPL;
    const int ei = i < m ? L.se_e[i] : 0, si = i < m ? L.gi_slot[i] : 0;
    if (NMPC_WCACHE && sv.wc_) {   // from the cached columns
#pragma unroll
        for (int q = 0; q < CPL; q++) {
            const int j = g * CPL + q;
            a[q] = (i < m && j < m) ? sv.wcv(L.gi_slot[j], si) : 0.0;
        }
    } else {
#pragma unroll
    for (int q = 0; q < CPL; q++) {
        const int j = g * CPL + q;
        if constexpr (UNCOND_GATHER<EPL>) {
            const int jj = j < m ? j : 0;
            const double w = sv.w(p, L.se_e[jj], L.gi_slot[jj], ei, si);
            a[q] = (i < m && j < m) ? w : 0.0;
        } else {
            a[q] = (i < m && j < m) ? sv.w(p, L.se_e[j], L.gi_slot[j], ei, si) : 0.0;
        }
    }
    }
#pragma unroll
    for (int q = 0; q < CPL; q++)
        if (g * CPL + q == i && i < m) L.wdg[i] = a[q];
    CLF_SYNC();
}
template <int WSM, class LdsT>
__device__ __forceinline__ void sweep_store(LdsT &L, int i, int g, const double (&a)[HGeom<WSM>::CPL])
{
    constexpr int CPL = HGeom<WSM>::CPL;
#pragma unroll
    for (int q = 0; q < CPL; q++) L.hm[i][g * CPL + q] = -a[q];
    CLF_SYNC();
}

// The symmetric sweep for sets of up to 16, inlined into its caller: a run-time pivot loop over the lane's CPL
// register entries (the index a register move).
template <typename T, int WSM, int EPL, class LdsT>
__device__ __forceinline__ bool sweep_inverse_rt(const ClFastParams<T> &p, LdsT &L, const SlotView<EPL> &sv, int m, int lane)
{
    constexpr int CPL = HGeom<WSM>::CPL;
    const int i = lane % WSM, g = lane / WSM;
    double a[CPL];
    sweep_gather<T, WSM>(p, L, sv, m, i, g, a);
    bool pd = true;
#pragma unroll
    for (int k = 0; k < WSM; k++) {
        if (k >= m) break;
        if (g == k / CPL) L.vb1[i] = a[k % CPL];
        CLF_SYNC();
        const double ci = L.vb1[i], d0 = L.vb1[k], wkk = L.wdg[k];
        pd = pd && wkk > 0.0;
        const double d = d0 > 1e-9 * wkk ? d0 : fmax(d0, 0.0) + 1e-6 * wkk;
        const double f = rcp_nr(d);
        // rows i != k: a_ij - c_i f c_j; row k (a_kj = c_j by symmetry): a_kj - (1 - f) c_j = c_j f
        const double cif = i == k ? 1.0 - f : ci * f;
#pragma unroll
        for (int q = 0; q < CPL; q++) a[q] = fma(-cif, L.vb1[g * CPL + q], a[q]);
        if (g == k / CPL) a[k % CPL] = i == k ? -f : ci * f;
    }
    sweep_store<WSM>(L, i, g, a);
    return pd;
}

// Sets of 17..32 (the force shape, WSM 32) keep the form the compiler outlines: its run-time pivot loop keeps a[]
// in scratch memory, and measured faster there than the inlined form, which costs the force kernels registers
// (-10 % at B = 1024 and 8192, profiles/r6n_sweep_inline_ab.jsonl). Sets of up to 16 (GI's H for quad13 / jerk)
// take sweep_inverse_rt, inlined (quad13 +6.8 %, same A/B).
template <typename T, int WSM, int EPL, class LdsT>
__device__ bool sweep_inverse(const ClFastParams<T> &p, LdsT &L, const SlotView<EPL> &sv, int m, int lane)
{
    if constexpr (WSM <= 16) return sweep_inverse_rt<T, WSM>(p, L, sv, m, lane);   // sets of up to 16: inlined
    constexpr int CPL = HGeom<WSM>::CPL;
    const int i = lane % WSM, g = lane / WSM;
    double a[CPL];
    const int ei = i < m ? L.se_e[i] : 0, si = i < m ? L.gi_slot[i] : 0;
#pragma unroll
    for (int q = 0; q < CPL; q++) {
        const int j = g * CPL + q;
        if constexpr (UNCOND_GATHER<EPL>) {
            const int jj = j < m ? j : 0;
            const double w = sv.w(p, L.se_e[jj], L.gi_slot[jj], ei, si);
            a[q] = (i < m && j < m) ? w : 0.0;
        } else {
            a[q] = (i < m && j < m) ? sv.w(p, L.se_e[j], L.gi_slot[j], ei, si) : 0.0;
        }
    }
#pragma unroll
    for (int q = 0; q < CPL; q++)
        if (g * CPL + q == i && i < m) L.wdg[i] = a[q];
    CLF_SYNC();
    bool pd = true;
    if constexpr (LdsT::sweep2) {
        // pivots k = k0 + kk with kk unrolled, so a[kk] is a compile-time register; the runtime loop below
        // indexes the register row dynamically and copies it per pivot. Same arithmetic, same order. Measured
        // (force B = 1024, one wavefront per SIMD) +3 % over the runtime loop; its register use costs the
        // second wavefront per SIMD at B = 8192 (-22 %), hence only in the CLF_ONE variant
        for (int k0 = 0; k0 < m; k0 += CPL) {
            const bool own = g == k0 / CPL;   // this lane's registers hold the group's columns
#pragma clang loop unroll(full)
            for (int kk = 0; kk < CPL; kk++) {
                const int k = k0 + kk;
                if (k < m) {
                    if (own) L.vb1[i] = a[kk];
                    CLF_SYNC();
                    const double ci = L.vb1[i], d0 = L.vb1[k], wkk = L.wdg[k];
                    pd = pd && wkk > 0.0;
                    const double d = d0 > 1e-9 * wkk ? d0 : fmax(d0, 0.0) + 1e-6 * wkk;
                    const double f = rcp_nr(d);
                    const double cif = i == k ? 1.0 - f : ci * f;
#pragma unroll
                    for (int q = 0; q < CPL; q++) a[q] = fma(-cif, L.vb1[g * CPL + q], a[q]);
                    if (own) a[kk] = i == k ? -f : ci * f;
                }
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < WSM; k++) {
            if (k >= m) break;
            if (g == k / CPL) L.vb1[i] = a[k % CPL];
            CLF_SYNC();
            const double ci = L.vb1[i], d0 = L.vb1[k], wkk = L.wdg[k];
            pd = pd && wkk > 0.0;
            const double d = d0 > 1e-9 * wkk ? d0 : fmax(d0, 0.0) + 1e-6 * wkk;
            const double f = rcp_nr(d);
            // rows i != k: a_ij - c_i f c_j; row k (a_kj = c_j by symmetry): a_kj - (1 - f) c_j = c_j f
            const double cif = i == k ? 1.0 - f : ci * f;
#pragma unroll
            for (int q = 0; q < CPL; q++) a[q] = fma(-cif, L.vb1[g * CPL + q], a[q]);
            if (g == k / CPL) a[k % CPL] = i == k ? -f : ci * f;
        }
    }
#pragma unroll
    for (int q = 0; q < CPL; q++) L.hm[i][g * CPL + q] = -a[q];
    CLF_SYNC();
    return pd;
}

// y_i = sum_j H_ij x_j with x all-gathered in LDS (x_j = 0 outside the set): the row's CPL-column
// partial sums, reduced over the row's lanes; y_i on every lane of row i
template <int WSM, class LdsT>
__device__ double h_matvec(const LdsT &L, const double *x, int lane)
{
    constexpr int CPL = HGeom<WSM>::CPL;
    const int i = lane % WSM, g = lane / WSM;
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < CPL; q++) s = fma(L.hm[i][g * CPL + q], x[g * CPL + q], s);
    if (WSM == 16) s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    return s;
}

// x . y over the set positions for two all-gathered vectors (every lane gets the sum)
template <int WSM>
__device__ double h_dot(const double *x, const double *y, int lane)
{
    constexpr int CPL = HGeom<WSM>::CPL;
    const int g = lane / WSM;
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < CPL; q++) s = fma(x[g * CPL + q], y[g * CPL + q], s);
    if (WSM == 16) s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    return s;
}

// bordering: position q (free: row and column q of H zero) joins with r = H W[S, p] all-gathered in
// L.vb2 (r_q = 0) and Schur complement theta = W_pp - W[S, p] . r > 0: H += r r^T / theta,
// H_iq = H_qi = -r_i / theta, H_qq = 1 / theta
template <int WSM, class LdsT>
__device__ void h_add(LdsT &L, int q, double theta, int lane)
{
    constexpr int CPL = HGeom<WSM>::CPL;
    const int i = lane % WSM, g = lane / WSM;
    const double it = rcp_nr(theta), rit = L.vb2[i] * it;
#pragma unroll
    for (int c = 0; c < CPL; c++) {
        const int j = g * CPL + c;
        const double rj = L.vb2[j];
        double v = fma(rit, rj, L.hm[i][j]);
        if (j == q) v = i == q ? it : -rit;
        if (i == q) v = j == q ? it : -rj * it;
        L.hm[i][j] = v;
    }
    CLF_SYNC();
}

// position k leaves: H_ij -= H_ik H_kj / H_kk (the inverse of the set without k), row and column k zeroed.
// One wavefront: every lane's reads of a column group precede the writes to it (LDS program order)
template <int WSM, class LdsT>
__device__ void h_drop(LdsT &L, int k, int lane)
{
    constexpr int CPL = HGeom<WSM>::CPL;
    const int i = lane % WSM, g = lane / WSM;
    const double f = L.hm[i][k] * rcp_nr(L.hm[k][k]);
#pragma unroll
    for (int c = 0; c < CPL; c++) {
        const int j = g * CPL + c;
        const double v = fma(-f, L.hm[k][j], L.hm[i][j]);
        L.hm[i][j] = (i == k || j == k) ? 0.0 : v;
    }
    CLF_SYNC();
}

// the active positions (bitmask am) as a compacted list for w_combo_slots: elements to L.cl_e, the
// coefficients (lane i < WSM holds position i's) to L.cl_c; returns the count
template <int WSM, class LdsT>
__device__ int compact_set(LdsT &L, unsigned am, int lane, double coef)
{
    const bool act = lane < WSM && ((am >> lane) & 1u);
    const unsigned long long b = __ballot(act);
    if (act) {
        const int to = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(b >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)b, 0u));
        L.cl_e[to] = L.se_e[lane];
        L.cl_s[to] = L.gi_slot[lane];
        L.cl_c[to] = coef;
    }
    CLF_SYNC();
    return __popcll(b);
}

// acc[j] += sum_i W[e_i][e_j] c_i at every slot j of the lane (padding slots untouched) for the m
// elements el (LDS) with coefficients cf (LDS): the set in batches of QB, each batch's loads for all the
// lane's slots in flight together (one memory latency per batch, not one per slot and batch); per slot
// the sum runs in list order, in the accumulator's precision A (fp64 for both storage precisions: the
// terms of an ill-conditioned set cancel)
template <typename T, int EPL, typename A>
__device__ void w_combo_slots(const ClFastParams<T> &p, const int *el, const int *sl, const SlotView<EPL> sv,
                              const double *cf, int m, A (&acc)[EPL])
{
#ifndef NMPC_QB34
#define NMPC_QB34 4
#endif
    constexpr int QB = EPL <= 2 ? 8 : (EPL <= 4 ? NMPC_QB34 : 2);
    int e[EPL];
#pragma unroll
    for (int j = 0; j < EPL; j++) e[j] = sv.e(j);
    if (NMPC_WCACHE && sv.wc_) {   // the cached columns: LDS reads, same order of terms
        for (int i = 0; i < m; i++) {
            const A c = (A)cf[i];
            const double *col = sv.wcol_ + sv.wcolof_[sl[i]] * sv.wcld_;
#pragma unroll
            for (int j = 0; j < EPL; j++)
                if (e[j] >= 0) acc[j] = fma((A)col[j * 64 + sv.lane], c, acc[j]);
        }
        return;
    }
    for (int i0 = 0; i0 < m; i0 += QB) {
        double w[QB][EPL];
#pragma unroll
        for (int q = 0; q < QB; q++) {
            const int row = i0 + q < m ? el[i0 + q] : 0, rs = i0 + q < m ? sl[i0 + q] : 0;
#pragma unroll
            for (int j = 0; j < EPL; j++) {
                if constexpr (UNCOND_GATHER<EPL>) {
                    const double wl = sv.w(p, row, rs, e[j] >= 0 ? e[j] : 0, e[j] >= 0 ? j * 64 + sv.lane : 0);
                    w[q][j] = (i0 + q < m && e[j] >= 0) ? wl : 0.0;
                } else {
                    w[q][j] = (i0 + q < m && e[j] >= 0) ? sv.w(p, row, rs, e[j], j * 64 + sv.lane) : 0.0;
                }
            }
        }
#pragma unroll
        for (int q = 0; q < QB; q++)
            if (i0 + q < m) {
                const A c = (A)cf[i0 + q];
#pragma unroll
                for (int j = 0; j < EPL; j++)
                    if (e[j] >= 0) acc[j] = fma((A)w[q][j], c, acc[j]);
            }
    }
}

// the set of flag bits wf in LDS in slot order (= element order): element, sign (-1 lower, 1 upper),
// b - z_0, slot; pos[j] = the held slot's position in the set. Returns the set size (not written when
// larger than WSM).
template <typename T, int EPL, int WSM, class LdsT>
__device__ int load_set(LdsT &L, const SlotView<EPL> sv, int lane, unsigned wf, const T (&z0)[EPL], int (&pos)[EPL])
{
    unsigned long long bal[EPL];
    int m = 0;
#pragma unroll
    for (int j = 0; j < EPL; j++) {
        bal[j] = __ballot(((wf >> (2 * j)) & 3u) != 0);
        m += __popcll(bal[j]);
    }
    int base = 0;
#pragma unroll
    for (int j = 0; j < EPL; j++) {
        const unsigned f = (wf >> (2 * j)) & 3u;
        pos[j] = -1;
        if (f && m <= WSM) {
            pos[j] = base + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bal[j] >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal[j], 0u));
            L.se_e[pos[j]] = sv.e(j);
            L.se_s[pos[j]] = f == 1u ? -1 : 1;
            L.se_t[pos[j]] = (f == 1u ? sv.lb(j) : sv.ub(j)) - (double)z0[j];   // fp64: b_S is met to 1e-9
            L.gi_slot[pos[j]] = j * 64 + lane;
        }
        base += __popcll(bal[j]);
    }
    CLF_SYNC();
    return m;
}

// Primal-dual active-set steps on W (oracle/c/riccati_ipm.c fast_finish): wf holds the set (warm
// start, or empty: the first set from z_0's violations — the violated inputs and each state
// component's most violated stage), z z_0 at the lane's slots. Each round solves W_SS nu = b_S - z_0,S: W_SS gathered
// into LDS over 8 x 8 lane tiles, a right-looking Cholesky (column scaling by lanes, trailing update
// over lane tiles), the two triangular solves with the right-hand side lane-distributed (lane i holds
// row i, the pivot broadcast by readlane); then z = z_0 + W[:, S] nu at the lane's slots, accepted
// when the held bounds are met (1e-9), no other bound is violated (1e-13) and every multiplier has its
// sign (displacement nu_i W_ii to 1e-10 (1 + |b - z_0|)); otherwise removals and additions as the
// finish's PDAS rule. An emptied set restarts from z_0 (one round). Result: ok | m << 8 | steps << 16
// (z in L.zb, the set in L.se_*); not ok: a set larger than WSM, W_SS not positive definite, or no
// acceptance in polish_steps rounds. z: z_0 in, the solution out (when accepted); wf: the set the rounds start from
// in, the set they reached out (the dual fallback starts from it)
template <int WSM, int EPL>
using WCacheOf = WCache<WSM + 1, EPL * 64>;

template <typename T, int NX, int NU, int EPL, int WSM, class LdsT>
__device__ int wsteps_run(const ClFastParams<T> &p, LdsT &L, const SlotView<EPL> sv, int lane, T (&z)[EPL], unsigned &wf,
                          int rounds, WCacheOf<WSM, EPL> *wc = nullptr)
{
    constexpr int NZ = NX + NU;
    static_assert(WSM <= 64, "active sets are lane-distributed");
    const int ne = p.ne;
    int wsteps = 0;
    T z0[EPL];
#pragma unroll
    for (int j = 0; j < EPL; j++) z0[j] = z[j];
    auto comp = [&](int j) {   // the slot's component r (or -1: padding slot)
        const int e = sv.e(j);
        return e >= 0 ? e % NZ : -1;
    };
    auto done = [&](int m) { return 1 | (m << 8) | (wsteps << 16); };
    // per state component: the most violated slot (argmax by LDS atomics, ties to the first stage)
    auto argmax_states = [&](const double (&v)[EPL]) {
        if (lane < NZ) {
            L.vmax[lane] = 0ull;
            L.vslot[lane] = 0x7fffffff;
        }
        CLF_SYNC();
#pragma unroll
        for (int j = 0; j < EPL; j++) {
            const int r = comp(j);
            if (r >= 0 && r < NX && v[j] > 0.0) atomicMax(&L.vmax[r], __builtin_bit_cast(unsigned long long, v[j]));
        }
        CLF_SYNC();
#pragma unroll
        for (int j = 0; j < EPL; j++) {
            const int r = comp(j);
            if (r >= 0 && r < NX && v[j] > 0.0 && __builtin_bit_cast(unsigned long long, v[j]) == L.vmax[r])
                atomicMin(&L.vslot[r], sv.e(j));
        }
        CLF_SYNC();
    };
    auto add_states = [&](const double (&v)[EPL], unsigned sgn, unsigned &w) {
        // no violated state bound anywhere: nothing to add (the argmax's LDS atomics and three wave syncs
        // skipped; the slowest quad13 instances spend a third of a PDAS round there)
        bool sv_ = false;
#pragma unroll
        for (int j = 0; j < EPL; j++) {
            const int r = comp(j);
            sv_ |= r >= 0 && r < NX && v[j] > 0.0;
        }
        if (!__any(sv_)) return;
        argmax_states(v);
#pragma unroll
        for (int j = 0; j < EPL; j++) {
            const int r = comp(j);
            if (r >= 0 && r < NX && v[j] > 0.0 && L.vslot[r] == sv.e(j)) w |= ((sgn >> (2 * j)) & 3u) << (2 * j);
        }
        CLF_SYNC();
    };
    for (int ws = 0, first = 1; ws < rounds; first = 0) {
        CLF_T(tm0);
        int m = 0;
#pragma unroll
        for (int j = 0; j < EPL; j++) m += __popcll(__ballot(((wf >> (2 * j)) & 3u) != 0));
        CLF_TADD(L, 22, tm0);
        if (m == 0) {
            // no bound held: the iterate is z_0 — accepted if feasible, else the set from its violations
            if (!first) ws++;
            bool bad = false;
            double v[EPL];
            unsigned sgn = 0;
#pragma unroll
            for (int j = 0; j < EPL; j++) {
                const double zj = (double)z0[j];
                const bool lo = zj < sv.lo(j), hi = zj > sv.hi(j);
                bad |= lo || hi || !isfinite(zj);
                v[j] = lo ? sv.lb(j) - zj : (hi ? zj - sv.ub(j) : 0.0);
                sgn |= (lo ? 1u : (hi ? 2u : 0u)) << (2 * j);
                if (comp(j) >= NX && (lo || hi)) wf |= (lo ? 1u : 2u) << (2 * j);   // inputs join at once
            }
            if (!__any(bad)) {
#pragma unroll
                for (int j = 0; j < EPL; j++) z[j] = z0[j];   // (a restart: z holds the last round's trial)
                return done(0);
            }
            add_states(v, sgn, wf);
            continue;
        }
        if (m > WSM) break;
        int pos[EPL];
        CLF_T(tl_set);
        load_set<T, EPL, WSM>(L, sv, lane, wf, z0, pos);
        if (NMPC_WCACHE && sv.wc_) wc_fill<T, EPL>(p, *wc, sv, lane < m ? L.gi_slot[lane] : 0, m, 0u, lane);   // the set's columns
        CLF_TADD(L, 18, tl_set);
        // nu = W_SS^-1 (b - z_0)_S, lane i holding row i: Gauss-Jordan in registers for sets of up to 16
        // (one lane per row) and 32 (two lanes per row: register rows of 32 would go to scratch), the LDS
        // Cholesky beyond
        bool pd = true;
        double y;
        CLF_T(ts0);
        if (WSM <= 16 || m <= 16) {
            y = solve_set_gj<T, (WSM < 16 ? WSM : 16)>(p, L, sv, m, lane, lane < m ? L.se_t[lane] : 0.0, pd);
        } else {
            // sets of 17..WSM: the sweep's explicit inverse, nu = H (b - z_0)_S
            pd = sweep_inverse<T, WSM>(p, L, sv, m, lane);
            if (lane < WSM) L.vb2[lane] = lane < m ? L.se_t[lane] : 0.0;
            CLF_SYNC();
            y = h_matvec<WSM>(L, L.vb2, lane);
            y = lane < m ? y : 0.0;
        }
        CLF_TADD(L, 3, ts0);
        CLF_TCNT(L, 10, 1);
        if (!pd) break;
        CLF_T(tmu0);
        // multiplier signs as displacements nu_i W_ii (lower: >= 0, upper: <= 0) to 1e-10 (1 + |b - z_0|)
        bool rmv = false;
        if (lane < m) {
            L.se_nu[lane] = y;
            const double tol = 1e-10 * (1.0 + fabs(L.se_t[lane])), dsp = y * L.wdg[lane];
            const int sg = L.se_s[lane];
            rmv = (sg < 0 && dsp < -tol) || (sg > 0 && dsp > tol) || !isfinite(y);
        }
        const unsigned long long remm = __ballot(rmv);
        CLF_SYNC();
        CLF_TADD(L, 21, tmu0);
        const int round = ws++;
        wsteps++;
        const int nrem = __popcll(remm);
        const bool addok = round == 0 || nrem == 0;
        bool bad = nrem > 0;
        double v[EPL];
        unsigned sgn = 0, nwf = wf;
        // z = z_0 + W[:, S] nu and its checks in fp64 (T = float: the stored z_0 and W widened)
        double zd[EPL];
#pragma unroll
        for (int j = 0; j < EPL; j++) zd[j] = (double)z0[j];
        CLF_T(tc0);
        w_combo_slots<T, EPL>(p, L.se_e, L.gi_slot, sv, L.se_nu, m, zd);
        CLF_TADD(L, 4, tc0);
        CLF_T(tk0);
#pragma unroll
        for (int j = 0; j < EPL; j++) {
            v[j] = 0.0;
            const int e = sv.e(j);
            if (e < 0) {
                z[j] = z0[j];
                continue;
            }
            double zz = zd[j];
            const unsigned f = (wf >> (2 * j)) & 3u;
            if (f) {
                const double bb = f == 1u ? sv.lb(j) : sv.ub(j);
                bad |= !(fabs(zz - bb) <= 1e-9 * (1.0 + fabs(bb)));
                zz = bb;
                if ((remm >> pos[j]) & 1ull) nwf &= ~(3u << (2 * j));
            } else {
                const bool lo = zz < sv.lo(j), hi = zz > sv.hi(j);
                bad |= lo || hi || !isfinite(zz);
                v[j] = lo ? sv.lb(j) - zz : (hi ? zz - sv.ub(j) : 0.0);
                sgn |= (lo ? 1u : (hi ? 2u : 0u)) << (2 * j);
                if (e % NZ >= NX && (lo || hi)) nwf |= (lo ? 1u : 2u) << (2 * j);   // inputs join at once
            }
            z[j] = (T)zz;
        }
        CLF_TADD(L, 23, tk0);
        if (!__any(bad)) {
            CLF_TADD(L, 19, tk0);
            return done(m);
        }
        CLF_T(tad0);
        if (addok) add_states(v, sgn, nwf);
        CLF_TADD(L, 20, tad0);
        wf = nwf;
        CLF_SYNC();
        CLF_TADD(L, 19, tk0);
    }
#pragma unroll
    for (int j = 0; j < EPL; j++) z[j] = z0[j];   // not accepted: z_0 back to the caller
    return wsteps << 16;
}

// The fast path's fallback when the PDAS rounds do not settle — degenerate sets, cycling
// (oracle/c/riccati_ipm.c gi_set): the Goldfarb-Idnani dual active-set method on W, which converges for
// any strictly convex QP. Bounds are constraints n_i^T z >= b_i, n_i = +e (lower) / -e (upper), sign
// sg_i. From z = z_0 and an empty set the most violated inactive bound p enters (ties: the first slot):
// with a = W[S, p] and H = W_SS^-1 (L.hm, kept up to date by bordering / downdating instead of being
// refactored), r = H a, theta = W_pp - a . r (the curvature along p), the multipliers' rate
// r_i' = sg_p sg_i r_i, dz = sg_p (W[:, p] - W[:, S] r); the full step t2 = -sg_p (z_p - b_p) / theta
// makes p active (h_add), the partial step t1 = min u_i / r_i' (r_i' > 0; ties: the earliest entry) drops
// the bound whose multiplier reaches zero first (h_drop); z += t dz, u -= t r', u_p += t. theta ~ 0 (p
// dependent on the set) only drops; no blocking bound then: infeasible. Set positions stay fixed (am:
// the occupied ones, se_ord: entry order); multipliers on lanes i < WSM. true: no inactive bound violated
// beyond 1e-13, the set in wf (per-lane flag bits), for wsteps_run to solve exactly and check. z_0 is not
// modified.
template <typename T, int NX, int NU, int EPL, int WSM, class LdsT>
__device__ bool gi_set(const ClFastParams<T> &p, LdsT &L, const SlotView<EPL> sv, int lane, const T (&z0)[EPL],
                       unsigned w0, unsigned &wf, int &iters, WCacheOf<WSM, EPL> *wc = nullptr)
{
    constexpr int CPL = HGeom<WSM>::CPL;
    const int ne = p.ne, hi_ = lane % WSM, hg = lane / WSM;
    double z[EPL];   // the iterate in fp64 for both storage precisions
#pragma unroll
    for (int j = 0; j < EPL; j++) z[j] = (double)z0[j];
    unsigned am = 0;                      // occupied set positions (wave-uniform)
    int ps = -1, sp = 0, ep = 0, ord = 0; // the entering bound: slot, sign (+1 lower, -1 upper), element
    double u = 0.0, up = 0.0;             // lane i < WSM: the multiplier u_i of position i; up: the entering bound's
    const bool pl = lane < WSM;
    // warm start: the set the PDAS rounds started from (w0), made dual feasible — its equality-constrained
    // solution nu = W_SS^-1 (b - z_0)_S, u_i = sg_i nu_i; the negative ones leave (downdates), re-solved
    // until none is left — and z = z_0 + W[:, S] nu
    {
        int pos[EPL];
        int m = load_set<T, EPL, WSM>(L, sv, lane, w0, z0, pos);
        wf = m <= WSM ? w0 : 0u;
        if (m > WSM) m = 0;
        if (m > 0) {
            if (NMPC_WCACHE && sv.wc_) wc_fill<T, EPL>(p, *wc, sv, lane < m ? L.gi_slot[lane] : 0, m, 0u, lane);
            sweep_inverse<T, WSM>(p, L, sv, m, lane);
            am = m == 32 ? 0xffffffffu : ((1u << m) - 1u);
        } else {
#pragma unroll
            for (int c = 0; c < CPL; c++) L.hm[hi_][hg * CPL + c] = 0.0;
        }
        if (pl) L.se_ord[lane] = lane;
        ord = m;
        double nu = 0.0;
        while (am) {
            if (pl) L.vb2[lane] = ((am >> lane) & 1u) ? L.se_t[lane] : 0.0;
            CLF_SYNC();
            nu = h_matvec<WSM>(L, L.vb2, lane);
            u = (pl && ((am >> lane) & 1u)) ? (double)(-L.se_s[lane]) * nu : 0.0;
            const unsigned long long neg = __ballot(pl && ((am >> lane) & 1u) && u < 0.0);
            if (!neg) break;
            for (unsigned long long d_ = neg; d_; d_ &= d_ - 1) {
                const int k = (int)__builtin_ctzll(d_);
                const int sk = L.gi_slot[k];
                if (lane == (sk & 63)) wf &= ~(3u << (2 * (sk >> 6)));
                h_drop<WSM>(L, k, lane);
                am &= ~(1u << k);
            }
        }
        if (am) {
            const int mc = compact_set<WSM>(L, am, lane, nu);
            w_combo_slots<T, EPL>(p, L.cl_e, L.cl_s, sv, L.cl_c, mc, z);
            CLF_SYNC();
        }
    }
    const int cap = 3 * WSM + 16;
    int it = 0;
    for (; it < cap; it++) {
        CLF_T(tg_sel);
        if (ps < 0) {
            double v[EPL], vm = 0.0;
#pragma unroll
            for (int j = 0; j < EPL; j++) {
                const bool held = ((wf >> (2 * j)) & 3u) != 0;
                const bool lo = !held && z[j] < sv.lo(j), hi = !held && z[j] > sv.hi(j);
                v[j] = lo ? sv.lb(j) - z[j] : (hi ? z[j] - sv.ub(j) : 0.0);
                vm = fmax(vm, v[j]);
            }
            vm = wave_max(vm);
            if (!(vm > 0.0)) break;
#pragma unroll
            for (int j = EPL - 1; j >= 0; j--) {
                const unsigned long long bal = __ballot(v[j] == vm);
                if (bal) ps = j * 64 + (int)__builtin_ctzll(bal);
            }
            ep = sv.e_[ps];
            up = 0.0;
        }
        CLF_TADD(L, 14, tg_sel);
        CLF_T(tg_sol);
        // a = W[S, p] (occupied positions) and W_pp, loads issued together
        const bool occ = pl && ((am >> lane) & 1u);
        if (NMPC_WCACHE && sv.wc_) {   // the entering bound's column, keeping the set's
            const unsigned keep = occ ? 1u << wc->colof[L.gi_slot[lane]] : 0u;
            wc_fill<T, EPL>(p, *wc, sv, ps, 1, keep, lane);
        }
        double ai;
        double wpj[EPL];   // (UNCOND_GATHER) W[p, slots] of the step direction, issued with a
        if constexpr (UNCOND_GATHER<EPL>) {
            const double aw = sv.w(p, occ ? L.se_e[lane] : ep, occ ? L.gi_slot[lane] : ps, ep, ps);
            ai = occ ? aw : 0.0;
#pragma unroll
            for (int j = 0; j < EPL; j++) {
                const int e = sv.e(j);
                wpj[j] = sv.w(p, ep, ps, e >= 0 ? e : 0, e >= 0 ? j * 64 + lane : 0);
            }
        } else if (NMPC_WCACHE && sv.wc_) {
            ai = occ ? sv.wcv(ps, L.gi_slot[lane]) : 0.0;
        } else {
            ai = occ ? sv.w(p, L.se_e[lane], L.gi_slot[lane], ep, ps) : 0.0;
        }
        const double wpp = (NMPC_WCACHE && sv.wc_) ? sv.wcv(ps, ps) : sv.w(p, ep, ps, ep, ps);
        double zc = 0.0;
#pragma unroll
        for (int j = 0; j < EPL; j++)
            if (j == (ps >> 6)) zc = z[j];
        const double zp = bcast(zc, ps & 63);
        if (up == 0.0) sp = zp < sv.lo_[ps] ? 1 : -1;   // entering: the violated side
        const double bp = sp > 0 ? sv.lb_[ps] : sv.ub_[ps];
        if (pl) L.vb1[lane] = ai;
        CLF_SYNC();
        const double r_ = h_matvec<WSM>(L, L.vb1, lane);   // r = H a
        if (pl) L.vb2[lane] = r_;
        CLF_SYNC();
        const double theta = wpp - h_dot<WSM>(L.vb1, L.vb2, lane);
        const double ri = occ ? (double)sp * (double)(-L.se_s[lane]) * r_ : 0.0;
        const double q = (occ && ri > 0.0) ? u / ri : INFINITY;
        const double t1 = wave_min(q);
        const double t2 = theta > 1e-12 * wpp ? -(double)sp * (zp - bp) / theta : INFINITY;
        if (t1 == INFINITY && t2 == INFINITY) break;   // infeasible
        const bool full = t2 <= t1;
        const double t = full ? t2 : t1;
        CLF_TADD(L, 15, tg_sol);
        CLF_T(tg_cmb);
        if (t2 < INFINITY) {
            const int mc = compact_set<WSM>(L, am, lane, r_);
            double comb[EPL];
#pragma unroll
            for (int j = 0; j < EPL; j++) comb[j] = 0.0;
            w_combo_slots<T, EPL>(p, L.cl_e, L.cl_s, sv, L.cl_c, mc, comb);
#pragma unroll
            for (int j = 0; j < EPL; j++) {
                const int e = sv.e(j);
                if (e >= 0) {
                    double wj;
                    if constexpr (UNCOND_GATHER<EPL>) wj = wpj[j];
                    else wj = (NMPC_WCACHE && sv.wc_) ? sv.wcv(ps, j * 64 + lane) : sv.w(p, ep, ps, e, j * 64 + lane);
                    z[j] = fma(t, (double)sp * (wj - comb[j]), z[j]);
                }
            }
            CLF_SYNC();
        }
        CLF_TADD(L, 16, tg_cmb);
        CLF_T(tg_upd);
        if (occ) u = fma(-t, ri, u);
        up += t;
        if (full) {
            if (__popc(am) >= WSM) break;
            const int qn = (int)__builtin_ctz(~am);   // the lowest free position
            h_add<WSM>(L, qn, theta, lane);
            if (lane == qn) {
                L.se_e[qn] = ep;
                L.se_s[qn] = sp > 0 ? -1 : 1;
                L.gi_slot[qn] = ps;
                L.se_ord[qn] = ord;
                u = up;
            }
            ord++;
            am |= 1u << qn;
            if (lane == (ps & 63)) wf |= (sp > 0 ? 1u : 2u) << (2 * (ps >> 6));
            ps = -1;
            CLF_SYNC();
        } else {
            // the blocking bound (ties: the earliest entry, as the oracle's list order)
            const bool tie = occ && ri > 0.0 && q == t1;
            const unsigned long long kb = __ballot(tie);
            int kk = (int)__builtin_ctzll(kb);
            if (__popcll(kb) > 1) {
                const int o = tie ? L.se_ord[lane] : 0x7fffffff;
                int om = o;
#pragma unroll
                for (int s_ = 32; s_ > 0; s_ >>= 1) om = min(om, __shfl_xor(om, s_));
                kk = (int)__builtin_ctzll(__ballot(tie && o == om));
            }
            const int sk = L.gi_slot[kk];
            if (lane == (sk & 63)) wf &= ~(3u << (2 * (sk >> 6)));
            h_drop<WSM>(L, kk, lane);
            am &= ~(1u << kk);
        }
        CLF_TADD(L, 17, tg_upd);
    }
    iters = it;
    return ps < 0 && it < cap;
}

// interval certificate (oracle/c/riccati_ipm.c infeasible_stage): lane i < NX carries state i of
// X_k in midpoint / radius form, X_{k+1} = hull([A B] X_k x U + c) meets the state box of stage
// k + 1; an empty intersection proves the QP infeasible. x_0 in L.xs; [A B], c from the workgroup's
// LDS copy (the model's own values: zero outside its structure); the stage exchange by readlane.
template <typename T, int NX, int NU, class LdsT>
__device__ bool certificate_infeasible(const ClFastParams<T> &p, LdsT &L, const double *abl, const double *cl, int lane)
{
    constexpr int NZ = NX + NU;
    const int i = lane < NX ? lane : 0;
    double m = lane < NX ? L.xs[lane] : 0.0, r = 0.0;
    double a[NX];
#pragma unroll
    for (int j = 0; j < NX; j++) a[j] = abl[i * NZ + j];
    // the stage-invariant operands ahead of the stage chain (the same arithmetic, in the same order): the
    // input box's midpoint and radius terms, the state bounds of the inner stages and of the last one
    double bu[NU], bm[NU], br[NU];
#pragma unroll
    for (int j = 0; j < NU; j++) {
        const double l = p.lbnd[NX + j], h = p.ubnd[NX + j];
        const bool bb = has_b(l) && has_b(h);
        bu[j] = abl[i * NZ + NX + j];
        bm[j] = bb ? 0.5 * (l + h) : 0.0;
        br[j] = bb ? 0.5 * (h - l) : (double)INFINITY;
    }
    const double lb1 = p.lbnd[NZ + i], ub1 = p.ubnd[NZ + i], lb2 = p.lbnd[2 * NZ + i], ub2 = p.ubnd[2 * NZ + i];
    // the skipped zero terms only matter against an infinite radius (0 x inf): with every radius finite,
    // fma(0, r, tr) = tr, so the chains run without the per-term selects — the same bits, half the chain
    // (a select pair per term doubled the radius chain's latency); the wave-uniform test per stage
    bool binf = false;
#pragma unroll
    for (int j = 0; j < NU; j++) binf |= !(br[j] <= DBL_MAX);
    bool rinf = false;   // (r = 0 at stage 0)
    for (int k = 0; k < p.N; k++) {
        double s = cl[i], tr = 0.0;
        if (!rinf) {
#pragma unroll
            for (int j = 0; j < NX; j++) {
                const double mj = bcast(m, j), rj = bcast(r, j);
                s = fma(a[j], mj, s);
                tr = fma(fabs(a[j]), rj, tr);
            }
        } else {
#pragma unroll
            for (int j = 0; j < NX; j++) {
                const double mj = bcast(m, j), rj = bcast(r, j);
                s = fma(a[j], mj, s);
                if (a[j] != 0.0) tr = fma(fabs(a[j]), rj, tr);
            }
        }
        if (!binf) {
#pragma unroll
            for (int j = 0; j < NU; j++) {
                s = fma(bu[j], bm[j], s);
                tr = fma(fabs(bu[j]), br[j], tr);
            }
        } else {
#pragma unroll
            for (int j = 0; j < NU; j++) {
                s = fma(bu[j], bm[j], s);
                if (bu[j] != 0.0) tr = fma(fabs(bu[j]), br[j], tr);
            }
        }
        const bool last = k + 1 == p.N;
        const double lb = last ? lb2 : lb1, ub = last ? ub2 : ub1;
        double lo = s - tr, hi = s + tr;
        if (has_b(lb) && lb > lo) lo = lb;
        if (has_b(ub) && ub < hi) hi = ub;
        // the first empty intersection proves it (the oracle's first infeasible stage): the remaining
        // stages of the chain are not run
        if (__any(lane < NX && lo > hi + 1e-9 * (1.0 + fabs(hi)))) return true;
        const bool fin = isfinite(lo) && isfinite(hi);
        m = fin ? 0.5 * (lo + hi) : s;
        r = fin ? 0.5 * (hi - lo) : tr;
        rinf = __any(lane < NX && !(r <= DBL_MAX));   // (NaN too: the selecting chain)
    }
    return false;
}

// plant step + noise, lane-distributed: lane i < NX returns x_i after the step (nmpc_cl_device.h
// cl_advance_group's arithmetic). Plant 0: the controller's own discrete model, row i of [A B] from the
// workgroup's LDS copy (the structure's nonzeros, in column order), x from L.xs, u0 wave-uniform;
// plants 1 / 2: the Crazyflie plant with the force / jerk converter, evaluated wave-uniformly.
template <typename T, int NX, int NU, class SP>
__device__ __forceinline__ double plant_step(const ClFastParams<T> &p, const double *abl, const double *cl,
                                             const double *xs, double xl, const double (&u0)[NU], double w, int lane)
{
    constexpr int NZ = NX + NU;
    if (p.plant == 0) {
        const int i = lane < NX ? lane : 0;
        double s = cl[i];
#pragma unroll
        for (int j = 0; j < NX; j++) s = fma(abl[i * NZ + j], xs[j], s);
#pragma unroll
        for (int j = 0; j < NU; j++) s = fma(abl[i * NZ + NX + j], u0[j], s);
        return lane < NX ? s + (lane < p.noise_dims ? w : 0.0) : 0.0;
    } else if constexpr ((NX == 4 && NU == 2) || (NX == 6 && NU == 2)) {
        double x4[4], f[4];
#pragma unroll
        for (int i = 0; i < 4; i++) x4[i] = xs[i];
        const double inv_m = 1.0 / p.mass;
        double xn = xl;
        // the converter hands the plant theta = atan2(Fx, Fz) and F_d = |F| (force_model/ocp.py:106-115,
        // jerk_model/ocp.py:106-116) and the plant uses F_d sin(theta), F_d cos(theta)
        // (force_model/dynamics.py:54-79): the composition is (Fx, Fz) itself, so the kernel passes the
        // components with F_d = 1 (no atan2 / sin / cos; the oracle keeps the reference's operations, which
        // agree to rounding)
        if (NX == 4) {
            const double s_ = u0[0], c_ = u0[1], Fd = 1.0, h = p.dt;
            double k1[4], k2[4], k3[4], k4[4], tt[4];
            crazyflie_rhs(x4, s_, c_, Fd, inv_m, p.g, k1);
            for (int i = 0; i < 4; i++) tt[i] = x4[i] + 0.5 * h * k1[i];
            crazyflie_rhs(tt, s_, c_, Fd, inv_m, p.g, k2);
            for (int i = 0; i < 4; i++) tt[i] = x4[i] + 0.5 * h * k2[i];
            crazyflie_rhs(tt, s_, c_, Fd, inv_m, p.g, k3);
            for (int i = 0; i < 4; i++) tt[i] = x4[i] + h * k3[i];
            crazyflie_rhs(tt, s_, c_, Fd, inv_m, p.g, k4);
            for (int i = 0; i < 4; i++) x4[i] += h / 6.0 * (k1[i] + 2.0 * k2[i] + 2.0 * k3[i] + k4[i]);
#pragma unroll
            for (int i = 0; i < 4; i++)
                if (lane == i) xn = x4[i] + w;
        } else {
            double a0 = xs[4 % NX], a1 = xs[5 % NX];
            const double h0 = u0[0], h1 = u0[1];
            for (int j = 0; j < p.substeps; j++) {
                a0 = a0 + h0 * p.dt_conv;
                a1 = a1 + h1 * p.dt_conv;
                crazyflie_rhs(x4, p.mass * a0, p.mass * a1, 1.0, inv_m, p.g, f);
                for (int i = 0; i < 4; i++) x4[i] += p.dt_conv * f[i];
            }
#pragma unroll
            for (int i = 0; i < 4; i++)
                if (lane == i) xn = x4[i] + w;
            if (lane == 4 % NX) xn = a0;
            if (lane == 5 % NX) xn = a1;
        }
        return xn;
    }
    return xl;
}

// z_0 of element e = k nz + r as sf_kernel wrote it (the unconstrained solution, unclamped)
template <typename T, int NX, int NU>
__device__ __forceinline__ T z0_from_outputs(const ClFastParams<T> &p, int inst, int e)
{
    constexpr int NZ = NX + NU;
    const int k = e / NZ, r = e % NZ;
    return r < NX ? p.xout[((size_t)inst * (p.N + 1) + k) * NX + r] : p.uout[((size_t)inst * p.N + k) * NU + (r - NX)];
}

// trajectory outputs of an instance's last solve: x_0 the state, the bounded elements the lane's slots
// (z of the accepted solve — held bounds exact — clamped onto the bounds), the unbounded decision
// elements (p.s_free) z_0 from the full tables plus the accepted active-set step W[:, S] nu; a failed
// last step (status 4) outputs the initial point for every element. x_0 in L.xs.
template <typename T, int NX, int NU, int EPL, class LdsT>
__device__ void write_outputs(const ClFastParams<T> &p, LdsT &L, const SlotView<EPL> sv, int lane, int inst, int t,
                              int status, int m, const T (&zs)[EPL])
{
    constexpr int NZ = NX + NU;
    const int N = p.N, ne = p.ne;
    auto put = [&](int e, T z) {
        CLF_CHECK(e >= 0 && e < ne, 10, e);
        const int k = e / NZ, r = e % NZ;
        if (r < NX) p.xout[((size_t)inst * (N + 1) + k) * NX + r] = z;
        else p.uout[((size_t)inst * N + k) * NU + (r - NX)] = z;
    };
    if (status != 0) {
#pragma unroll 1
        for (int e = lane; e < ne; e += 64) {
            const int k = e / NZ, r = e % NZ;
            if (k == N && r >= NX) continue;
            put(e, init_point(p, NX, NZ, k, r, t, r < NX ? (T)L.xs[r] : T(0)));
        }
        return;
    }
    if (lane < NX) put(lane, (T)L.xs[lane]);
#pragma unroll
    for (int j = 0; j < EPL; j++) {
        const int e = sv.e(j);
        if (e >= 0) put(e, fmin(fmax(zs[j], (T)sv.lb(j)), (T)sv.ub(j)));
    }
#pragma unroll 1
    for (int q = lane; q < p.nfree; q += 64) {
        const int e = p.s_free[q];
        double z;
        if (p.z0all) {   // the solve finish: z_0 from the GEMM
            z = (double)p.z0all[(size_t)inst * p.z0_ld + e];
        } else if (p.z0_xu) {   // the fp64 solve's finish: z_0 as sf_kernel wrote it
            z = (double)z0_from_outputs<T, NX, NU>(p, inst, e);
        } else {
            const T *tr = p.txfull + (size_t)e * NX;
            double s0 = (double)p.vfull[(size_t)t * ne + e], s1 = 0.0;   // fp64 sums (the set's terms cancel)
#pragma unroll
            for (int c = 0; c + 1 < NX; c += 2) {
                s0 = fma((double)tr[c], L.xs[c], s0);
                s1 = fma((double)tr[c + 1], L.xs[c + 1], s1);
            }
            if (NX % 2) s0 = fma((double)tr[NX - 1], L.xs[NX - 1], s0);
            z = s0 + s1;
        }
        // W[S, e] nu in batches of 4 (the loads of a batch issued together)
        for (int i0 = 0; i0 < m; i0 += 4) {
            double wv[4];
#pragma unroll
            for (int q = 0; q < 4; q++) wv[q] = i0 + q < m ? p.W[(size_t)L.se_e[i0 + q] * ne + e] : 0.0;
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (i0 + q < m) z = fma(wv[q], L.se_nu[i0 + q], z);
        }
        put(e, (T)z);
    }
}

// The rare path of one step (the instance's wavefront): PDAS rounds from the warm set wf; if they do not
// settle, the interval certificate (oracle/c/riccati_ipm.c infeasible_stage: status 4), else the dual
// active-set fallback finds the set and one more PDAS run solves and checks it; else the step parks. An
// instance whose last solve failed (cert_first) tries the certificate first: infeasible QPs come in runs.
// The first PDAS run takes at most PDAS_ROUNDS rounds (its long runs are cycles, which the fallback
// resolves in a few steps) — one round when the instance's previous step of this launch needed the
// fallback (gi_prev: saturation arcs, where the shifted set is right or the fallback is needed again) —
// the run after the fallback polish_steps. z: z_0 in, the solution out when accepted. Returns status |
// accepted << 8 | ran the fallback << 9 | set size << 10 | (status 4 ? 0 : 1 + active-set steps) << 18.
template <typename T, int NX, int NU, int EPL, int WSM, class LdsT>
__device__ int slow_step(const ClFastParams<T> &p, LdsT &L, const SlotView<EPL> sv0, int lane, const double *abl,
                         const double *cl, T (&z)[EPL], unsigned wf, bool cert_first, bool gi_prev,
                         WCacheOf<WSM, EPL> *wc = nullptr)
{
    int r = 0, steps_ = 0, status = 0;
    bool ran_gi = false;
    unsigned wset = wf;
    // the workgroup's W column cache for this step, if no other wavefront holds it
    SlotView<EPL> sv = sv0;
    if (wc) {
        int got = 0;
        if (lane == 0) {
            int expect = -1;
            got = __hip_atomic_compare_exchange_strong(&wc->owner, &expect, 1, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_WORKGROUP) ? 1 : 0;
        }
        sv.wc_ = __builtin_amdgcn_readfirstlane(got) != 0;
        sv.wcol_ = &wc->col[0][0];
        sv.wcolof_ = wc->colof;
        sv.wcld_ = EPL * 64;
    }
    CLF_T(tcf);
    if (cert_first && certificate_infeasible<T, NX, NU>(p, L, abl, cl, lane)) status = 4;
    CLF_TADD(L, 6, tcf);
    for (int pass = 0; pass < 2 && status != 4; pass++) {
        const int rounds = pass == 1 ? p.polish_steps : (gi_prev ? 1 : min(p.polish_steps, PDAS_ROUNDS));
        CLF_T(tw0);
        r = wsteps_run<T, NX, NU, EPL, WSM>(p, L, sv, lane, z, wset, rounds, wc);
        CLF_TADD(L, 2, tw0);
        steps_ += r >> 16;
        if ((r & 1) || pass == 1) break;
        CLF_T(tc1);
        const bool infeas = !cert_first && certificate_infeasible<T, NX, NU>(p, L, abl, cl, lane);
        CLF_TADD(L, 6, tc1);
        if (infeas) {
            status = 4;
            break;
        }
        if (!p.gi) break;   // test knob: no fallback, the step parks
        int git = 0;
        ran_gi = true;
        CLF_T(tg0);
        // from the set the PDAS rounds reached (wsteps_run leaves it in wset), made dual feasible — not the warm set
        // they started from (oracle/c/riccati_ipm.c: quad13 longest chain 44 -> 36 set steps, force B = 1024 -15 %)
        const bool found = gi_set<T, NX, NU, EPL, WSM>(p, L, sv, lane, z, wset, wset, git, wc);
        CLF_TADD(L, 5, tg0);
        CLF_TCNT(L, 11, git);
        steps_ += git;
        if (!found) break;
    }
    if (NMPC_WCACHE && sv.wc_) {   // the cache's columns and tags written before the next owner takes it
        CLF_SYNC();
        if (lane == 0) __hip_atomic_store(&wc->owner, -1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    const bool ok = (r & 1) != 0;
    const int m_acc = ok ? (r >> 8) & 0xff : 0;
    const int iters = status == 4 ? 0 : 1 + steps_;
    return status | (ok ? 1 << 8 : 0) | (ran_gi ? 1 << 9 : 0) | (m_acc << 10) | (min(iters, 0x3fff) << 18);
}

// One instance's closed-loop steps up to p.target on the whole wavefront (cl_fast_kernel's instance loop,
// and the lockstep kernel's rare path): record load, per step the warm-start shift, the explicit form
// (explicit_form(z, vt): z = v_t + T_x x at the lane's slots, x in L.xs), the bound test, slow_step when
// needed, flags, u0, cost / AED, the outputs at the last step, the plant; write-back (or park).
template <typename T, int NX, int NU, int EPL, int WSM, class SP, class LdsT, class ExplicitF>
__device__ __forceinline__ void run_instance(const ClFastParams<T> &p, LdsT &L, const SlotView<EPL> sv, int lane,
                                             const double *abl, const double *cl, int inst, ExplicitF &&explicit_form,
                                             WCacheOf<WSM, EPL> *wc = nullptr)
{
    constexpr int NZ = NX + NU, NSLOT = EPL * 64;
    const int nref = p.ncl > p.aed_dims ? p.ncl : p.aed_dims;   // reference components of cost / AED
    const double wl = lane < p.ncl ? (double)p.wcl[lane] : 0.0;   // this lane's cost weight
    double uin[NU];                                                // inputs of a failed step (mid-box)
#pragma unroll
    for (int i = 0; i < NU; i++) uin[i] = (double)p.uinit[i];
    CLF_T(tr0);
    const long long inst_t0 = p.iter_log ? wall_clock64() : 0;
    CLF_CHECK(inst >= 0 && inst < p.B, 7, inst);
    // the instance's record, issued together: step, state (lane i < NX holds x_i), active flags of the
    // last solution by slot (bit 2j lower, 2j+1 upper; meaningful after step 0), offset, status
    int step = p.istep[inst];
    double xl = lane < NX ? (double)p.state[(size_t)inst * NX + lane] : 0.0;
    signed char fb[EPL];
#pragma unroll
    for (int j = 0; j < EPL; j++) {
        const int s = j * 64 + lane;
        fb[j] = s < p.nslot ? p.flags[(size_t)inst * p.nslot + s] : 0;
    }
    const unsigned off = (unsigned)p.offset[inst];
    const int st_prev = p.status[inst];
    if (step >= p.target) return;
    CLF_CHECK(step >= p.step0, 8, step - p.step0);
    unsigned fl = 0;
    if (step > 0) {
#pragma unroll
        for (int j = 0; j < EPL; j++) fl |= (fb[j] < 0 ? 1u : (fb[j] > 0 ? 2u : 0u)) << (2 * j);
    }
    int t = (int)((off % (unsigned)p.period + (unsigned)step % (unsigned)p.period) % (unsigned)p.period);
    double cost = 0.0, aed = 0.0;   // this lane's terms (component lane), summed over the wave at the end
    int nfail = 0, nst = 0;
    int last_status = step > 0 ? st_prev : 0, last_iters = 0;
    int nslow = 0;          // rare-path steps of this launch (the next launch claims such instances first)
    bool last_gi = false;   // the previous step of this launch ran the dual fallback
    bool parked = false;
    // v_t at the slots one step ahead (the step's first dependency); the reference component and the
    // noise draw are issued at the top of the step and consumed after the solve
    T vtn[EPL];
    auto fetch_v = [&](int tt) {
        CLF_CHECK(tt >= 0 && tt < p.period, 3, tt);
        const T *vp = p.vb + (size_t)tt * NSLOT;
#pragma unroll
        for (int j = 0; j < EPL; j++) vtn[j] = vp[j * 64 + lane];
    };
    fetch_v(t);
    CLF_TADD(L, 9, tr0);
    for (; step < p.target; step++) {
        const long long clk0 = p.iter_log ? wall_clock64() : 0;
        CLF_T(tp0);
        T vt[EPL];
#pragma unroll
        for (int j = 0; j < EPL; j++) vt[j] = vtn[j];
        const int tn = t + 1 == p.period ? 0 : t + 1;
        if (step + 1 < p.target) fetch_v(tn);
        CLF_CHECK(t >= 0 && t < p.period, 6, t);
        CLF_CHECK(step - p.step0 >= 0 && step - p.step0 < p.noise_ld, 5, step - p.step0);
        const double xr = lane < nref ? (double)p.table[(size_t)t * p.table_cols + lane] : 0.0;
        const double w = p.noise[(size_t)inst * p.noise_ld + (step - p.step0)];
        if (lane < NX) L.xs[lane] = xl;
        // ---- warm start: the last solution's flags shifted by one stage (slot source)
        unsigned wf = 0;
        if (__any(fl != 0)) {
#pragma unroll
            for (int j = 0; j < EPL; j++) L.fl[j * 64 + lane] = flag_of(fl, j);
            CLF_SYNC();
#pragma unroll
            for (int j = 0; j < EPL; j++) {
                // the slot's source code (nmpc_api.cpp clf_setup): the flag of the same component one stage later;
                // kinds 1 / 2 (state slots of stages N - 1 / N - 2): a bound held at N - 1 but not at N - 2 stays at
                // N - 1 (the horizon's end holds it; oracle closed loop mode 1)
                const int code = sv.src(j), sr_ = (code & 0xfff) - 1, ps = ((code >> 12) & 0xfff) - 1, kind = code >> 24;
                signed char f = sr_ >= 0 ? L.fl[sr_] : (signed char)0;
                if (kind != 0) {
                    const signed char own = L.fl[j * 64 + lane], par = L.fl[ps];
                    if (kind == 1 && own != 0 && par == 0) f = own;
                    if (kind == 2 && par != 0 && own == 0) f = 0;
                }
                wf |= bits_of(f) << (2 * j);
            }
        }
        CLF_SYNC();
        CLF_TADD(L, 0, tp0);
        CLF_T(te0);
        // ---- explicit unconstrained solution at the lane's slots (the kernel's functor; x in L.xs)
        T z[EPL];
        explicit_form(z, vt);
        bool ok = false;
        int status = 0, iters = 1, m_acc = 0;
        const bool gi_prev = last_gi;
        last_gi = false;
        if (!__any(wf != 0)) {
            bool bad = false;
#pragma unroll
            for (int j = 0; j < EPL; j++) bad |= !(z[j] >= (T)sv.lo(j) && z[j] <= (T)sv.hi(j));   // NaN: bad
            ok = !__any(bad);
        }
        CLF_TADD(L, 1, te0);
        CLF_TCNT(L, 13, 1);
        if (!ok) {
            CLF_TCNT(L, 12, 1);
            nslow++;
            const int sr = slow_step<T, NX, NU, EPL, WSM>(p, L, sv, lane, abl, cl, z, wf, last_status == 4, gi_prev, wc);
            status = sr & 0xff;
            last_gi = (sr >> 9) & 1;
            ok = (sr >> 8) & 1;
            m_acc = (sr >> 10) & 0xff;
            iters = sr >> 18;
            if (!ok && status != 4) {
                parked = true;
                break;
            }
        }
        // ---- the solution's active flags (z on a bound to 1e-7): the next step's warm start
        fl = 0;
        if (status == 0) {
#pragma unroll
            for (int j = 0; j < EPL; j++)
                fl |= (z[j] <= (T)sv.onl(j) ? 1u : (z[j] >= (T)sv.onu(j) ? 2u : 0u)) << (2 * j);
        }
        // ---- u0 (slots 0..nu-1: lanes 0..nu-1 of j = 0), clamped onto its bound
        const T z0c = fmin(fmax(z[0], (T)sv.lb(0)), (T)sv.ub(0));
        double u0[NU];
#pragma unroll
        for (int i = 0; i < NU; i++) u0[i] = status == 0 ? bcast((double)z0c, i) : uin[i];
        // ---- cost (controller.py:40-41) at x_0 = the state, or x_1 (jerk loop), and the AED numerator:
        // lane i adds component i
        {
            double xo = xl;
            if (p.cost_stage != 0) {
                const double x1 = __shfl((double)z0c, p.x1_slot + lane);
                xo = status == 0 ? x1 : (lane < NX ? (double)init_point(p, NX, NZ, 1, lane, t, T(0)) : 0.0);
            }
            const double e = xo - xr;
            if (lane < p.ncl) cost = fma(wl * e, e, cost);
            if (lane < p.aed_dims) aed += fabs(xr - xl);
        }
        nfail += status != 0;
        nst++;
        last_status = status;
        last_iters = iters;
        // ---- the trajectory outputs of the instance's last step of the run
        CLF_T(to0);
        if (p.traj_out && step + 1 == p.target) write_outputs<T, NX, NU, EPL>(p, L, sv, lane, inst, t, status, m_acc, z);
        CLF_TADD(L, 7, to0);
        CLF_T(tl0);
        // ---- plant step + noise
        xl = plant_step<T, NX, NU, SP>(p, abl, cl, L.xs, xl, u0, w, lane);
        CLF_TADD(L, 8, tl0);
        t = tn;
        if (p.iter_log && lane == 0) {
            const long long kc = wall_clock64() - clk0;   // constant-rate ticks (hipDeviceAttributeWallClockRate)
            p.iter_log[(size_t)(step - p.step0) * p.B + inst] =
                (iters < 255 ? iters : 255) | (status << 8) | ((int)(kc < 32767 ? kc : 32767) << 16);
        }
    }
    // ---- write back: state, sums, step, flags, status
    CLF_T(tb0);
    const bool fl_end = __any(fl != 0u);   // the next launch's first step starts from a nonempty warm set
    cost = wave_sum(cost);
    aed = wave_sum(aed);
    if (lane < NX) p.state[(size_t)inst * NX + lane] = (T)xl;
    if (lane < 4)   // lanes 0..3: [cost, AED numerator, failures, steps], added in the L2 (no return:
                    // nothing waits for the old sums; each instance's sums have one writer)
        unsafeAtomicAdd(p.acc + (size_t)inst * 4 + lane, lane == 0 ? cost : lane == 1 ? aed : lane == 2 ? (double)nfail : (double)nst);
    if (lane == 0) {
        p.istep[inst] = step;
        if (p.demoted) p.demoted[inst] = (unsigned char)((nslow < 127 ? nslow : 127) | (fl_end ? 128 : 0));
        if (parked) {
            const int pos = atomicAdd(p.park_count, 1);
            p.park_list[pos] = inst;
        } else {
            p.status[inst] = last_status;
            p.iters[inst] = last_iters;
        }
    }
#pragma unroll
    for (int j = 0; j < EPL; j++) {
        const int s = j * 64 + lane;
        if (s < p.nslot) p.flags[(size_t)inst * p.nslot + s] = flag_of(fl, j);
    }
    if (p.iter_log && lane == 0) {   // the instance's start and end in this launch (rows target - step0 + 0 / 1,
        // wall-clock ticks, low 31 bits)
        p.iter_log[(size_t)(p.target - p.step0) * p.B + inst] = (int)(inst_t0 & 0x7fffffff);
        p.iter_log[(size_t)(p.target - p.step0 + 1) * p.B + inst] = (int)(wall_clock64() & 0x7fffffff);
    }
#ifdef NMPC_CLF_TIMING
    CLF_TADD(L, 9, tb0);
    CLF_SYNC();
    if (p.cycles && lane < CLF_NT) p.cycles[(size_t)inst * CLF_NT + lane] += (unsigned long long)L.tacc[lane];
    CLF_SYNC();
    if (lane < CLF_NT) L.tacc[lane] = 0;
#endif
    CLF_SYNC();   // L.xs / L.fl of this instance are read before the next one overwrites them
}

constexpr int LOCK_QCAP = 512;   // demoted instances per workgroup (the host checks B / grid <= LOCK_QCAP)

// A workgroup's claim order over its range [lo, lo + cnt) (cnt <= 65536), by one wavefront, longest
// first. `hard` holds one byte per instance from the previous launch: bit 7 = its last solution left
// bounds active (a nonempty warm start: its first step takes the rare path), bits 0-6 = its rare-path
// steps (capped). Groups: bit 7 set, then any rare-path steps, then the rest (buckets = 1: each of the
// first two split by the rare-path steps, >= 8 / 1-7 / 0 and >= 8 / 1-7); instance order within a group
// (hard null: instance order)
// Returns how many of the ordered instances fall in the first `lead` groups (0 without the order bytes).
__device__ inline int claim_order(unsigned short *ord, const unsigned char *hard, const int *map, int lo, int cnt, int lane,
                                  int buckets, int lead = 0)
{
    const unsigned long long lt = (1ull << lane) - 1ull;
    constexpr int MN[2][6] = {{128, 1, 0, 0, 0, 0}, {136, 129, 128, 8, 1, 0}}, MX[2][6] = {{255, 127, 0, 0, 0, 0}, {255, 135, 128, 127, 7, 0}};
    const int nb = hard ? (buckets ? 6 : 3) : 1;
    int pos = 0, warm = 0;
    for (int b = 0; b < nb; b++) {
        const int mn = nb == 1 ? 0 : MN[buckets ? 1 : 0][b], mx = nb == 1 ? 255 : MX[buckets ? 1 : 0][b];
        for (int c = 0; c < cnt; c += 64) {
            const bool in = c + lane < cnt;
            const int h = in && hard ? (int)hard[map ? map[lo + c + lane] : lo + c + lane] : 0;
            const bool d = in && h >= mn && h <= mx;
            const unsigned long long m = __ballot(d);
            if (d) ord[pos + __popcll(m & lt)] = (unsigned short)(c + lane);
            pos += __popcll(m);
        }
        if (nb > 1 && b < lead) warm = pos;
    }
    return warm;
}

// The host-driven rounds' park count without a copy behind the kernel (a blit launch on the stream, ≈5 µs
// per round): every wavefront counts itself out at the kernel's end; the last one reads the count and
// stores it to the pinned host word (a system-scope store, written through), then rezeroes the exit counter
// for the next launch (stream order). No fences: a wavefront's park atomic returned (its list position was
// used) before its exit atomic is issued, the atomics are performed at the device's coherence point, and the
// list entries themselves are read by the next kernel only (an agent-scope release here would write back the
// XCD's L2 at every wavefront's exit: jerk 358M -> 325M). Every wavefront reaches the kernels' ends (no early
// exit but the asynchronous rounds' run_if, which have no host word).
template <typename T>
__device__ __forceinline__ void report_exit(const ClFastParams<T> &p, int lane)
{
    if (!p.park_host) return;
    if (lane == 0) {
        const unsigned total = gridDim.x * (blockDim.x >> 6);
        if (__hip_atomic_fetch_add(p.exit_count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == total - 1u) {
            const int v = __hip_atomic_load(p.park_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(p.park_host, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            // the next launch's park count and claim counter (the parked list stays for the list-mode solve,
            // whose length the host passes)
            __hip_atomic_store(p.park_count, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(p.park_count + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(p.exit_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// The launch's noise draws of the workgroup's own instances (per-workgroup claim ranges), written before the
// workgroup's first barrier, so its wavefronts read them as they read the noise kernel's (the chunk's noise
// kernel and its launch gap, ≈12 µs per host-driven round, saved; noise_draw: the same bits)
template <typename T>
__device__ __forceinline__ void gen_noise(const ClFastParams<T> &p, int wg_lo, int wg_hi)
{
    const int ld = p.noise_ld, cnt = (wg_hi - wg_lo) * ld;
    for (int q = threadIdx.x; q < cnt; q += blockDim.x) {
        const int r = q / ld, s = q - r * ld;
        const int b = p.inst_map ? p.inst_map[wg_lo + r] : wg_lo + r;
        p.noise_gen[(size_t)b * ld + s] = noise_draw(p.seed, p.inst_base, p.noise_std, p.noise_table, p.noise_len, b, p.step0 + s);
    }
}

// WPB wavefronts per workgroup (the slot tables in LDS are shared by them), MW the occupancy target
// (waves per SIMD; 0: none)
template <typename T, int NX, int NU, int EPL, int WSM, int WPB, int MW, class SP, bool WL = false, bool SW2 = false>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(MW > 0 ? MW : 1, 8))) void cl_fast_kernel(ClFastParams<T> p)
{
    if (p.run_if && __builtin_amdgcn_readfirstlane(*p.run_if) == 0) return;   // an empty asynchronous round
    constexpr int NZ = NX + NU, NSLOT = EPL * 64;
    static_assert(NX < 32 && NZ <= 64, "lane-distributed state");
    __shared__ Lds<NSLOT, NZ, WSM, SW2> lds_all[WPB];
    // workgroup constants: [A B], c (plant), the slots' bounds, thresholds, elements and warm-start sources
    __shared__ double abl[NX * NZ], cl[NX], slb[NSLOT], sub[NSLOT], slo[NSLOT], shi[NSLOT], sol[NSLOT], sou[NSLOT];
    __shared__ int sse[NSLOT], ssrc[NSLOT];
    // the slots' T_x rows, pairs of components per word (txl[c][s] = (T_x(s, 2c), T_x(s, 2c + 1))):
    // lanes read consecutive words, one ds_read_b128 (fp32: b64) per slot and pair
    constexpr int NXP = (NX + 1) / 2;
    using TP = typename std::conditional<std::is_same<T, float>::value, float2, double2>::type;
    __shared__ TP txl[NXP][NSLOT];
    for (int e = threadIdx.x; e < NXP * NSLOT; e += 64 * WPB) {
        const int c = e / NSLOT, s_ = e % NSLOT;
        const bool v = s_ < p.nslot;
        TP w;
        w.x = v ? p.s_tx[(size_t)s_ * NX + 2 * c] : T(0);
        w.y = v && 2 * c + 1 < NX ? p.s_tx[(size_t)s_ * NX + 2 * c + 1] : T(0);
        txl[c][s_] = w;
    }
    for (int e = threadIdx.x; e < NX * NZ; e += 64 * WPB) {
        const int i = e / NZ, j = e % NZ;
        abl[e] = SP::ab(i, j) ? (double)p.AB[e] : 0.0;   // the plant rows: the structure's nonzeros
    }
    for (int e = threadIdx.x; e < NX; e += 64 * WPB) cl[e] = (double)p.c[e];
    for (int s = threadIdx.x; s < NSLOT; s += 64 * WPB) {
        const bool v = s < p.nslot;
        const double l = v ? (double)p.s_lb[s] : -1e30, u = v ? (double)p.s_ub[s] : 1e30;
        const bool hl = has_b(l), hu = has_b(u);
        slb[s] = l;
        sub[s] = u;
        slo[s] = hl ? l - ClfTol<T>::viol * (1.0 + fabs(l)) : -DBL_MAX;
        shi[s] = hu ? u + ClfTol<T>::viol * (1.0 + fabs(u)) : DBL_MAX;
        sol[s] = hl ? l + ClfTol<T>::onb * (1.0 + fabs(l)) : -DBL_MAX;
        sou[s] = hu ? u - ClfTol<T>::onb * (1.0 + fabs(u)) : DBL_MAX;
        sse[s] = v ? p.s_e[s] : -1;
        ssrc[s] = v ? p.s_src[s] : 0;
    }
    // WL: W over the slots in LDS (lower triangle; the rare path's gathers and W[:, S] nu combinations
    // then wait on LDS instead of L2 — the force shape, whose steps are mostly active-set steps)
    constexpr int NTRI = WL ? NSLOT * (NSLOT + 1) / 2 : 1;
    __shared__ double wtri[NTRI];
    if constexpr (WL) {
        for (int e = threadIdx.x; e < NTRI; e += 64 * WPB) {
            int r = (int)((sqrtf(8.0f * (float)e + 1.0f) - 1.0f) * 0.5f);   // row of triangle entry e
            while ((r + 1) * (r + 2) / 2 <= e) r++;
            while (r * (r + 1) / 2 > e) r--;
            const int c = e - r * (r + 1) / 2;
            wtri[e] = (r < p.nslot && c < p.nslot) ? p.W[(size_t)p.s_e[r] * p.ne + p.s_e[c]] : 0.0;
        }
    }
    __shared__ int wg_next;   // the workgroup's next instance (offset into its range)
    __shared__ unsigned short ord[LOCK_QCAP];   // claim order (offsets into the workgroup's range)
    // the W column cache (sets of up to 16: quad13, jerk; not with W in LDS)
    constexpr bool WCACHE = NMPC_WCACHE && WSM <= 16 && !WL;
    using WCT = typename std::conditional<WCACHE, WCacheOf<WSM, EPL>, char>::type;
    __shared__ WCT wcache_;
    WCacheOf<WSM, EPL> *wcp = nullptr;
    if constexpr (WCACHE) {
        wc_init(wcache_);
        if (p.wcache) wcp = &wcache_;
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    Lds<NSLOT, NZ, WSM, SW2> &L = lds_all[wave];
    if (lane < 32) L.xs[lane] = 0.0;
#ifdef NMPC_CLF_TIMING
    if (lane < CLF_NT) L.tacc[lane] = 0;
#endif
    if (threadIdx.x == 0) wg_next = 0;
    const int per_wg = (p.B + (int)gridDim.x - 1) / (int)gridDim.x;
    const int wg_lo = p.claim_global ? 0 : (int)blockIdx.x * per_wg, wg_hi = p.claim_global ? p.B : min(p.B, wg_lo + per_wg);
    // the previous launch's rare-path instances first (longest first: the workgroup's makespan), when the
    // range fits the order table
    const bool ordered = !p.claim_global && p.demoted && wg_hi - wg_lo <= LOCK_QCAP;
    if (ordered && wave == 0) claim_order(ord, p.demoted, p.inst_map, wg_lo, wg_hi - wg_lo, lane, p.order_buckets);
    if (p.noise_gen && !p.claim_global) gen_noise(p, wg_lo, wg_hi);
    __syncthreads();
    const SlotView<EPL> sv{slb, sub, slo, shi, sol, sou, sse, ssrc, lane, wtri, WL};

    const int nref = p.ncl > p.aed_dims ? p.ncl : p.aed_dims;   // reference components of cost / AED
    const double wl = lane < p.ncl ? (double)p.wcl[lane] : 0.0;   // this lane's cost weight
    double uin[NU];                                                // inputs of a failed step (mid-box)
#pragma unroll
    for (int i = 0; i < NU; i++) uin[i] = (double)p.uinit[i];

    // persistent wavefronts: the workgroup owns a contiguous range of instances, its wavefronts take the
    // next one from a counter in LDS until none is left (an instance's cost varies 10x with its active
    // sets; every wavefront reaches the exit). Against one device-wide counter: jerk +14 %, force
    // B = 8192 -6 % (less balancing across workgroups), quad13 unchanged (r4e / r4f)
    // (p.claim_global: one device-wide counter instead, p.park_count[1] — the force shape, whose instances'
    // costs vary most, balances across workgroups)
    for (;;) {
        int next = 0;
        if (lane == 0) next = p.claim_global ? atomicAdd(p.park_count + 1, 1) : atomicAdd(&wg_next, 1);
        next = __builtin_amdgcn_readfirstlane(next);
        if (wg_lo + next >= wg_hi) break;
        const int pos = wg_lo + (ordered ? (int)ord[next] : next);
        const int inst = p.claim_global ? (p.gorder ? p.gorder[pos] : pos) : (p.inst_map ? p.inst_map[pos] : pos);
        // explicit unconstrained solution at the lane's slots: T_x pairs from LDS against x pairs broadcast
        run_instance<T, NX, NU, EPL, WSM, SP>(p, L, sv, lane, abl, cl, inst, [&](T(&z)[EPL], const T(&vt)[EPL]) {
            T z1[EPL];
#pragma unroll
            for (int j = 0; j < EPL; j++) {
                z[j] = vt[j];
                z1[j] = T(0);
            }
#pragma unroll
            for (int c = 0; c < NXP; c++) {
                const double2 xx = *reinterpret_cast<const double2 *>(&L.xs[2 * c]);
                const T x0 = (T)xx.x, x1 = (T)xx.y;
#pragma unroll
                for (int j = 0; j < EPL; j++) {
                    const TP tt = txl[c][j * 64 + lane];
                    z[j] = fma(tt.x, x0, z[j]);
                    z1[j] = fma(tt.y, x1, z1[j]);
                }
            }
#pragma unroll
            for (int j = 0; j < EPL; j++) z[j] += z1[j];
        }, wcp);
    }
    report_exit(p, lane);
}


// ------------------------------------------------------------------------------------------------------
// The exact finish of fp32 handles' solves (nmpc_solve / solve_async; fp64 handles finish inside the IPM
// kernel). The fp32 IPM stops at tol_comp 1e-7 in fp32 arithmetic, 1e-3..1e-2 from the exact solution on
// the force OCP (condition ~4e4); the finish takes its active bounds as the warm set and runs the lean
// loop's machinery on them — PDAS on the projected inverse Hessian W (fp64), the dual fallback, the fp64
// KKT acceptance — so an accepted solution is the exact QP solution of the fp32-stored problem data.
//
// Step 1 (fin32_z0_kernel): the unconstrained solution of every element, linear in the pinned state and the
// reference, z_0 = M [x0; yref] + vc (M = [T_x | V_y], host-built from the unconstrained Riccati tables), as
// a batched GEMM on v_mfma_f32_16x16x4_f32 (A[i][k] = lane 16k + i, B[k][j] = lane 16k + j, D[4 (l >> 4) +
// r][l & 15]): rows = elements in tiles of 16, columns = 16 instances per workgroup, K = nx + the stage-
// stacked reference in steps of 4; each wavefront of the workgroup takes every WPB-th element tile.
template <int WPB>
__global__ __launch_bounds__(64 * WPB) void fin32_z0_kernel(Fin32Z0Params p)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int j = lane & 15, kl = lane >> 4;
    const int ib = (int)blockIdx.x * 16 + j;   // this lane's instance (B operand column)
    const bool iv = ib < p.B;
    const int ntile = p.m16 / 16, K = p.nx + p.ystride;
    for (int et = wave; et < ntile; et += WPB) {
        using f4 = __attribute__((__vector_size__(4 * sizeof(float)))) float;
        f4 acc;
#pragma unroll
        for (int r = 0; r < 4; r++) acc[r] = p.vc[et * 16 + 4 * kl + r];
        const float *mrow = p.M + (size_t)(et * 16 + j) * p.kp;   // A operand row (element et * 16 + j)
        for (int k0 = 0; k0 < p.kp; k0 += 4) {
            const int k = k0 + kl;
            const float a = mrow[k];
            float b = 0.f;
            if (iv && k < K) b = k < p.nx ? p.x0[(size_t)ib * p.nx + k] : p.yref[(size_t)ib * p.ystride + (k - p.nx)];
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
        }
        if (iv) {
            float4 v;
            v.x = acc[0];
            v.y = acc[1];
            v.z = acc[2];
            v.w = acc[3];
            *reinterpret_cast<float4 *>(p.z0 + (size_t)ib * p.m16 + et * 16 + 4 * kl) = v;
        }
    }
}

// Step 2: one wavefront per instance (persistent). An instance the IPM did not solve (status != 0) keeps
// its result. Otherwise: z_0 at the slots from step 1; the warm set = the bounds the IPM solution sits on
// (within 1e-3 (1 + |b|) — the fp32 interior point's distance from an active bound); no set and z_0
// feasible: the unconstrained solution; else slow_step (PDAS rounds, certificate, dual fallback). Accepted:
// the outputs are rewritten from the exact solution (free elements z_0 + W[:, S] nu) and the finish's
// active-set steps are added to qp_iter; not accepted: the IPM's solution stays.
template <int NX, int NU, int EPL, int WSM, int WPB>
__global__ __launch_bounds__(64 * WPB) void fin32_kernel(ClFastParams<float> p)
{
    using T = float;
    constexpr int NZ = NX + NU, NSLOT = EPL * 64;
    __shared__ Lds<NSLOT, NZ, WSM> lds_all[WPB];
    __shared__ double abl[NX * NZ], cl[NX], slb[NSLOT], sub[NSLOT], slo[NSLOT], shi[NSLOT], sol[NSLOT], sou[NSLOT];
    __shared__ int sse[NSLOT], ssrc[NSLOT];
    for (int e = threadIdx.x; e < NX * NZ; e += 64 * WPB) abl[e] = (double)p.AB[e];
    for (int e = threadIdx.x; e < NX; e += 64 * WPB) cl[e] = (double)p.c[e];
    for (int s = threadIdx.x; s < NSLOT; s += 64 * WPB) {
        const bool v = s < p.nslot;
        const double l = v ? (double)p.s_lb[s] : -1e30, u = v ? (double)p.s_ub[s] : 1e30;
        const bool hl = has_b(l), hu = has_b(u);
        slb[s] = l;
        sub[s] = u;
        slo[s] = hl ? l - ClfTol<T>::viol * (1.0 + fabs(l)) : -DBL_MAX;
        shi[s] = hu ? u + ClfTol<T>::viol * (1.0 + fabs(u)) : DBL_MAX;
        sol[s] = hl ? l + 1e-3 * (1.0 + fabs(l)) : -DBL_MAX;   // the IPM solution's active bounds
        sou[s] = hu ? u - 1e-3 * (1.0 + fabs(u)) : DBL_MAX;
        sse[s] = v ? p.s_e[s] : -1;
        ssrc[s] = 0;
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    Lds<NSLOT, NZ, WSM> &L = lds_all[wave];
    if (lane < 32) L.xs[lane] = 0.0;
#ifdef NMPC_CLF_TIMING
    if (lane < CLF_NT) L.tacc[lane] = 0;
#endif
    __syncthreads();
    const SlotView<EPL> sv{slb, sub, slo, shi, sol, sou, sse, ssrc, lane};
    for (int inst = (int)blockIdx.x * WPB + wave; inst < p.B; inst += (int)gridDim.x * WPB) {
        if (p.status[inst] != 0) continue;   // wave-uniform
        if (lane < NX) L.xs[lane] = (double)p.x0in[(size_t)inst * NX + lane];
        T z[EPL];
        unsigned wf = 0;
#pragma unroll
        for (int j = 0; j < EPL; j++) {
            const int e = sv.e(j);
            z[j] = e >= 0 ? p.z0all[(size_t)inst * p.z0_ld + e] : T(0);
            if (e >= 0) {
                const int k = e / NZ, r = e % NZ;
                const T zi = r < NX ? p.xout[((size_t)inst * (p.N + 1) + k) * NX + r]
                                    : p.uout[((size_t)inst * p.N + k) * NU + (r - NX)];
                wf |= (zi <= (T)sv.onl(j) ? 1u : (zi >= (T)sv.onu(j) ? 2u : 0u)) << (2 * j);
            }
        }
        CLF_SYNC();
        bool ok = false;
        int m_acc = 0, steps = 0;
        if (!__any(wf != 0)) {
            bool bad = false;
#pragma unroll
            for (int j = 0; j < EPL; j++) bad |= !(z[j] >= (T)sv.lo(j) && z[j] <= (T)sv.hi(j));
            ok = !__any(bad);
        }
        if (!ok) {
            const int sr = slow_step<T, NX, NU, EPL, WSM>(p, L, sv, lane, abl, cl, z, wf, false, false);
            ok = ((sr >> 8) & 1) && (sr & 0xff) == 0;
            m_acc = (sr >> 10) & 0xff;
            steps = sr >> 18;
        }
        if (ok) {
            write_outputs<T, NX, NU, EPL>(p, L, sv, lane, inst, 0, 0, m_acc, z);
            if (lane == 0) p.iters[inst] += steps;
        }
        CLF_SYNC();
    }
}

// ------------------------------------------------------------------------------------------------------
// The finish of the fp64 general solve: the instances sf_kernel (nmpc_solve_fast.hip) listed because their
// unconstrained solution violates a bound, one wavefront per instance (persistent over the list): z_0 at the
// slots from the outputs sf_kernel wrote, then slow_step from an empty warm set (the first set from z_0's
// violations; PDAS rounds on W, the certificate, the dual fallback; oracle/c/riccati_ipm.c
// riccati_ipm_solve_batch_fast). Accepted: the outputs are rewritten from the exact solution, status 0,
// qp_iter = 1 + the active-set steps. Otherwise (a certified-infeasible QP or no settled set) the instance is
// parked for the full IPM (ipm_lpc_kernel in list mode).
template <int NX, int NU, int EPL, int WSM, int WPB>
__global__ __launch_bounds__(64 * WPB) void fin64_kernel(ClFastParams<double> p)
{
    using T = double;
    constexpr int NZ = NX + NU, NSLOT = EPL * 64;
    const int cnt = __builtin_amdgcn_readfirstlane(*p.work_count);
    if ((int)blockIdx.x * WPB >= cnt) return;   // nothing for this workgroup: no table setup
    __shared__ Lds<NSLOT, NZ, WSM> lds_all[WPB];
    __shared__ double abl[NX * NZ], cl[NX], slb[NSLOT], sub[NSLOT], slo[NSLOT], shi[NSLOT], sol[NSLOT], sou[NSLOT];
    __shared__ int sse[NSLOT], ssrc[NSLOT];
    for (int e = threadIdx.x; e < NX * NZ; e += 64 * WPB) abl[e] = p.AB[e];
    for (int e = threadIdx.x; e < NX; e += 64 * WPB) cl[e] = p.c[e];
    for (int s = threadIdx.x; s < NSLOT; s += 64 * WPB) {
        const bool v = s < p.nslot;
        const double l = v ? p.s_lb[s] : -1e30, u = v ? p.s_ub[s] : 1e30;
        const bool hl = has_b(l), hu = has_b(u);
        slb[s] = l;
        sub[s] = u;
        slo[s] = hl ? l - ClfTol<T>::viol * (1.0 + fabs(l)) : -DBL_MAX;
        shi[s] = hu ? u + ClfTol<T>::viol * (1.0 + fabs(u)) : DBL_MAX;
        sol[s] = hl ? l + ClfTol<T>::onb * (1.0 + fabs(l)) : -DBL_MAX;
        sou[s] = hu ? u - ClfTol<T>::onb * (1.0 + fabs(u)) : DBL_MAX;
        sse[s] = v ? p.s_e[s] : -1;
        ssrc[s] = 0;
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    Lds<NSLOT, NZ, WSM> &L = lds_all[wave];
    if (lane < 32) L.xs[lane] = 0.0;
#ifdef NMPC_CLF_TIMING
    if (lane < CLF_NT) L.tacc[lane] = 0;
#endif
    __syncthreads();
    const SlotView<EPL> sv{slb, sub, slo, shi, sol, sou, sse, ssrc, lane};
    for (int w = (int)blockIdx.x * WPB + wave; w < cnt; w += (int)gridDim.x * WPB) {
        const int inst = __builtin_amdgcn_readfirstlane(p.work_list[w]);
        if (lane < NX) L.xs[lane] = p.x0in[(size_t)inst * NX + lane];
        T z[EPL];
#pragma unroll
        for (int j = 0; j < EPL; j++) {
            const int e = sv.e(j);
            z[j] = e >= 0 ? z0_from_outputs<T, NX, NU>(p, inst, e) : T(0);
        }
        CLF_SYNC();
        const int sr = slow_step<T, NX, NU, EPL, WSM>(p, L, sv, lane, abl, cl, z, 0u, false, false);
        const bool ok = ((sr >> 8) & 1) && (sr & 0xff) == 0;
        if (ok) {
            write_outputs<T, NX, NU, EPL>(p, L, sv, lane, inst, 0, 0, (sr >> 10) & 0xff, z);
            if (lane == 0) {
                p.status[inst] = 0;
                p.iters[inst] = sr >> 18;
            }
        } else if (lane == 0) {
            const int pos = atomicAdd(p.park_count, 1);
            p.park_list[pos] = inst;
        }
        CLF_SYNC();
    }
}

// ------------------------------------------------------------------------------------------------------
// The lockstep closed loop (quad13-class shapes: controller-model plant, cost on x_0): four instances per
// wavefront advance together and the step's dense products run on the matrix cores. Two phases per
// workgroup, so the lockstep registers and the single-instance rare path never coexist:
//
// Phase 1, lockstep (the common path):
//   * explicit form Z = V + T_x X for four instances at once on v_mfma_f64_4x4x4_4b_f64: M = slots in tiles
//     of 16 (4 blocks of 4 rows), K = state components in chunks of 4, N = the 4 instances
//     (A[b][i][k] = lane 16k + 4b + i, B[b][k][n] = lane 16k + 4b + n, D[b][i][n] = lane 16i + 4b + n,
//     pinned by tools/ubench/mfma_f64_layout.hip). T_x sits in LDS in A-operand order (one conflict-free
//     8-byte read per lane per MFMA), the states X are the B operand straight from registers (lane
//     16k + 4b + n holds component 4 kc + k of instance n, all four blocks), V (the window's v_t at the
//     lane's slots, loaded one step ahead) the accumulators' initial value. Lane l owns instance n = l & 3
//     and the slots 16 t + 4 ((l >> 2) & 3) + (l >> 4), t < NT;
//   * the bound test and the warm-start flags per lane, one ballot per wave: an instance whose z_0 meets
//     every bound (1e-13) and whose last solution touched none is solved (cl_fast_kernel's fast path);
//   * the plant X' = [A B] [X; U] + c as five more MFMAs (K = 16 states + 4 inputs), the result moved back
//     into the B-operand layout by four lane permutes; cost / AED on the lanes of block 0;
//   * an instance that needs the rare path (a violated bound, or a nonempty warm set) is demoted: its
//     record goes back to memory (state, step, flags, sums so far) and into the workgroup's LDS queue, and
//     the slot takes the next instance. Its last step's trajectory outputs are written from the lockstep
//     layout.
// Phase 2: each wavefront whose slots ran dry takes demoted instances from the queue and runs them to the
// target with the single-instance code (run_instance: slow_step's PDAS on W, certificate, dual fallback,
// parks; the explicit form on the same MFMA tiles), until every wavefront of the workgroup has left phase 1
// and the queue is empty (all of a workgroup's wavefronts are co-resident: the wait always ends).
// Same decisions, thresholds and outputs as cl_fast_kernel (oracle/c/riccati_ipm.c mode 1); only the
// summation order of the explicit form and the plant differs (rounding).

template <typename T, int NX, int NU, int EPL, int WSM, int WPB, int MW, class SP>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(MW > 0 ? MW : 1, MW > 0 ? MW : 8))) void cl_lock_kernel(ClFastParams<T> p)
{
    if (p.run_if && __builtin_amdgcn_readfirstlane(*p.run_if) == 0) return;   // an empty asynchronous round
    constexpr int NZ = NX + NU, NSLOT = EPL * 64, NT = NSLOT / 16, KC = (NX + 3) / 4, KU = (NU + 3) / 4;
    static_assert(NX <= 16 && NU <= 4 && NZ <= 64 && NT <= 32, "lockstep layout: states in 4 chunks, inputs in one");
    __shared__ Lds<NSLOT, NZ, WSM> lds_all[WPB];
    __shared__ double zb_all[WPB][NSLOT];               // z staging in slot order (phase 2's explicit form)
    __shared__ signed char flb_all[WPB][4][NSLOT];      // each slot's last solution flags, slot order
    __shared__ double abl[NX * NZ], cl[NX], slb[NSLOT], sub[NSLOT], slo[NSLOT], shi[NSLOT], sol[NSLOT], sou[NSLOT];
    __shared__ int sse[NSLOT], ssrc[NSLOT];
    __shared__ double txA[NT][KC][64];                  // T_x in A-operand order
    __shared__ double2 lohi[NSLOT], onb[NSLOT];         // (lo, hi) violation / (onl, onu) on-bound thresholds
    __shared__ int dq[LOCK_QCAP];                       // demoted instances (-1: slot not yet written)
    __shared__ unsigned short ord[LOCK_QCAP];           // claim order (offsets into the workgroup's range)
    __shared__ int wg_next, dq_tail, dq_head, ph1_done;
    constexpr bool WCACHE = NMPC_WCACHE && WSM <= 16;   // the W column cache of the rare path
    using WCT = typename std::conditional<WCACHE, WCacheOf<WSM, EPL>, char>::type;
    __shared__ WCT wcache_;
    WCacheOf<WSM, EPL> *wcp = nullptr;
    if constexpr (WCACHE) {
        wc_init(wcache_);
        if (p.wcache) wcp = &wcache_;
    }
    for (int e = threadIdx.x; e < NT * KC * 64; e += 64 * WPB) {
        const int t = e / (KC * 64), kc = (e / 64) % KC, l = e % 64;
        const int s_ = 16 * t + 4 * ((l >> 2) & 3) + (l & 3), c = 4 * kc + (l >> 4);
        txA[t][kc][l] = (s_ < p.nslot && c < NX) ? (double)p.s_tx[(size_t)s_ * NX + c] : 0.0;
    }
    for (int e = threadIdx.x; e < NX * NZ; e += 64 * WPB) {
        const int i = e / NZ, j = e % NZ;
        abl[e] = SP::ab(i, j) ? (double)p.AB[e] : 0.0;
    }
    for (int e = threadIdx.x; e < NX; e += 64 * WPB) cl[e] = (double)p.c[e];
    for (int s = threadIdx.x; s < NSLOT; s += 64 * WPB) {
        const bool v = s < p.nslot;
        const double l = v ? (double)p.s_lb[s] : -1e30, u = v ? (double)p.s_ub[s] : 1e30;
        const bool hl = has_b(l), hu = has_b(u);
        slb[s] = l;
        sub[s] = u;
        slo[s] = hl ? l - ClfTol<T>::viol * (1.0 + fabs(l)) : -DBL_MAX;
        shi[s] = hu ? u + ClfTol<T>::viol * (1.0 + fabs(u)) : DBL_MAX;
        sol[s] = hl ? l + ClfTol<T>::onb * (1.0 + fabs(l)) : -DBL_MAX;
        sou[s] = hu ? u - ClfTol<T>::onb * (1.0 + fabs(u)) : DBL_MAX;
        lohi[s] = make_double2(slo[s], shi[s]);
        onb[s] = make_double2(sol[s], sou[s]);
        sse[s] = v ? p.s_e[s] : -1;
        ssrc[s] = v ? p.s_src[s] : 0;
    }
    for (int e = threadIdx.x; e < LOCK_QCAP; e += 64 * WPB) dq[e] = -1;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    Lds<NSLOT, NZ, WSM> &L = lds_all[wave];
    double *zb = zb_all[wave];
    signed char(*flb)[NSLOT] = flb_all[wave];
    if (lane < 32) L.xs[lane] = 0.0;
#ifdef NMPC_CLF_TIMING
    if (lane < CLF_NT) L.tacc[lane] = 0;
#endif
    if (threadIdx.x == 0) wg_next = dq_tail = dq_head = ph1_done = 0;
    // the workgroup's contiguous instance range (persistent grid)
    const int per_wg = (p.B + (int)gridDim.x - 1) / (int)gridDim.x;
    const int wg_lo = (int)blockIdx.x * per_wg, wg_hi = min(p.B, wg_lo + per_wg);
    // claim order: the instances the previous launch demoted first (the launch's longest chains start at its
    // beginning, not behind the lockstep ones), then the rest, each group in instance order. Only the
    // schedule changes: an instance runs lockstep until its first rare step wherever it is claimed
    // The instances that start from a nonempty warm set take the rare path at their first step: lockstep would
    // demote them at once (slow = ... || flany), so they go straight to the phase-2 queue, where the early
    // workers start their chains at the launch's beginning (env NMPC_LOCK_DIRECT=0: through lockstep). The same
    // steps on the same path (the record is read by run_instance either way).
    if (wave == 0) {
        // (lock_direct = the leading claim-order groups routed: 1 = the warm-started ones, the default; more
        // groups also route instances with rare-path steps in the previous launch — a tuning experiment)
        const int warm = claim_order(ord, p.demoted, p.inst_map, wg_lo, wg_hi - wg_lo, lane, p.order_buckets,
                                     p.lock_workers > 0 ? p.lock_direct : 0);
        if (warm > 0) {
            for (int q = lane; q < warm; q += 64) {
                int inst_ = wg_lo + (int)ord[q];
                if (p.inst_map) inst_ = p.inst_map[inst_];
                dq[q] = inst_;
            }
            if (lane == 0) {
                dq_tail = warm;
                wg_next = warm;
            }
        }
    }
    if (p.noise_gen) gen_noise(p, wg_lo, wg_hi);
    __syncthreads();
    const SlotView<EPL> sv{slb, sub, slo, shi, sol, sou, sse, ssrc, lane};
    const int n = lane & 3, ti = lane >> 4, tb = (lane >> 2) & 3;   // instance slot; D-layout slot offset
    const int prow = lane & 15, drow = 4 * tb + ti;                 // plant A-operand row; D row
    auto slot_of = [&](int q) { return 16 * q + 4 * tb + ti; };

    // ================= phase 1: lockstep (the workgroup's last p.lock_workers wavefronts start as phase-2
    // workers, so the queued chains start at once: env NMPC_LOCK_WORKERS, default 1)
    if (wave < WPB - p.lock_workers) {
        // per-instance state, replicated on the 16 lanes of its slot
        int inst = -1, step = 0, t = 0, last_status = 0, nfail = 0, nst = 0;
        bool flany = false;
        double cost = 0.0, aed = 0.0;
        long long inst_t0 = 0;
        double xr[KC];
        T vt[NT];
#pragma unroll
        for (int kc = 0; kc < KC; kc++) xr[kc] = 0.0;
#pragma unroll
        for (int q = 0; q < NT; q++) vt[q] = T(0);
        auto fetch_v = [&](int tt) {
            CLF_CHECK(tt >= 0 && tt < p.period, 3, tt);
            const T *vp = p.vb + (size_t)tt * NSLOT;
#pragma unroll
            for (int q = 0; q < NT; q++) vt[q] = vp[slot_of(q)];
        };
        // a new instance for every slot that wants one (lane q < 4 claims for slot q) and its record:
        // step, state (B-operand layout), flags (slot order, LDS), offset, status; v of its first step
        auto claim = [&](bool want) {
            int nx_ = 0;
            if (lane < 4 && want) nx_ = atomicAdd(&wg_next, 1);
            nx_ = __shfl(nx_, n);
            if (!want) return;
            CLF_CHECK(nx_ >= wg_hi - wg_lo || nx_ < LOCK_QCAP, 1, nx_);
            inst = nx_ < wg_hi - wg_lo ? wg_lo + (int)ord[nx_] : -1;
            if (inst >= 0 && p.inst_map) inst = p.inst_map[inst];
            CLF_CHECK(inst < p.B, 2, inst);
            flany = false;
            cost = aed = 0.0;
            nfail = nst = 0;
            if (inst < 0) return;
            inst_t0 = p.iter_log ? wall_clock64() : 0;
            step = p.istep[inst];
            const unsigned off = (unsigned)p.offset[inst];
            last_status = step > 0 ? p.status[inst] : 0;
            t = (int)((off % (unsigned)p.period + (unsigned)step % (unsigned)p.period) % (unsigned)p.period);
#pragma unroll
            for (int kc = 0; kc < KC; kc++) {
                const int c = 4 * kc + ti;
                xr[kc] = c < NX ? (double)p.state[(size_t)inst * NX + c] : 0.0;
            }
            bool any = false;
            for (int s = 4 * tb + ti; s < NSLOT; s += 16) {   // the slot's 16 lanes cover its flags
                const signed char f = (s < p.nslot && step > 0) ? p.flags[(size_t)inst * p.nslot + s] : (signed char)0;
                flb[n][s] = f;
                any |= f != 0;
            }
            flany = (__ballot(any) & (0x1111111111111111ull << n)) != 0;
            if (step < p.target) fetch_v(t);
        };
        // the instance's record back to memory (its slot's lanes): state, the sums so far (no-return f64
        // atomics), step, status, flags; demote: into the workgroup queue for phase 2 (the record stores
        // complete and are released at workgroup scope before the queue entry appears)
        auto write_back = [&](bool demote) {
            const long long t1 = p.iter_log ? wall_clock64() : 0;
            double c_ = cost, a_ = aed;
#pragma unroll
            for (int o = 4; o < 64; o <<= 1) {
                c_ += __shfl_xor(c_, o);
                a_ += __shfl_xor(a_, o);
            }
            if (tb == 0) {
#pragma unroll
                for (int kc = 0; kc < KC; kc++) {
                    const int c = 4 * kc + ti;
                    if (c < NX) p.state[(size_t)inst * NX + c] = (T)xr[kc];
                }
            }
            for (int s = 4 * tb + ti; s < p.nslot; s += 16) p.flags[(size_t)inst * p.nslot + s] = flany ? flb[n][s] : (signed char)0;
            if (lane == n) {
                if (nst > 0 || c_ != 0.0 || a_ != 0.0) {
                    unsafeAtomicAdd(p.acc + (size_t)inst * 4 + 0, c_);
                    unsafeAtomicAdd(p.acc + (size_t)inst * 4 + 1, a_);
                    unsafeAtomicAdd(p.acc + (size_t)inst * 4 + 2, (double)nfail);
                    unsafeAtomicAdd(p.acc + (size_t)inst * 4 + 3, (double)nst);
                }
                p.istep[inst] = step;
                p.status[inst] = last_status;
                if (p.demoted) p.demoted[inst] = demote ? 1 : (flany ? 128 : 0);
                if (!demote) p.iters[inst] = 1;
                if (p.iter_log && !demote) {
                    p.iter_log[(size_t)(p.target - p.step0) * p.B + inst] = (int)(inst_t0 & 0x7fffffff);
                    p.iter_log[(size_t)(p.target - p.step0 + 1) * p.B + inst] = (int)(t1 & 0x7fffffff);
                }
            }
            if (demote) {
                __builtin_amdgcn_s_waitcnt(0);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (lane == n) {
                    const int pos = atomicAdd(&dq_tail, 1);
                    CLF_CHECK(pos < LOCK_QCAP, 4, pos);
                    __hip_atomic_store(&dq[pos], inst, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
        };
        claim(true);
        for (;;) {
            CLF_T(tk_idle);
            // slots whose instance is already at the target move on
            for (int guard = 0; guard < per_wg + 4; guard++) {
                const bool idle = inst >= 0 && step >= p.target;
                if (!__any(idle)) break;
                if (idle && nst > 0) write_back(false);   // finished here (nothing to write for one claimed at the target)
                claim(idle);
            }
            CLF_TADD(L, 0, tk_idle);
            if (!__any(inst >= 0)) break;
            const bool act = inst >= 0;
            const long long clk0 = p.iter_log ? wall_clock64() : 0;
            CLF_T(tk_mf);
            // ---- explicit unconstrained solutions of the four instances: Z = V + T_x X on the matrix cores
            T z[NT];
#pragma unroll
            for (int q = 0; q < NT; q++) z[q] = vt[q];
#pragma unroll
            for (int kc = 0; kc < KC; kc++) {
                __builtin_amdgcn_sched_barrier(0);   // one K-chunk's A operands in flight at a time
#pragma unroll
                for (int q = 0; q < NT; q++) z[q] = __builtin_amdgcn_mfma_f64_4x4x4f64(txA[q][kc][lane], xr[kc], z[q], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            CLF_TADD(L, 1, tk_mf);
            CLF_T(tk_bt);
            const int tn = t + 1 == p.period ? 0 : t + 1;
            // ---- bound test and flags (lanes of instance n)
            bool bad = false;
            unsigned long long flm = 0;   // 2 bits per tile
#pragma unroll
            for (int q = 0; q < NT; q++) {
                const double2 lh = lohi[slot_of(q)], ob = onb[slot_of(q)];
                const double zz = (double)z[q];
                bad |= !(zz >= lh.x && zz <= lh.y);   // NaN: bad
                flm |= (unsigned long long)(zz <= ob.x ? 1u : (zz >= ob.y ? 2u : 0u)) << (2 * q);
            }
            const unsigned long long mslot = 0x1111111111111111ull << n;
            const bool slow = act && ((__ballot(bad) & mslot) != 0 || flany);
            const bool fany = (__ballot(flm != 0) & mslot) != 0;
            const bool adv = act && !slow;
            // the demoted: record back, into the queue; their slots refill below
            if (slow) write_back(true);
            // fast instances: flags (slot order, only when some bound is touched), u0 (slots 0..nu-1: tile 0,
            // block 0, lanes 16 i + n) clamped
            if (adv && fany) {
#pragma unroll
                for (int q = 0; q < NT; q++) flb[n][slot_of(q)] = flag_of((unsigned)(flm >> (q >= 16 ? 32 : 0)), q & 15);
            }
            if (adv) flany = fany;
            double u0v = 0.0;
            if (tb == 0 && ti < NU) u0v = fmin(fmax((double)z[0], slb[ti]), sub[ti]);
            CLF_TADD(L, 19, tk_bt);
            CLF_T(tk_out);
            // the trajectory outputs of a fast instance's last step (write_outputs' success branch with an
            // empty set): x_0 the state, the bounded elements z clamped, the unbounded ones from the full tables
            if (p.traj_out && __any(adv && step + 1 == p.target)) {
                double xa[NX];   // the instance's whole state on each of its lanes
#pragma unroll
                for (int c = 0; c < NX; c++) xa[c] = __shfl(xr[c / 4], 16 * (c % 4) + n);
                if (adv && step + 1 == p.target) {
                    if (tb == 0) {
#pragma unroll
                        for (int kc = 0; kc < KC; kc++)
                            if (4 * kc + ti < NX) p.xout[(size_t)inst * (p.N + 1) * NX + 4 * kc + ti] = (T)xr[kc];
                    }
#pragma unroll
                    for (int q = 0; q < NT; q++) {
                        const int s_ = slot_of(q), e = sse[s_];
                        if (e < 0) continue;
                        CLF_CHECK(e < p.ne, 10, e);
                        const T zc = fmin(fmax(z[q], (T)slb[s_]), (T)sub[s_]);
                        const int k = e / NZ, r = e % NZ;
                        if (r < NX) p.xout[((size_t)inst * (p.N + 1) + k) * NX + r] = zc;
                        else p.uout[((size_t)inst * p.N + k) * NU + (r - NX)] = zc;
                    }
                    for (int qf = 4 * tb + ti; qf < p.nfree; qf += 16) {
                        const int e = p.s_free[qf];
                        const T *tr = p.txfull + (size_t)e * NX;
                        T zz = p.vfull[(size_t)t * p.ne + e];
#pragma unroll
                        for (int c = 0; c < NX; c++) zz = fma(tr[c], (T)xa[c], zz);
                        const int k = e / NZ, r = e % NZ;
                        if (r < NX) p.xout[((size_t)inst * (p.N + 1) + k) * NX + r] = zz;
                        else p.uout[((size_t)inst * p.N + k) * NU + (r - NX)] = zz;
                    }
                }
            }
            CLF_TADD(L, 7, tk_out);
            CLF_T(tk_ld);
            // ---- the next step's v (one step ahead), this step's reference row and noise draw
            double w = 0.0;
            if (adv) {
                CLF_CHECK(step - p.step0 >= 0 && step - p.step0 < p.noise_ld, 5, step - p.step0);
                CLF_CHECK(t >= 0 && t < p.period, 6, t);
                w = p.noise[(size_t)inst * p.noise_ld + (step - p.step0)];
            }
            double xrf[KC];
#pragma unroll
            for (int kc = 0; kc < KC; kc++) {
                const int c = 4 * kc + ti;
                xrf[kc] = (adv && tb == 0 && c < NX && (c < p.ncl || c < p.aed_dims)) ? (double)p.table[(size_t)t * p.table_cols + c] : 0.0;
            }
            if (adv && step + 1 < p.target) fetch_v(tn);
            CLF_TADD(L, 18, tk_ld);
            CLF_T(tk_pl);
            // ---- cost (controller.py:40-41) at x_0, or at x_1 (the jerk loop, cost_stage 1: x_1's components
            // are the slots x1_slot + c < 64, z of tile (s >> 4) on lane 16 (s & 3) + 4 ((s >> 2) & 3) + n, clamped
            // as run_instance's z0c), and the AED numerator at x_0: lanes 16 k + n (block 0)
            double xo[KC];
#pragma unroll
            for (int kc = 0; kc < KC; kc++) xo[kc] = xr[kc];
            if constexpr (NX == 6 && NU == 2) {
              if (p.cost_stage != 0) {   // wave-uniform
#pragma unroll
                for (int kc = 0; kc < KC; kc++) {
                    const int c = 4 * kc + ti, s_ = p.x1_slot + (c < NX ? c : 0);
                    const int src = 16 * (s_ & 3) + 4 * ((s_ >> 2) & 3) + n;
                    double v = 0.0;
#pragma unroll
                    for (int q = 0; q < 4 && q < NT; q++) {
                        const double zq = __shfl((double)z[q], src);
                        if ((s_ >> 4) == q) v = zq;
                    }
                    xo[kc] = s_ < NSLOT ? fmin(fmax(v, slb[s_]), sub[s_]) : 0.0;
                }
              }
            }
            if (adv && tb == 0) {
#pragma unroll
                for (int kc = 0; kc < KC; kc++) {
                    const int c = 4 * kc + ti;
                    if (c < NX) {
                        const double e = xo[kc] - xrf[kc];
                        if (c < p.ncl) cost = fma((double)p.wcl[c] * e, e, cost);
                        if (c < p.aed_dims) aed += fabs(xrf[kc] - xr[kc]);
                    }
                }
            }
            if constexpr (NX == 6 && NU == 2) {
                if (p.plant == 2) {
                    // ---- the jerk converter plant (plant_step's arithmetic, src/plant.py): every lane of
                    // instance n evaluates it on the instance's gathered state and inputs
                    double x4[4], f[4];
#pragma unroll
                    for (int c = 0; c < 4; c++) x4[c] = __shfl(xr[0], 16 * c + n);
                    double a0 = __shfl(xr[1], n), a1 = __shfl(xr[1], 16 + n);
                    const double h0 = __shfl(u0v, n), h1 = __shfl(u0v, 16 + n), inv_m = 1.0 / p.mass;
                    for (int j = 0; j < p.substeps; j++) {
                        a0 = a0 + h0 * p.dt_conv;
                        a1 = a1 + h1 * p.dt_conv;
                        crazyflie_rhs(x4, p.mass * a0, p.mass * a1, 1.0, inv_m, p.g, f);
#pragma unroll
                        for (int i = 0; i < 4; i++) x4[i] += p.dt_conv * f[i];
                    }
                    if (adv) {
                        double x0n = 0.0;
#pragma unroll
                        for (int i = 0; i < 4; i++)
                            if (ti == i) x0n = x4[i] + w;
                        xr[0] = x0n;
                        xr[1] = ti == 0 ? a0 : (ti == 1 ? a1 : 0.0);
                    }
                }
            }
            // ---- plant X' = [A B] [X; U] + c + noise on the matrix cores: A operand [A B] (row prow, columns
            // 4 kc + (lane >> 4); the inputs' chunk last) from the workgroup's copy, C = c + noise
            if (p.plant == 0) {
                double d = (drow < NX ? cl[drow] : 0.0) + ((drow < p.noise_dims && drow < NX) ? w : 0.0);
#pragma unroll
                for (int kc = 0; kc < KC; kc++) {
                    const int c = 4 * kc + (lane >> 4);
                    const double a = (prow < NX && c < NX) ? abl[prow * NZ + c] : 0.0;
                    d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, xr[kc], d, 0, 0, 0);
                }
                const double ub = __shfl(u0v, lane & 0x33);   // U[k][n] from lane 16 k + n
#pragma unroll
                for (int ku = 0; ku < KU; ku++) {
                    const int c = 4 * ku + (lane >> 4);
                    const double a = (prow < NX && c < NU) ? abl[prow * NZ + NX + c] : 0.0;
                    d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, ub, d, 0, 0, 0);
                }
                double xn[KC];
#pragma unroll
                for (int kc = 0; kc < KC; kc++) xn[kc] = __shfl(d, (lane & 0x33) | (kc << 2));
                if (adv) {
#pragma unroll
                    for (int kc = 0; kc < KC; kc++) xr[kc] = xn[kc];
                }
            }
            CLF_TADD(L, 8, tk_pl);
            CLF_T(tk_bk);
            // ---- step bookkeeping
            if (adv) {
                nst++;
                last_status = 0;
                if (p.iter_log && lane == n) {
                    const long long kc_ = wall_clock64() - clk0;
                    p.iter_log[(size_t)(step - p.step0) * p.B + inst] = 1 | ((int)(kc_ < 32767 ? kc_ : 32767) << 16);
                }
                step++;
                t = tn;
            }
            CLF_SYNC();
            claim(slow);   // the demoted instances' slots refill
            CLF_TADD(L, 9, tk_bk);
            CLF_TCNT(L, 13, 4);
        }
#ifdef NMPC_CLF_TIMING
        // phase 1's wave totals into the row of the workgroup's instance wg_lo + wave (tools/clf_phases.py sums)
        CLF_SYNC();
        if (p.cycles && lane < CLF_NT && wg_lo + wave < wg_hi) p.cycles[(size_t)(wg_lo + wave) * CLF_NT + lane] += (unsigned long long)L.tacc[lane];
        CLF_SYNC();
        if (lane < CLF_NT) L.tacc[lane] = 0;
#endif
    }
    if (lane == 0) atomicAdd(&ph1_done, 1);
    // phase 2 carries the launch's critical chains (an instance with an active-set step at most steps sets
    // the launch time): its wavefronts issue ahead of the lockstep ones sharing their SIMD (env
    // NMPC_LOCK_PRIO=0: equal priority)
    if (p.lock_prio) __builtin_amdgcn_s_setprio(3);

    // ================= phase 2: the demoted instances, one at a time on the whole wavefront
    for (;;) {
        int got = -1, fin = 0;
        if (lane == 0) {
            for (;;) {
                const int h = __hip_atomic_load(&dq_head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                const int tl = __hip_atomic_load(&dq_tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (h < tl) {
                    if (atomicCAS(&dq_head, h, h + 1) == h) {
                        int v;
                        while ((v = __hip_atomic_load(&dq[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < 0)
                            __builtin_amdgcn_s_sleep(1);
                        got = v;
                        break;
                    }
                    continue;
                }
                if (__hip_atomic_load(&ph1_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == WPB &&
                    __hip_atomic_load(&dq_tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == h) {
                    fin = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        fin = __builtin_amdgcn_readfirstlane(fin);
        if (fin) break;
        const int inst = __builtin_amdgcn_readfirstlane(got);
        CLF_CHECK(inst >= 0 && inst < p.B, 9, inst);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        // explicit form of one instance on the same MFMA tiles: all four B columns the instance's x (L.xs),
        // the n = 0 lanes' results staged to slot order
        run_instance<T, NX, NU, EPL, WSM, SP>(p, L, sv, lane, abl, cl, inst, [&](T(&z)[EPL], const T(&vt)[EPL]) {
            T zq[NT];
#pragma unroll
            for (int q = 0; q < NT; q++) zq[q] = T(0);
#pragma unroll
            for (int kc = 0; kc < KC; kc++) {
                __builtin_amdgcn_sched_barrier(0);
                const double xk = L.xs[4 * kc + (lane >> 4)];
#pragma unroll
                for (int q = 0; q < NT; q++) zq[q] = __builtin_amdgcn_mfma_f64_4x4x4f64(txA[q][kc][lane], xk, zq[q], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            if (n == 0) {
#pragma unroll
                for (int q = 0; q < NT; q++) zb[slot_of(q)] = (double)zq[q];
            }
            CLF_SYNC();
#pragma unroll
            for (int j = 0; j < EPL; j++) z[j] = vt[j] + (T)zb[j * 64 + lane];
            CLF_SYNC();
        }, wcp);
    }
    report_exit(p, lane);
}

}  // namespace clf

int cl_fast_epl(int nx, int nu)
{
    if (nx == 13 && nu == 4) return 4;   // quad13: 251 bounded elements at N = 20
    if (nx == 6 && nu == 2) return 5;    // jerk: 314 at N = 40
    if (nx == 4 && nu == 2) return 2;    // force: 116 at N = 20
    return 0;
}

// largest active set of the fast path per shape (oracle/cref.py WSMAX restates it): the saturating
// force model rides input bounds over long arcs (its closed loop needs up to ~20), quad13 and jerk 16
// (the dual active-set fallback's sets on the bench workloads)
int cl_fast_wsmax(int nx, int nu)
{
    return (nx == 4 && nu == 2) ? 32 : 16;
}

// one compiled variant per shape, as a tag type
template <typename T_, int NX_, int NU_, int EPL_, int WSM_, int WPB_, int MW_, class SP_, bool WL_ = false, bool SW2_ = false>
struct Variant {
    static constexpr int WPB = WPB_;
    static constexpr auto kernel() { return clf::cl_fast_kernel<T_, NX_, NU_, EPL_, WSM_, WPB_, MW_, SP_, WL_, SW2_>; }
};
// the lockstep kernel (four instances per wavefront, MFMA explicit form and plant)
template <typename T_, int NX_, int NU_, int EPL_, int WSM_, int WPB_, int MW_, class SP_>
struct LockVariant {
    static constexpr int WPB = WPB_;
    static constexpr auto kernel() { return clf::cl_lock_kernel<T_, NX_, NU_, EPL_, WSM_, WPB_, MW_, SP_>; }
};

// whether the shape has a lockstep kernel (quad13; jerk, whose plant may be its converter and whose cost may
// sit on x_1: the host checks plant and cost stage)
bool cl_lock_shape(int nx, int nu) { return (nx == 13 && nu == 4) || (nx == 6 && nu == 2); }
bool cl_wlds_shape(int nx, int nu) { return nx == 4 && nu == 2; }
bool cl_one_shape(int nx, int nu) { return nx == 4 && nu == 2; }

// calls f(Variant<...>{}) for the shape's compiled variant; false: none. NMPC_CLF_VARIANT=1 (tuning):
// an occupancy target (quad13 4 waves per SIMD: spills, measured 10 % slower than the default)
template <typename T, class F>
static bool clf_dispatch(int nx, int nu, int sid, int kind, F &&f)
{
    static const int var = std::getenv("NMPC_CLF_VARIANT") ? std::atoi(std::getenv("NMPC_CLF_VARIANT")) : 0;
    // (the force variants come first: the code object emits the kernels in this order, so the force kernels'
    // placement does not move with the other shapes' code sizes)
    if (nx == 4 && nu == 2 && kind != CLF_LOCK) {
        if (kind == CLF_WLDS) f(Variant<T, 4, 2, 2, 32, 4, 0, lpc::DenseStructure<4, 2>, true>{});
        else if (kind == CLF_ONE) f(Variant<T, 4, 2, 2, 32, 4, 0, lpc::DenseStructure<4, 2>, false, true>{});
        else if (var == 1) f(Variant<T, 4, 2, 2, 32, 4, 2, lpc::DenseStructure<4, 2>>{});
        else f(Variant<T, 4, 2, 2, 32, 4, 0, lpc::DenseStructure<4, 2>>{});
        return true;
    }
    if (kind == CLF_LOCK) {   // fp64 only (the f64 MFMA tiles)
        if constexpr (std::is_same<T, double>::value) {
            if (nx == 13 && nu == 4 && sid == lpc::Quad13Structure::id) f(LockVariant<T, 13, 4, 4, 16, 8, 0, lpc::Quad13Structure>{});
            else if (nx == 13 && nu == 4) f(LockVariant<T, 13, 4, 4, 16, 8, 0, lpc::DenseStructure<13, 4>>{});
            // jerk: 20 tiles of z and v_t per lane — one wavefront per SIMD with the whole register file (four
            // per workgroup; B = 4096 is one round of 1024 wavefronts)
            else if (nx == 6 && nu == 2) f(LockVariant<T, 6, 2, 5, 16, 4, 1, lpc::DenseStructure<6, 2>>{});
            else return false;
            return true;
        }
        return false;
    }
    if (nx == 13 && nu == 4 && sid == lpc::Quad13Structure::id) {
        if (var == 1) f(Variant<T, 13, 4, 4, 16, 8, 4, lpc::Quad13Structure>{});
        else f(Variant<T, 13, 4, 4, 16, 8, 0, lpc::Quad13Structure>{});
    } else if (nx == 13 && nu == 4) {
        f(Variant<T, 13, 4, 4, 16, 8, 0, lpc::DenseStructure<13, 4>>{});
    } else if (nx == 6 && nu == 2) {
        f(Variant<T, 6, 2, 5, 16, 8, 0, lpc::DenseStructure<6, 2>>{});
    } else {
        return false;
    }
    return true;
}

// the workgroups of the shape's kernel that `device` holds at once (the persistent grid), queried for
// the given device at nmpc_closed_loop_init and kept on the handle (no process-wide cache)
int cl_fast_resident(int nx, int nu, int sid, int kind, bool f64, int device)
{
    int res = 0;
    auto occ = [&](auto v) {
        using V = decltype(v);
        int per_cu = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, V::kernel(), 64 * V::WPB, 0) != hipSuccess || per_cu < 1) return;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus < 1) return;
        res = per_cu * cus;
    };
    if (f64) clf_dispatch<double>(nx, nu, sid, kind, occ);
    else clf_dispatch<float>(nx, nu, sid, kind, occ);
    return res;
}

// grid: min(workgroups for one wavefront per instance, the resident workgroups)
bool cl_fast_fits(int nx, int nu, int sid, int kind, bool f64, int waves, int resident)
{
    bool fits = false;
    auto g = [&](auto v) {
        using V = decltype(v);
        const int wv = kind == CLF_LOCK ? (waves + 3) / 4 : waves;
        fits = std::min((wv + V::WPB - 1) / V::WPB, resident) * V::WPB >= wv;
    };
    if (f64) clf_dispatch<double>(nx, nu, sid, kind, g);
    else clf_dispatch<float>(nx, nu, sid, kind, g);
    return fits;
}

int cl_fast_grid(int nx, int nu, int sid, int kind, bool f64, int waves, int resident)
{
    int blocks = 0;
    auto g = [&](auto v) {
        using V = decltype(v);
        const int wv = kind == CLF_LOCK ? (waves + 3) / 4 : waves;
        blocks = std::max(1, std::min((wv + V::WPB - 1) / V::WPB, resident));
    };
    if (f64) clf_dispatch<double>(nx, nu, sid, kind, g);
    else clf_dispatch<float>(nx, nu, sid, kind, g);
    return blocks;
}

template <typename T>
hipError_t cl_fast_launch(int nx, int nu, int sid, int kind, const ClFastParams<T> &p, int waves, int resident,
                          hipStream_t s)
{
    const bool ok = clf_dispatch<T>(nx, nu, sid, kind, [&](auto v) {
        using V = decltype(v);
        // the lockstep kernel: four instances per wavefront
        const int wv = kind == CLF_LOCK ? (waves + 3) / 4 : waves;
        const int blocks = std::max(1, std::min((wv + V::WPB - 1) / V::WPB, resident));
        NMPC_LAUNCH(V::kernel(), dim3(blocks), dim3(64 * V::WPB), 0, s, p);
    });
    return ok ? hipGetLastError() : hipErrorInvalidValue;
}

template hipError_t cl_fast_launch<double>(int, int, int, int, const ClFastParams<double> &, int, int, hipStream_t);

namespace clf {
// one workgroup of 1024 threads: each thread a contiguous run of instances; per group the runs' counts, their
// exclusive scan over the workgroup (wavefront scans by shuffles, then the wavefront totals), then every thread
// writes its run's instances at its offsets — the same order as claim_order's three groups, batch-wide
__global__ __launch_bounds__(1024) void clf_order_kernel(const unsigned char *hard, int B, int *gorder)
{
    __shared__ int wtot[16][3];
    __shared__ int gbase[3];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int per = (B + 1023) / 1024, b0 = min(B, t * per), b1 = min(B, b0 + per);
    int c[3] = {0, 0, 0};
    for (int b = b0; b < b1; b++) {
        const int h = hard[b];
        c[h >= 128 ? 0 : (h > 0 ? 1 : 2)]++;
    }
    int x[3];
#pragma unroll
    for (int g = 0; g < 3; g++) {
        int v = c[g];
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int u = __shfl_up(v, o);
            if (lane >= o) v += u;
        }
        x[g] = v - c[g];   // exclusive within the wavefront
        if (lane == 63) wtot[wv][g] = v;
    }
    __syncthreads();
    if (t < 3) {   // the wavefront totals' scan and the groups' bases
        int acc = 0;
        for (int w = 0; w < 16; w++) {
            const int v = wtot[w][t];
            wtot[w][t] = acc;
            acc += v;
        }
        gbase[t] = acc;   // (the group's total for now)
    }
    __syncthreads();
    const int base[3] = {0, gbase[0], gbase[0] + gbase[1]};
    int pos[3];
#pragma unroll
    for (int g = 0; g < 3; g++) pos[g] = base[g] + wtot[wv][g] + x[g];
    for (int b = b0; b < b1; b++) {
        const int h = hard[b], g = h >= 128 ? 0 : (h > 0 ? 1 : 2);
        gorder[pos[g]++] = b;
    }
}
}  // namespace clf

hipError_t clf_order_launch(const unsigned char *hard, int B, int *gorder, hipStream_t s)
{
    NMPC_LAUNCH(clf::clf_order_kernel, dim3(1), dim3(1024), 0, s, hard, B, gorder);
    return hipGetLastError();
}

hipError_t fin32_z0_launch(const Fin32Z0Params &p, hipStream_t s)
{
    if (p.m16 % 16 || p.kp % 4 || p.B < 1) return hipErrorInvalidValue;
    NMPC_LAUNCH(clf::fin32_z0_kernel<4>, dim3((p.B + 15) / 16), dim3(256), 0, s, p);
    return hipGetLastError();
}

// the finish's compiled shapes: the lean loop's slot layouts (one wavefront per instance), with more slots
// per lane for longer horizons (force N <= 20 / 31 / 42, jerk N <= 40 / 56, quad13 N <= 20 / 30)
template <class F>
static bool fin32_dispatch(int nx, int nu, int nslot, F &&f)
{
    if (nx == 13 && nu == 4 && nslot <= 256) f(clf::fin32_kernel<13, 4, 4, 16, 8>, 8);
    else if (nx == 13 && nu == 4 && nslot <= 384) f(clf::fin32_kernel<13, 4, 6, 16, 4>, 4);
    else if (nx == 6 && nu == 2 && nslot <= 320) f(clf::fin32_kernel<6, 2, 5, 16, 8>, 8);
    else if (nx == 6 && nu == 2 && nslot <= 448) f(clf::fin32_kernel<6, 2, 7, 16, 4>, 4);
    else if (nx == 4 && nu == 2 && nslot <= 128) f(clf::fin32_kernel<4, 2, 2, 32, 4>, 4);
    else if (nx == 4 && nu == 2 && nslot <= 192) f(clf::fin32_kernel<4, 2, 3, 32, 4>, 4);
    else if (nx == 4 && nu == 2 && nslot <= 256) f(clf::fin32_kernel<4, 2, 4, 32, 4>, 4);
    else return false;
    return true;
}

int fin32_resident(int nx, int nu, int nslot, int device)
{
    int res = 0;
    fin32_dispatch(nx, nu, nslot, [&](auto k, int wpb) {
        int per_cu = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 64 * wpb, 0) != hipSuccess || per_cu < 1) return;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus < 1) return;
        res = per_cu * cus;
    });
    return res;
}

// the fp64 solve finish's shapes: as fin32 (the lean loop's slot layouts)
template <class F>
static bool fin64_dispatch(int nx, int nu, int nslot, F &&f)
{
    if (nx == 13 && nu == 4 && nslot <= 256) f(clf::fin64_kernel<13, 4, 4, 16, 8>, 8);
    else if (nx == 13 && nu == 4 && nslot <= 384) f(clf::fin64_kernel<13, 4, 6, 16, 4>, 4);
    else if (nx == 6 && nu == 2 && nslot <= 320) f(clf::fin64_kernel<6, 2, 5, 16, 8>, 8);
    else if (nx == 6 && nu == 2 && nslot <= 448) f(clf::fin64_kernel<6, 2, 7, 16, 4>, 4);
    else if (nx == 4 && nu == 2 && nslot <= 128) f(clf::fin64_kernel<4, 2, 2, 32, 4>, 4);
    else if (nx == 4 && nu == 2 && nslot <= 192) f(clf::fin64_kernel<4, 2, 3, 32, 4>, 4);
    else if (nx == 4 && nu == 2 && nslot <= 256) f(clf::fin64_kernel<4, 2, 4, 32, 4>, 4);
    else return false;
    return true;
}

int fin64_resident(int nx, int nu, int nslot, int device)
{
    int res = 0;
    fin64_dispatch(nx, nu, nslot, [&](auto k, int wpb) {
        int per_cu = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 64 * wpb, 0) != hipSuccess || per_cu < 1) return;
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus < 1) return;
        res = per_cu * cus;
    });
    return res;
}

// grid: the resident workgroups, at most one per wpb instances of the batch. The list's length is known on the device
// only (sf_kernel fills it on the same stream), so the grid covers the longest list the persistent loop may meet;
// workgroups past the list's end return before any setup. hipErrorInvalidValue: no compiled finish for the shape
hipError_t fin64_launch(int nx, int nu, const ClFastParams<double> &p, int resident, hipStream_t s)
{
    hipError_t e = hipErrorInvalidValue;
    fin64_dispatch(nx, nu, p.nslot, [&](auto k, int wpb) {
        const int blocks = std::max(1, std::min((p.B + wpb - 1) / wpb, resident));
        NMPC_LAUNCH(k, dim3(blocks), dim3(64 * wpb), 0, s, p);
        e = hipGetLastError();
    });
    return e;
}

bool fin32_launch(int nx, int nu, int, const ClFastParams<float> &p, int resident, hipStream_t s)
{
    return fin32_dispatch(nx, nu, p.nslot, [&](auto k, int wpb) {
        const int blocks = std::max(1, std::min((p.B + wpb - 1) / wpb, resident));
        NMPC_LAUNCH(k, dim3(blocks), dim3(64 * wpb), 0, s, p);
    });
}
template hipError_t cl_fast_launch<float>(int, int, int, int, const ClFastParams<float> &, int, int, hipStream_t);

}  // namespace nmpc
