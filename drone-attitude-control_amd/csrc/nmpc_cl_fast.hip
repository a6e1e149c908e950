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
//     unconstrained problem (z = z_0 + W[:, S] nu, W_SS nu = b_S - z_0,S, sets of <= WSMAX bounds,
//     KKT acceptance with the multiplier signs measured as displacements nu_i W_ii);
//   * a QP the interval certificate proves infeasible returns status 4 with the initial point's
//     inputs (the lane-per-component kernel's failure output);
//   * anything else is parked: the instance stops, and the host runs one full solve (IPM + exact
//     finish, ipm_lpc_kernel in list mode) for every parked instance before the next round.
//
// Layout: only the bounded elements of z matter for the test (quad13: 251 of 357), so the wavefront's
// 64 lanes own them in "slots" s = j * 64 + lane (j < EPL, stage-major order: stage 0's inputs are
// slots 0..nu-1, stage 1's bounded elements follow). Each lane keeps its slots' T_x rows, bounds and
// element indices in registers for the whole launch (loaded once per wavefront), so a step costs one
// coalesced load of the window's v_t slots, EPL x nx FMAs per lane and a few wave reductions; the
// state, the plant step and the sums are wave-uniform. No per-step stores: the solution's active flags
// stay in a register mask, the trajectory outputs are written once, at the instance's last step.
// The unbounded elements (quaternions, the terminal stage) are formed only for those outputs.

#include <hip/hip_runtime.h>

#include "nmpc_cl_device.h"
#include "nmpc_internal.h"
#include "nmpc_lpc_geom.h"

namespace nmpc {
namespace clf {

constexpr int WSMAX = 8;   // largest active set of the fast path (the lane-per-component kernel's)
constexpr int WPB = 4;     // wavefronts per workgroup

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

__device__ __forceinline__ unsigned long long ballot(bool b) { return __ballot(b); }

// per-wavefront LDS: active flags by slot (the warm-start shift), the set of an active-set step
// (element, sign, target b - z_0, multiplier), the per-component argmax of the violated states, and
// the certificate's stage exchange
template <int NSLOT, int NZ>
struct Lds {
    double zb[NSLOT];          // z_0 into / z out of the active-set steps
    signed char fl[NSLOT];     // flags: the warm-start shift buffer; the active-set steps' set
    double se_t[WSMAX], se_nu[WSMAX], wdg[WSMAX], wss[WSMAX][WSMAX];
    int se_e[WSMAX], se_s[WSMAX];
    unsigned long long vmax[NZ];
    int vslot[NZ];
    double cm[32], cr[32], xs[32];   // certificate exchange; x_0 for the certificate and the outputs
};

// the workgroup's slot constants (LDS), seen from one lane: slot j of this lane is j * 64 + lane
template <int EPL>
struct SlotView {
    const double *lb_, *ub_;
    const int *e_, *src_;
    int lane;
    __device__ double lb(int j) const { return lb_[j * 64 + lane]; }
    __device__ double ub(int j) const { return ub_[j * 64 + lane]; }
    __device__ int e(int j) const { return e_[j * 64 + lane]; }
    __device__ int src(int j) const { return src_[j * 64 + lane]; }
};

// 2-bit flags of a per-lane mask (bit 2j lower, 2j+1 upper) <-> -1 / 0 / 1
__device__ __forceinline__ signed char flag_of(unsigned m, int j)
{
    const unsigned b = (m >> (2 * j)) & 3u;
    return b == 1u ? (signed char)-1 : (b == 2u ? (signed char)1 : (signed char)0);
}
__device__ __forceinline__ unsigned bits_of(signed char f) { return f < 0 ? 1u : (f > 0 ? 2u : 0u); }

// a bound violated beyond the fast path's 1e-13 (relative to 1 + |b|)
template <typename T>
__device__ __forceinline__ bool violated(T z, T l, T u)
{
    return (has_b(l) && z < l - T(1e-13) * (T(1) + fabs(l))) || (has_b(u) && z > u + T(1e-13) * (T(1) + fabs(u)));
}

#define CLF_SYNC()                                               \
    do {                                                         \
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   \
        __builtin_amdgcn_wave_barrier();                         \
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   \
    } while (0)

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

// Primal-dual active-set steps on W (oracle/c/riccati_ipm.c fast_finish; the lane-per-component
// kernel's W steps): wf holds the set (warm start, or empty: the first set from z_0's violations —
// the violated inputs and each state component's most violated stage). Each round solves
// W_SS nu = b_S - z_0,S (Cholesky on every lane, the set broadcast through LDS, W_SS by wave-uniform
// loads), sets z = z_0 + W[:, S] nu at the lane's slots and accepts when the held bounds are met
// (1e-9), no other bound is violated (1e-13) and every multiplier has its sign (displacement nu_i W_ii
// to 1e-10 (1 + |b - z_0|)); otherwise removals and additions as the finish's PDAS rule. An emptied
// set restarts from z_0 (one round). false: set larger than WSMAX, W_SS not positive definite, or no
// acceptance in polish_steps rounds.
template <typename T, int NX, int NU, int EPL, class LdsT>
__device__ int wsteps_run(const ClFastParams<T> &p, LdsT &L, const SlotView<EPL> sv, int lane)
{
    constexpr int NZ = NX + NU;
    const int ne = p.ne;
    int se[EPL], sr[EPL], wsteps = 0;
    T lb[EPL], ub[EPL], z0[EPL], z[EPL];
    unsigned wf = 0;
#pragma unroll
    for (int j = 0; j < EPL; j++) {
        se[j] = sv.e(j);
        sr[j] = se[j] >= 0 ? se[j] % NZ : -1;
        lb[j] = (T)sv.lb(j);
        ub[j] = (T)sv.ub(j);
        z0[j] = (T)L.zb[j * 64 + lane];
        wf |= bits_of(L.fl[j * 64 + lane]) << (2 * j);
    }
    auto done = [&](int m) {   // accepted: z to LDS; result word ok | m << 8 | steps << 16
#pragma unroll
        for (int j = 0; j < EPL; j++) L.zb[j * 64 + lane] = (double)z[j];
        CLF_SYNC();
        return 1 | (m << 8) | (wsteps << 16);
    };
    // per state component: the most violated slot (argmax by LDS atomics, ties to the first stage)
    auto argmax_states = [&](const double (&v)[EPL]) {
        if (lane < NZ) {
            L.vmax[lane] = 0ull;
            L.vslot[lane] = 0x7fffffff;
        }
        CLF_SYNC();
#pragma unroll
        for (int j = 0; j < EPL; j++)
            if (sr[j] >= 0 && sr[j] < NX && v[j] > 0.0) atomicMax(&L.vmax[sr[j]], __builtin_bit_cast(unsigned long long, v[j]));
        CLF_SYNC();
#pragma unroll
        for (int j = 0; j < EPL; j++)
            if (sr[j] >= 0 && sr[j] < NX && v[j] > 0.0 && __builtin_bit_cast(unsigned long long, v[j]) == L.vmax[sr[j]])
                atomicMin(&L.vslot[sr[j]], se[j]);
        CLF_SYNC();
    };
    for (int ws = 0, first = 1; ws < p.polish_steps; first = 0) {
        unsigned long long bal[EPL];
        int m = 0;
#pragma unroll
        for (int j = 0; j < EPL; j++) {
            bal[j] = __ballot(((wf >> (2 * j)) & 3u) != 0);
            m += __popcll(bal[j]);
        }
        if (m == 0) {
            // no bound held: the iterate is z_0 — accepted if feasible, else the set from its violations
            if (!first) ws++;
            bool bad = false;
            double v[EPL];
            unsigned sgn = 0;
#pragma unroll
            for (int j = 0; j < EPL; j++) {
                const T tl = T(1e-13) * (T(1) + fabs(lb[j])), tu = T(1e-13) * (T(1) + fabs(ub[j]));
                const bool lo = has_b(lb[j]) && z0[j] < lb[j] - tl, hi = has_b(ub[j]) && z0[j] > ub[j] + tu;
                bad |= lo || hi || (se[j] >= 0 && !isfinite(z0[j]));
                v[j] = lo ? (double)(lb[j] - z0[j]) : (hi ? (double)(z0[j] - ub[j]) : 0.0);
                sgn |= (lo ? 1u : (hi ? 2u : 0u)) << (2 * j);
                if (sr[j] >= NX && (lo || hi)) wf |= (lo ? 1u : 2u) << (2 * j);   // inputs join at once
            }
            if (!__any(bad)) {
#pragma unroll
                for (int j = 0; j < EPL; j++) z[j] = z0[j];
                return done(0);
            }
            argmax_states(v);
#pragma unroll
            for (int j = 0; j < EPL; j++)
                if (sr[j] >= 0 && sr[j] < NX && v[j] > 0.0 && L.vslot[sr[j]] == se[j]) wf |= ((sgn >> (2 * j)) & 3u) << (2 * j);
            CLF_SYNC();
            continue;
        }
        if (m > WSMAX) return wsteps << 16;
        // the set in LDS: element, sign, b - z_0
        int base = 0;
#pragma unroll
        for (int j = 0; j < EPL; j++) {
            const unsigned f = (wf >> (2 * j)) & 3u;
            if (f) {
                const int pos = base + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bal[j] >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal[j], 0u));
                L.se_e[pos] = se[j];
                L.se_s[pos] = f == 1u ? -1 : 1;
                L.se_t[pos] = (double)((f == 1u ? lb[j] : ub[j]) - z0[j]);
            }
            base += __popcll(bal[j]);
        }
        CLF_SYNC();
        // W_SS in LDS, entry (i, j) on lane 8 i + j; right-looking Cholesky (the lower triangle), then
        // the triangular solves for nu on every lane from LDS (wave-uniform reads)
        {
            const int i = lane >> 3, j = lane & 7;
            const bool in = i < m && j < m && j <= i;
            const double wij = in ? (double)p.W[(size_t)L.se_e[j] * ne + L.se_e[i]] : 0.0;
            L.wss[i][j] = wij;
            if (in && i == j) L.wdg[i] = wij;
        }
        CLF_SYNC();
        bool pd = true;
        for (int c = 0; c < m; c++) {
            const double d = L.wss[c][c];
            pd = pd && d > 0.0;
            const double lcc = d > 0.0 ? sqrt(d) : 1.0;
            const int i = lane >> 3, j = lane & 7;
            CLF_SYNC();
            if (j == c && i >= c && i < m) L.wss[i][c] = i == c ? lcc : L.wss[i][c] / lcc;
            CLF_SYNC();
            if (j > c && j <= i && i < m) L.wss[i][j] -= L.wss[i][c] * L.wss[j][c];
            CLF_SYNC();
        }
        if (!pd) return wsteps << 16;
        // nu = L^-T L^-1 (b - z_0)_S into L.se_nu (lane 0 writes, every lane reads; m <= WSMAX rows)
#pragma unroll 1
        for (int i = 0; i < m; i++) {
            double s_ = L.se_t[i];
#pragma unroll 1
            for (int l = 0; l < i; l++) s_ = fma(-L.wss[i][l], L.se_nu[l], s_);
            CLF_SYNC();
            if (lane == 0) L.se_nu[i] = s_ / L.wss[i][i];
            CLF_SYNC();
        }
#pragma unroll 1
        for (int i = m - 1; i >= 0; i--) {
            double s_ = L.se_nu[i];
#pragma unroll 1
            for (int l = i + 1; l < m; l++) s_ = fma(-L.wss[l][i], L.se_nu[l], s_);
            CLF_SYNC();
            if (lane == 0) L.se_nu[i] = s_ / L.wss[i][i];
            CLF_SYNC();
        }
        const int round = ws++;
        wsteps++;
        // multiplier signs as displacements nu_i W_ii (lower: >= 0, upper: <= 0) to 1e-10 (1 + |b - z_0|)
        unsigned remm = 0;
#pragma unroll 1
        for (int i = 0; i < m; i++) {
            const double nui = L.se_nu[i], tol = 1e-10 * (1.0 + fabs(L.se_t[i])), dsp = nui * L.wdg[i];
            const int sg = L.se_s[i];
            if ((sg < 0 && dsp < -tol) || (sg > 0 && dsp > tol) || !isfinite(nui)) remm |= 1u << i;
        }
        const int nrem = __popc(remm);
        const bool addok = round == 0 || nrem == 0;
        bool bad = nrem > 0;
        double v[EPL];
        unsigned sgn = 0, nwf = wf;
#pragma unroll
        for (int j = 0; j < EPL; j++) {
            v[j] = 0.0;
            if (se[j] < 0) {
                z[j] = z0[j];
                continue;
            }
            T zz = z0[j];
#pragma unroll 1
            for (int i = 0; i < m; i++) zz = fma(p.W[(size_t)L.se_e[i] * ne + se[j]], (T)L.se_nu[i], zz);
            const unsigned f = (wf >> (2 * j)) & 3u;
            if (f) {
                const T bb = f == 1u ? lb[j] : ub[j];
                bad |= !(fabs(zz - bb) <= T(1e-9) * (T(1) + fabs(bb)));
                zz = bb;
#pragma unroll 1
                for (int i = 0; i < m; i++)
                    if (((remm >> i) & 1u) && L.se_e[i] == se[j]) nwf &= ~(3u << (2 * j));
            } else {
                const T tl = T(1e-13) * (T(1) + fabs(lb[j])), tu = T(1e-13) * (T(1) + fabs(ub[j]));
                const bool lo = has_b(lb[j]) && zz < lb[j] - tl, hi = has_b(ub[j]) && zz > ub[j] + tu;
                bad |= lo || hi || !isfinite(zz);
                v[j] = lo ? (double)(lb[j] - zz) : (hi ? (double)(zz - ub[j]) : 0.0);
                sgn |= (lo ? 1u : (hi ? 2u : 0u)) << (2 * j);
                if (sr[j] >= NX && (lo || hi)) nwf |= (lo ? 1u : 2u) << (2 * j);   // inputs join at once
            }
            z[j] = zz;
        }
        if (!__any(bad)) return done(m);
        if (addok) {
            argmax_states(v);
#pragma unroll
            for (int j = 0; j < EPL; j++)
                if (sr[j] >= 0 && sr[j] < NX && v[j] > 0.0 && L.vslot[sr[j]] == se[j]) nwf |= ((sgn >> (2 * j)) & 3u) << (2 * j);
        }
        wf = nwf;
        CLF_SYNC();
    }
    return wsteps << 16;
}

// interval certificate (oracle/c/riccati_ipm.c infeasible_stage): lane i < NX carries state i of
// X_k in midpoint / radius form, X_{k+1} = hull([A B] X_k x U + c) meets the state box of stage
// k + 1; an empty intersection proves the QP infeasible
template <typename T, int NX, int NU, class LdsT>
__device__ bool certificate_infeasible(const ClFastParams<T> &p, LdsT &L, int lane)
{
    // x_0 in L.xs (the caller's copy)
    constexpr int NZ = NX + NU;
    T m = lane < NX ? (T)L.xs[lane] : T(0), r = 0;
    T mu[NU], ru[NU];
#pragma unroll
    for (int j = 0; j < NU; j++) {
        const T l = p.lbnd[NX + j], h = p.ubnd[NX + j];
        const bool bb = has_b(l) && has_b(h);
        mu[j] = bb ? T(0.5) * (l + h) : T(0);
        ru[j] = bb ? T(0.5) * (h - l) : T(INFINITY);
    }
    bool infeas = false;
    const int i = lane < NX ? lane : 0;
    for (int k = 0; k < p.N; k++) {
        if (lane < NX) {
            L.cm[lane] = (double)m;
            L.cr[lane] = (double)r;
        }
        CLF_SYNC();
        T s = p.c[i], tr = 0;
#pragma unroll
        for (int j = 0; j < NX; j++) {
            const T a = p.AB[i * NZ + j];
            s = fma(a, (T)L.cm[j], s);
            if (a != T(0)) tr = fma(fabs(a), (T)L.cr[j], tr);
        }
#pragma unroll
        for (int j = 0; j < NU; j++) {
            const T b = p.AB[i * NZ + NX + j];
            s = fma(b, mu[j], s);
            if (b != T(0)) tr = fma(fabs(b), ru[j], tr);
        }
        CLF_SYNC();
        const int ty = k + 1 == p.N ? 2 : 1;
        const T lb = p.lbnd[ty * NZ + i], ub = p.ubnd[ty * NZ + i];
        T lo = s - tr, hi = s + tr;
        if (has_b(lb) && lb > lo) lo = lb;
        if (has_b(ub) && ub < hi) hi = ub;
        infeas |= lane < NX && lo > hi + T(1e-9) * (T(1) + fabs(hi));
        const bool fin = isfinite(lo) && isfinite(hi);
        m = fin ? T(0.5) * (lo + hi) : s;
        r = fin ? T(0.5) * (hi - lo) : tr;
    }
    return __any(infeas);
}

// plant step + noise on the wave-uniform state (nmpc_cl_device.h cl_advance_group's arithmetic):
// plant 0 the controller's own discrete model [A B] (structure SP), 1 / 2 the Crazyflie plant with
// the force / jerk converter
template <typename T, int NX, int NU, class SP>
__device__ __forceinline__ void plant_step(const ClFastParams<T> &p, const double *abl, const double *cl, T (&x)[NX],
                                           const double (&u0)[NU], double w)
{
    constexpr int NZ = NX + NU;
    if (p.plant == 0) {
        // [A B] and c from the workgroup's LDS copy (wave-uniform reads; kept out of SGPRs)
        T xn[NX];
#pragma unroll
        for (int i = 0; i < NX; i++) {
            double s = cl[i];
#pragma unroll
            for (int j = 0; j < NX; j++)
                if (SP::ab(i, j)) s += abl[i * NZ + j] * (double)x[j];
#pragma unroll
            for (int j = 0; j < NU; j++)
                if (SP::ab(i, NX + j)) s += abl[i * NZ + NX + j] * u0[j];
            xn[i] = (T)(s + (i < p.noise_dims ? w : 0.0));
        }
#pragma unroll
        for (int i = 0; i < NX; i++) x[i] = xn[i];
    } else if constexpr ((NX == 4 && NU == 2) || (NX == 6 && NU == 2)) {
        double xs[4], f[4];
#pragma unroll
        for (int i = 0; i < 4; i++) xs[i] = (double)x[i];
        const double inv_m = 1.0 / p.mass;
        if (NX == 4) {
            const double Fx = u0[0], Fz = u0[1];
            const double th = atan2(Fx, Fz), Fd = sqrt(Fx * Fx + Fz * Fz);
            const double s_ = sin(th), c_ = cos(th), h = p.dt;
            double k1[4], k2[4], k3[4], k4[4], tt[4];
            crazyflie_rhs(xs, s_, c_, Fd, inv_m, p.g, k1);
            for (int i = 0; i < 4; i++) tt[i] = xs[i] + 0.5 * h * k1[i];
            crazyflie_rhs(tt, s_, c_, Fd, inv_m, p.g, k2);
            for (int i = 0; i < 4; i++) tt[i] = xs[i] + 0.5 * h * k2[i];
            crazyflie_rhs(tt, s_, c_, Fd, inv_m, p.g, k3);
            for (int i = 0; i < 4; i++) tt[i] = xs[i] + h * k3[i];
            crazyflie_rhs(tt, s_, c_, Fd, inv_m, p.g, k4);
            for (int i = 0; i < 4; i++) xs[i] += h / 6.0 * (k1[i] + 2.0 * k2[i] + 2.0 * k3[i] + k4[i]);
            for (int i = 0; i < 4; i++) x[i] = (T)(xs[i] + w);
        } else {
            double a0 = (double)x[4 % NX], a1 = (double)x[5 % NX];
            const double h0 = u0[0], h1 = u0[1];
            for (int j = 0; j < p.substeps; j++) {
                a0 = a0 + h0 * p.dt_conv;
                a1 = a1 + h1 * p.dt_conv;
                const double Fx = p.mass * a0, Fz = p.mass * a1;
                const double th = atan2(Fx, Fz), Fd = sqrt(Fx * Fx + Fz * Fz);
                crazyflie_rhs(xs, sin(th), cos(th), Fd, inv_m, p.g, f);
                for (int i = 0; i < 4; i++) xs[i] += p.dt_conv * f[i];
            }
            for (int i = 0; i < 4; i++) x[i] = (T)(xs[i] + w);
            x[4 % NX] = (T)a0;
            x[5 % NX] = (T)a1;
        }
    }
}

// trajectory outputs of an instance's last solve (lanes over the (N+1) nz elements): z_0 from the
// full tables plus the accepted active-set step (LDS), held bounds exact, bounded elements clamped;
// a failed last step (status 4) outputs the initial point
template <typename T, int NX, int NU, int EPL, class LdsT>
__device__ void write_outputs(const ClFastParams<T> &p, LdsT &L, int lane, int inst, int t, int status, int m)
{
    // x_0 in L.xs (the caller's copy)
    constexpr int NZ = NX + NU;
    const int N = p.N, ne = p.ne;
    T x0[NX];
#pragma unroll
    for (int c = 0; c < NX; c++) x0[c] = (T)L.xs[c];
#pragma unroll 1
    for (int e = lane; e < ne; e += 64) {
        const int k = e / NZ, r = e % NZ;
        if (k == N && r >= NX) continue;
        T x0r = 0;
#pragma unroll
        for (int c = 0; c < NX; c++)
            if (c == r) x0r = x0[c];
        const int ty = k == 0 ? 0 : (k == N ? 2 : 1);
        const T lb = p.lbnd[ty * NZ + r], ub = p.ubnd[ty * NZ + r];
        T z;
        if (status != 0) {
            z = init_point(p, NX, NZ, k, r, t, x0r);
        } else if (k == 0 && r < NX) {
            z = x0r;
        } else {
            const T *tr = p.txfull + (size_t)e * NX;
            T s0 = p.vfull[(size_t)t * ne + e], s1 = 0;
#pragma unroll
            for (int c = 0; c + 1 < NX; c += 2) {
                s0 = fma(tr[c], x0[c], s0);
                s1 = fma(tr[c + 1], x0[c + 1], s1);
            }
            if (NX % 2) s0 = fma(tr[NX - 1], x0[NX - 1], s0);
            z = s0 + s1;
            int held = 0;
            for (int i = 0; i < m; i++) {
                z = fma(p.W[(size_t)L.se_e[i] * ne + e], (T)L.se_nu[i], z);
                if (L.se_e[i] == e) held = L.se_s[i];
            }
            if (held) z = held < 0 ? lb : ub;
            if (has_b(lb)) z = fmax(z, lb);
            if (has_b(ub)) z = fmin(z, ub);
        }
        if (r < NX) p.xout[((size_t)inst * (N + 1) + k) * NX + r] = z;
        else p.uout[((size_t)inst * N + k) * NU + (r - NX)] = z;
    }
}

template <typename T, int NX, int NU, int EPL, class SP>
__global__ __launch_bounds__(64 * WPB) void cl_fast_kernel(ClFastParams<T> p)
{
    constexpr int NZ = NX + NU, NSLOT = EPL * 64;
    __shared__ Lds<NSLOT, NZ> lds_all[WPB];
    // workgroup constants: [A B], c (plant), the slots' bounds, elements and warm-start sources
    __shared__ double abl[NX * NZ], cl[NX], slb[NSLOT], sub[NSLOT];
    __shared__ int sse[NSLOT], ssrc[NSLOT];
    // the slots' T_x rows, component-major (txl[c][s]: lanes read consecutive words, no bank conflicts),
    // shared by the workgroup's wavefronts — registers stay free for occupancy
    // pairs of components per 16-byte word (txl[c / 2][s] = (T_x(s, c), T_x(s, c + 1))): one ds_read_b128
    // per slot and pair
    constexpr int NXP = (NX + 1) / 2;
    __shared__ double2 txl[NXP][NSLOT];
    for (int e = threadIdx.x; e < NXP * NSLOT; e += 64 * WPB) {
        const int c = e / NSLOT, s_ = e % NSLOT;
        const bool v = s_ < p.nslot;
        txl[c][s_] = make_double2(v ? (double)p.s_tx[(size_t)s_ * NX + 2 * c] : 0.0,
                                  v && 2 * c + 1 < NX ? (double)p.s_tx[(size_t)s_ * NX + 2 * c + 1] : 0.0);
    }
    for (int e = threadIdx.x; e < NX * NZ; e += 64 * WPB) abl[e] = (double)p.AB[e];
    for (int e = threadIdx.x; e < NX; e += 64 * WPB) cl[e] = (double)p.c[e];
    for (int s = threadIdx.x; s < NSLOT; s += 64 * WPB) {
        const bool v = s < p.nslot;
        slb[s] = v ? (double)p.s_lb[s] : -1e30;
        sub[s] = v ? (double)p.s_ub[s] : 1e30;
        sse[s] = v ? p.s_e[s] : -1;
        ssrc[s] = v ? p.s_src[s] : -1;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    Lds<NSLOT, NZ> &L = lds_all[wave];
    const int gw = blockIdx.x * WPB + wave, nw = gridDim.x * WPB;
    const SlotView<EPL> sv{slb, sub, sse, ssrc, lane};

    const int nref = p.ncl > p.aed_dims ? p.ncl : p.aed_dims;   // reference components of cost / AED

    for (int inst = gw; inst < p.B; inst += nw) {
        int step = p.istep[inst];
        if (step >= p.target) continue;
        T x[NX];
#pragma unroll
        for (int c = 0; c < NX; c++) x[c] = p.state[(size_t)inst * NX + c];
        // active flags of the last solution by slot: bit 2j lower, 2j+1 upper
        unsigned fl = 0;
        if (step > 0) {
#pragma unroll
            for (int j = 0; j < EPL; j++) {
                const int s = j * 64 + lane;
                const signed char f = s < p.nslot ? p.flags[(size_t)inst * p.nslot + s] : 0;
                fl |= (f < 0 ? 1u : (f > 0 ? 2u : 0u)) << (2 * j);
            }
        }
        int t = (int)(((long long)p.offset[inst] + step) % p.period);
        double cost = 0.0, aed = 0.0, nfail = 0.0, nst = 0.0;
        int last_status = 0, last_iters = 0;
        bool parked = false;
        // v_t at the slots one step ahead (the step's first dependency); the reference row and the noise
        // draw are issued at the top of the step and consumed after the solve
        constexpr int NR = NX < 8 ? NX : 8;   // reference components of cost / AED (nmpc_closed_loop_init: <= 8)
        T vtn[EPL];
        auto fetch_v = [&](int tt) {
            const T *vp = p.vb + (size_t)tt * NSLOT;
#pragma unroll
            for (int j = 0; j < EPL; j++) vtn[j] = vp[j * 64 + lane];
        };
        fetch_v(t);
        for (; step < p.target; step++) {
            T vt[EPL], xr[NR];
#pragma unroll
            for (int j = 0; j < EPL; j++) vt[j] = vtn[j];
            const int tn = t + 1 == p.period ? 0 : t + 1;
            if (step + 1 < p.target) fetch_v(tn);
            {
                const T *xp = p.table + (size_t)t * p.table_cols;
#pragma unroll
                for (int i = 0; i < NR; i++) xr[i] = i < nref ? xp[i] : T(0);
            }
            const double w = p.noise[(size_t)inst * p.noise_ld + (step - p.step0)];
            // ---- warm start: the last solution's flags shifted by one stage (slot source)
            unsigned wf = 0;
            if (__any(fl != 0)) {
#pragma unroll
                for (int j = 0; j < EPL; j++) L.fl[j * 64 + lane] = flag_of(fl, j);
                CLF_SYNC();
#pragma unroll
                for (int j = 0; j < EPL; j++) {
                    const int sr_ = sv.src(j);
                    wf |= bits_of(sr_ >= 0 ? L.fl[sr_] : (signed char)0) << (2 * j);
                }
                CLF_SYNC();
            }
            // ---- explicit unconstrained solution at the lane's slots
            T z[EPL], z1[EPL];
#pragma unroll
            for (int j = 0; j < EPL; j++) {
                z[j] = vt[j];
                z1[j] = T(0);
            }
            // x in LDS for the rolled pair loop (its component pair is wave-uniform)
#pragma unroll
            for (int c = 0; c < NX; c++)
                if (lane == c) L.xs[c] = (double)x[c];
            if (lane == NX) L.xs[NX] = 0.0;
            CLF_SYNC();
#pragma unroll 1
            for (int c = 0; c < NXP; c++) {
                const double xa = L.xs[2 * c], xb = L.xs[2 * c + 1];
#pragma unroll
                for (int j = 0; j < EPL; j++) {
                    const double2 tt = txl[c][j * 64 + lane];
                    z[j] = fma((T)tt.x, (T)xa, z[j]);
                    z1[j] = fma((T)tt.y, (T)xb, z1[j]);
                }
            }
#pragma unroll
            for (int j = 0; j < EPL; j++) z[j] += z1[j];
            bool ok = false;
            int status = 0, iters = 1, m_acc = 0;
            if (!__any(wf != 0)) {
                bool bad = false;
#pragma unroll
                for (int j = 0; j < EPL; j++) bad |= violated(z[j], (T)sv.lb(j), (T)sv.ub(j)) || !isfinite(z[j]);
                ok = !__any(bad);
            }
            if (!ok) {
                // ---- active-set steps on W (rare), the set and z_0 / z through LDS
#pragma unroll
                for (int j = 0; j < EPL; j++) {
                    L.zb[j * 64 + lane] = (double)z[j];
                    L.fl[j * 64 + lane] = flag_of(wf, j);
                }
                CLF_SYNC();
                const int r = wsteps_run<T, NX, NU, EPL>(p, L, sv, lane);
                ok = (r & 1) != 0;
                m_acc = ok ? (r >> 8) & 0xff : 0;
                iters = 1 + (r >> 16);
                if (ok) {
#pragma unroll
                    for (int j = 0; j < EPL; j++) z[j] = (T)L.zb[j * 64 + lane];
                } else {
                    // ---- interval certificate (oracle/c/riccati_ipm.c infeasible_stage)
#pragma unroll
                    for (int c = 0; c < NX; c++)
                        if (lane == c) L.xs[c] = (double)x[c];
                    CLF_SYNC();
                    if (certificate_infeasible<T, NX, NU>(p, L, lane)) {
                        status = 4;
                        iters = 0;
                    } else {
                        parked = true;
                        break;
                    }
                }
            }
            // ---- the solution's active flags (z on a bound to 1e-7): the next step's warm start
            fl = 0;
            if (status == 0) {
#pragma unroll
                for (int j = 0; j < EPL; j++) {
                    const T l = (T)sv.lb(j), u = (T)sv.ub(j);
                    const bool onl = has_b(l) && z[j] <= l + T(1e-7) * (T(1) + fabs(l));
                    const bool onu = has_b(u) && z[j] >= u - T(1e-7) * (T(1) + fabs(u));
                    fl |= (onl ? 1u : (onu ? 2u : 0u)) << (2 * j);
                }
            }
            // ---- u0 (slots 0..nu-1: lanes 0..nu-1 of j = 0), clamped onto its bound
            const T z0c = fmin(fmax(z[0], (T)sv.lb(0)), (T)sv.ub(0));
            double u0[NU];
#pragma unroll
            for (int i = 0; i < NU; i++) u0[i] = status == 0 ? bcast((double)z0c, i) : (double)p.uinit[i];
            // ---- cost (controller.py:40-41) at x_0 = the state, or x_1 (jerk loop), and the AED numerator
            double cc = 0.0, aa = 0.0;
#pragma unroll
            for (int i = 0; i < NR; i++) {
                if (i < p.ncl) {
                    double xo = (double)x[i];
                    if (p.cost_stage != 0) {
                        xo = status == 0 ? bcast((double)z0c, p.x1_slot + i) : (double)init_point(p, NX, NZ, 1, i, t, T(0));
                    }
                    const double e = xo - (double)xr[i];
                    cc += (double)p.wcl[i] * e * e;
                }
                if (i < p.aed_dims) aa += fabs((double)xr[i] - (double)x[i]);
            }
            cost += cc;
            aed += aa;
            nfail += status != 0 ? 1.0 : 0.0;
            nst += 1.0;
            last_status = status;
            last_iters = iters;
            // ---- the trajectory outputs of the instance's last step of the run
            if (step + 1 == p.target) {
#pragma unroll
                for (int c = 0; c < NX; c++)
                    if (lane == c) L.xs[c] = (double)x[c];
                CLF_SYNC();
                write_outputs<T, NX, NU, EPL>(p, L, lane, inst, t, status, m_acc);
            }
            // ---- plant step + noise
            plant_step<T, NX, NU, SP>(p, abl, cl, x, u0, w);
            t = tn;
        }
        // ---- write back: state, sums, step, flags, status
        if (lane == 0) {
#pragma unroll
            for (int c = 0; c < NX; c++) p.state[(size_t)inst * NX + c] = x[c];
            double *a = p.acc + (size_t)inst * 4;
            a[0] += cost;
            a[1] += aed;
            a[2] += nfail;
            a[3] += nst;
            p.istep[inst] = step;
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
    }
}

}  // namespace clf

int cl_fast_epl(int nx, int nu)
{
    if (nx == 13 && nu == 4) return 4;   // quad13: 251 bounded elements at N = 20
    if (nx == 6 && nu == 2) return 5;    // jerk: 314 at N = 40
    if (nx == 4 && nu == 2) return 2;    // force: 116 at N = 20
    return 0;
}

template <typename T>
hipError_t cl_fast_launch(int nx, int nu, int sid, const ClFastParams<T> &p, int waves, hipStream_t s)
{
    const int blocks = (waves + clf::WPB - 1) / clf::WPB;
    if (nx == 13 && nu == 4 && sid == lpc::Quad13Structure::id)
        hipLaunchKernelGGL((clf::cl_fast_kernel<T, 13, 4, 4, lpc::Quad13Structure>), dim3(blocks), dim3(64 * clf::WPB), 0, s, p);
    else if (nx == 13 && nu == 4)
        hipLaunchKernelGGL((clf::cl_fast_kernel<T, 13, 4, 4, lpc::DenseStructure<13, 4>>), dim3(blocks), dim3(64 * clf::WPB), 0, s, p);
    else if (nx == 6 && nu == 2)
        hipLaunchKernelGGL((clf::cl_fast_kernel<T, 6, 2, 5, lpc::DenseStructure<6, 2>>), dim3(blocks), dim3(64 * clf::WPB), 0, s, p);
    else if (nx == 4 && nu == 2)
        hipLaunchKernelGGL((clf::cl_fast_kernel<T, 4, 2, 2, lpc::DenseStructure<4, 2>>), dim3(blocks), dim3(64 * clf::WPB), 0, s, p);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

template hipError_t cl_fast_launch<double>(int, int, int, const ClFastParams<double> &, int, hipStream_t);

}  // namespace nmpc
