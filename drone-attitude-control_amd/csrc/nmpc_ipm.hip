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
//   * Mehrotra predictor-corrector IPM. Each iteration is four sweeps over the N stages:
//       A  backward: Riccati factorisation + predictor right-hand side (and the lazily
//          applied step of the previous iteration),
//       B  forward: predictor direction + its ratio test and centring sums,
//       C  backward: corrector right-hand side,
//       D  forward: corrector direction + step length + the new complementarity measure
//          (closed form in alpha, so no extra elementwise sweep is needed);
//   * the stage matrices (P, M = P[A B] stored transposed, F = [A B]'M + H + Sigma) live in
//     LDS; the lanes form a (column c, row group rg) grid and each lane keeps its column of
//     [A B] in registers, so every LDS operand is a broadcast read;
//   * input-block gains in explicit form, K = -F_uu^{-1} F_ux and F_uu^{-1}: the forward
//     sweeps are then a matrix-vector product per stage, with no triangular solve on the
//     stage-to-stage dependency chain;
//   * per-stage iterates and gains stream through a per-instance HBM scratch region; every
//     sweep prefetches the next stage's data one stage ahead so global latency overlaps
//     the current stage's LDS/VALU work;
//   * lanes of one wavefront exchange LDS data without barriers: LDS operations of one
//     wavefront execute in issue order, so a wavefront-scope fence (compiler ordering only)
//     between writer and reader phases suffices. Global scratch hand-offs between lanes are
//     ordered by one workgroup-scope fence per sweep.
//
// The algorithm is the one in oracle/c/riccati_ipm.c (the CPU baseline), step for step; its
// results are checked against the KKT-certified dense oracle (oracle/qp.py).

#include <hip/hip_runtime.h>

#include <cstdlib>

#include "nmpc_internal.h"

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
struct ScratchLayout {
    size_t z, ll, lu, gc, gf, dza, dz, re, pr, kst, finv, kff, total;
    __host__ __device__ ScratchLayout(int N, int nx, int nu)
    {
        const size_t nz = (size_t)nx + nu, S = (size_t)(N + 1) * nz;
        z = 0;
        ll = z + S;
        lu = ll + S;
        gc = lu + S;
        gf = gc + S;
        dza = gf + S;
        dz = dza + S;
        re = dz + S;
        pr = re + (size_t)N * nx;
        kst = pr + (size_t)N * nx;            // K_k  [nu][nx] row-major
        finv = kst + (size_t)N * nu * nx;     // Cholesky factor of F_uu, packed (inverse diagonal)
        kff = finv + (size_t)N * (nu * (nu + 1) / 2);   // feed-forward -F_uu^-1 h_u [nu]
        total = kff + (size_t)N * nu;
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
    // per-instance work area
    static constexpr int I_FP = 0, I_MT = I_FP + NZ * LDZ, I_ZV = I_MT + NZ * LDX, I_SV = I_ZV + 2 * LDZ,
                         I_RV = I_SV + 2 * LDZ, I_VV = I_RV + 2 * LDX, I_HV = I_VV + LDX, I_PV = I_HV + LDZ,
                         I_KL = I_PV + LDX, I_DX = I_KL + NU * LDX, I_DU = I_DX + 2 * LDX, I_TOT = I_DU + LDU;
    static constexpr int LDS_ELEMS = C_TOT + WPB * IPW * I_TOT;
    static_assert(R >= 1, "lane group narrower than the stage width");
};

template <typename T, int NX, int NU, int IPW, int WPB, int MW>
__global__ __launch_bounds__(64 * WPB, MW) void ipm_kernel(IpmParams<T> p)
{
    using Gm = Geometry<T, NX, NU, IPW, WPB>;
    constexpr int NZ = Gm::NZ, G = Gm::G, R = Gm::R, RM = Gm::RM, RF = Gm::RF;
    constexpr int LDZ = Gm::LDZ, LDX = Gm::LDX;

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
    T *w = lds + Gm::C_TOT + (wave * IPW + grp) * Gm::I_TOT;
    T *fp = w + Gm::I_FP, *mt = w + Gm::I_MT, *hv = w + Gm::I_HV, *vv = w + Gm::I_VV, *pv = w + Gm::I_PV;
    T *kl = w + Gm::I_KL, *du_l = w + Gm::I_DU;

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
    // bounds of this lane's component for the three stage types (0, 1..N-1, N)
    const int lc = ll < NZ ? ll : 0;

    const ScratchLayout L(N, NX, NU);
    // wave-uniform bases (SGPRs) + 32-bit lane offsets: global loads take the saddr form
    const unsigned wave_u = __builtin_amdgcn_readfirstlane(wave);
    const size_t inst0 = ((size_t)blockIdx.x * WPB + wave_u) * IPW;
    Scr<T> S;
    S.r = __builtin_amdgcn_make_buffer_rsrc(p.scratch + inst0 * L.total, 0,
                                            (int)(IPW * L.total * sizeof(T)), 0x00020000);
    S.go = (unsigned)grp * (unsigned)(L.total * sizeof(T));
    const unsigned Lz = L.z, Lll = L.ll, Llu = L.lu, Lgc = L.gc, Lgf = L.gf, Ldza = L.dza, Ldz = L.dz;
    const unsigned Lre = L.re, Lpr = L.pr, Lkst = L.kst, Lfinv = L.finv, Lkff = L.kff;
    const T *yref = p.yref + (size_t)inst * ((size_t)N * p.ny + p.ny_e);
    const T *x0 = p.x0 + (size_t)inst * NX;
    const int nel = (N + 1) * NZ;
    auto stype = [&](int k) { return k == 0 ? 0 : (k == N ? 2 : 1); };
    auto LBR = [&](int k) { return clb[stype(k) * LDZ + lc]; };
    auto UBR = [&](int k) { return cub[stype(k) * LDZ + lc]; };

    // ------------------------------------------------------------------ initial point
    for (int e = ll; e < nel; e += G) {
        const int k = e / NZ, i = e % NZ;
        T z = 0, lam_l = 0, lam_u = 0, gc = 0;
        if (k < N || i < NX) {
            const T *yk = yref + (size_t)k * p.ny;
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
    bool active = inst_ok;
    int status = 2, iters = 0;
    bool fail = false, pending = false;
    T alpha = 0, smu = 0;      // step and sigma*mu of the pending (lazily applied) update

    // component lanes: lane ll owns component ll of every stage vector
    auto nzk = [&](int k) { return k == N ? NX : NZ; };

    // P1: (lazy update,) Sigma and z of stage k -> LDS buffer (k & 1)
    auto stage_p1 = [&](int k, T z, T lam_l, T lam_u, T dz, T dza, T &zreg) {
        if (ll < nzk(k)) {
            const int e = k * NZ + ll;
            const T lb = LBR(k), ub = UBR(k);
            if (pending) {
                if (lam_l > T(0)) {
                    const T t = z - lb, it_ = frcp(t), dla = -lam_l * (T(1) + dza * it_);
                    lam_l += alpha * ((smu - lam_l * t - dla * dza - lam_l * dz) * it_);
                }
                if (lam_u > T(0)) {
                    const T t = ub - z, it_ = frcp(t), dla = -lam_u * (T(1) - dza * it_);
                    lam_u += alpha * ((smu - lam_u * t + dla * dza + lam_u * dz) * it_);
                }
                z += alpha * dz;
                S.st(Lz + k * NZ, ll, z);
                S.st(Lll + k * NZ, ll, lam_l);
                S.st(Llu + k * NZ, ll, lam_u);
            }
            T sig = 0;
            if (lam_l > T(0)) sig += lam_l * frcp(z - lb);
            if (lam_u > T(0)) sig += lam_u * frcp(ub - z);
            w[Gm::I_ZV + (k & 1) * LDZ + ll] = z;
            w[Gm::I_SV + (k & 1) * LDZ + ll] = sig;
            zreg = z;
        }
    };
    // P2: objective gradient g_k (predictor rhs) and dynamics residual re_k -> LDS (k & 1)
    auto stage_p2 = [&](int k, T gc, T zprev, T &greg) {
        const T *zv = w + Gm::I_ZV + (k & 1) * LDZ;
        if (ll < nzk(k)) {
            T g;
            if (k < N) {
                g = dot2<NZ>(gc, [&](int b) { return ch[ll * LDZ + b]; }, [&](int b) { return zv[b]; });
            } else {
                g = dot2<NX>(gc, [&](int b) { return che[ll * LDX + b]; }, [&](int b) { return zv[b]; });
            }
            greg = g;
            S.st(Lgf + k * NZ, ll, g);
        }
        if (k < N && ll < NX) {
            const T r = dot2<NZ>(cc[ll] - zprev, [&](int j) { return cab[ll * LDZ + j]; },
                                 [&](int j) { return zv[j]; });
            w[Gm::I_RV + (k & 1) * LDX + ll] = r;
            S.st(Lre + k * NX, ll, r);
        }
    };
    struct Pre {
        T z, l, u, dz, dza, gc;
    };
    // Prefetches are unconditional (no phi at a branch join, so the compiler does not drain
    // vmcnt there); lanes / stages outside the valid range read harmless data or, past the
    // end of the buffer resource, zeros.
    auto prefetch_a = [&](int k, Pre &q) {
        const unsigned e = (unsigned)(k < 0 ? 0 : k) * NZ;
        q.z = S.ld(Lz + e, ll);
        q.l = S.ld(Lll + e, ll);
        q.u = S.ld(Llu + e, ll);
        q.gc = S.ld(Lgc + e, ll);
        q.dz = S.ld(Ldz + e, ll);
        q.dza = S.ld(Ldza + e, ll);
    };

    // forward sweep shared by predictor (corr = false) and corrector (corr = true);
    // returns the group's step bound and, for the corrector, the closed-form mu sums
    auto forward = [&](bool corr, unsigned dst, T &amax, T &s0, T &s1, T &s2) {
        T *dxb = w + Gm::I_DX;
        if (ll < NX) dxb[ll] = T(0);
        amax = T(1);
        s0 = s1 = s2 = T(0);
        // stage-0 data; every later stage is fetched one stage ahead (K after its last use)
        T krow[NX], kff = 0, re = 0, z = 0, lam_l = 0, lam_u = 0, dza = 0;
        auto fetch_k = [&](int k) {
#pragma unroll
            for (int i = 0; i < NX; i++) krow[i] = S.ld(Lkst + k * NU * NX + i, ll * NX);
        };
        auto fetch_v = [&](int k, T &kf, T &r, T &zz, T &la, T &lu, T &da) {
            const unsigned kk = (unsigned)(k < N ? k : N - 1);
            kf = S.ld(Lkff + kk * NU, ll);
            r = S.ld(Lre + kk * NX, ll);
            const unsigned e = k * NZ;
            zz = S.ld(Lz + e, ll);
            la = S.ld(Lll + e, ll);
            lu = S.ld(Llu + e, ll);
            da = S.ld(Ldza + e, ll);
        };
        fetch_k(0);
        fetch_v(0, kff, re, z, lam_l, lam_u, dza);
        WAVE_SYNC();
        int cur = 0;
        for (int k = 0; k <= N; k++) {
            const T *dxc = dxb + cur * LDX;
            T *dxn = dxb + (1 - cur) * LDX;
            T kff_n = 0, re_n = 0, z_n = 0, ll_n = 0, lu_n = 0, dza_n = 0;
            if (k < N) {
                fetch_v(k + 1, kff_n, re_n, z_n, ll_n, lu_n, dza_n);
                // du = kff + K dx
                if (ll < NU) {
                    du_l[ll] = dot2<NX>(kff, [&](int i) { return krow[i]; }, [&](int i) { return dxc[i]; });
                }
                fetch_k(k + 1 < N ? k + 1 : N - 1);
                WAVE_SYNC();
                if (ll < NX) {
                    dxn[ll] = dot2<NZ>(re, [&](int j) { return cab[ll * LDZ + j]; },
                                       [&](int j) { return j < NX ? dxc[j] : du_l[j - NX]; });
                }
            }
            // stage k direction component + ratio test / sums
            if (ll < nzk(k)) {
                const T dz = ll < NX ? dxc[ll] : du_l[ll - NX];
                S.st(dst + k * NZ, ll, dz);
                const T lb = LBR(k), ub = UBR(k);
                if (lam_l > T(0)) {
                    const T t = z - lb, it_ = frcp(t);
                    if (!corr) {
                        const T dl = -lam_l * (T(1) + dz * it_);
                        if (dz < T(0)) amax = fmin(amax, -t * frcp(dz));
                        if (dl < T(0)) amax = fmin(amax, -lam_l * frcp(dl));
                        s0 += lam_l * t;
                        s2 += lam_l * dz * (t + dz) * it_;
                    } else {
                        const T dla = -lam_l * (T(1) + dza * it_);
                        const T dl = (smu - lam_l * t - dla * dza - lam_l * dz) * it_;
                        if (dz < T(0)) amax = fmin(amax, -t * frcp(dz));
                        if (dl < T(0)) amax = fmin(amax, -lam_l * frcp(dl));
                        s0 += lam_l * t;
                        s1 += dla * dza;
                        s2 += dl * dz;
                    }
                }
                if (lam_u > T(0)) {
                    const T t = ub - z, it_ = frcp(t);
                    if (!corr) {
                        const T dl = -lam_u * (T(1) - dz * it_);
                        if (dz > T(0)) amax = fmin(amax, t * frcp(dz));
                        if (dl < T(0)) amax = fmin(amax, -lam_u * frcp(dl));
                        s0 += lam_u * t;
                        s2 += lam_u * dz * (dz - t) * it_;
                    } else {
                        const T dla = -lam_u * (T(1) - dza * it_);
                        const T dl = (smu - lam_u * t + dla * dza + lam_u * dz) * it_;
                        if (dz > T(0)) amax = fmin(amax, t * frcp(dz));
                        if (dl < T(0)) amax = fmin(amax, -lam_u * frcp(dl));
                        s0 += lam_u * t;
                        s1 += -dla * dza;
                        s2 += -dl * dz;
                    }
                }
            }
            if (k < N) {
                kff = kff_n;
                re = re_n;
                z = z_n;
                lam_l = ll_n;
                lam_u = lu_n;
                dza = dza_n;
                cur = 1 - cur;
                WAVE_SYNC();
            }
        }
        SWEEP_FENCE();
        amax = group_min<G>(amax);
        s0 = group_sum<G>(s0);
        s1 = group_sum<G>(s1);
        s2 = group_sum<G>(s2);
    };

    int it = 0;
    for (;; it++) {
        const bool conv = mu <= p.tol_comp && theta * r0 <= p.tol_res;
        const bool bad = !isfinite(mu) || !isfinite(theta) || fail;
        if (active && (conv || bad)) {
            active = false;
            status = conv && !bad ? 0 : 4;
            iters = it;
        }
        if (active && it >= p.max_iter) {
            active = false;
            status = 2;
            iters = it;
        }
        if (!__any(active)) break;

        // ============================ A: backward factorisation + predictor vector
        {
            Pre q{}, qn{};
            T zreg_k = 0, zreg_km1 = 0, greg = 0, greg_n = 0;
            prefetch_a(N, q);
            stage_p1(N, q.z, q.l, q.u, q.dz, q.dza, zreg_k);
            prefetch_a(N - 1, qn);
            WAVE_SYNC();
            stage_p2(N, q.gc, T(0), greg);
            stage_p1(N - 1, qn.z, qn.l, qn.u, qn.dz, qn.dza, zreg_km1);
            // P_N = He + Sigma_N, p_N = g_N
            if (gridl && col < NX) {
#pragma unroll
                for (int qq = 0; qq < RM; qq++) {
                    const int i = rg + R * qq;
                    if (i < NX)
                        fp[i * LDZ + col] = (che[i * LDX + col]) + (i == col ? w[Gm::I_SV + (N & 1) * LDZ + col] : T(0));
                }
            }
            if (ll < NX) pv[ll] = greg;
            const T gc_km1 = qn.gc;
            WAVE_SYNC();
            stage_p2(N - 1, gc_km1, zreg_k, greg);
            WAVE_SYNC();
            for (int k = N - 1; k >= 0; k--) {
                const int b = k & 1;
                const T *rv = w + Gm::I_RV + b * LDX;
                const T *sv = w + Gm::I_SV + b * LDZ;
                // next stage's (k-1) global data in flight during this stage
                Pre qk{};
                prefetch_a(k - 1, qk);
                // B: Pr = P re, v = Pr + p, M^T = (P [A B])^T
                T abcol[NX];
                load_abcol(abcol);
                if (ll < NX) {
                    const T s = dot2<NX>(T(0), [&](int l) { return fp[ll * LDZ + l]; }, [&](int l) { return rv[l]; });
                    S.st(Lpr + k * NX, ll, s);
                    vv[ll] = s + pv[ll];
                }
                if (gridl) {
#pragma unroll 1
                    for (int qq = 0; qq < RM; qq++) {
                        const int i = rg + R * qq;
                        if (i < NX) {
                            mt[col * LDX + i] = dot2<NX>(T(0), [&](int l) { return fp[i * LDZ + l]; },
                                                         [&](int l) { return abcol[l]; });
                        }
                    }
                }
                WAVE_SYNC();
                // C: F = [A B]' M + H + Sigma (row col), h = [A B]' v + g
                if (gridl) {
#pragma unroll 1
                    for (int qq = 0; qq < RF; qq++) {
                        const int bb = rg + R * qq;
                        if (bb < NZ) {
                            T s = dot2<NX>(ch[col * LDZ + bb], [&](int l) { return abcol[l]; },
                                           [&](int l) { return mt[bb * LDX + l]; });
                            if (bb == col) s += sv[col];
                            fp[col * LDZ + bb] = s;
                        }
                    }
                    if (rg == 0) {
                        hv[col] = dot2<NX>(greg, [&](int l) { return abcol[l]; }, [&](int l) { return vv[l]; });
                    }
                }
                WAVE_SYNC();
                // D: F_uu^-1 (wave-uniform Cholesky), K = -F_uu^-1 F_ux, kff, p_k; P1(k-1)
                constexpr int NUT = NU * (NU + 1) / 2;
                T lf[NUT];
#pragma unroll
                for (int i = 0; i < NU; i++)
#pragma unroll
                    for (int j = 0; j <= i; j++) {
                        T s = fp[(NX + i) * LDZ + NX + j];
#pragma unroll
                        for (int l = 0; l < j; l++) s -= lf[tri(i, l)] * lf[tri(j, l)];
                        if (i == j) {
                            const bool pd = s > T(0);
                            fail |= active & !pd;
                            lf[tri(i, i)] = frsq(pd ? s : T(1));
                        } else {
                            lf[tri(i, j)] = s * lf[tri(j, j)];
                        }
                    }
                T hu[NU];
#pragma unroll
                for (int j = 0; j < NU; j++) hu[j] = hv[NX + j];
                if (ll < NX) {
                    T kc[NU];
#pragma unroll
                    for (int j = 0; j < NU; j++) kc[j] = fp[ll * LDZ + NX + j];
                    chol_solve<T, NU>(lf, kc);
                    T s = hv[ll];
#pragma unroll
                    for (int u = 0; u < NU; u++) {
                        kc[u] = -kc[u];
                        kl[u * LDX + ll] = kc[u];
                        S.st(Lkst + k * NU * NX + u * NX, ll, kc[u]);
                        s += kc[u] * hu[u];
                    }
                    if (k > 0) pv[ll] = s;
                }
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
                    if (ll < NU) S.st(Lkff + k * NU, ll, mine);
                    if (ll < NUT) S.st(Lfinv + k * NUT, ll, lmine);
                }
                T zreg_km2 = 0;
                if (k > 0) stage_p1(k - 1, qk.z, qk.l, qk.u, qk.dz, qk.dza, zreg_km2);
                WAVE_SYNC();
                // E: P_k = F_xx + F_xu K ; P2(k-1)
                if (k > 0) {
                    if (gridl && col < NX) {
                        T fu[NU];
#pragma unroll
                        for (int u = 0; u < NU; u++) fu[u] = fp[col * LDZ + NX + u];
#pragma unroll 1
                        for (int qq = 0; qq < RF; qq++) {
                            const int i = rg + R * qq;
                            if (i < NX) {
                                T s = fp[col * LDZ + i];   // F_xx entry, overwritten in place by P
#pragma unroll
                                for (int u = 0; u < NU; u++) s += fu[u] * kl[u * LDX + i];
                                fp[col * LDZ + i] = s;
                            }
                        }
                    }
                    stage_p2(k - 1, qk.gc, zreg_km1, greg);
                    zreg_km1 = zreg_km2;
                }
                WAVE_SYNC();
            }
            pending = false;
        }
        SWEEP_FENCE();

        // ============================ B: forward predictor
        T a_aff, S0, S1, S2;
        forward(false, Ldza, a_aff, S0, S1, S2);
        // mu_aff = [(1 - a) S0 - a^2 S2'] / m  with S2' = sum lam dz (t + dz) / t (closed form)
        const T mu_aff = ((T(1) - a_aff) * S0 - a_aff * a_aff * S2) * p.inv_m;
        const T sg = mu > T(0) ? fmax(mu_aff, T(0)) * frcp(mu) : T(0);
        const T smu_new = sg * sg * sg * mu;

        // ============================ C: backward corrector vector
        {
            smu = smu_new;
            auto corr_grad = [&](int k, T gf, T z, T lam_l, T lam_u, T dza) -> T {
                T g = gf;
                const T lb = LBR(k), ub = UBR(k);
                if (lam_l > T(0)) {
                    const T t = z - lb, it_ = frcp(t), dl = -lam_l * (T(1) + dza * it_);
                    g += (dl * dza - smu) * it_;
                }
                if (lam_u > T(0)) {
                    const T t = ub - z, it_ = frcp(t), dl = -lam_u * (T(1) - dza * it_);
                    g += (dl * dza + smu) * it_;
                }
                return g;
            };
            constexpr int NUT = NU * (NU + 1) / 2;
            struct PreC {
                T gf, z, l, u, dza, pr;
            };
            auto fetch_c = [&](int k, PreC &q) {
                const unsigned kc_ = (unsigned)(k < 0 ? 0 : k);
                const unsigned e = kc_ * NZ;
                q.gf = S.ld(Lgf + e, ll);
                q.z = S.ld(Lz + e, ll);
                q.l = S.ld(Lll + e, ll);
                q.u = S.ld(Llu + e, ll);
                q.dza = S.ld(Ldza + e, ll);
                q.pr = S.ld(Lpr + (kc_ < (unsigned)N ? kc_ : N - 1) * NX, ll);
            };
            PreC qN{};
            fetch_c(N, qN);
            if (ll < NX) pv[ll] = corr_grad(N, qN.gf, qN.z, qN.l, qN.u, qN.dza);
            PreC q{};
            fetch_c(N - 1, q);
            WAVE_SYNC();
            for (int k = N - 1; k >= 0; k--) {
                T abcol[NX];
                load_abcol(abcol);
                // this stage's factors (used two phases later) and the next stage's vectors
                T lf[NUT], kc[NU];
#pragma unroll
                for (int j = 0; j < NUT; j++) lf[j] = S.ld(Lfinv + k * NUT + j, 0);
#pragma unroll
                for (int u = 0; u < NU; u++) kc[u] = S.ld(Lkst + k * NU * NX + u * NX, ll);
                PreC qn{};
                fetch_c(k - 1, qn);
                T greg = 0;
                if (ll < NZ) greg = corr_grad(k, q.gf, q.z, q.l, q.u, q.dza);
                if (ll < NX) vv[ll] = q.pr + pv[ll];
                WAVE_SYNC();
                if (ll < NZ) {
                    hv[ll] = dot2<NX>(greg, [&](int l) { return abcol[l]; }, [&](int l) { return vv[l]; });
                }
                WAVE_SYNC();
                T hu[NU], x[NU];
#pragma unroll
                for (int j = 0; j < NU; j++) x[j] = hu[j] = hv[NX + j];
                chol_solve<T, NU>(lf, x);
                T mine = 0;
#pragma unroll
                for (int j = 0; j < NU; j++) mine = (ll == j) ? -x[j] : mine;
                if (ll < NU) S.st(Lkff + k * NU, ll, mine);
                if (k > 0 && ll < NX) {
                    T s = hv[ll];
#pragma unroll
                    for (int u = 0; u < NU; u++) s += kc[u] * hu[u];
                    pv[ll] = s;
                }
                q = qn;
                WAVE_SYNC();
            }
        }
        SWEEP_FENCE();

        // ============================ D: forward corrector, step length, new mu
        T amax, T0, C1, C2;
        forward(true, Ldz, amax, T0, C1, C2);
        const T a = fmin(T(1), T(0.995) * amax);
        if (active) {
            // m mu_new = (1 - a) S0 + a (m smu - C1) + a^2 C2
            mu = ((T(1) - a) * T0 + a * (smu * m_bounds - C1) + a * a * C2) * p.inv_m;
            theta *= (T(1) - a);
            alpha = a;
            pending = true;
        }
    }

    // ------------------------------------------------------------------ apply pending step, outputs
    if (!inst_ok) return;
    T *xo = p.xout + (size_t)inst * (N + 1) * NX;
    T *uo = p.uout + (size_t)inst * N * NU;
    for (int e = ll; e < nel; e += G) {
        const int k = e / NZ, i = e % NZ;
        if (k == N && i >= NX) continue;
        T z = S.ld(Lz, e);
        if (pending) z += alpha * S.ld(Ldz, e);
        if (i < NX) xo[k * NX + i] = z;
        else uo[k * NU + (i - NX)] = z;
    }
    if (ll == 0) {
        p.status[inst] = status;
        p.iters[inst] = iters;
    }
}

// ---------------------------------------------------------------------- dispatch table
template <typename T, int NX, int NU, int IPW, int WPB, int MW>
static hipError_t launch_ipm(const IpmParams<T> &p, hipStream_t s)
{
    const int waves = (p.B + IPW - 1) / IPW;
    const int blocks = (waves + WPB - 1) / WPB;
    hipLaunchKernelGGL((ipm_kernel<T, NX, NU, IPW, WPB, MW>), dim3(blocks), dim3(64 * WPB), 0, s, p);
    return hipGetLastError();
}

template <typename T>
struct IpmEntry {
    int nx, nu, ipw, wpb, mw;
    hipError_t (*fn)(const IpmParams<T> &, hipStream_t);
    int lds_bytes;
};

// MW: minimum wavefronts per SIMD requested from the register allocator (__launch_bounds__)
template <typename T, int NX, int NU, int IPW, int WPB, int MW = 1>
static constexpr IpmEntry<T> entry()
{
    return IpmEntry<T>{NX, NU, IPW, WPB, MW, &launch_ipm<T, NX, NU, IPW, WPB, MW>,
                       (int)(sizeof(T) * Geometry<T, NX, NU, IPW, WPB>::LDS_ELEMS)};
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
        entry<T, 13, 4, 1, 4, 3>(),
    };
    *n = (int)(sizeof(t) / sizeof(t[0]));
    return t;
}

template <typename T>
int ipm_find(int nx, int nu, int ipw_req, int *ipw_out, int *lds_out, int *wpb_out)
{
    int n;
    const IpmEntry<T> *t = table<T>(&n);
    int best = -1;
    // NMPC_VARIANT=k picks the k-th compiled kernel of this (nx, nu) (tuning runs)
    const char *var = getenv("NMPC_VARIANT");
    if (var) {
        int want = atoi(var), seen = 0;
        for (int i = 0; i < n; i++) {
            if (t[i].nx != nx || t[i].nu != nu) continue;
            if (seen++ == want) {
                *ipw_out = t[i].ipw;
                *lds_out = t[i].lds_bytes;
                if (wpb_out) *wpb_out = t[i].wpb;
                return i;
            }
        }
    }
    for (int i = 0; i < n; i++) {
        if (t[i].nx != nx || t[i].nu != nu) continue;
        if (ipw_req > 0) {
            if (t[i].ipw == ipw_req) best = i;
        } else if (best < 0 || t[i].ipw > t[best].ipw) {
            best = i;
        }
    }
    if (best < 0) return -1;
    *ipw_out = t[best].ipw;
    *lds_out = t[best].lds_bytes;
    if (wpb_out) *wpb_out = t[best].wpb;
    return best;
}

template <typename T>
hipError_t ipm_launch(int idx, const IpmParams<T> &p, hipStream_t s)
{
    int n;
    const IpmEntry<T> *t = table<T>(&n);
    return t[idx].fn(p, s);
}

template int ipm_find<double>(int, int, int, int *, int *, int *);
template int ipm_find<float>(int, int, int, int *, int *, int *);
template hipError_t ipm_launch<double>(int, const IpmParams<double> &, hipStream_t);
template hipError_t ipm_launch<float>(int, const IpmParams<float> &, hipStream_t);

}  // namespace nmpc
