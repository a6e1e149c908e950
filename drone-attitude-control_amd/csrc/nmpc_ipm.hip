// nmpc_ipm.hip — batched box-constrained LQ-OCP solver for CDNA4 (gfx950).
//
// Replaces, per trajectory instance, one `AcadosOcpSolver.solve()` of the reference
// (src/force_model/controller.py:32, src/jerk_model/controller.py:33): acados SQP-GN over
// an LTI model with LINEAR_LS cost and box constraints is exactly one QP, which acados
// hands to HPIPM's Riccati-based interior-point method (force_model/ocp.py:83). This file
// is a from-scratch interior-point solver of that QP laid out for the MI355X:
//
//   * one 64-lane wavefront per workgroup; the wavefront owns IPW instances, G = 64/IPW
//     lanes per instance (IPW = 1 for nx=13, nu=4: one wavefront per trajectory instance);
//   * Mehrotra predictor-corrector IPM; each Newton system is solved by a backward Riccati
//     factorisation over the N stages and two forward sweeps (predictor, corrector);
//   * the stage matrices of the Riccati step (P, M = P[A B], F = [A B]'M + H + Sigma) live
//     in LDS; the wave's lanes form a (column c, row-group rg) grid over them and each lane
//     keeps its column of [A B] in registers, so every LDS operand read is a broadcast;
//   * per-stage iterates and factors (z, lambda, Delta z, L_uu, L_xu, ...) stream through a
//     per-instance HBM scratch region; elementwise IPM passes read it coalesced;
//   * the lanes of one wave exchange LDS data without barriers: LDS operations of one
//     wavefront execute in issue order, so a wavefront-scope fence (compiler ordering only)
//     between the writing and the reading phase suffices. Global scratch hand-offs between
//     lanes are ordered by a workgroup-scope fence once per sweep.
//
// The algorithm is, step for step, the one in oracle/c/riccati_ipm.c (the CPU baseline);
// its numerics are checked against the KKT-certified dense oracle (oracle/qp.py).

#include <hip/hip_runtime.h>

#include "nmpc_internal.h"

namespace nmpc {

#define WAVE_SYNC()                                              \
    do {                                                         \
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   \
        __builtin_amdgcn_wave_barrier();                         \
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   \
    } while (0)

// global scratch written by some lanes and read by others of the same wave (once per sweep)
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

template <typename T>
__device__ __forceinline__ bool has_bound(T b)
{
    return fabs(b) < T(1e20);
}

// scratch layout (elements of T) for one instance
struct ScratchLayout {
    size_t z, ll, lu, gc, gf, dza, dz, re, pr, luu, lxu, luv, total;
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
        luu = pr + (size_t)N * nx;
        lxu = luu + (size_t)N * nu * nu;
        luv = lxu + (size_t)N * nx * nu;
        total = luv + (size_t)N * nu;
        total = (total + 31) & ~size_t(31);  // 256-B aligned regions for fp64
    }
};

size_t scratch_elems_per_instance(int N, int nx, int nu) { return ScratchLayout(N, nx, nu).total; }

template <typename T, int NX, int NU, int IPW>
struct Geometry {
    static constexpr int NZ = NX + NU;
    static constexpr int G = 64 / IPW;          // lanes per instance
    static constexpr int R = G / NZ;            // row groups of the lane grid
    static constexpr int RM = (NX + R - 1) / R; // rounds for M (NX rows)
    static constexpr int RF = (NZ + R - 1) / R; // rounds for F (NZ rows)
    static constexpr int NUT = NU * (NU + 1) / 2;
    // per-instance LDS vector block
    static constexpr int V_ZV = 0, V_SV = V_ZV + NZ, V_RV = V_SV + NZ, V_VV = V_RV + NX,
                         V_HV = V_VV + NX, V_PV = V_HV + NZ, V_LX = V_PV + NX,
                         V_DX = V_LX + NX * NU, V_TV = V_DX + 2 * NX, V_DU = V_TV + NU,
                         VEC = V_DU + NU;
    static_assert(R >= 1, "lane group too narrow for the stage width");
    static_assert(G % NZ == 0 || R >= 1, "");
};

template <typename T, int NX, int NU, int IPW>
__global__ __launch_bounds__(64) void ipm_kernel(IpmParams<T> p)
{
    using Gm = Geometry<T, NX, NU, IPW>;
    constexpr int NZ = Gm::NZ, G = Gm::G, R = Gm::R, RM = Gm::RM, RF = Gm::RF;

    __shared__ T s_ab[NX * NZ];            // [A B] row-major, shared by the wave's instances
    __shared__ T s_fp[IPW][NZ * NZ];       // F, and P_{k+1} in its leading NX x NX block
    __shared__ T s_m[IPW][NX * NZ];        // M = P [A B]
    __shared__ T s_v[IPW][Gm::VEC];        // stage vectors

    const int lane = threadIdx.x;
    const int grp = lane / G;
    const int ll = lane % G;
    const int inst_raw = blockIdx.x * IPW + grp;
    const bool inst_ok = inst_raw < p.B;
    const int inst = inst_ok ? inst_raw : p.B - 1;   // tail groups shadow the last instance
    const int col = ll % NZ;
    const int rg = ll / NZ;
    const bool gridl = rg < R;
    const int N = p.N;

    T *fp = s_fp[grp], *mm = s_m[grp], *vv = s_v[grp];

    for (int e = lane; e < NX * NZ; e += 64) s_ab[e] = p.AB[e];
    T abcol[NX];
#pragma unroll
    for (int l = 0; l < NX; l++) abcol[l] = p.AB[l * NZ + col];

    const ScratchLayout L(N, NX, NU);
    T *scr = p.scratch + (size_t)inst_raw * L.total;   // tail groups get their own region
    T *sz = scr + L.z, *sll = scr + L.ll, *slu = scr + L.lu, *sgc = scr + L.gc, *sgf = scr + L.gf;
    T *sdza = scr + L.dza, *sdz = scr + L.dz, *sre = scr + L.re, *spr = scr + L.pr;
    T *sluu = scr + L.luu, *slxu = scr + L.lxu, *sluv = scr + L.luv;
    const T *yref = p.yref + (size_t)inst * ((size_t)N * p.ny + p.ny_e);
    const T *x0 = p.x0 + (size_t)inst * NX;
    const int nel = (N + 1) * NZ;

    auto lbk = [&](int k, int i) -> T { return p.lbnd[(k == 0 ? 0 : (k == N ? 2 : 1)) * NZ + i]; };
    auto ubk = [&](int k, int i) -> T { return p.ubnd[(k == 0 ? 0 : (k == N ? 2 : 1)) * NZ + i]; };

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
                const T lb = lbk(k, i), ub = ubk(k, i);
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
        sz[e] = z;
        sll[e] = lam_l;
        slu[e] = lam_u;
        sgc[e] = gc;
    }
    SWEEP_FENCE();

    // initial residual scale r0 (pi = 0) and complementarity mu
    T r0 = 0, mu = 0;
    for (int e = ll; e < nel; e += G) {
        const int k = e / NZ, i = e % NZ;
        if (k == N && i >= NX) continue;
        const T *zk = sz + (size_t)k * NZ;
        if (!(k == 0 && i < NX)) {
            T g = sgc[e];
            if (k < N) {
                for (int b = 0; b < NZ; b++) g += p.H[i * NZ + b] * zk[b];
            } else {
                for (int b = 0; b < NX; b++) g += p.He[i * NX + b] * zk[b];
            }
            r0 = fmax(r0, fabs(g - sll[e] + slu[e]));
            const T z = zk[i];
            if (sll[e] > T(0)) mu += sll[e] * (z - lbk(k, i));
            if (slu[e] > T(0)) mu += slu[e] * (ubk(k, i) - z);
        }
        if (k < N && i < NX) {
            T r = p.c[i] - zk[NZ + i];
            for (int j = 0; j < NZ; j++) r += p.AB[i * NZ + j] * zk[j];
            r0 = fmax(r0, fabs(r));
        }
    }
    r0 = group_max<G>(r0);
    mu = group_sum<G>(mu) * p.inv_m;

    T theta = 1;
    bool active = inst_ok;
    int status = 2, iters = 0;
    bool fail = false;
    int it = 0;
    __syncthreads();   // s_ab visible

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

        // ============================ backward: factorisation + predictor vector
        T zprev = 0;     // z_{k+1}[ll] for the dynamics residual
        T freg[RF];
#pragma unroll
        for (int q = 0; q < RF; q++) freg[q] = 0;
        for (int k = N; k >= 0; k--) {
            const int nzk = (k == N) ? NX : NZ;
            // P1: stage data -> LDS
            T zreg = 0, sig = 0;
            if (ll < nzk) {
                const int e = k * NZ + ll;
                zreg = sz[e];
                const T lam_l = sll[e], lam_u = slu[e];
                if (lam_l > T(0)) sig += lam_l / (zreg - lbk(k, ll));
                if (lam_u > T(0)) sig += lam_u / (ubk(k, ll) - zreg);
                vv[Gm::V_ZV + ll] = zreg;
                vv[Gm::V_SV + ll] = sig;
            }
            WAVE_SYNC();
            // P2: objective gradient (predictor rhs) and dynamics residual
            T greg = 0;
            if (ll < nzk) {
                T g = sgc[k * NZ + ll];
                if (k < N) {
#pragma unroll
                    for (int b = 0; b < NZ; b++) g += p.H[ll * NZ + b] * vv[Gm::V_ZV + b];
                } else {
#pragma unroll
                    for (int b = 0; b < NX; b++) g += p.He[ll * NX + b] * vv[Gm::V_ZV + b];
                }
                greg = g;
                sgf[k * NZ + ll] = g;
            }
            if (k < N && ll < NX) {
                T r = p.c[ll] - zprev;
#pragma unroll
                for (int j = 0; j < NZ; j++) r += s_ab[ll * NZ + j] * vv[Gm::V_ZV + j];
                vv[Gm::V_RV + ll] = r;
                sre[k * NX + ll] = r;
            }
            zprev = zreg;
            if (k == N) {
                // P_N = He + Sigma_N, p_N = grad f_N
                if (gridl && col < NX) {
#pragma unroll
                    for (int q = 0; q < RM; q++) {
                        const int i = rg + R * q;
                        if (i < NX) fp[i * NZ + col] = p.He[i * NX + col] + (i == col ? vv[Gm::V_SV + col] : T(0));
                    }
                }
                if (ll < NX) vv[Gm::V_PV + ll] = greg;
                WAVE_SYNC();
                continue;
            }
            WAVE_SYNC();
            // B: Pr = P re, v = Pr + p, M = P [A B]
            if (ll < NX) {
                T s = 0;
#pragma unroll
                for (int l = 0; l < NX; l++) s += fp[ll * NZ + l] * vv[Gm::V_RV + l];
                spr[k * NX + ll] = s;
                vv[Gm::V_VV + ll] = s + vv[Gm::V_PV + ll];
            }
            if (gridl) {
#pragma unroll
                for (int q = 0; q < RM; q++) {
                    const int i = rg + R * q;
                    if (i < NX) {
                        T s = 0;
#pragma unroll
                        for (int l = 0; l < NX; l++) s += fp[i * NZ + l] * abcol[l];
                        mm[i * NZ + col] = s;
                    }
                }
            }
            WAVE_SYNC();
            // C: F = [A B]' M + H + Sigma (row `col`), h = [A B]' v + g
            if (gridl) {
#pragma unroll
                for (int q = 0; q < RF; q++) {
                    const int b = rg + R * q;
                    if (b < NZ) {
                        T s = p.H[col * NZ + b];
#pragma unroll
                        for (int l = 0; l < NX; l++) s += abcol[l] * mm[l * NZ + b];
                        if (b == col) s += vv[Gm::V_SV + col];
                        freg[q] = s;
                        fp[col * NZ + b] = s;
                    }
                }
                if (rg == 0) {
                    T s = greg;
#pragma unroll
                    for (int l = 0; l < NX; l++) s += abcol[l] * vv[Gm::V_VV + l];
                    vv[Gm::V_HV + col] = s;
                }
            }
            WAVE_SYNC();
            // D: L_uu = chol(F_uu), l_u = L_uu^-1 h_u (wave-uniform); L_xu rows; p_k
            T luu[NU][NU];
            T luv[NU];
            {
#pragma unroll
                for (int i = 0; i < NU; i++)
#pragma unroll
                    for (int j = 0; j <= i; j++) {
                        T s = fp[(NX + i) * NZ + NX + j];
#pragma unroll
                        for (int l = 0; l < j; l++) s -= luu[i][l] * luu[j][l];
                        if (i == j) {
                            if (!(s > T(0))) {
                                fail = fail || active;
                                s = T(1);
                            }
                            luu[i][i] = sqrt(s);
                        } else {
                            luu[i][j] = s / luu[j][j];
                        }
                    }
#pragma unroll
                for (int j = 0; j < NU; j++) {
                    T s = vv[Gm::V_HV + NX + j];
#pragma unroll
                    for (int l = 0; l < j; l++) s -= luu[j][l] * luv[l];
                    luv[j] = s / luu[j][j];
                }
            }
            if (ll < NX) {
                T lx[NU];
#pragma unroll
                for (int j = 0; j < NU; j++) {
                    T s = fp[ll * NZ + NX + j];
#pragma unroll
                    for (int l = 0; l < j; l++) s -= lx[l] * luu[j][l];
                    lx[j] = s / luu[j][j];
                    vv[Gm::V_LX + ll * NU + j] = lx[j];
                    slxu[(size_t)k * NX * NU + ll * NU + j] = lx[j];
                }
                if (k > 0) {
                    T s = vv[Gm::V_HV + ll];
#pragma unroll
                    for (int j = 0; j < NU; j++) s -= lx[j] * luv[j];
                    vv[Gm::V_PV + ll] = s;
                }
            }
            if (ll < NU) {
                // lane j stores row j of L_uu and l_u[j]
#pragma unroll
                for (int j = 0; j < NU; j++)
                    if (j == ll) {
#pragma unroll
                        for (int l = 0; l < NU; l++) sluu[(size_t)k * NU * NU + j * NU + l] = l <= j ? luu[j][l] : T(0);
                        sluv[(size_t)k * NU + j] = luv[j];
                    }
            }
            WAVE_SYNC();
            // E: P_k = F_xx - L_xu L_xu'
            if (k > 0 && gridl && col < NX) {
#pragma unroll
                for (int q = 0; q < RF; q++) {
                    const int i = rg + R * q;
                    if (i < NX) {
                        T s = freg[q];
#pragma unroll
                        for (int j = 0; j < NU; j++) s -= vv[Gm::V_LX + col * NU + j] * vv[Gm::V_LX + i * NU + j];
                        fp[col * NZ + i] = s;
                    }
                }
            }
            WAVE_SYNC();
        }
        SWEEP_FENCE();

        // ============================ forward sweep (direction into dst)
        auto forward = [&](T *dst) {
            if (ll < NX) vv[Gm::V_DX + ll] = T(0);
            int cur = 0;
            WAVE_SYNC();
            for (int k = 0; k < N; k++) {
                const T *dxc = vv + Gm::V_DX + cur * NX;
                T *dxn = vv + Gm::V_DX + (1 - cur) * NX;
                if (ll < NU) {
                    T s = sluv[(size_t)k * NU + ll];
#pragma unroll
                    for (int i = 0; i < NX; i++) s += slxu[(size_t)k * NX * NU + i * NU + ll] * dxc[i];
                    vv[Gm::V_TV + ll] = s;
                }
                WAVE_SYNC();
                T du[NU];
#pragma unroll
                for (int j = NU - 1; j >= 0; j--) {
                    T s = vv[Gm::V_TV + j];
#pragma unroll
                    for (int l = j + 1; l < NU; l++) s -= sluu[(size_t)k * NU * NU + l * NU + j] * du[l];
                    du[j] = s / sluu[(size_t)k * NU * NU + j * NU + j];
                }
#pragma unroll
                for (int j = 0; j < NU; j++) du[j] = -du[j];
                if (ll < NX) {
                    T s = sre[k * NX + ll];
#pragma unroll
                    for (int j = 0; j < NX; j++) s += s_ab[ll * NZ + j] * dxc[j];
#pragma unroll
                    for (int j = 0; j < NU; j++) s += s_ab[ll * NZ + NX + j] * du[j];
                    dxn[ll] = s;
                    dst[k * NZ + ll] = dxc[ll];
                }
                if (ll < NU) {
#pragma unroll
                    for (int j = 0; j < NU; j++)
                        if (j == ll) dst[k * NZ + NX + j] = du[j];
                }
                cur = 1 - cur;
                WAVE_SYNC();
            }
            if (ll < NX) dst[N * NZ + ll] = vv[Gm::V_DX + cur * NX + ll];
            SWEEP_FENCE();
        };
        forward(sdza);

        // ============================ affine step length and centring
        T a_aff = 1;
        for (int e = ll; e < nel; e += G) {
            const int k = e / NZ, i = e % NZ;
            const T lam_l = sll[e], lam_u = slu[e];
            if (lam_l > T(0) || lam_u > T(0)) {
                const T z = sz[e], dz = sdza[e];
                if (lam_l > T(0)) {
                    const T t = z - lbk(k, i), dl = -lam_l * (T(1) + dz / t);
                    if (dz < T(0)) a_aff = fmin(a_aff, -t / dz);
                    if (dl < T(0)) a_aff = fmin(a_aff, -lam_l / dl);
                }
                if (lam_u > T(0)) {
                    const T t = ubk(k, i) - z, dl = -lam_u * (T(1) - dz / t);
                    if (dz > T(0)) a_aff = fmin(a_aff, t / dz);
                    if (dl < T(0)) a_aff = fmin(a_aff, -lam_u / dl);
                }
            }
        }
        a_aff = group_min<G>(a_aff);
        T mu_aff = 0;
        for (int e = ll; e < nel; e += G) {
            const int k = e / NZ, i = e % NZ;
            const T lam_l = sll[e], lam_u = slu[e];
            if (lam_l > T(0) || lam_u > T(0)) {
                const T z = sz[e], dz = sdza[e];
                if (lam_l > T(0)) {
                    const T t = z - lbk(k, i), dl = -lam_l * (T(1) + dz / t);
                    mu_aff += (t + a_aff * dz) * (lam_l + a_aff * dl);
                }
                if (lam_u > T(0)) {
                    const T t = ubk(k, i) - z, dl = -lam_u * (T(1) - dz / t);
                    mu_aff += (t - a_aff * dz) * (lam_u + a_aff * dl);
                }
            }
        }
        mu_aff = group_sum<G>(mu_aff) * p.inv_m;
        const T sg = mu_aff / mu;
        const T smu = sg * sg * sg * mu;

        // ============================ backward: corrector vector sweep
        auto corr_grad = [&](int k, int i) -> T {
            const int e = k * NZ + i;
            T g = sgf[e];
            const T lam_l = sll[e], lam_u = slu[e];
            if (lam_l > T(0) || lam_u > T(0)) {
                const T z = sz[e], dz = sdza[e];
                if (lam_l > T(0)) {
                    const T t = z - lbk(k, i), dl = -lam_l * (T(1) + dz / t);
                    g += (dl * dz - smu) / t;
                }
                if (lam_u > T(0)) {
                    const T t = ubk(k, i) - z, dl = -lam_u * (T(1) - dz / t);
                    g += (dl * dz + smu) / t;
                }
            }
            return g;
        };
        if (ll < NX) vv[Gm::V_PV + ll] = corr_grad(N, ll);
        WAVE_SYNC();
        for (int k = N - 1; k >= 0; k--) {
            T greg = 0;
            if (ll < NZ) greg = corr_grad(k, ll);
            if (ll < NX) vv[Gm::V_VV + ll] = spr[k * NX + ll] + vv[Gm::V_PV + ll];
            WAVE_SYNC();
            if (ll < NZ) {
                T s = greg;
#pragma unroll
                for (int l = 0; l < NX; l++) s += abcol[l] * vv[Gm::V_VV + l];
                vv[Gm::V_HV + ll] = s;
            }
            WAVE_SYNC();
            T luv[NU];
#pragma unroll
            for (int j = 0; j < NU; j++) {
                T s = vv[Gm::V_HV + NX + j];
#pragma unroll
                for (int l = 0; l < j; l++) s -= sluu[(size_t)k * NU * NU + j * NU + l] * luv[l];
                luv[j] = s / sluu[(size_t)k * NU * NU + j * NU + j];
            }
            if (ll < NU) {
#pragma unroll
                for (int j = 0; j < NU; j++)
                    if (j == ll) sluv[(size_t)k * NU + j] = luv[j];
            }
            if (k > 0 && ll < NX) {
                T s = vv[Gm::V_HV + ll];
#pragma unroll
                for (int j = 0; j < NU; j++) s -= slxu[(size_t)k * NX * NU + ll * NU + j] * luv[j];
                vv[Gm::V_PV + ll] = s;
            }
            WAVE_SYNC();
        }
        SWEEP_FENCE();
        forward(sdz);

        // ============================ step length, update, new mu
        T alpha = 1;
        for (int e = ll; e < nel; e += G) {
            const int k = e / NZ, i = e % NZ;
            const T lam_l = sll[e], lam_u = slu[e];
            if (lam_l > T(0) || lam_u > T(0)) {
                const T z = sz[e], dz = sdz[e], dza = sdza[e];
                if (lam_l > T(0)) {
                    const T t = z - lbk(k, i), dla = -lam_l * (T(1) + dza / t);
                    const T dl = (smu - lam_l * t - dla * dza - lam_l * dz) / t;
                    if (dz < T(0)) alpha = fmin(alpha, -t / dz);
                    if (dl < T(0)) alpha = fmin(alpha, -lam_l / dl);
                }
                if (lam_u > T(0)) {
                    const T t = ubk(k, i) - z, dla = -lam_u * (T(1) - dza / t);
                    const T dl = (smu - lam_u * t + dla * dza + lam_u * dz) / t;
                    if (dz > T(0)) alpha = fmin(alpha, t / dz);
                    if (dl < T(0)) alpha = fmin(alpha, -lam_u / dl);
                }
            }
        }
        alpha = fmin(T(1), T(0.995) * group_min<G>(alpha));
        T mu_new = 0;
        for (int e = ll; e < nel; e += G) {
            const int k = e / NZ, i = e % NZ;
            if (k == 0 && i < NX) continue;
            if (k == N && i >= NX) continue;
            const T lam_l = sll[e], lam_u = slu[e];
            const T z = sz[e], dz = sdz[e], dza = sdza[e];
            const T zn = active ? z + alpha * dz : z;
            if (lam_l > T(0)) {
                const T lb = lbk(k, i), t = z - lb, dla = -lam_l * (T(1) + dza / t);
                const T dl = (smu - lam_l * t - dla * dza - lam_l * dz) / t;
                const T ln = active ? lam_l + alpha * dl : lam_l;
                sll[e] = ln;
                mu_new += ln * (zn - lb);
            }
            if (lam_u > T(0)) {
                const T ub = ubk(k, i), t = ub - z, dla = -lam_u * (T(1) - dza / t);
                const T dl = (smu - lam_u * t + dla * dza + lam_u * dz) / t;
                const T ln = active ? lam_u + alpha * dl : lam_u;
                slu[e] = ln;
                mu_new += ln * (ub - zn);
            }
            sz[e] = zn;
        }
        if (active) {
            mu = group_sum<G>(mu_new) * p.inv_m;
            theta *= (T(1) - alpha);
        } else {
            (void)group_sum<G>(mu_new);
        }
        SWEEP_FENCE();
    }

    // ------------------------------------------------------------------ outputs
    if (!inst_ok) return;
    T *xo = p.xout + (size_t)inst * (N + 1) * NX;
    T *uo = p.uout + (size_t)inst * N * NU;
    for (int e = ll; e < nel; e += G) {
        const int k = e / NZ, i = e % NZ;
        if (i < NX) xo[k * NX + i] = sz[e];
        else if (k < N) uo[k * NU + (i - NX)] = sz[e];
    }
    if (ll == 0) {
        p.status[inst] = status;
        p.iters[inst] = iters;
    }
}

// ---------------------------------------------------------------------- dispatch table
template <typename T, int NX, int NU, int IPW>
static hipError_t launch_ipm(const IpmParams<T> &p, hipStream_t s)
{
    const int blocks = (p.B + IPW - 1) / IPW;
    hipLaunchKernelGGL((ipm_kernel<T, NX, NU, IPW>), dim3(blocks), dim3(64), 0, s, p);
    return hipGetLastError();
}

template <typename T>
struct IpmEntry {
    int nx, nu, ipw;
    hipError_t (*fn)(const IpmParams<T> &, hipStream_t);
    int lds_bytes;
};

template <typename T, int NX, int NU, int IPW>
static constexpr IpmEntry<T> entry()
{
    using Gm = Geometry<T, NX, NU, IPW>;
    return IpmEntry<T>{NX, NU, IPW, &launch_ipm<T, NX, NU, IPW>,
                       (int)(sizeof(T) * (NX * Gm::NZ + IPW * (Gm::NZ * Gm::NZ + NX * Gm::NZ + Gm::VEC)))};
}

template <typename T>
static const IpmEntry<T> *table(int *n)
{
    static const IpmEntry<T> t[] = {
        entry<T, 4, 2, 1>(),  entry<T, 4, 2, 2>(),  entry<T, 4, 2, 4>(),  entry<T, 4, 2, 8>(),
        entry<T, 6, 2, 1>(),  entry<T, 6, 2, 2>(),  entry<T, 6, 2, 4>(),
        entry<T, 13, 4, 1>(),
    };
    *n = (int)(sizeof(t) / sizeof(t[0]));
    return t;
}

template <typename T>
int ipm_find(int nx, int nu, int ipw_req, int *ipw_out, int *lds_out)
{
    int n;
    const IpmEntry<T> *t = table<T>(&n);
    int best = -1;
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
    return best;
}

template <typename T>
hipError_t ipm_launch(int idx, const IpmParams<T> &p, hipStream_t s)
{
    int n;
    const IpmEntry<T> *t = table<T>(&n);
    return t[idx].fn(p, s);
}

template int ipm_find<double>(int, int, int, int *, int *);
template int ipm_find<float>(int, int, int, int *, int *);
template hipError_t ipm_launch<double>(int, const IpmParams<double> &, hipStream_t);
template hipError_t ipm_launch<float>(int, const IpmParams<float> &, hipStream_t);

}  // namespace nmpc
