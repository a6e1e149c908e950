// nmpc_cl_device.h — per-instance closed-loop advance shared by the step kernels
// (nmpc_closed_loop.hip) and the fused closed loop inside the solve kernels (nmpc_ipm.hip,
// nmpc_ipm_lpc.hip): one thread advances one instance by one NMPC step.
//
//   cost:  closed-loop cost of the step (force_model/controller.py:40-41)
//   AED:   |reference - state| numerator (store_results.py:233-236)
//   plant: converter + Crazyflie plant (force_model/dynamics.py:54-79 + ocp.py:106-115;
//          jerk_model/dynamics.py:59-83 + jerk_model/ocp.py:106-116) or the controller's own
//          discrete model (synthetic instances), then one scalar N(0, sigma) noise draw per
//          (instance, step) added to the plant states (ocp.py:114), from Philox4x32-10 keyed by
//          (seed, global instance id, step) so results do not depend on the sharding.
#pragma once

#include <hip/hip_runtime.h>

#include "nmpc_internal.h"

namespace nmpc {

__device__ __forceinline__ void philox4x32(uint32_t ctr[4], uint32_t k0, uint32_t k1)
{
#pragma unroll
    for (int r = 0; r < 10; r++) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * ctr[0];
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * ctr[2];
        const uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0;
        const uint32_t h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
        const uint32_t n0 = h1 ^ ctr[1] ^ k0, n2 = h0 ^ ctr[3] ^ k1;
        ctr[0] = n0;
        ctr[1] = l1;
        ctr[2] = n2;
        ctr[3] = l0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

// standard normal from Philox(seed; instance, step) via Box-Muller (fp64)
__device__ __forceinline__ double philox_normal_dev(uint64_t seed, uint64_t inst, uint64_t step)
{
    uint32_t c[4] = {(uint32_t)step, (uint32_t)(step >> 32), (uint32_t)inst, (uint32_t)(inst >> 32)};
    philox4x32(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const double u1 = ((double)c[0] + 1.0) * (1.0 / 4294967296.0);   // (0, 1]
    const double u2 = (double)c[1] * (1.0 / 4294967296.0);
    return sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
}

// instance b's noise draw at closed-loop step `step`: the recorded table's value (0 past its end), else
// noise_std x the Philox normal (cl_noise_kernel, the lean kernels' in-launch draws and cl_advance_instance
// share it: the same bits on every path)
__device__ __forceinline__ double noise_draw(uint64_t seed, long long inst_base, double noise_std, const double *table,
                                             int table_len, int b, int step)
{
    if (table) return step < table_len ? table[(size_t)b * table_len + step] : 0.0;
    if (noise_std > 0) return noise_std * philox_normal_dev(seed, (unsigned long long)(inst_base + b), (unsigned long long)step);
    return 0.0;
}

__device__ __forceinline__ void crazyflie_rhs(const double x[4], double st, double ct, double Fd, double inv_m,
                                              double g, double f[4])
{
    f[0] = x[2];
    f[1] = x[3];
    f[2] = inv_m * Fd * st;
    f[3] = inv_m * Fd * ct - g;
}

// Advance instance b by closed-loop step `step` (p.step is ignored): reads the solve's x / u
// outputs and status, updates the state and the per-instance sums [cost, AED, failures, steps].
// NXC > 0: the controller-model plant at that compile-time size (registers, no scratch arrays);
// NXC = 0: runtime sizes. Both keep the arithmetic order of cl_advance_kernel.
template <typename T, int NXC = 0, int NUC = 0>
__device__ void cl_advance_instance(const ClParams<T> &p, int b, int step, int status)
{
    // plants a model of this size can drive (nmpc_closed_loop_init checks the pairing)
    constexpr bool PL1 = NXC == 0 || (NXC == 4 && NUC == 2), PL2 = NXC == 0 || (NXC == 6 && NUC == 2);
    const int nx = NXC > 0 ? NXC : p.nx, nu = NXC > 0 ? NUC : p.nu;
    const int t = (p.offset[b] + step) % p.period;
    const T *xref = p.table + (size_t)t * p.table_cols;
    T *st = p.state + (size_t)b * nx;
    const T *xo = p.xout + ((size_t)b * (p.N + 1) + p.cost_stage) * nx;
    const T *u0 = p.uout + (size_t)b * p.N * nu;
    double cost = 0.0, aed = 0.0;
    for (int i = 0; i < p.ncl; i++) {
        const double e = (double)xo[i] - (double)xref[i];
        cost += (double)p.wcl[i] * e * e;
    }
    for (int i = 0; i < p.aed_dims; i++) aed += fabs((double)xref[i] - (double)st[i]);
    const double w = noise_draw(p.seed, p.inst_base, p.noise_std, p.noise_table, p.noise_len, b, step);
    if (p.plant == 0) {
        // controller's own discrete model
        constexpr int NXA = NXC > 0 ? NXC : 32, NUA = NUC > 0 ? NUC : 32;
        double xs[NXA], us[NUA], xn[NXA];
#pragma unroll
        for (int i = 0; i < NXA; i++)
            if (i < nx) xs[i] = (double)st[i];
#pragma unroll
        for (int j = 0; j < NUA; j++)
            if (j < nu) us[j] = (double)u0[j];
#pragma unroll
        for (int i = 0; i < NXA; i++) {
            if (i >= nx) break;
            double s = (double)p.c[i];
#pragma unroll
            for (int j = 0; j < NXA; j++)
                if (j < nx) s += (double)p.A[i * nx + j] * xs[j];
#pragma unroll
            for (int j = 0; j < NUA; j++)
                if (j < nu) s += (double)p.Bm[i * nu + j] * us[j];
            xn[i] = s;
        }
#pragma unroll
        for (int i = 0; i < NXA; i++)
            if (i < nx) st[i] = (T)(xn[i] + (i < p.noise_dims ? w : 0.0));
    } else if constexpr (PL1 || PL2) {
        double x[4], f[4];
        for (int i = 0; i < 4; i++) x[i] = (double)st[i];
        const double inv_m = 1.0 / p.mass;
        if (PL1 && p.plant == 1) {
            // force converter (atan2, |F|) + RK4 over dt
            const double Fx = (double)u0[0], Fz = (double)u0[1];
            const double th = atan2(Fx, Fz), Fd = sqrt(Fx * Fx + Fz * Fz);
            const double s_ = sin(th), c_ = cos(th), h = p.dt;
            double k1[4], k2[4], k3[4], k4[4], tt[4];
            crazyflie_rhs(x, s_, c_, Fd, inv_m, p.g, k1);
            for (int i = 0; i < 4; i++) tt[i] = x[i] + 0.5 * h * k1[i];
            crazyflie_rhs(tt, s_, c_, Fd, inv_m, p.g, k2);
            for (int i = 0; i < 4; i++) tt[i] = x[i] + 0.5 * h * k2[i];
            crazyflie_rhs(tt, s_, c_, Fd, inv_m, p.g, k3);
            for (int i = 0; i < 4; i++) tt[i] = x[i] + h * k3[i];
            crazyflie_rhs(tt, s_, c_, Fd, inv_m, p.g, k4);
            for (int i = 0; i < 4; i++) x[i] += h / 6.0 * (k1[i] + 2.0 * k2[i] + 2.0 * k3[i] + k4[i]);
            for (int i = 0; i < 4; i++) st[i] = (T)(x[i] + w);
        } else if (PL2) {
            // jerk converter: a <- a + h dt_conv per sub-step, F = m a, Euler plant over dt_conv
            double a0 = (double)st[4], a1 = (double)st[5];
            const double h0 = (double)u0[0], h1 = (double)u0[1];
            for (int j = 0; j < p.substeps; j++) {
                a0 = a0 + h0 * p.dt_conv;
                a1 = a1 + h1 * p.dt_conv;
                const double Fx = p.mass * a0, Fz = p.mass * a1;
                const double th = atan2(Fx, Fz), Fd = sqrt(Fx * Fx + Fz * Fz);
                crazyflie_rhs(x, sin(th), cos(th), Fd, inv_m, p.g, f);
                for (int i = 0; i < 4; i++) x[i] += p.dt_conv * f[i];
            }
            for (int i = 0; i < 4; i++) st[i] = (T)(x[i] + w);
            st[4] = (T)a0;
            st[5] = (T)a1;
        }
    }
    double *acc = p.acc + (size_t)b * 4;
    acc[0] += cost;
    acc[1] += aed;
    acc[2] += status != 0 ? 1.0 : 0.0;
    acc[3] += 1.0;
}

}  // namespace nmpc

namespace nmpc {

// The same advance run by the lanes of one instance's lane group inside the fused closed loop
// (nmpc_ipm_lpc.hip / nmpc_ipm.hip): lane r < nx of the controller-model plant computes state
// row r (the dot products in cl_advance_instance's order), the Crazyflie plants run on lane 0,
// lane 0 adds the cost / AED / failure sums. w: the step's noise draw, precomputed by
// cl_noise_launch (no Box-Muller in the solve kernels). The group's solve outputs must be visible
// (the caller fences); every lane reads the old state before any lane stores a new row (each
// store depends on all of its lane's loads and the wavefront executes in lockstep).
template <typename T, int NX, int NU>
__device__ __forceinline__ void cl_advance_group(const ClParams<T> &p, int b, int step, int status, int r, double w)
{
    constexpr bool PL1 = NX == 4 && NU == 2, PL2 = NX == 6 && NU == 2;
    T *st = p.state + (size_t)b * NX;
    const T *u0 = p.uout + (size_t)b * p.N * NU;
    double cost = 0.0, aed = 0.0;
    if (r == 0) {
        const int t = (p.offset[b] + step) % p.period;
        const T *xref = p.table + (size_t)t * p.table_cols;
        const T *xo = p.xout + ((size_t)b * (p.N + 1) + p.cost_stage) * NX;
        for (int i = 0; i < p.ncl; i++) {
            const double e = (double)xo[i] - (double)xref[i];
            cost += (double)p.wcl[i] * e * e;
        }
        for (int i = 0; i < p.aed_dims; i++) aed += fabs((double)xref[i] - (double)st[i]);
    }
    if (p.plant == 0) {
        if (r < NX) {
            double s = (double)p.c[r];
#pragma unroll
            for (int j = 0; j < NX; j++) s += (double)p.A[r * NX + j] * (double)st[j];
#pragma unroll
            for (int j = 0; j < NU; j++) s += (double)p.Bm[r * NU + j] * (double)u0[j];
            st[r] = (T)(s + (r < p.noise_dims ? w : 0.0));
        }
    } else if constexpr (PL1 || PL2) {
        if (r == 0) {
            double x[4], f[4];
            for (int i = 0; i < 4; i++) x[i] = (double)st[i];
            const double inv_m = 1.0 / p.mass;
            if (PL1) {
                const double Fx = (double)u0[0], Fz = (double)u0[1];
                const double th = atan2(Fx, Fz), Fd = sqrt(Fx * Fx + Fz * Fz);
                const double s_ = sin(th), c_ = cos(th), h = p.dt;
                double k1[4], k2[4], k3[4], k4[4], tt[4];
                crazyflie_rhs(x, s_, c_, Fd, inv_m, p.g, k1);
                for (int i = 0; i < 4; i++) tt[i] = x[i] + 0.5 * h * k1[i];
                crazyflie_rhs(tt, s_, c_, Fd, inv_m, p.g, k2);
                for (int i = 0; i < 4; i++) tt[i] = x[i] + 0.5 * h * k2[i];
                crazyflie_rhs(tt, s_, c_, Fd, inv_m, p.g, k3);
                for (int i = 0; i < 4; i++) tt[i] = x[i] + h * k3[i];
                crazyflie_rhs(tt, s_, c_, Fd, inv_m, p.g, k4);
                for (int i = 0; i < 4; i++) x[i] += h / 6.0 * (k1[i] + 2.0 * k2[i] + 2.0 * k3[i] + k4[i]);
                for (int i = 0; i < 4; i++) st[i] = (T)(x[i] + w);
            } else {
                double a0 = (double)st[4], a1 = (double)st[5];
                const double h0 = (double)u0[0], h1 = (double)u0[1];
                for (int j = 0; j < p.substeps; j++) {
                    a0 = a0 + h0 * p.dt_conv;
                    a1 = a1 + h1 * p.dt_conv;
                    const double Fx = p.mass * a0, Fz = p.mass * a1;
                    const double th = atan2(Fx, Fz), Fd = sqrt(Fx * Fx + Fz * Fz);
                    crazyflie_rhs(x, sin(th), cos(th), Fd, inv_m, p.g, f);
                    for (int i = 0; i < 4; i++) x[i] += p.dt_conv * f[i];
                }
                for (int i = 0; i < 4; i++) st[i] = (T)(x[i] + w);
                st[4] = (T)a0;
                st[5] = (T)a1;
            }
        }
    }
    if (r == 0) {
        double *acc = p.acc + (size_t)b * 4;
        acc[0] += cost;
        acc[1] += aed;
        acc[2] += status != 0 ? 1.0 : 0.0;
        acc[3] += 1.0;
    }
}

}  // namespace nmpc
