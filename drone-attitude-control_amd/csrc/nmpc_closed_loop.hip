// nmpc_closed_loop.hip — on-device closed loop around the batched solve.
//
// One closed-loop step of every instance, kept resident in HBM between steps:
//   prepare:  yref window from a shared reference table + per-instance start row
//             (set_up_ocp, force_model/ocp.py:117-122; table = generate_trajectory.py:7-28),
//             x0_bar <- current state (force_model/controller.py:29-31, jerk :30-32)
//   solve:    nmpc_ipm.hip
//   advance:  closed-loop cost (controller.py:40-41), AED numerator (store_results.py:233-236),
//             converter + plant + noise (force_model/dynamics.py:54-79 + ocp.py:106-115;
//             jerk_model/dynamics.py:59-83 + jerk_model/ocp.py:106-116), or the controller's own
//             discrete model for synthetic instances.
// Noise: one scalar N(0, sigma) per (instance, step) added to every plant state (ocp.py:114),
// drawn from Philox4x32-10 keyed by (seed, global instance id, step) so results do not depend
// on how instances are sharded over GPUs.

#include <hip/hip_runtime.h>

#include <algorithm>

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
__device__ double philox_normal_dev(uint64_t seed, uint64_t inst, uint64_t step)
{
    uint32_t c[4] = {(uint32_t)step, (uint32_t)(step >> 32), (uint32_t)inst, (uint32_t)(inst >> 32)};
    philox4x32(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const double u1 = ((double)c[0] + 1.0) * (1.0 / 4294967296.0);   // (0, 1]
    const double u2 = (double)c[1] * (1.0 / 4294967296.0);
    return sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
}

template <typename T>
__global__ __launch_bounds__(256) void cl_prepare_kernel(ClParams<T> p)
{
    const int per = p.N * p.ny + p.ny_e;
    const size_t total = (size_t)p.B * per;
    for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < total;
         idx += (size_t)gridDim.x * blockDim.x) {
        const int b = (int)(idx / per), e = (int)(idx % per);
        const int t = (p.offset[b] + p.step) % p.period;
        int row, col;
        if (e < p.N * p.ny) {
            row = t + e / p.ny;
            col = e % p.ny;
        } else {
            row = t + p.N;
            col = e - p.N * p.ny;
        }
        p.yref[idx] = p.table[(size_t)row * p.table_cols + col];
    }
    const size_t nxs = (size_t)p.B * p.nx;
    for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < nxs; idx += (size_t)gridDim.x * blockDim.x)
        p.x0[idx] = p.state[idx];
}

__device__ __forceinline__ void crazyflie_rhs(const double x[4], double st, double ct, double Fd, double inv_m,
                                              double g, double f[4])
{
    f[0] = x[2];
    f[1] = x[3];
    f[2] = inv_m * Fd * st;
    f[3] = inv_m * Fd * ct - g;
}

template <typename T>
__global__ __launch_bounds__(256) void cl_advance_kernel(ClParams<T> p)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= p.B) return;
    const int nx = p.nx, nu = p.nu;
    const int t = (p.offset[b] + p.step) % p.period;
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
    double w = 0.0;
    if (p.noise_table) {
        if (p.step < p.noise_len) w = p.noise_table[(size_t)b * p.noise_len + p.step];
    } else if (p.noise_std > 0) {
        w = p.noise_std * philox_normal_dev(p.seed, (unsigned long long)(p.inst_base + b), (unsigned long long)p.step);
    }
    if (p.plant == 0) {
        // controller's own discrete model
        double xn[32];
        for (int i = 0; i < nx; i++) {
            double s = (double)p.c[i];
            for (int j = 0; j < nx; j++) s += (double)p.A[i * nx + j] * (double)st[j];
            for (int j = 0; j < nu; j++) s += (double)p.Bm[i * nu + j] * (double)u0[j];
            xn[i] = s;
        }
        for (int i = 0; i < nx; i++) st[i] = (T)(xn[i] + (i < p.noise_dims ? w : 0.0));
    } else {
        double x[4], f[4];
        for (int i = 0; i < 4; i++) x[i] = (double)st[i];
        const double inv_m = 1.0 / p.mass;
        if (p.plant == 1) {
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
        } else {
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
    acc[2] += p.status[b] != 0 ? 1.0 : 0.0;
    acc[3] += 1.0;
}

// The controller-model plant (plant == 0) at a compile-time size: the model matrices live in LDS
// (one broadcast read per entry instead of a global load per thread and entry) and the state,
// input and successor state in registers (the generic kernel's runtime-sized arrays spill to
// scratch). Same arithmetic order as cl_advance_kernel.
template <typename T, int NX, int NU>
__global__ __launch_bounds__(256) void cl_model_advance_kernel(ClParams<T> p)
{
    __shared__ double sA[NX * NX], sB[NX * NU], sc[NX];
    for (int e = threadIdx.x; e < NX * NX; e += blockDim.x) sA[e] = (double)p.A[e];
    for (int e = threadIdx.x; e < NX * NU; e += blockDim.x) sB[e] = (double)p.Bm[e];
    for (int e = threadIdx.x; e < NX; e += blockDim.x) sc[e] = (double)p.c[e];
    __syncthreads();
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= p.B) return;
    const int t = (p.offset[b] + p.step) % p.period;
    const T *xref = p.table + (size_t)t * p.table_cols;
    T *st = p.state + (size_t)b * NX;
    const T *xo = p.xout + ((size_t)b * (p.N + 1) + p.cost_stage) * NX;
    const T *u0 = p.uout + (size_t)b * p.N * NU;
    double x[NX], u[NU];
#pragma unroll
    for (int i = 0; i < NX; i++) x[i] = (double)st[i];
#pragma unroll
    for (int j = 0; j < NU; j++) u[j] = (double)u0[j];
    double cost = 0.0, aed = 0.0;
    for (int i = 0; i < p.ncl; i++) {
        const double e = (double)xo[i] - (double)xref[i];
        cost += (double)p.wcl[i] * e * e;
    }
    for (int i = 0; i < p.aed_dims; i++) aed += fabs((double)xref[i] - (double)st[i]);
    double w = 0.0;
    if (p.noise_table) {
        if (p.step < p.noise_len) w = p.noise_table[(size_t)b * p.noise_len + p.step];
    } else if (p.noise_std > 0) {
        w = p.noise_std * philox_normal_dev(p.seed, (unsigned long long)(p.inst_base + b), (unsigned long long)p.step);
    }
#pragma unroll
    for (int i = 0; i < NX; i++) {
        double s = sc[i];
#pragma unroll
        for (int j = 0; j < NX; j++) s += sA[i * NX + j] * x[j];
#pragma unroll
        for (int j = 0; j < NU; j++) s += sB[i * NU + j] * u[j];
        st[i] = (T)(s + (i < p.noise_dims ? w : 0.0));
    }
    double *acc = p.acc + (size_t)b * 4;
    acc[0] += cost;
    acc[1] += aed;
    acc[2] += p.status[b] != 0 ? 1.0 : 0.0;
    acc[3] += 1.0;
}

template <typename T>
hipError_t cl_prepare_launch(const ClParams<T> &p, hipStream_t s)
{
    const size_t total = (size_t)p.B * (p.N * p.ny + p.ny_e);
    const int blocks = (int)std::min<size_t>((total + 255) / 256, 4096);
    hipLaunchKernelGGL(cl_prepare_kernel<T>, dim3(blocks), dim3(256), 0, s, p);
    return hipGetLastError();
}

template <typename T>
hipError_t cl_advance_launch(const ClParams<T> &p, hipStream_t s)
{
    if (p.plant == 0 && p.nx == 13 && p.nu == 4) {   // quad13 (the headline model)
        hipLaunchKernelGGL((cl_model_advance_kernel<T, 13, 4>), dim3((p.B + 255) / 256), dim3(256), 0, s, p);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(cl_advance_kernel<T>, dim3((p.B + 255) / 256), dim3(256), 0, s, p);
    return hipGetLastError();
}

template hipError_t cl_prepare_launch<double>(const ClParams<double> &, hipStream_t);
template hipError_t cl_prepare_launch<float>(const ClParams<float> &, hipStream_t);
template hipError_t cl_advance_launch<double>(const ClParams<double> &, hipStream_t);
template hipError_t cl_advance_launch<float>(const ClParams<float> &, hipStream_t);

}  // namespace nmpc
