// nmpc_plant.hip — device step of the reference's plant simulator.
//
// Replaces AcadosSimSolver on the nonlinear 2-D Crazyflie plant (src/plant.py:27-33):
//   x = [px, pz, vx, vz], u = [theta, F_d],
//   x' = [vx, vz, F_d sin(theta)/m, F_d cos(theta)/m - g].
// The force loop integrates it with ERK, 4 stages over dt (force_model/ocp.py:98-104,
// acados default integrator ERK); the jerk loop with ERK, 1 stage over dt_conv
// (jerk_model/ocp.py:97-104). One thread per instance: the state is four registers.

#include <hip/hip_runtime.h>

#include "nmpc_internal.h"

namespace nmpc {

__device__ __forceinline__ void plant_rhs(const double x[4], double st, double ct, double Fd, double inv_m,
                                          double g, double f[4])
{
    f[0] = x[2];
    f[1] = x[3];
    f[2] = inv_m * Fd * st;
    f[3] = inv_m * Fd * ct - g;
}

__global__ __launch_bounds__(256) void plant_step_kernel(int batch, int num_stages, double h, double mass, double g,
                                                         const double *__restrict__ x_in,
                                                         const double *__restrict__ u, double *__restrict__ x_out)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= batch) return;
    double x[4], f[4];
#pragma unroll
    for (int i = 0; i < 4; i++) x[i] = x_in[b * 4 + i];
    const double theta = u[b * 2 + 0], Fd = u[b * 2 + 1];
    const double st = sin(theta), ct = cos(theta), inv_m = 1.0 / mass;
    if (num_stages == 1) {
        plant_rhs(x, st, ct, Fd, inv_m, g, f);
#pragma unroll
        for (int i = 0; i < 4; i++) x[i] += h * f[i];
    } else {
        double k1[4], k2[4], k3[4], k4[4], t[4];
        plant_rhs(x, st, ct, Fd, inv_m, g, k1);
#pragma unroll
        for (int i = 0; i < 4; i++) t[i] = x[i] + 0.5 * h * k1[i];
        plant_rhs(t, st, ct, Fd, inv_m, g, k2);
#pragma unroll
        for (int i = 0; i < 4; i++) t[i] = x[i] + 0.5 * h * k2[i];
        plant_rhs(t, st, ct, Fd, inv_m, g, k3);
#pragma unroll
        for (int i = 0; i < 4; i++) t[i] = x[i] + h * k3[i];
        plant_rhs(t, st, ct, Fd, inv_m, g, k4);
#pragma unroll
        for (int i = 0; i < 4; i++) x[i] += h / 6.0 * (k1[i] + 2.0 * k2[i] + 2.0 * k3[i] + k4[i]);
    }
#pragma unroll
    for (int i = 0; i < 4; i++) x_out[b * 4 + i] = x[i];
}

hipError_t plant_step_launch(int batch, int num_stages, double T, double mass, double g, const double *x_in,
                             const double *u, double *x_out, hipStream_t s)
{
    const int blocks = (batch + 255) / 256;
    NMPC_LAUNCH(plant_step_kernel, dim3(blocks), dim3(256), 0, s, batch, num_stages, T, mass, g, x_in, u,
                       x_out);
    return hipGetLastError();
}

}  // namespace nmpc
