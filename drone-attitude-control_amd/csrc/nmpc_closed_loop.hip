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
// The advance itself (and the noise stream) is nmpc_cl_device.h, shared with the fused closed
// loop that the lane-per-component and wavefront solve kernels run without per-step launches.

#include <hip/hip_runtime.h>

#include <algorithm>

#include "nmpc_cl_device.h"
#include "nmpc_internal.h"

namespace nmpc {

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

template <typename T>
__global__ __launch_bounds__(256) void cl_advance_kernel(ClParams<T> p)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= p.B) return;
    cl_advance_instance<T>(p, b, p.step, p.status[b]);
}

// the controller-model plant at a compile-time size (state / input in registers)
template <typename T, int NX, int NU>
__global__ __launch_bounds__(256) void cl_model_advance_kernel(ClParams<T> p)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= p.B) return;
    cl_advance_instance<T, NX, NU>(p, b, p.step, p.status[b]);
}

template <typename T>
__global__ __launch_bounds__(256) void cl_noise_kernel(ClParams<T> p, int step0, int nsteps, double *out, int *zero2)
{
    // (zero2: two counters of the next kernel reset here, one stream operation fewer than a memset)
    if (zero2 && blockIdx.x == 0 && threadIdx.x < 2) zero2[threadIdx.x] = 0;
    const size_t total = (size_t)p.B * nsteps;
    for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < total;
         idx += (size_t)gridDim.x * blockDim.x) {
        const int b = (int)(idx / nsteps), step = step0 + (int)(idx % nsteps);
        out[idx] = noise_draw(p.seed, p.inst_base, p.noise_std, p.noise_table, p.noise_len, b, step);
    }
}

template <typename T>
hipError_t cl_noise_launch(const ClParams<T> &p, int step0, int nsteps, double *out, hipStream_t s, int *zero2)
{
    const size_t total = (size_t)p.B * nsteps;
    const int blocks = (int)std::max<size_t>(1, std::min<size_t>((total + 255) / 256, 4096));
    NMPC_LAUNCH(cl_noise_kernel<T>, dim3(blocks), dim3(256), 0, s, p, step0, nsteps, out, zero2);
    return hipGetLastError();
}

template <typename T>
hipError_t cl_prepare_launch(const ClParams<T> &p, hipStream_t s)
{
    const size_t total = (size_t)p.B * (p.N * p.ny + p.ny_e);
    const int blocks = (int)std::min<size_t>((total + 255) / 256, 4096);
    NMPC_LAUNCH(cl_prepare_kernel<T>, dim3(blocks), dim3(256), 0, s, p);
    return hipGetLastError();
}

template <typename T>
hipError_t cl_advance_launch(const ClParams<T> &p, hipStream_t s)
{
    if (p.plant == 0 && p.nx == 13 && p.nu == 4) {   // quad13 (the headline model)
        NMPC_LAUNCH((cl_model_advance_kernel<T, 13, 4>), dim3((p.B + 255) / 256), dim3(256), 0, s, p);
        return hipGetLastError();
    }
    NMPC_LAUNCH(cl_advance_kernel<T>, dim3((p.B + 255) / 256), dim3(256), 0, s, p);
    return hipGetLastError();
}

template hipError_t cl_prepare_launch<double>(const ClParams<double> &, hipStream_t);
template hipError_t cl_prepare_launch<float>(const ClParams<float> &, hipStream_t);
template hipError_t cl_advance_launch<double>(const ClParams<double> &, hipStream_t);
template hipError_t cl_advance_launch<float>(const ClParams<float> &, hipStream_t);
template hipError_t cl_noise_launch<double>(const ClParams<double> &, int, int, double *, hipStream_t, int *);
template hipError_t cl_noise_launch<float>(const ClParams<float> &, int, int, double *, hipStream_t, int *);

}  // namespace nmpc
