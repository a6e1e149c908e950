// nmpc_internal.h — device-side parameter blocks shared by the HIP kernels and the C-ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>

namespace nmpc {

// Kernel parameters of the batched IPM solve (nmpc_ipm.hip). All pointers are device
// pointers. Model data (AB..ubnd) is shared by every instance of a handle.
template <typename T>
struct IpmParams {
    int B;          // instances
    int N;          // horizon
    int ny, ny_e;   // LINEAR_LS residual sizes
    int yref_is_z;  // y = [x; u] (selection Vx, Vu): use yref as the initial guess
    int max_iter;
    T tol_comp, tol_res, mu0, inv_m;
    const T *AB;    // [nx][nx+nu]   discrete [A B], row-major
    const T *ABt;   // [nx+nu][nx]   its transpose
    const T *c;     // [nx]
    const T *H;     // [nz][nz]      stage Hessian (cost-scaled), z = [x; u]
    const T *He;    // [nx][nx]
    const T *G;     // [nz][ny]      stage gradient map: g_k = G yref_k
    const T *Ge;    // [nx][ny_e]
    const T *lbnd;  // [3][nz]       bounds: stage 0 (x entries absent), 1..N-1, N
    const T *ubnd;  // [3][nz]
    const T *x0;    // [B][nx]
    const T *yref;  // [B][N*ny + ny_e]
    T *xout;        // [B][N+1][nx]
    T *uout;        // [B][N][nu]
    int *status;    // [B]
    int *iters;     // [B]
    T *scratch;     // [ceil(B/(IPW*WPB))*IPW*WPB][scratch_elems_per_instance]
    unsigned long long *cycles;   // optional [B][5] clock cycles per sweep type A..D + total (tuning, env NMPC_SWEEP_CYCLES)
};

size_t scratch_elems_per_instance(int N, int nx, int nu);

// returns an index into the kernel table (or -1), the chosen instances-per-wave, the
// static LDS bytes per workgroup and the wavefronts per workgroup. ipw_req <= 0 picks the
// widest packing compiled. Scratch must cover ceil(B / (ipw*wpb)) * ipw * wpb instances.
template <typename T>
int ipm_find(int nx, int nu, int ipw_req, int batch, int *ipw_out, int *lds_out, int *wpb_out);
template <typename T>
hipError_t ipm_launch(int idx, const IpmParams<T> &p, hipStream_t s);
// scratch elements (of T) the kernel `idx` needs for a batch of B instances, horizon N
template <typename T>
size_t ipm_scratch_elems(int idx, int B, int N);
// kernel family of entry `idx`: 0 wavefront per instance block, 1 lane per component
template <typename T>
int ipm_kind(int idx);
// structure-specialised twin of entry idx that the model (host [A B] row-major nx x (nx+nu),
// H, He) fits, else idx; and the structure id of an entry (0 dense)
template <typename T>
int ipm_refine(int idx, const double *AB, const double *H, const double *He);
template <typename T>
int ipm_structure(int idx);

// closed-loop step kernels (nmpc_closed_loop.hip)
template <typename T>
struct ClParams {
    int B, N, ny, ny_e, nx, nu;
    int plant;        // 0 controller model, 1 Crazyflie + force converter, 2 Crazyflie + jerk converter
    int period;       // reference rows per period (start row = (offset + step) % period)
    int table_cols;
    int step;
    int cost_stage;   // X_opt = x_{cost_stage} (0: force_model/controller.py:39, 1: jerk :39)
    int ncl, aed_dims, noise_dims, substeps;
    long long inst_base;
    unsigned long long seed;
    double noise_std, mass, g, dt, dt_conv;
    const T *table;   // [rows][table_cols]
    const int *offset;
    T *state;         // [B][nx]
    T *x0;            // engine input [B][nx]
    T *yref;          // engine input [B][N*ny + ny_e]
    const T *xout, *uout;
    const int *status;
    const T *A, *Bm, *c;   // plant == 0
    const T *wcl;     // [ncl]
    const double *noise_table;   // optional [B][noise_len] (replaces Philox draws)
    int noise_len;
    double *acc;      // [B][4] cost, aed numerator, failures, steps
};
template <typename T>
hipError_t cl_prepare_launch(const ClParams<T> &p, hipStream_t s);
template <typename T>
hipError_t cl_advance_launch(const ClParams<T> &p, hipStream_t s);

// plant simulator (nmpc_plant.hip)
hipError_t plant_step_launch(int batch, int num_stages, double T, double mass, double g,
                             const double *x_in, const double *u, double *x_out, hipStream_t s);

}  // namespace nmpc
