// nmpc_internal.h — device-side parameter blocks shared by the HIP kernels and the C-ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>

#include <vector>

// A kernel launch whose error check sees that launch alone: hipLaunchKernelGGL reports through the thread's
// sticky last-error word, so a failure of an earlier, unrelated call (already reported at its own call site —
// every HIP return in nmpc_api.cpp is checked) is cleared first instead of being blamed on this launch.
#define NMPC_LAUNCH(...)        \
    do {                        \
        (void)hipGetLastError(); \
        hipLaunchKernelGGL(__VA_ARGS__); \
    } while (0)

namespace nmpc {

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
// Kernel parameters of the batched IPM solve (nmpc_ipm.hip). All pointers are device
// pointers. Model data (AB..ubnd) is shared by every instance of a handle.
template <typename T>
struct IpmParams {
    int B;          // instances
    int N;          // horizon
    int ny, ny_e;   // LINEAR_LS residual sizes
    int yref_is_z;  // y = [x; u] (selection Vx, Vu): use yref as the initial guess
    int g_diag;     // yref_is_z and G, Ge diagonal (diagonal W): g_c = G_rr y_r
    int max_iter;
    T tol_comp, tol_res, mu0, inv_m;
    T polish_mu;    // exact finish threshold (0: off)
    T polish_rho;   // penalty on the identified active bounds in the finish
    int polish_steps;   // active-set Newton steps per finish run
    int polish_first;   // ... in the first run of a solve (the warm-started one in the closed loop)
    T polish_drop;      // after a rejected run the next one waits for mu <= polish_drop * mu
    int warm_shift;     // fused closed loop: warm-start flags shifted by one stage (1) or as solved (0)
    int fast_mode;      // fused closed loop: fast exact finish on an empty warm set (1; 0 off, 2 not at a launch's first step)
    const T *AB;    // [nx][nx+nu]   discrete [A B], row-major
    const T *ABt;   // [nx+nu][nx]   its transpose
    const T *c;     // [nx]
    const T *H;     // [nz][nz]      stage Hessian (cost-scaled), z = [x; u]
    const T *He;    // [nx][nx]
    const T *G;     // [nz][ny]      stage gradient map: g_k = G yref_k
    const T *Ge;    // [nx][ny_e]
    const T *lbnd;  // [3][nz]       bounds: stage 0 (x entries absent), 1..N-1, N
    const T *ubnd;  // [3][nz]
    const T *lqr;   // [N][nz][nz+1] unconstrained Riccati records (nmpc_api.cpp lqr_table), or null
    const T *lqrf;  // [N][nz][1+2nu+nx] the fast finish's rollout records (lqr_table), or null
    const T *lqrw;  // [(N+1)nz]^2 projected inverse Hessian of the unconstrained problem (lqr_wmat), or null
    const T *x0;    // [B][nx]
    const T *yref;  // [B][N*ny + ny_e]
    T *xout;        // [B][N+1][nx]
    T *uout;        // [B][N][nu]
    int *status;    // [B]
    int *iters;     // [B]
    T *scratch;     // [ceil(B/(IPW*WPB))*IPW*WPB][scratch_elems_per_instance]
    unsigned long long *cycles;   // optional [B][5] clock cycles per sweep type A..D + total (tuning, env NMPC_SWEEP_CYCLES)
    int ipw;                      // lane-per-instance kernel: instances per wavefront (lanes 0 .. ipw-1)
    long long lpi_stride;         // lane-per-instance kernel: scratch elements between words (>= slots)
    // fused closed loop (lane-per-component and wavefront kernels): > 0 runs cl_steps closed-loop
    // steps per instance inside the solve kernel — yref window and x0 read from cl.table / cl.state,
    // the plant advance (cl_advance_instance) after each solve — with no grid-wide step barrier
    int cl_steps;
    ClParams<T> cl;
    const double *cl_noise;   // [B][cl_steps] noise draws of the launch's steps (cl_noise_launch)
    int *iter_log;            // optional [cl_steps][B]: finish steps | IPM iterations << 8 | status << 16 per fused step
    // fused closed loop, explicit unconstrained solution (nmpc_closed_loop_init): z_0 = T_x x_0 + v_t
    const T *cl_tx;           // [(N+1) nz][nx]
    const T *cl_v;            // [period][(N+1) nz]
    // list mode (lane-per-component kernel, cl_steps = 1): the fallback of the lean closed loop —
    // one cold full solve + plant step for each listed instance at its own step cl_istep[inst];
    // noise cl_noise[inst * cl_noise_ld + step - cl_noise_step0]; the solution's active flags to
    // cl_flags[inst][cl_eslot[k nz + r]] (bounded elements)
    const int *cl_list;
    int cl_count;                 // list length; with cl_count_dev: the grid's capacity (an upper bound)
    const int *cl_count_dev;      // or null: the list length on the device (read by the kernel), so the list can be
                                  // filled by an earlier kernel of the same stream with no host round trip
    int *cl_istep;
    int cl_noise_ld, cl_noise_step0;
    signed char *cl_flags;
    const int *cl_eslot;
    int cl_nslot;
};

// Lean fused closed loop (nmpc_cl_fast.hip): the exact finish's fast path, one wavefront per
// instance at a time, the bounded elements of z in per-lane "slots" (s = j * 64 + lane)
template <typename T>
struct ClFastParams {
    int B, N, ne, nslot;          // ne = (N + 1)(nx + nu); nslot = bounded elements (slot count)
    int period, table_cols, cost_stage, ncl, aed_dims, noise_dims, plant, substeps, ny, ny_e;
    double mass, g, dt, dt_conv;
    int target;                   // run every instance up to this closed-loop step
    int step0, noise_ld;          // noise[b][step - step0], row length noise_ld
    int polish_steps;             // active-set rounds of the fast path
    int gi;                       // 1: the dual active-set fallback runs; 0 (test knob): such steps park
    int lock_workers;             // lockstep kernel: wavefronts per workgroup that start in phase 2
    int lock_prio;                // lockstep kernel: phase-2 wavefronts at raised issue priority
    int lock_direct;              // lockstep kernel: the leading claim-order groups straight to the phase-2 queue (1: warm-started)
    int claim_global;             // cl_fast_kernel: instances from one device-wide counter (park_count[1])
    int wcache;                   // 1: the rare path's W column cache in LDS (quad13 / jerk shapes; env NMPC_CLF_WCACHE=0: off)
    const int *gorder;            // or null: claim position -> instance of the device-wide claim (clf_order_launch)
    const int *inst_map;          // or null: position -> instance of the per-workgroup claim ranges (nmpc_api.cpp
                                  // clf_xcd_map: each XCD's workgroups own a contiguous stretch of reference-table rows)
    unsigned char *demoted;       // [B] the previous launch's rare-path steps | 128 if its last solution left bounds
                                  // active (lockstep: 1 at demotion), or null: the claim order's key
    int order_buckets;            // claim order: 0 three groups (warm start, rare path, rest); 1 six
    int x1_slot;                  // slot (lane, j = 0) of x_1[0] (cost of the jerk loop: cost_stage 1)
    const T *table;               // reference table [rows][table_cols]
    const int *offset;            // [B]
    T *state;                     // [B][nx]
    double *acc;                  // [B][4] cost, AED numerator, failures, steps
    int *istep;                   // [B] closed-loop step each instance has reached
    signed char *flags;           // [B][nslot] the last solution's active flags (-1 lower, 1 upper)
    const double *noise;          // [B][noise_ld]
    const int *s_e, *s_src;       // [nslot] element index k nz + r; warm-start source code (nmpc_api.cpp clf_setup)
    const int *s_free;            // [nfree] the decision elements without a bound (outputs only)
    int nfree;
    const T *s_lb, *s_ub;         // [nslot]
    const T *s_tx;                // [nslot][nx] rows of T_x
    const T *vb;                  // [period][EPL * 64] v_t at the slots
    const T *vfull;               // [period][ne]
    const T *txfull;              // [ne][nx]
    const double *W;              // [ne][ne] projected inverse Hessian (lqr_wmat), fp64 for both precisions
    const T *lbnd, *ubnd;         // [3][nz]
    const T *AB, *c;              // [nx][nz], [nx]: the controller model (plant 0, certificate)
    const T *wcl;                 // [ncl]
    const T *uinit;               // [nu] inputs of the solver's initial point (failure output)
    T *xout, *uout;               // trajectories of the last solve (written at the last step when traj_out)
    int traj_out;                 // closed loop: 1 writes the last step's x / u trajectories (opt-in,
                                  // nmpc_closed_loop_set_outputs); the loop itself reads only u_0 / x_1
    int *status, *iters;
    int *park_count, *park_list;  // instances that need a full solve (list mode of ipm_lpc_kernel)
    const int *run_if;            // or null: the launch runs only if *run_if != 0 (the lean loop's asynchronous rounds:
                                  // the previous round's park count), else every workgroup returns at entry
    int *park_host;               // or null: the launch's last wavefront to exit writes the park count here (pinned
                                  // host word; the host-driven rounds read it after the stream wait, no copy)
    unsigned *exit_count;         // ... counting the exited wavefronts (device word, 0 between launches)
    // or null: each workgroup first writes its instances' noise draws of the launch's steps here ([B][noise_ld],
    // the buffer `noise` reads; per-workgroup claims only) — the chunk's noise kernel launch saved
    double *noise_gen;
    unsigned long long seed;
    long long inst_base;
    double noise_std;
    const double *noise_table;
    int noise_len;
    int *iter_log;                // optional [steps][B]: active-set steps (<= 255) | status << 8 | wall-clock ticks (<= 32767) << 16
    unsigned long long *cycles;   // diagnostic builds (NMPC_CLF_TIMING): [B][14] phase cycles / counts per instance
    unsigned *check;              // checked builds (NMPC_CLF_CHECK): bit mask of the failed index checks
    // the fp32 solve finish (fin32_kernel): z_0 of every element per instance ([B][z0_ld], fin32_z0_kernel),
    // the pinned states x0 [B][nx]; the lean loop leaves them null (z_0 from T_x x + v_t)
    const T *z0all;
    int z0_ld;
    const T *x0in;
    // the fp64 general solve's finish (fin64_kernel): the instances sf_kernel listed (work_list[0 .. *work_count)),
    // whose unconstrained solutions z_0 sf_kernel wrote to xout / uout (z0_xu = 1: z_0 read from there)
    const int *work_list, *work_count;
    int z0_xu;
};
// fp32 handles' exact finish of a solve (nmpc_cl_fast.hip): z_0 = M [x0; yref] + vc for every element on the
// f32 matrix cores, then per instance the lean loop's active-set machinery (fp64 W, solves and acceptance)
// from the IPM solution's active bounds. M: [m16 rows][kp] (rows = elements, zero-padded), vc [m16].
struct Fin32Z0Params {
    int B, nx, ystride, kp, m16;
    const float *M, *vc, *x0, *yref;
    float *z0;   // [B][m16]
};
hipError_t fin32_z0_launch(const Fin32Z0Params &p, hipStream_t s);
// false: no compiled finish for the shape and slot count (p.nslot)
bool fin32_launch(int nx, int nu, int sid, const ClFastParams<float> &p, int resident, hipStream_t s);
// resident workgroups of the finish for (nx, nu, nslot) on `device`; 0: none compiled
int fin32_resident(int nx, int nu, int nslot, int device);
// The fp64 general solve's common path (nmpc_solve_fast.hip sf_kernel): the unconstrained solution of every
// instance by the Riccati recursion on the shared factorisation (f64 MFMA, four instances per block group),
// x / u written unclamped, the bound test; instances with a violated bound listed for fin64_kernel.
struct SfParams {
    int B, N, ny, ystride;
    const double *tab;            // [N][sf_table_words] per-stage matrices / vectors (nmpc_api.cpp sf_setup)
    const double *gd;             // [nz] diagonal gradient map G_rr, then [nx] Ge_rr
    const double *AB, *c;         // [nx][nz], [nx]
    const double *lbnd, *ubnd;    // [3][nz]
    const double *x0, *yref;      // [B][nx], [B][ystride]
    double *xout, *uout;
    int *status, *iters;
    int *list_count, *list;       // instances whose unconstrained solution violates a bound
    int *next_counts;             // the next solve's [list, park] counters, zeroed by workgroup 0 (or null)
    unsigned long long *cycles;   // diagnostic builds (NMPC_SF_TIMING): [waves][8] phase clocks, or null
};
// per-stage table words for (nx, nu) (0: no compiled sf_kernel), its dynamic LDS bytes at horizon N
int sf_table_words(int nx, int nu);
size_t sf_lds_bytes(int nx, int nu, int N);
hipError_t sf_launch(int nx, int nu, const SfParams &p, hipStream_t s);
// the active-set finish of the instances sf_kernel listed (fp64; shapes and slot counts as fin32); the list's
// length is read on the device
hipError_t fin64_launch(int nx, int nu, const ClFastParams<double> &p, int resident, hipStream_t s);
int fin64_resident(int nx, int nu, int nslot, int device);
// compiled fast kernels: EPL slots per lane (0 if none for this shape)
int cl_fast_epl(int nx, int nu);
// largest active set of the fast path for the shape (oracle/cref.py WSMAX)
int cl_fast_wsmax(int nx, int nu);
// whether the shape has the lockstep kernel cl_lock_kernel (four instances per wavefront, MFMA explicit form;
// quad13 with the controller-model plant, jerk with the model or its converter plant; cost on x_0 or x_1)
bool cl_lock_shape(int nx, int nu);
// whether the shape has a cl_fast_kernel variant with W over the slots in LDS (the force shape)
bool cl_wlds_shape(int nx, int nu);
bool cl_one_shape(int nx, int nu);
// lean-loop kernel kinds: one instance per wavefront (W from L2 / from LDS), the lockstep kernel
// CLF_ONE: cl_fast_kernel compiled for one wavefront per SIMD (the whole register file; batches no larger than
// the device's SIMD count)
constexpr int CLF_FAST = 0, CLF_LOCK = 1, CLF_WLDS = 2, CLF_ONE = 3;
// workgroups of the shape's cl_fast_kernel (lock: cl_lock_kernel, fp64 only) in the handle's precision
// that `device` holds at once (the persistent grid), or 0
int cl_fast_resident(int nx, int nu, int sid, int kind, bool f64, int device);
// the lean-loop launch's workgroup count for `waves` (instances) and `resident` (cl_fast_launch's grid)
int cl_fast_grid(int nx, int nu, int sid, int kind, bool f64, int waves, int resident);
// every instance has its own wavefront from the launch's start (no claim order can matter)
bool cl_fast_fits(int nx, int nu, int sid, int kind, bool f64, int waves, int resident);
// grid = min(waves / wavefronts per workgroup, resident); waves = instances (lock: instances / 4)
template <typename T>
hipError_t cl_fast_launch(int nx, int nu, int sid, int kind, const ClFastParams<T> &p, int waves, int resident,
                          hipStream_t s);
// the device-wide claim's order for the next launch: the instances whose last solution left bounds active, then those
// with rare-path steps in the previous launch, then the rest, each group in instance order (one workgroup)
hipError_t clf_order_launch(const unsigned char *hard, int B, int *gorder, hipStream_t s);

size_t scratch_elems_per_instance(int N, int nx, int nu);

// returns an index into the kernel table (or -1), the chosen instances-per-wave, the
// static LDS bytes per workgroup and the wavefronts per workgroup. ipw_req <= 0 picks the
// widest packing compiled. Scratch must cover ceil(B / (ipw*wpb)) * ipw * wpb instances.
template <typename T>
int ipm_find(int nx, int nu, int ipw_req, int batch, int *ipw_out, int *lds_out, int *wpb_out);
template <typename T>
hipError_t ipm_launch(int idx, const IpmParams<T> &p, hipStream_t s);
// first dense compiled entry of family `kind` (0 wavefront, 1 lane per component) for (nx, nu), or -1
template <typename T>
int ipm_find_family(int nx, int nu, int kind);
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

// Condensed IPM (nmpc_cond.hip): one wavefront per instance, states eliminated on the host
// (nmpc_cond_host.cpp). Matrices are shared by every instance; layouts noted per field.
template <typename T>
struct CondParams {
    int B, N, nx, nu, n, nb, mx, ldg, nY, ny, yref_is_z, max_iter;
    int wave_elems;    // LDS elements per wavefront (cond_wave_elems)
    T tol_comp, tol_res, mu0, inv_m;
    const T *Gx;       // [16 nb][ldg] Gamma_x column-major (rows = bounded x rows), zero padded
    const T *H0;       // [n][n] condensed Hessian, column-major
    const T *H0t;      // lower 16x16 tiles of H0 (tile I(I+1)/2 + J, column-major within the tile)
    const T *Fx;       // [nx][n]  f = fc + Fx x0 + Fy yref (column-major)
    const T *Fy;       // [nY][n]
    const T *fc;       // [n]
    const T *Phx;      // [nx][mx] x-row offsets xf = dx + Phx x0 (column-major)
    const T *dx;       // [mx]
    const T *lox, *hix;   // [mx] x-row bounds (|b| >= 1e20: none)
    const T *lou, *hiu;   // [n] input bounds
    const int *xcols;  // [mx] nonzero columns of each x row (k nu)
    const int *rstart; // [n] first x row with a nonzero in column i
    const int *ks;     // [nb] first 4-row step of Gx with a nonzero in tile column block I
    const T *Gall;     // [n][(N+1) nx] outputs X = Phall x0 + dall + Gall U (column-major)
    const T *Phall;    // [nx][(N+1) nx]
    const T *dall;     // [(N+1) nx]
    const T *x0;       // [B][nx]
    const T *yref;     // [B][nY]
    T *xout, *uout;
    int *status, *iters;
    unsigned long long *cycles;   // optional [B][9] phase cycles (NMPC_COND_TIMING builds)
};
template <typename T>
hipError_t cond_launch(const CondParams<T> &p, int wpb, size_t lds_bytes, hipStream_t s);
template <typename T>
size_t cond_wave_elems(int nb, int ldg);

// host condensing of the stage-wise QP data (double); returns false if the dims are outside
// what the condensed kernels are compiled for (n <= 128, n + mx <= 512)
struct CondHost {
    int n = 0, nb = 0, mx = 0, ldg = 0, nY = 0;
    std::vector<double> Gx, H0, H0t, Fx, Fy, fc, Phx, dx, lox, hix, lou, hiu, Gall, Phall, dall;
    std::vector<int> xcols, rstart, ks;
};
bool cond_build(int nx, int nu, int N, int ny, int ny_e, const std::vector<double> &A, const std::vector<double> &Bm,
                const std::vector<double> &c, const std::vector<double> &H, const std::vector<double> &G,
                const std::vector<double> &He, const std::vector<double> &Ge, const std::vector<double> &lbnd,
                const std::vector<double> &ubnd, CondHost &out);

template <typename T>
hipError_t cl_prepare_launch(const ClParams<T> &p, hipStream_t s);
// noise draws of steps [step0, step0 + nsteps) for every instance: out[b][s] (cl_advance_instance's
// draw: the user table if given, else Philox / Box-Muller, else 0)
template <typename T>
hipError_t cl_noise_launch(const ClParams<T> &p, int step0, int nsteps, double *out, hipStream_t s, int *zero2 = nullptr);
template <typename T>
hipError_t cl_advance_launch(const ClParams<T> &p, hipStream_t s);

// plant simulator (nmpc_plant.hip)
hipError_t plant_step_launch(int batch, int num_stages, double T, double mass, double g,
                             const double *x_in, const double *u, double *x_out, hipStream_t s);

}  // namespace nmpc
