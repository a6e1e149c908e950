/*
 * nmpc.h — C-ABI of the MI355X batched NMPC solve engine (libnmpc_hip.so).
 *
 * Drop-in boundary for the reference's hot path. In the reference every closed-loop step
 * goes Python -> acados_template (ctypes) -> the generated `libacados_ocp_solver_<model>.so`:
 *
 *   reference call site                                   replaced by
 *   ---------------------------------------------------   -----------------------------------
 *   AcadosOcpSolver(ocp, json_file=...)                    nmpc_create()
 *     force_model/ocp.py:95-96, jerk_model/ocp.py:94-95     (JSON render + CasADi codegen +
 *     [ext: <name>_acados_create / ocp_nlp_* setup]          make + dlopen -> one C call)
 *   ocp_solver.set(k, 'yref', v)                           nmpc_set(h, inst, k, "yref", v, n)
 *     force_model/ocp.py:120-122, jerk_model/ocp.py:121-123
 *     [ext: ocp_nlp_cost_model_set(..., "yref")]
 *   ocp_solver.set(0, 'lbx'/'ubx', x0_bar)                 nmpc_set(h, inst, 0, "lbx"/"ubx", ...)
 *     force_model/controller.py:30-31, jerk_model/controller.py:31-32
 *     [ext: ocp_nlp_constraints_model_set(..., "lbx")]
 *   status = ocp_solver.solve()                            nmpc_solve(h)
 *     force_model/controller.py:32, jerk_model/controller.py:33
 *     [ext: <name>_acados_solve]
 *   ocp_solver.get(k, 'u' / 'x')                           nmpc_get(h, inst, k, "u"/"x", out, n)
 *     force_model/controller.py:37,39, jerk_model/controller.py:38-39
 *     [ext: ocp_nlp_out_get(..., "u")]
 *   ocp_solver.get_cost(), print_statistics()              nmpc_get_cost(), nmpc_get_stats()
 *     force_model/ocp.py:164, force_model/controller.py:34
 *   AcadosSimSolver.set/solve/get (plant step)             nmpc_sim_plant()
 *     force_model/ocp.py:108-112, jerk_model/ocp.py:110-113
 *
 * Every handle carries a batch dimension: `instance` selects one of `batch` independent
 * OCPs (instance = -1 in nmpc_set broadcasts to all). Batched host/device entry points
 * (nmpc_set_batch / nmpc_get_batch / nmpc_device_ptr) serve the batched drivers.
 *
 * Conventions: the engine owns its device buffers, the caller owns host buffers (copied in
 * and out). Return codes: >= 0 are acados solver status codes (src/Readme.md:14-20:
 * 0 success, 1 failure, 2 max iterations, 3 min step, 4 QP solver failed); < 0 are API
 * errors (NMPC_E*), with a message from nmpc_last_error(). One handle per host thread;
 * every handle runs on its own HIP stream unless nmpc_set_stream() supplies one.
 * All matrices are row-major doubles. A bound with |value| >= 1e20 means "no bound"
 * (acados ACADOS_INFTY convention).
 */
#ifndef NMPC_H
#define NMPC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NMPC_ABI_VERSION 2

/* solver status codes (acados, src/Readme.md:14-20) */
#define NMPC_SUCCESS 0
#define NMPC_FAILURE 1
#define NMPC_MAXITER 2
#define NMPC_MINSTEP 3
#define NMPC_QP_FAILURE 4

/* API error codes */
#define NMPC_EINVAL -1
#define NMPC_EDEVICE -2
#define NMPC_ENOMEM -3
#define NMPC_EUNSUPPORTED -4
#define NMPC_ESTATE -5

/* precision */
#define NMPC_FP64 0
#define NMPC_FP32 1

/* dynamics description */
#define NMPC_DYN_CONTINUOUS_AFFINE 0 /* x' = A x + B u + c, integrated by `integrator` */
#define NMPC_DYN_DISCRETE_AFFINE 1   /* x+ = A x + B u + c */

/* integrator_type (acados solver_options.integrator_type) */
#define NMPC_IRK 0 /* Gauss-Legendre collocation, num_stages (acados default 4) */
#define NMPC_ERK 1 /* explicit Runge-Kutta: 1 = Euler, 2 = midpoint, 4 = classic RK4 */

/* cost_scaling */
#define NMPC_COST_SCALING_TIME_STEPS 0 /* stage cost x time step, terminal x 1 (acados) */
#define NMPC_COST_SCALING_NONE 1

typedef struct nmpc_ocp_desc {
    int abi_version; /* = NMPC_ABI_VERSION */
    const char *name;
    /* dims (AcadosOcp.dims) */
    int nx, nu, N, ny, ny_e;
    /* dynamics (AcadosModel f_expl_expr of an affine model; replaces the CasADi-generated
     * integrator sensitivities of force_model/dynamics.py:32-47, jerk_model/dynamics.py:35-52) */
    int dyn_type;
    const double *A; /* nx*nx */
    const double *B; /* nx*nu */
    const double *c; /* nx */
    int integrator_type, num_stages, num_steps;
    double tf; /* horizon length; time step = tf / N (ocp.py:92-93) */
    /* LINEAR_LS cost (force_model/ocp.py:28-58) */
    const double *W, *Vx, *Vu; /* ny*ny, ny*nx, ny*nu */
    const double *W_e, *Vx_e;  /* ny_e*ny_e, ny_e*nx */
    const double *yref, *yref_e; /* initial cost.yref (ny) / cost.yref_e (ny_e); may be NULL */
    int cost_scaling;
    /* box constraints BGH (force_model/ocp.py:62-78); x at stage 0 is pinned by lbx=ubx */
    int nbu;
    const int *idxbu;
    const double *lbu, *ubu;
    int nbx;
    const int *idxbx;
    const double *lbx, *ubx; /* stages 1..N-1 */
    int nbx_e;
    const int *idxbx_e;
    const double *lbx_e, *ubx_e;
    const double *x0; /* constraints.x0 initial value (nx); may be NULL */
    /* QP / IPM options (solver_options.qp_solver_*) */
    int qp_solver_iter_max;    /* <= 0: 50 */
    double qp_solver_tol_comp; /* <= 0: 1e-15 (fp64) / 1e-7 (fp32); fp32 clamps to >= 1e-7 */
    double qp_solver_tol_res;  /* <= 0: 1e-12 (fp64) / 1e-5 (fp32); fp32 clamps to >= 1e-5 */
    double qp_solver_mu0;      /* <= 0: 1e-2 */
    /* exact finish (oracle/c/riccati_ipm.c): once mu <= qp_solver_polish_mu, a
     * primal-dual active-set run of at most qp_solver_polish_steps Newton steps from the current
     * iterate (active bounds held by a penalty, the others dropped; the first active set is
     * where the IPM multiplier exceeds the slack), then one refinement step; accepted when the
     * QP's KKT sign and bound conditions hold, else the IPM goes on and the next run waits for
     * mu to drop 100-fold. 0: 1 (first run at the start for the default mu0; fp64 handles only,
     * fp32 handles never run it); < 0: off. fp32 handles instead end each solve in their own
     * exact finish (the IPM's active bounds as the warm set of active-set steps on the fp64
     * projected inverse Hessian, fp64 KKT acceptance; env NMPC_FIN32=0 off) */
    double qp_solver_polish_mu;
    int qp_solver_polish_steps; /* <= 0: 12 */
} nmpc_ocp_desc;

typedef struct nmpc_solver nmpc_solver;

/* library / device */
int nmpc_abi_version(void);
int nmpc_device_count(void);
const char *nmpc_last_error_global(void);

/* lifecycle */
int nmpc_create(const nmpc_ocp_desc *desc, int batch, int device, int precision, nmpc_solver **out);
void nmpc_destroy(nmpc_solver *h);
const char *nmpc_last_error(const nmpc_solver *h);
int nmpc_set_stream(nmpc_solver *h, void *hip_stream); /* NULL: back to the handle's own stream */
void *nmpc_get_stream(nmpc_solver *h);

/* discrete model actually used on the device (after integration): A (nx*nx), B (nx*nu), c (nx) */
int nmpc_get_model(const nmpc_solver *h, double *A, double *B, double *c);

/* per-instance field access (AcadosOcpSolver.set/get). Fields:
 *   set: "yref" (stage 0..N-1: ny values, stage N: ny_e), "lbx"/"ubx" (stage 0 only: nx,
 *        must end up equal = x0_bar), "x0" (stage ignored: nx, sets lbx=ubx)
 *   get: "x" (stage 0..N: nx), "u" (stage 0..N-1: nu)
 * instance = -1 in nmpc_set applies the value to every instance. */
int nmpc_set(nmpc_solver *h, int instance, int stage, const char *field, const double *value, int n);
int nmpc_get(nmpc_solver *h, int instance, int stage, const char *field, double *out, int n);

/* batched host access. Fields and layouts (row-major, instance-major):
 *   "x0"   batch*nx                 (set)
 *   "yref" batch*(N*ny + ny_e)      (set; stage-stacked horizon window)
 *   "x"    batch*(N+1)*nx           (get)
 *   "u"    batch*N*nu               (get)
 *   "status", "qp_iter"  batch int32 (get; use nmpc_get_batch_int)
 * `count` = number of doubles supplied / requested, checked against the layout. */
int nmpc_set_batch(nmpc_solver *h, const char *field, const double *values, size_t count);
int nmpc_get_batch(nmpc_solver *h, const char *field, double *out, size_t count);
int nmpc_get_batch_int(nmpc_solver *h, const char *field, int32_t *out, size_t count);

/* device-resident access for batched drivers: the engine's own device buffer for a field
 * ("x0", "yref", "x", "u", "status", "qp_iter"), element type double (NMPC_FP64) or float
 * (NMPC_FP32) / int32. Writing "x0"/"yref" there before nmpc_solve_async() skips the copy. */
int nmpc_device_ptr(nmpc_solver *h, const char *field, void **out);

/* solve all instances. nmpc_solve: upload host-staged inputs, launch, wait, download; returns
 * the max status over instances (0 when every instance succeeded) or < 0 on API error.
 * nmpc_solve_async: launch on the handle's stream using the device buffers as they are;
 * returns immediately (no host staging). The solve is complete in stream order: with the fast solve
 * (nmpc_get_launch_info out[8]) its three launches (sf_kernel, fin64_kernel for the instances with a violated
 * bound, the full IPM in list mode for what the finish parks) read their list lengths on the device, so a
 * kernel or copy the caller enqueues behind nmpc_solve_async on the handle's stream (nmpc_set_stream) reads
 * the final x / u / status / qp_iter of every instance. Back-to-back nmpc_solve_async calls write the same
 * device outputs, each complete before the next starts. nmpc_synchronize waits for the stream. */
int nmpc_solve(nmpc_solver *h);
int nmpc_solve_async(nmpc_solver *h);
int nmpc_synchronize(nmpc_solver *h);

/* cost of the current solution of one instance (AcadosOcpSolver.get_cost, acados
 * LINEAR_LS semantics: sum_k s_k 1/2|y_k - yref_k|^2_W + 1/2|y_N - yref_N|^2_We) */
int nmpc_get_cost(nmpc_solver *h, int instance, double *cost);

/* statistics of the last solve: stats[0] = max qp_iter, stats[1] = mean qp_iter,
 * stats[2] = number of instances with status != 0, stats[3] = device time of the last
 * solve in ms (HIP events), stats[4] = sqp_iter (always 1: one QP solves an LQ-OCP),
 * stats[5] / stats[6] = the last fast solve's instances listed for the active-set finish / parked for the
 * full IPM (0 without the fast solve); n <= 7 values are written. stats[0..2] describe the outputs last
 * downloaded (nmpc_solve / nmpc_get_batch*), stats[3], [5], [6] the last solve waited for */
int nmpc_get_stats(nmpc_solver *h, double *stats, int n);

/* kernel geometry chosen for this handle: out[0] = instances per wavefront,
 * out[1] = workgroups per launch, out[2] = threads per workgroup, out[3] = LDS bytes/WG,
 * out[4] = kernel family (1: lane per component — the default, nx+nu lanes per instance;
 * 0: one wavefront per instance block, env NMPC_KERNEL=wave), out[5] = model structure the
 * kernel is specialised for (0: dense; 1 force, 2 jerk, 3 quad13; env NMPC_STRUCT=0 forces dense),
 * out[6] = the closed loop's kernel after nmpc_closed_loop_init (1: the lean loop, cl_fast_kernel; 2: the
 * lean loop's lockstep kernel cl_lock_kernel, four instances per wavefront on MFMA; 0: the fused / per-step
 * launches of the family above), out[7] = the lean loop's largest active set, out[8] = 1 when this handle's
 * plain solves (nmpc_solve / nmpc_solve_async) take the fast solve (fp64 handles of the compiled shapes:
 * sf_kernel's unconstrained solution + bound test, fin64_kernel's active-set steps for the instances with a
 * violated bound, the full IPM in list mode for what they leave; env NMPC_SOLVE_FAST=0 or an explicit
 * NMPC_KERNEL family: 0, every QP on the full IPM + exact finish) */
int nmpc_get_launch_info(const nmpc_solver *h, int *out, int n);

/* ------------------------------------------------------------------ batched closed loop
 * On-device closed loop around the solve: every step builds each instance's
 * yref window from a shared reference table (set_up_ocp, force_model/ocp.py:117-122), pins
 * x0 = current state, solves, accumulates the closed-loop cost (controller.py:40-41) and the
 * AED numerator (store_results.py:233-236), and advances the plant with one scalar noise draw
 * per step (ocp.py:114). Instances never exchange data; results are independent of sharding. */
#define NMPC_PLANT_MODEL 0           /* the controller's own discrete model x+ = A x + B u0 + c */
#define NMPC_PLANT_CRAZYFLIE_FORCE 1 /* src/plant.py, force converter, ERK4 over dt */
#define NMPC_PLANT_CRAZYFLIE_JERK 2  /* src/plant.py, jerk converter, substeps x Euler over dt_conv */

typedef struct nmpc_closed_loop_desc {
    int plant;
    const double *ref_table; /* ref_rows x ref_cols; yref_k = row[t+k][0:ny], yref_N = row[t+N][0:ny_e] */
    int ref_rows, ref_cols, ref_period; /* start row t = (offset + step) % ref_period */
    const int32_t *offsets;  /* batch start rows */
    const double *x_init;    /* batch*nx initial states (controller state: plant state [+ acceleration]) */
    long long instance_base; /* global id of this handle's instance 0 (noise stream key) */
    unsigned long long seed;
    double noise_std;
    int noise_dims;            /* NMPC_PLANT_MODEL: noise added to the first noise_dims states */
    const double *noise_table; /* optional batch*noise_len draws used instead of Philox (parity runs) */
    int noise_len;
    int cost_stage;            /* closed-loop cost on x_{cost_stage} of the solution (force 0, jerk 1) */
    int ncl;
    const double *w_cl;        /* ncl diagonal weights of the closed-loop cost */
    int aed_dims;              /* AED over the first aed_dims state components */
    double mass, g, dt, dt_conv;
    int substeps;
} nmpc_closed_loop_desc;

/* bind the closed loop to a solver handle (allocates the table/state/accumulators on the device) */
int nmpc_closed_loop_init(nmpc_solver *h, const nmpc_closed_loop_desc *d);
/* enqueue `steps` closed-loop steps on the handle's stream; sync != 0 waits for completion (polling the
 * stream: one host core busy for the wait; env NMPC_SPIN_WAIT=0 sleeps in hipStreamSynchronize).
 * Paths (the same results on every one; the choice may change from run to run on one handle):
 *   - the lean loop (nmpc_cl_fast.hip; quad13 / jerk / force shapes, fp64 and fp32 — fp32: fp32 tables
 *     and explicit form, fp64 W, set solves and acceptance — the default): launches of at
 *     most 64 steps; a step the fast path cannot solve parks, and the parked instances get their full solve
 *     in list mode, after which the fast kernel continues them. sync != 0: after each launch the host reads the
 *     park count and enqueues only the rounds needed. sync = 0: nothing waits — each chunk enqueues all its
 *     possible rounds (chunk length + 1 fast launches and list-mode solves), each guarded by the count of the
 *     round before on the device (an empty round returns at entry), so the run is asynchronous and complete
 *     in stream order, at the cost of the empty rounds' launches. fp32 handles: the list-mode full solve is
 *     the fp32 IPM without the exact finish (1e-3..1e-2 from the exact step solution, which the plant then
 *     carries);
 *     on the bench workloads no step parks (tests/test_gpu_bench_parity.py forces parks with
 *     NMPC_CLF_NO_GI=1 to measure it);
 *   - fused (lane-per-component and wavefront kernel families, NMPC_CL_FAST=0): each solve launch
 *     carries up to 64 steps of every instance (prepare + solve + advance per instance, no step barrier
 *     between instances); asynchronous with sync = 0;
 *   - per step (env NMPC_CL_FUSED=0): one prepare / solve / advance launch per step. */
int nmpc_closed_loop_run(nmpc_solver *h, int steps, int sync);
/* out[0] sum closed-loop cost, out[1] sum AED numerator, out[2] failed solves, out[3] instance-steps,
 * out[4] total device ms of the solve kernel launches of the last run (HIP events around each),
 * out[5] solve launches in the last run, out[6] mean qp_iter of the last step, out[7] closed-loop
 * steps of the last run, out[8] solves of the last run that parked (lean loop: list-mode full solves),
 * out[9] lean-loop fast-kernel launches of the last run; n <= 10 values are written */
int nmpc_closed_loop_stats(nmpc_solver *h, double *out, int n);
/* per-instance accumulators, batch*4: [cost sum, AED numerator, failed solves, steps] of each
 * instance (the Monte-Carlo distribution behind nmpc_closed_loop_stats' sums) */
int nmpc_closed_loop_instance_stats(nmpc_solver *h, double *out, size_t count);
/* tuning aid: with env NMPC_ITER_LOG set, the per-step solve record of the last run, rows*batch values
 * [row][instance]; returns the row count (out = NULL: the row count only, 0: no log). Layouts:
 *   - fused lane-per-component / wavefront kernels (NMPC_CL_FAST=0): the run's last launch, one row per
 *     step = finish steps | IPM iterations << 8 | status << 16;
 *   - the lean loop: the run's last launch (<= 64 steps) + 2 rows. Step rows = active-set steps (<= 255)
 *     | status << 8 | wall-clock ticks of the step (100 MHz, <= 32767) << 16; a step the list-mode
 *     fallback solved keeps the marker -1. The last two rows: each instance's start and end in that
 *     launch (wall-clock ticks, low 31 bits). */
int nmpc_closed_loop_iter_log(nmpc_solver *h, int32_t *out, size_t count);
/* the lean loop's trajectory outputs (opt-in; default off). The loop reads only u_0 and x_1 of each step's
 * solution (controller.py:37-41), so by default no trajectory is written to HBM. With on != 0, every later
 * nmpc_closed_loop_run on the lean loop writes each instance's last-step solution (x_0 = the state the
 * step started from) and downloads it with that step's status and qp_iter when the run ends: nmpc_get /
 * nmpc_get_batch / nmpc_get_batch_int then read them (nmpc_get_cost refuses: the loop's windows come
 * from its reference table). The fused and per-step paths (NMPC_CL_FAST=0 / NMPC_CL_FUSED=0) do not
 * expose their outputs either way. */
int nmpc_closed_loop_set_outputs(nmpc_solver *h, int on);
/* current closed-loop states, batch*nx */
int nmpc_closed_loop_get_state(nmpc_solver *h, double *out, size_t count);

/* plant simulator (AcadosSimSolver for src/plant.py:27-43): one step of the nonlinear 2-D
 * Crazyflie plant x=[px,pz,vx,vz], u=[theta, F_d] on the device for `batch` states.
 *   method NMPC_ERK, num_stages 4 over T (force_model/ocp.py:98-104), or
 *   method NMPC_ERK, num_stages 1 over T (jerk_model/ocp.py:97-104).
 * x_in/x_out: batch*4, u: batch*2 (host pointers). mass, g: plant constants. */
int nmpc_sim_plant(int device, int batch, int num_stages, double T, double mass, double g,
                   const double *x_in, const double *u, double *x_out);

#ifdef __cplusplus
}
#endif
#endif /* NMPC_H */
