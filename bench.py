"""Benchmark: batched NMPC closed-loop steps/s on MI355X (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W --model quad13 --batch 8192 --precision fp64]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Workload (BASELINE.json metric "NMPC steps/sec (batched trajectories), N=20 nx=13 nu=4"):
the synthetic quad13 OCP (nx=13, nu=4, horizon N=20, no reference counterpart: SURVEY §0),
B = 8192 independent closed-loop trajectories per GPU (weak scaling), fp64. One step = for
every instance: build the yref window + pin x0 (set_up_ocp, ocp.py:117-122), solve the OCP
(AcadosOcpSolver.solve, controller.py:32) to its exact solution (the lean closed loop,
cl_fast_kernel: explicit unconstrained solution, warm-started primal-dual active-set steps, the
dual active-set fallback, KKT-checked; full IPM + finish for what is left), advance
the plant with Philox noise and accumulate cost/AED — all resident in HBM. value = instances x steps / wall time (max over ranks) for all ranks together. Ranks
exchange nothing during the run; RCCL (torch.distributed "nccl") reduces the cost/AED/failure
statistics once at the end.

Also reported (one JSON line on rank 0):
  roofline — the closed-loop kernel (the dominant kernel: cl_fast_kernel, or the fused solve kernel
    with NMPC_CL_FAST=0), bound "valu_fp64": achieved = the FP64 flops per instance-step that the CPU
    baseline executes on the same closed loop (the same algorithm, counted per path it takes:
    explicit solution 2 nx per element, active-set steps m^3/3 + 2 m^2 + 2 ne m, the dual fallback's
    iterations, full solves SURVEY §8d's F_iter per Newton system, plant 2 nx nz)
    x B / the kernel's mean duration per step from HIP events around each launch; peak = MI355X
    FP64 78.6 TFLOP/s (the FP64 vector and matrix peaks are equal). executed_frac = the FP64 flops
    the kernel really issues (SQ_INSTS_VALU_FLOPS_FP64 of the committed rocprofv3 PMC pass, idle
    lanes included) / kernel time / peak. traffic = memory-side bytes per step (FETCH_SIZE +
    WRITE_SIZE) from the same PMC pass (profiles/pmc_traffic.json) when one matches, else null.
  cpu_baseline — oracle/c/riccati_ipm.c's closed loop in mode 1 (the GPU's algorithm: warm-started
    fast finish, fp64, OpenMP over instances) on the host cores, rank 0 at N=1 only, over the same
    instances and steps as the timed GPU run.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_TFLOPS = {"fp64": 78.6, "fp32": 157.3}   # MI355X vector = matrix peaks (MI355X_MICROARCH)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="quad13", choices=["quad13", "force", "jerk"])
    ap.add_argument("--batch", type=int, default=8192, help="instances per GPU")
    ap.add_argument("--horizon", type=int, default=None)
    ap.add_argument("--precision", default="fp64", choices=["fp64", "fp32"])
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--repeats", type=int, default=10,
                    help="timed regions of --steps steps each; value = the median region (BASELINE.md: median of >= 10)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--python-loop-steps", type=int, default=100,
                    help="steps of the B=1 Python drop-in loop timed for BASELINE config 1 (0: skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL over xGMI, the default); gloo only to rehearse several ranks "
                         "on a one-GPU box (ranks then share the visible GPUs round-robin)")
    return ap.parse_args()


def ipm_tolerances(model, N, precision="fp64"):
    """(tol_comp, tol_res, polish_mu, polish_steps) the engine runs with: the model's OCP solver
    options (library defaults 1e-15 / 1e-12 when unset), clamped to >= 1e-7 / 1e-5 for fp32
    handles exactly as nmpc_create does (nmpc_api.cpp); the exact finish (from mu <= 1, <= 12
    active-set steps) on fp64 handles only (include/nmpc.h qp_solver_polish_*)."""
    from drone_attitude_control_amd.models import OCPS
    from oracle import cref
    o = OCPS[model](N).solver_options
    tc, tr = float(o.qp_solver_tol_comp or 1e-15), float(o.qp_solver_tol_stat or 1e-12)
    pm = getattr(o, "qp_solver_polish_mu", None) or 0.0
    pm = 0.0 if pm < 0 or precision != "fp64" else (pm or cref.DEFAULT_POLISH_MU)
    ps = int(getattr(o, "qp_solver_polish_steps", None) or cref.DEFAULT_POLISH_STEPS)
    if precision == "fp32":
        tc, tr = max(tc, 1e-7), max(tr, 1e-5)
    return tc, tr, pm, ps


def cpu_baseline(model, N, table, offsets, x_init, warmup, steps, seconds, precision, seed):
    """Time the C oracle's closed loop in mode 1 — the GPU's algorithm (warm-started fast finish on
    the shared factorisation, full IPM + finish where it fails; fp64 arithmetic, the handle's
    options) — on the same instances and steps as the timed GPU run: `warmup` untimed steps, then
    `steps` timed ones (all host threads; fewer instances if the whole batch would take longer than
    ~`seconds`), then a single-thread figure on a slice. Also returns the FP64 flops per
    instance-step it executed over the timed steps (the roofline credit)."""
    from oracle import cref, models
    spec = models.MODELS[model](N)
    tc, tr, pm, ps = ipm_tolerances(model, N, precision)

    def loop(n, threads, nsteps):
        cl = cref.ClosedLoopRef(spec, model, table, offsets[:n], x_init[:n], mode=1, seed=seed,
                                tol_comp=tc, tol_res=tr, polish_mu=pm, polish_steps=ps)
        cl.run(warmup, nthreads=threads)
        c0 = cl.stats()
        t0 = time.perf_counter()
        cl.run(nsteps, nthreads=threads)
        el = time.perf_counter() - t0
        c1 = cl.stats()
        return el, {k: c1[k] - c0[k] for k in c1}

    threads = cref.RiccatiIpmRef(spec).max_threads()
    B = len(offsets)
    # probe the rate on a slice, then size the sample to ~`seconds`
    n0, s0 = min(B, 256), max(1, min(steps, 20))
    el, _ = loop(n0, threads, s0)
    n = int(min(B, max(n0, n0 * s0 / max(el, 1e-6) * seconds / max(1, steps))))
    el, st = loop(n, threads, steps)
    n1 = min(n, 128)
    e1, _ = loop(n1, 1, steps)
    solves = max(1.0, st["solves"])
    paths = {k: st[k] / solves for k in ("fast_unconstrained", "fast_set", "full", "failed")}
    return {"value": n * steps / el, "unit": "NMPC steps/s", "cores": threads, "kind": "port",
            "sample": f"{n} of the {B} bench instances, closed-loop steps {warmup}..{warmup + steps - 1} ({model}, "
                      f"N={N}, fp64 arithmetic) in {el:.2f} s after {warmup} untimed steps: oracle/c/riccati_ipm.c "
                      f"riccati_ipm_closed_loop mode 1 (the GPU's algorithm: warm-started fast finish, explicit "
                      f"unconstrained solution, active-set steps on the shared factorisation, full IPM + exact finish "
                      f"where they fail; tol_comp {tc:g} / tol_res {tr:g}), OpenMP over instances, -O3 -march=x86-64-v3",
            "paths_per_step": paths, "flops_per_instance_step": st["flops"] / solves,
            "single_core": {"value": n1 * steps / e1, "cores": 1,
                            "sample": f"{n1} of those instances, the same steps, in {e1:.2f} s"}}, st["flops"] / solves


def load_pmc(model, N, batch, precision, kernel):
    """The committed rocprofv3 PMC summary entry (profiles/pmc_traffic.json) for this config and
    solve kernel, if one matches: memory-side bytes per launch and MFMA instructions per launch."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return {}
    try:
        d = json.load(open(path))
        for e in d.get("entries", []):
            if (e.get("model"), e.get("N"), e.get("batch"), e.get("precision")) == (model, N, batch, precision) \
                    and e.get("kernel", kernel) == kernel:
                return e
    except (ValueError, OSError):
        return {}
    return {}


def python_loop_rate(N, steps):
    """BASELINE config 1: the reference's single-trajectory closed loop (force_model/controller.py
    :25-54) as the drop-in sees it — per step 31 yref set() calls, lbx/ubx, solve(), get(), the
    converter and one plant step, each a Python -> C-ABI call (the QP and the plant on the GPU)."""
    from drone_attitude_control_amd import controllers
    from drone_attitude_control_amd.models import gen_circle_traj
    ref = gen_circle_traj(500, N, 6, 2)
    x0 = np.array([1.0, 0, 0, 0.62])
    controllers.force_follow_trajectory(ref[:, :4], ref[:, 4:6], x0, False, verbose=False, N=N, n_steps=3)
    t0 = time.perf_counter()
    controllers.force_follow_trajectory(ref[:, :4], ref[:, 4:6], x0, False, verbose=False, N=N, n_steps=steps)
    el = time.perf_counter() - t0
    return {"value": steps / el, "unit": "NMPC steps/s", "batch": 1,
            "sample": f"{steps} steps of controllers.force_follow_trajectory (force, N={N}, B=1, fp64) in {el:.2f} s"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    device = local_rank
    if world > 1:
        # torch first: its HIP runtime (soname libamdhip64.so.7) is then shared by libnmpc_hip
        import torch
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            torch.cuda.set_device(local_rank)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            device = local_rank % max(1, torch.cuda.device_count())
            dist.init_process_group("gloo")

    from drone_attitude_control_amd.batched import DEFAULT_N, ClosedLoop
    from drone_attitude_control_amd.sharding import rank_workload, reduce_run

    model = args.model
    N = args.horizon or DEFAULT_N[model]
    B = args.batch
    table, offsets_r, x_r, base = rank_workload(model, N, B, world, rank, args.seed)
    cl = ClosedLoop(model, B, N=N, device=device if world > 1 else 0, precision=args.precision,
                    table=table, offsets=offsets_r, x_init=x_r, instance_base=base, seed=args.seed)
    nx, nu = cl.solver.nx, cl.solver.nu

    # CPU baseline and the B=1 Python drop-in loop first (rank 0, single-GPU runs only)
    cpu, flops_cpu, pyloop = None, None, None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, flops_cpu = cpu_baseline(model, N, table, offsets_r, x_r, args.warmup, args.repeats * args.steps,
                                      args.cpu_seconds, args.precision, args.seed)
        if args.python_loop_steps > 0:
            pyloop = python_loop_rate(20, args.python_loop_steps)
            cpu["python_loop"] = pyloop

    def barrier():
        if dist is not None:
            dist.barrier()

    cl.run(args.warmup, sync=True)
    regions, kernel_ms_r = [], []
    for _ in range(max(1, args.repeats)):
        barrier()
        t0 = time.perf_counter()
        cl.run(args.steps, sync=True)
        t1 = time.perf_counter()
        barrier()
        regions.append(t1 - t0)
        st = cl.stats()
        # solve-kernel time per closed-loop step (a fused launch carries all the region's steps)
        kernel_ms_r.append(st["solve_kernel_ms"] / max(1, st["steps"]))
    regions = np.array(regions)
    st = cl.stats()
    red = np.array([st["cost_sum"], st["aed_sum"], st["failed"], st["instance_steps"]])
    # one SUM of the statistics and one MAX of the timings over RCCL, after the timed regions
    red, regions, kernel_ms_r = reduce_run(dist, red, regions, np.array(kernel_ms_r),
                                           device="cuda" if dist is not None and args.dist_backend == "nccl" else None)
    regions = np.atleast_1d(regions)
    kernel_ms_r = np.atleast_1d(kernel_ms_r)
    med = int(np.argsort(regions)[len(regions) // 2])
    elapsed = float(regions[med])
    kernel_ms = float(np.median(kernel_ms_r))

    if rank == 0:
        tols = ipm_tolerances(model, N, args.precision)
        value = world * B * args.steps / elapsed
        # credit: the FP64 flops per instance-step the CPU baseline executes on the same closed loop
        # (same algorithm, same steps); without it (multi-rank runs) the engine's own path mix is
        # unknown here and the credit falls back to one explicit unconstrained solution per step
        nz_, ne_ = nx + nu, (N + 1) * (nx + nu)
        fl_step = flops_cpu if flops_cpu is not None else 2.0 * nx * (ne_ - nx - nu) + 2.0 * nx * nz_
        fl_launch = fl_step * B
        achieved = fl_launch / (kernel_ms * 1e-3) / 1e12
        peak = PEAK_TFLOPS[args.precision]
        info = cl.solver.launch_info()
        kernel = info["closed_loop_kernel"] if info["closed_loop_kernel"] != "fused" else info["kernel"]
        pmc = load_pmc(model, N, B, args.precision, kernel)
        headline = model == "quad13" and N == 20
        metric = ("NMPC steps/sec (batched trajectories), N=20 nx=13 nu=4, 1/2/4/8 MI355X" if headline else
                  f"NMPC steps/sec (batched trajectories), N={N} nx={nx} nu={nu} ({model}), 1/2/4/8 MI355X")
        line = {
            "metric": metric,
            "value": value,
            "unit": "NMPC steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64" if args.precision == "fp64" else "f32",
            "data": "synthetic (seeded closed-loop Monte-Carlo instances on the reference circle)",
            "config": {"workload": f"{model} closed-loop NMPC step: yref window + x0 pin + IPM solve "
                                   f"(tol_comp {tols[0]:g}, tol_res {tols[1]:g}, exact finish from mu <= {tols[2]:g}, <= {tols[3]} active-set steps) + plant/noise advance",
                       "model": model, "nx": nx, "nu": nu, "horizon_N": N, "batch_per_gpu": B,
                       "global_batch": B * world, "parallelism": f"instance-sharded x{world}, "
                                                                    f"{'gloo' if args.dist_backend == 'gloo' else 'RCCL'} stats reduce",
                       "instances_per_wave": info["instances_per_wave"]},
            "timing": {"regions": len(regions), "steps_per_region": args.steps, "value_from": "median region",
                       "region_ms": [round(float(r) * 1e3, 4) for r in regions],
                       "spread": float((regions.max() - regions.min()) / elapsed),
                       "iqr_rel": float((np.percentile(regions, 75) - np.percentile(regions, 25)) / elapsed),
                       "note": "each region is one fused launch whose time is set by its slowest wavefront; "
                               "region-to-region differences below the IQR are not resolved"},
            "roofline": {"bound": "valu_fp64" if args.precision == "fp64" else "valu_fp32",
                         "pipe": ("FP64 FMA on the VALU" if args.precision == "fp64" else "FP32 FMA on the VALU")
                         + " (MI355X: FP64 matrix peak = FP64 vector peak; FP32 matrix peak = FP32 vector peak)",
                         "kernel": kernel, "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                         "frac": achieved / peak,
                         "credit": "FP64 flops per instance-step of the CPU baseline's run of the same algorithm on "
                                   "the same steps (oracle closed loop mode 1, counted per path: explicit solution "
                                   "2 nx per element, active-set steps m^3/3 + 2 m^2 + 2 ne m, full solves F_iter "
                                   "(SURVEY 8d) per Newton system, plant 2 nx nz) x B / kernel time per step",
                         "flops_per_instance_step": fl_step, "flops_per_launch": fl_launch, "kernel_ms": kernel_ms,
                         "executed_fp64_flops_per_step": pmc.get("fp64_flops_per_step"),
                         "executed_frac": (pmc["fp64_flops_per_step"] / (kernel_ms * 1e-3) / 1e12 / peak
                                           if pmc.get("fp64_flops_per_step") else None),
                         "executed_note": "FP64 flops the kernel issues (64 x SQ_INSTS_VALU_FLOPS_FP64 per step, idle "
                                          f"lanes included; {pmc.get('source', 'no PMC pass for this config')}) / this "
                                          "run's kernel time / peak",
                         "mfma_instructions_per_launch": pmc.get("mfma_insts_per_launch"),
                         "traffic": pmc.get("hbm_bytes_per_step", pmc.get("hbm_bytes_per_launch")),
                         "traffic_note": "FETCH_SIZE + WRITE_SIZE per closed-loop step (per launch / fused steps per "
                                         "launch) from the committed rocprofv3 PMC pass "
                                         f"({pmc.get('source', 'none for this config')}); no x2 FETCH_SIZE "
                                         "correction: the kernel's loads are 4/8-B per lane, the guide's x2 is "
                                         "calibrated for 16-B streams; includes Infinity-Cache hits",
                         "gpu_mean_qp_iter": st["mean_qp_iter"]},
            "solve_only": {"value": world * B / (kernel_ms * 1e-3), "unit": "QP solves/s",
                           "note": "solve kernel alone (median of the regions' mean launch durations, HIP events), "
                                   "all ranks"},
            "cpu_baseline": cpu,
            "closed_loop": {"mean_cost_per_step": red[0] / max(1.0, red[3]),
                            "aed": red[1] / max(1.0, red[3]) / (2 if model != "quad13" else 3),
                            "failed_solves": int(red[2]), "instance_steps": int(red[3])},
        }
        print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
