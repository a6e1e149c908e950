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
HBM_PEAK_GBS = 8000.0                           # MI355X HBM3E spec peak (MI355X_MICROARCH: 6.29 TB/s measured copy)


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
    ap.add_argument("--mode", default="closed_loop", choices=["closed_loop", "solve"],
                    help="closed_loop (default, the BASELINE metric): the batched closed loop; solve: the "
                         "general batched nmpc_solve on per-instance yref windows (the reference's "
                         "set(k,'yref') / solve() pattern, src/force_model/ocp.py:117-122, controller.py:32)")
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


def load_pmc(model, N, batch, precision, kernel, steps_per_launch, mode="closed_loop"):
    """The committed rocprofv3 PMC summary entry (profiles/pmc_traffic.json) for this config, kernel
    and launch length, if one matches: memory-side bytes per launch, executed FP64 flops and MFMA
    instructions. An entry measured on launches of another length is refused (a launch's fixed costs —
    the trajectory write-back, the per-instance record loads — are spread over its steps)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return {}
    try:
        d = json.load(open(path))
        for e in d.get("entries", []):
            if (e.get("model"), e.get("N"), e.get("batch"), e.get("precision")) == (model, N, batch, precision) \
                    and e.get("kernel", kernel) == kernel and e.get("mode", "closed_loop") == mode \
                    and e.get("steps_per_launch") == steps_per_launch:
                return e
    except (ValueError, OSError):
        return {}
    return {}


def min_bytes_per_instance_step(nx, nu, precision):
    """Minimal algorithmic bytes of one closed-loop instance-step with the shared reference table:
    x0 and the start offset (int32) in, u0 and x1 out ('with a shared reference table,
    per-instance input drops to x0 + offset')."""
    w = 8 if precision == "fp64" else 4
    return (2 * nx + nu) * w + 4


def mfma_block(pmc, kernel_ms, spl):
    """MFMA use of the timed kernel from the committed PMC pass at this launch length: the f64 matrix
    instructions (the lockstep kernel's v_mfma_f64_4x4x4_4b_f64: 4 blocks x 4x4x4 x 2 = 512 flops each), their
    flops against the FP64 matrix peak at this run's kernel time, and the MFMA pipe's busy fraction
    (SQ_VALU_MFMA_BUSY_CYCLES over GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)."""
    n = pmc.get("mfma_f64_insts_per_launch")
    if n is None:
        return None
    fl = 512.0 * n / spl   # per closed-loop step
    busy, gui = pmc.get("mfma_busy_cycles_per_launch"), pmc.get("gui_active_per_launch")
    return {"f64_insts_per_step": n / spl, "f64_flops_per_step": fl,
            "achieved_tflops": fl / (kernel_ms * 1e-3) / 1e12,
            "frac_of_fp64_matrix_peak": fl / (kernel_ms * 1e-3) / 1e12 / PEAK_TFLOPS["fp64"],
            "pipe_busy_frac": (busy / (gui / 8.0 * 1024.0)) if busy and gui else None,
            "wait_any_frac": pmc.get("wait_any_frac"),
            "note": "from the committed rocprofv3 PMC pass at this launch length (" + str(pmc.get("source")) + ")"}


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


def fail(msg, code=2):
    sys.stderr.write(f"bench.py: {msg}\n")
    sys.exit(code)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args):
    """`bench.py --gpus N` with N > 1 and no launcher around it (no WORLD_SIZE in the environment): start
    the N ranks ourselves — torch.distributed.run as a child process, one rank per GPU, rendezvous on
    127.0.0.1 — and relay rank 0's one JSON line. Runs before anything in this process imports torch or
    touches the GPU (the parent only waits; it never execs). Exits non-zero when a rank fails or when the
    line's n_gpus is not N."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", NMPC_BENCH_SELF_LAUNCH=str(args.gpus))
    sys.stderr.write("bench.py: starting %d ranks: %s\n" % (args.gpus, " ".join(cmd)))
    p = subprocess.run(cmd, stdout=subprocess.PIPE, env=env)
    out = p.stdout.decode(errors="replace")
    lines = [l for l in out.splitlines() if l.startswith("{")]
    if p.returncode != 0 or not lines:
        sys.stderr.write(out)
        fail(f"the {args.gpus}-rank run failed (exit {p.returncode})", p.returncode or 1)
    line = json.loads(lines[-1])
    if line.get("n_gpus") != args.gpus:
        fail(f"the run reported n_gpus {line.get('n_gpus')}, asked for --gpus {args.gpus}", 3)
    os.write(1, (lines[-1] + "\n").encode())
    sys.exit(0)


def init_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        fail(f"world size {world} (WORLD_SIZE) differs from --gpus {args.gpus}")
    dist = None
    device = local_rank
    # a process group whenever torch.distributed.run launched us (RANK in the environment), also at
    # world size 1: the RCCL reduction of the statistics then runs on a real communicator
    if world > 1 or "RANK" in os.environ:
        # torch first: its HIP runtime (soname libamdhip64.so.7) is then shared by libnmpc_hip
        import torch
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            # one GPU per rank (device_count() does not initialise the GPU on this image)
            if torch.cuda.device_count() < world:
                fail(f"backend nccl (RCCL) needs one GPU per rank: {world} ranks, "
                     f"{torch.cuda.device_count()} visible GPUs (use --dist-backend gloo to rehearse)")
            torch.cuda.set_device(local_rank)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            device = local_rank % max(1, torch.cuda.device_count())
            dist.init_process_group("gloo")
    return world, rank, dist, device


def parallelism_label(dist, world):
    """config.parallelism: the sharding and the backend of the process group that reduced the statistics
    (dist.get_backend() of the live group: "nccl" is RCCL on ROCm)."""
    if dist is None:
        return f"instance-sharded x{world}, single process (no collective)"
    be = dist.get_backend()
    how = (f", {world} ranks started by bench.py --gpus {world} (torch.distributed.run child)"
           if os.environ.get("NMPC_BENCH_SELF_LAUNCH") else "")
    return f"instance-sharded x{world}, {'RCCL' if be == 'nccl' else be} stats reduce ({be} process group){how}"


def timing_block(regions, elapsed, note):
    return {"regions": len(regions), "value_from": "median region",
            "region_ms": [round(float(r) * 1e3, 4) for r in regions],
            "spread": float((regions.max() - regions.min()) / elapsed),
            "iqr_rel": float((np.percentile(regions, 75) - np.percentile(regions, 25)) / elapsed),
            "note": note}


def workload_label(model, tols, paths, kernel):
    """config.workload: what the timed step runs (`kernel`: the closed-loop kernel launch_info reports),
    with the path mix of the CPU run of the same algorithm over the same steps (None on multi-rank runs,
    which skip the CPU baseline)."""
    mix = ("path mix not measured in this run (the CPU baseline, which counts it, runs at N=1 only)" if paths is None
           else f"of the solves {paths['fast_unconstrained']:.2%} the explicit unconstrained solution, "
                f"{paths['fast_set']:.2%} warm-started active-set steps on W (incl. the dual active-set fallback), "
                f"{paths['full']:.3%} the full IPM + exact finish, {paths['failed']:.3%} certified infeasible "
                f"(status 4) — counted by the CPU run of the same algorithm over the timed steps")
    what = {"cl_lock_kernel": "the lockstep lean loop (cl_lock_kernel: 4 instances per wavefront on the f64 matrix "
                              "cores, demoted instances on the single-instance path)",
            "cl_fast_kernel": "the lean loop (cl_fast_kernel: one wavefront per instance)"}.get(
        kernel, f"the fused closed loop ({kernel})")
    return (f"{model} closed-loop NMPC step on {what}: yref window from the shared "
            f"reference table + x0 pin + the QP solved to its exact, KKT-checked solution ({mix}; "
            f"full-solve options tol_comp {tols[0]:g}, tol_res {tols[1]:g}) + plant/noise advance + cost/AED")


_JSON_FD = None


def claim_stdout():
    """Keep stdout for the one JSON line: everything else written to fd 1 from here on — RCCL's version banner at
    the first collective, library prints — goes to stderr (the driver parses stdout)."""
    global _JSON_FD
    if _JSON_FD is None:
        sys.stdout.flush()
        _JSON_FD = os.dup(1)
        os.dup2(2, 1)


def emit(line):
    os.write(_JSON_FD if _JSON_FD is not None else 1, (json.dumps(line) + "\n").encode())


def main():
    args = parse()
    if args.gpus < 1:
        fail(f"--gpus {args.gpus}")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        launch_ranks(args)
    claim_stdout()
    world, rank, dist, device = init_dist(args)
    if args.mode == "solve":
        return main_solve(args, world, rank, dist, device)

    from drone_attitude_control_amd.batched import DEFAULT_N, ClosedLoop
    from drone_attitude_control_amd.sharding import rank_workload, reduce_run

    model = args.model
    N = args.horizon or DEFAULT_N[model]
    B = args.batch
    table, offsets_r, x_r, base = rank_workload(model, N, B, world, rank, args.seed)
    cl = ClosedLoop(model, B, N=N, device=device if world > 1 else 0, precision=args.precision,
                    table=table, offsets=offsets_r, x_init=x_r, instance_base=base, seed=args.seed)
    nx, nu = cl.solver.nx, cl.solver.nu
    info = cl.solver.launch_info()
    # the lean loop runs the exact fast path in both precisions (fp32: fp32 tables and explicit form, fp64
    # set solves and acceptance), so its CPU counterpart is the fp64 oracle loop with the exact finish
    lean = info["closed_loop_kernel"] != "fused"

    # (the CPU baseline runs after the timed regions: ahead of them it left the GPU idle for its 10-30 s and the
    # first regions ran while the clocks ramped up — 0.38 ms against 0.25-0.30 ms, profiles/r7/evidence_r7z2)
    x_cpu = np.array(x_r, copy=True)

    def barrier():
        if dist is not None:
            dist.barrier()

    cl.run(args.warmup, sync=True)
    regions, kernel_ms_r, parked = [], [], 0
    for _ in range(max(1, args.repeats)):
        barrier()
        t0 = time.perf_counter()
        cl.run(args.steps, sync=True)
        t1 = time.perf_counter()
        barrier()
        regions.append(t1 - t0)
        st = cl.stats()
        parked += st["parked"]
        # closed-loop kernel time per step (a launch carries up to 64 of the region's steps)
        kernel_ms_r.append(st["solve_kernel_ms"] / max(1, st["steps"]))
    regions = np.array(regions)
    st = cl.stats()
    red = np.array([st["cost_sum"], st["aed_sum"], st["failed"], st["instance_steps"]])
    # CPU baseline and the B=1 Python drop-in loop (rank 0, single-GPU runs only), from the same initial states
    cpu, flops_cpu, pyloop = None, None, None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, flops_cpu = cpu_baseline(model, N, table, offsets_r, x_cpu, args.warmup, args.repeats * args.steps,
                                      args.cpu_seconds, "fp64" if lean else args.precision, args.seed)
        if args.python_loop_steps > 0:
            pyloop = python_loop_rate(20, args.python_loop_steps)
            cpu["python_loop"] = pyloop
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
        # the pipe the credited flops run on: an fp32 handle on the lean loop does its credited work (active-set
        # solves, W combinations, acceptance) in fp64 — the PMC passes count ~20x more FP64 than FP32 flops there
        arith = "fp64" if args.precision == "fp64" or lean else "fp32"
        peak = PEAK_TFLOPS[arith]
        kernel = info["closed_loop_kernel"] if info["closed_loop_kernel"] != "fused" else info["kernel"]
        spl = min(args.steps, 64)   # steps per launch of the timed regions (clf_run / fused chunks)
        pmc = load_pmc(model, N, B, args.precision, kernel, spl)
        headline = model == "quad13" and N == 20
        metric = ("NMPC steps/sec (batched trajectories), N=20 nx=13 nu=4, 1/2/4/8 MI355X" if headline else
                  f"NMPC steps/sec (batched trajectories), N={N} nx={nx} nu={nu} ({model}), 1/2/4/8 MI355X")
        min_b = min_bytes_per_instance_step(nx, nu, args.precision) * B
        traffic = pmc.get("hbm_bytes_per_step")
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
            "dtype_note": None if args.precision == "fp64" or not lean else
            "fp32 handle on the lean loop: fp32 storage (explicit-form tables, bounds, state, trajectories), explicit "
            "form and fast-path bound tests in fp32; W kept in fp64, and active-set solves, W[:, S] nu combinations, "
            "set targets and KKT acceptance in fp64",
            "data": "synthetic (seeded closed-loop Monte-Carlo instances on the reference circle)",
            "config": {"workload": workload_label(model, tols, cpu and cpu.get("paths_per_step"), kernel),
                       "model": model, "nx": nx, "nu": nu, "horizon_N": N, "batch_per_gpu": B,
                       "global_batch": B * world, "parallelism": parallelism_label(dist, world),
                       "instances_per_wave": {"cl_lock_kernel": 4, "cl_fast_kernel": 1}.get(
                           kernel, info["instances_per_wave"]),
                       "steps_per_launch": spl},
            "timing": dict(timing_block(regions, elapsed, "each region is one closed-loop launch of --steps steps whose "
                                                          "time is set by its slowest wavefront; region-to-region "
                                                          "differences below the IQR are not resolved"),
                           steps_per_region=args.steps),
            "roofline": {"bound": "valu_fp64" if arith == "fp64" else "valu_fp32",
                         "pipe": ("FP64 FMA on the VALU" if arith == "fp64" else "FP32 FMA on the VALU")
                         + (" (fp32 handle: the credited active-set arithmetic runs in fp64)"
                            if arith != args.precision else "")
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
                                          f"lanes included; {pmc.get('source', 'no PMC pass for this config and launch length')}) "
                                          "/ this run's kernel time / peak",
                         "mfma_instructions_per_launch": pmc.get("mfma_insts_per_launch"),
                         "mfma": mfma_block(pmc, kernel_ms, spl),
                         "traffic": traffic,
                         "min_bytes_per_step": min_b,
                         "traffic_vs_min_bytes": traffic / min_b if traffic else None,
                         "traffic_note": "2 x FETCH_SIZE + WRITE_SIZE per closed-loop step (per launch / steps per "
                                         f"launch) from the committed rocprofv3 PMC pass on launches of {spl} steps "
                                         f"({pmc.get('source', 'none for this config and launch length')}); FETCH_SIZE x 2 "
                                         "is the gfx950 correction (MI355X_MICROARCH.md), calibrated for these 8-B "
                                         "coalesced loads on sf_kernel's known byte count (tools/pmc_summary.py); "
                                         "includes Infinity-Cache hits. min_bytes: x0 + offset in, u0 + x1 out per "
                                         "instance-step; the shared tables (v_t, T_x, W), which every XCD's L2 pulls "
                                         "once per launch, are not in it",
                         "gpu_mean_qp_iter": st["mean_qp_iter"]},
            "kernel_only": {"value": world * B / (kernel_ms * 1e-3), "unit": "NMPC steps/s",
                            "note": "closed-loop kernel time only (median of the regions' launch durations, HIP "
                                    "events; plant, cost and instance bookkeeping included), all ranks. Not a "
                                    "QP-solve rate: the general solve on per-instance windows is bench.py --mode solve"},
            "parked_solves": int(parked),
            "cpu_baseline": cpu,
            "closed_loop": {"mean_cost_per_step": red[0] / max(1.0, red[3]),
                            "aed": red[1] / max(1.0, red[3]) / (2 if model != "quad13" else 3),
                            "failed_solves": int(red[2]), "instance_steps": int(red[3])},
            "parity": {"checked_against": (
                "the builder's CPU oracle only (oracle/c/riccati_ipm.c closed loop: mode 0 exact KKT-certified QP "
                "solutions, mode 1 this engine's algorithm): quad13 is a synthetic model the reference does not "
                "have (SURVEY.md §0), so no acados run exists for it" if model == "quad13" else
                "the CPU oracle (oracle/c/riccati_ipm.c) and the reference's own recorded runs "
                "(tests/test_reference_plots.py: jerk reproduces acados's loop to 3e-7; force explained step by "
                "step as acados's interior-point termination, DESIGN.md §6)"),
                "tests": "tests/test_gpu_bench_parity.py: this workload against committed oracle goldens at every "
                         "region boundary (fp64 1e-6 relative, failure counts exact)"},
        }
        emit(line)
    if dist is not None:
        dist.destroy_process_group()


def main_solve(args, world, rank, dist, device):
    """--mode solve: the general batched solve (nmpc_solve_async on the handle's device buffers) of B
    QPs per GPU with per-instance yref windows staged in HBM — what the reference's per-step pattern
    (set(k, 'yref') for every stage, set(0, 'lbx'/'ubx'), solve(); src/force_model/ocp.py:117-122,
    controller.py:29-32) hits, with no shared reference table and no warm start. fp64: the fast solve
    (sf_kernel: every instance's unconstrained solution by the Riccati recursion on the shared factorisation,
    on the f64 matrix cores, with the bound test; fin64_kernel: primal-dual active-set steps on W and the dual
    fallback for the instances with a violated bound; the full IPM + exact finish only for what they leave);
    NMPC_SOLVE_FAST=0 (or fp32): the full IPM + exact finish for every QP. The QPs are the closed loop's
    first-step QPs of the bench workload (batched.first_step_qps). A step = one batched solve."""
    from drone_attitude_control_amd.acados import AcadosOcpSolver
    from drone_attitude_control_amd.batched import (DEFAULT_N, NY, first_step_qps, flops_per_iter,
                                                    unconstrained_solve_flops)
    from drone_attitude_control_amd.models import OCPS
    from drone_attitude_control_amd.sharding import rank_workload, reduce_run

    model = args.model
    N = args.horizon or DEFAULT_N[model]
    B = args.batch
    table, offsets_r, x_r, _ = rank_workload(model, N, B, world, rank, args.seed)
    x0, Y = first_step_qps(model, N, table, offsets_r, x_r)
    ocp = OCPS[model](N)
    s = AcadosOcpSolver(ocp, batch=B, device=device if world > 1 else 0, precision=args.precision)
    s.set_batch("x0", x0)
    s.set_batch("yref", Y)
    s.solve()                                   # uploads the windows once; they stay resident in HBM
    nx, nu = s.nx, s.nu
    info = s.launch_info()
    fast = info["solve_kernel"] == "sf_kernel"

    # the CPU baseline (after the timed regions: ahead of them the idle GPU's clocks ramp down)
    def cpu_part():
        cpu = None
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            from oracle import cref, models
            ref = cref.RiccatiIpmRef.for_options(models.MODELS[model](N), ocp.solver_options, args.precision)

            def run(n, threads):
                if fast:   # the same algorithm (riccati_ipm_solve_batch_fast); its tables are built once, untimed
                    ref.solve_fast(x0[:1], Y[:1], wsmax=cref.WSMAX[model], nthreads=1)
                    t0 = time.perf_counter()
                    _, _, st_c, it_c, cnt = ref.solve_fast(x0[:n], Y[:n], wsmax=cref.WSMAX[model], nthreads=threads)
                else:
                    t0 = time.perf_counter()
                    _, _, st_c, it_c = ref.solve(x0[:n], Y[:n], nthreads=threads)
                    cnt = None
                return time.perf_counter() - t0, st_c, it_c, cnt

            n0 = min(B, 256)
            el0 = run(n0, ref.max_threads())[0]
            n = int(min(B, max(n0, n0 / max(el0, 1e-6) * args.cpu_seconds)))
            el, st_c, it_c, cnt = run(n, ref.max_threads())
            n1 = min(n, 128)
            e1 = run(n1, 1)[0]
            algo = ("riccati_ipm_solve_batch_fast (the GPU's algorithm: unconstrained solution on the shared "
                    "factorisation, active-set steps on W, the dual fallback, the full IPM + exact finish for what is "
                    "left; fp64)" if fast else "riccati_ipm_solve_batch (the same cold IPM + exact finish, fp64)")
            cpu = {"value": n / el, "unit": "QP solves/s", "cores": ref.max_threads(), "kind": "port",
                   "sample": f"{n} of the {B} QPs in {el:.2f} s: oracle/c/riccati_ipm.c {algo}, OpenMP over instances",
                   "mean_newton_systems": float(np.mean(it_c)), "failed": int((st_c != 0).sum()),
                   "single_core": {"value": n1 / e1, "cores": 1, "sample": f"{n1} QPs in {e1:.2f} s"}}
            if cnt:
                cpu["paths"] = {k: cnt[k] / max(1.0, cnt["solves"]) for k in ("unconstrained", "set", "full", "failed")}
                cpu["flops_per_qp"] = cnt["flops"] / max(1.0, cnt["solves"])
        return cpu

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(max(1, args.warmup)):
        s.solve_async()
    s.synchronize()
    regions, kms = [], []
    for _ in range(max(1, args.repeats)):
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            s.solve_async()
        s.synchronize()
        t1 = time.perf_counter()
        barrier()
        regions.append(t1 - t0)
        kms.append(s.get_stats("time_tot") * 1e3)   # the region's last launch (HIP events)
    s.solve()                                   # one synchronous solve: outputs, status and qp_iter to the host
    cpu = cpu_part()
    counts = ({"listed": s.get_stats("fast_listed"), "parked": s.get_stats("fast_parked"),
               "note": "the final solve's instances listed for fin64_kernel / parked for the list-mode IPM; every timed "
                       "solve is complete in stream order (the three launches read their list lengths on the device)"}
              if fast else None)
    status = s.get_batch_int("status")
    iters = s.get_batch_int("qp_iter")
    red, regions, kms = reduce_run(dist, np.array([float((status != 0).sum()), float(iters.sum()), float(B)]),
                                   np.array(regions), np.array(kms),
                                   device="cuda" if dist is not None and args.dist_backend == "nccl" else None)
    regions, kms = np.atleast_1d(regions), np.atleast_1d(kms)
    med = int(np.argsort(regions)[len(regions) // 2])
    elapsed = float(regions[med])
    kernel_ms = float(np.median(kms))
    if rank == 0:
        kernel = info["solve_kernel"]
        w = 8 if args.precision == "fp64" else 4
        min_b = float(B * (nx + N * (nx + nu) + nx + N * nu + (N + 1) * nx) * w)
        pmc = load_pmc(model, N, B, args.precision, kernel, 1, mode="solve")
        traffic = pmc.get("hbm_bytes_per_step")
        peak = PEAK_TFLOPS[args.precision]
        if fast and cpu and cpu.get("flops_per_qp"):
            fl_solve = cpu["flops_per_qp"]
            credit = ("FP64 flops per QP of the CPU run of the same algorithm on the same QPs (riccati_ipm_solve_batch_"
                      "fast, counted per path: gradient G yref, the Riccati recursion on the shared factorisation, "
                      "active-set steps m^3/3 + 2 m^2 + 2 ne m, full solves F_iter per Newton system) x B / kernel time")
        elif fast:   # no CPU run to count the paths taken: every QP credited with the unconstrained path only
            fl_solve = unconstrained_solve_flops(nx, nu, N, *NY[model])
            credit = ("FP64 flops per QP of the unconstrained path alone (gradient G yref + the Riccati recursion on "
                      "the shared factorisation, as riccati_ipm_solve_batch_fast counts them; a lower bound: no CPU "
                      "run counted the active-set steps) x B / kernel time")
        else:
            n_newton = cpu["mean_newton_systems"] if cpu else float(red[1] / max(1.0, red[2]))
            fl_solve = flops_per_iter(nx, nu, N) * n_newton
            credit = ("SURVEY 8d F_iter (one Riccati factorisation + predictor/corrector sweeps + box elementwise per "
                      "Newton system) x the CPU baseline's mean Newton systems per QP on the same QPs x B / kernel time")
        achieved = fl_solve * B / (kernel_ms * 1e-3) / 1e12
        hbm_achieved = min_b / (kernel_ms * 1e-3) / 1e9
        # the fast solve reads each window once and writes each trajectory once: its roof is HBM (the algorithmic
        # bytes per launch over the launch time, against 8 TB/s); the full IPM's is the FP64 pipe
        if fast:
            roof = {"bound": "hbm", "achieved": hbm_achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": hbm_achieved / HBM_PEAK_GBS,
                    "algorithmic_bytes_per_launch": min_b,
                    "bytes_note": "x0 + yref window in, the full x / u trajectories out per QP (SURVEY 8d) x B",
                    "fp64": {"achieved": achieved, "peak": peak, "unit": "TFLOP/s", "frac": achieved / peak,
                             "credit": credit, "flops_per_solve": fl_solve}}
        else:
            roof = {"bound": "valu_fp64" if args.precision == "fp64" else "valu_fp32",
                    "achieved": achieved, "peak": peak, "unit": "TFLOP/s", "frac": achieved / peak,
                    "credit": credit, "flops_per_solve": fl_solve,
                    "hbm": {"achieved": hbm_achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": hbm_achieved / HBM_PEAK_GBS}}
        roof.update({"kernel": kernel, "kernel_ms": kernel_ms,
                     "executed_fp64_flops_per_step": pmc.get("fp64_flops_per_step"),
                     "mfma_instructions_per_launch": pmc.get("mfma_insts_per_launch"),
                     "traffic": traffic, "min_bytes_per_step": min_b,
                     "traffic_vs_min_bytes": traffic / min_b if traffic else None,
                     "traffic_note": "2 x FETCH_SIZE (the gfx950 correction) + WRITE_SIZE per batched solve from the "
                                     "committed PMC pass "
                                     f"({pmc.get('source', 'none for this config')}); min bytes = x0 + yref window "
                                     "in, full x/u trajectories out (SURVEY 8d)",
                     "kernel_ms_note": "HIP events around the solve's launches (fast solve: sf_kernel, fin64_kernel "
                                       "and the list-mode full IPM of the parked instances, the last two always "
                                       "enqueued and empty when nothing is listed / parked)",
                     "gpu_mean_qp_iter": float(red[1] / max(1.0, red[2]))})
        what = (f"fp64 fast solve (sf_kernel: unconstrained solution by the Riccati recursion on the shared "
                f"factorisation on the f64 matrix cores + bound test; fin64_kernel: active-set steps on W and the dual "
                f"fallback for the violated ones; full IPM + exact finish for what they leave)" if fast else
                f"full Mehrotra IPM + exact active-set finish ({kernel})")
        line = {
            "metric": f"QP solves/sec (batched nmpc_solve, per-instance yref windows), N={N} nx={nx} nu={nu} ({model})",
            "value": world * B * args.steps / elapsed,
            "unit": "QP solves/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f64" if args.precision == "fp64" else "f32",
            "data": "synthetic (the bench workload's first-step QPs, per-instance yref windows)",
            "config": {"workload": f"{model} batched cold QP solve: {B} independent QPs per GPU, each with its own "
                                   f"stage-stacked yref window and x0 resident in HBM, no shared table, no warm "
                                   f"start; {what}",
                       "model": model, "nx": nx, "nu": nu, "horizon_N": N, "batch_per_gpu": B, "global_batch": B * world,
                       "parallelism": parallelism_label(dist, world),
                       "instances_per_wave": (16 // (1 if nx <= 4 else 2 if nx <= 8 else 4)) if fast else info["instances_per_wave"]},
            "timing": dict(timing_block(regions, elapsed, "each region enqueues --steps batched solves back to back"),
                           steps_per_region=args.steps),
            "roofline": roof,
            "failed_solves": int(red[0]),
            "fast_counts": counts,
            "cpu_baseline": cpu,
        }
        emit(line)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
