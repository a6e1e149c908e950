"""Benchmark: batched NMPC closed-loop steps/s on MI355X (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W --model quad13 --batch 8192 --precision fp64]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Workload (BASELINE.json metric "NMPC steps/sec (batched trajectories), N=20 nx=13 nu=4"):
the synthetic quad13 OCP (nx=13, nu=4, horizon N=20, no reference counterpart: SURVEY §0),
B = 8192 independent closed-loop trajectories per GPU (weak scaling), fp64. One step = for
every instance: build the yref window + pin x0 (set_up_ocp, ocp.py:117-122), solve the OCP
(AcadosOcpSolver.solve, controller.py:32) to 1e-15 complementarity, advance the plant with
Philox noise and accumulate cost/AED — all resident in HBM. value = instances x steps /
wall time (max over ranks) for all ranks together. Ranks exchange nothing during the run;
RCCL (torch.distributed "nccl") reduces the cost/AED/failure statistics once at the end.

Also reported (one JSON line on rank 0):
  roofline — the solve kernel (the dominant kernel): algorithmic flops per launch = SURVEY
    §8d F_iter x n_ipm (mean IPM iterations of the CPU baseline on the same inputs) x B,
    divided by the kernel's mean duration from HIP events around each launch;
    bound "mfma" = the dense FP64 FMA roofline: peak = MI355X FP64 78.6 TFLOP/s, the rate of
    both the FP64 matrix and the FP64 vector pipe (half the 157.3 TFLOP/s F32 rate of
    MI355X_MICROARCH.md); the kernel issues its FP64 FMAs on the vector pipe (DESIGN.md §4
    explains why 17-wide stage operands do not pay on MFMA). traffic = memory-side bytes per
    launch (FETCH_SIZE + WRITE_SIZE) from the rocprofv3 PMC passes committed under profiles/
    (profiles/pmc_traffic.json) when one matches this config, else null.
  cpu_baseline — oracle/c/riccati_ipm.c (same algorithm, fp64, OpenMP over instances) on the
    host cores, rank 0 at N=1 only, on a bounded sample of the same instances.
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
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL over xGMI, the default); gloo only to rehearse several ranks "
                         "on a one-GPU box (ranks then share the visible GPUs round-robin)")
    return ap.parse_args()


def ipm_tolerances(model, N):
    """(tol_comp, tol_res) of the model's OCP solver options (library defaults when unset)."""
    from drone_attitude_control_amd.models import OCPS
    o = OCPS[model](N).solver_options
    return float(o.qp_solver_tol_comp or 1e-15), float(o.qp_solver_tol_stat or 1e-12)


def cpu_baseline(model, N, table, offsets, x_init, seconds):
    """Time the C oracle (same Riccati IPM, fp64, same tolerances) on a bounded sample of the
    same instances."""
    from oracle import cref, models
    spec = models.MODELS[model](N)
    tc, tr = ipm_tolerances(model, N)
    R = cref.RiccatiIpmRef(spec, tol_comp=tc, tol_res=tr)
    ny, nye = spec.ny, spec.nx
    nsamp = min(len(offsets), 4096)
    Y = np.stack([np.concatenate([table[t:t + N, :ny].ravel(), table[t + N, :nye]]) for t in offsets[:nsamp]])
    X0 = x_init[:nsamp]
    threads = R.max_threads()
    # n_ipm on exactly the first-step inputs of the GPU run
    _, _, st, it = R.solve(X0, Y, nthreads=threads)
    n_ipm = float(it[st == 0].mean()) if (st == 0).any() else float(it.mean())
    # bounded timing loop (~`seconds` of CPU work)
    solves, t0 = 0, time.perf_counter()
    while True:
        R.solve(X0, Y, nthreads=threads)
        solves += nsamp
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    # single-core figure, on a smaller slice of the same inputs (~1/5 of the time)
    n1 = max(1, min(nsamp, 256))
    s1, t1 = 0, time.perf_counter()
    while True:
        R.solve(X0[:n1], Y[:n1], nthreads=1)
        s1 += n1
        e1 = time.perf_counter() - t1
        if e1 >= seconds / 5:
            break
    return {"value": solves / el, "unit": "NMPC steps/s", "cores": threads, "kind": "port",
            "sample": f"{solves} solves of the first closed-loop step of {nsamp} bench instances "
                      f"({model}, N={N}, fp64) in {el:.1f} s, OpenMP over instances; "
                      f"oracle/c/riccati_ipm.c -O3 -march=x86-64-v3",
            "single_core": {"value": s1 / e1, "cores": 1,
                            "sample": f"{s1} solves of {n1} of those instances in {e1:.1f} s"}}, n_ipm


def load_traffic(model, N, batch, precision):
    """HBM bytes per solve launch from the committed rocprofv3 PMC summary, if one matches."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        for e in d.get("entries", []):
            if (e.get("model"), e.get("N"), e.get("batch"), e.get("precision")) == (model, N, batch, precision):
                return e.get("hbm_bytes_per_launch")
    except (ValueError, OSError):
        return None
    return None


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

    from drone_attitude_control_amd.batched import DEFAULT_N, ClosedLoop, flops_per_iter
    from drone_attitude_control_amd.sharding import rank_workload, reduce_run

    model = args.model
    N = args.horizon or DEFAULT_N[model]
    B = args.batch
    table, offsets_r, x_r, base = rank_workload(model, N, B, world, rank, args.seed)
    cl = ClosedLoop(model, B, N=N, device=device if world > 1 else 0, precision=args.precision,
                    table=table, offsets=offsets_r, x_init=x_r, instance_base=base, seed=args.seed)
    nx, nu = cl.solver.nx, cl.solver.nu

    # CPU baseline first (rank 0, single-GPU runs only), on this rank's first-step inputs
    cpu, n_ipm_cpu = None, None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu, n_ipm_cpu = cpu_baseline(model, N, table, offsets_r, x_r, args.cpu_seconds)

    def barrier():
        if dist is not None:
            dist.barrier()

    cl.run(args.warmup, sync=True)
    barrier()
    t0 = time.perf_counter()
    cl.run(args.steps, sync=True)
    t1 = time.perf_counter()
    barrier()
    elapsed = t1 - t0
    st = cl.stats()
    red = np.array([st["cost_sum"], st["aed_sum"], st["failed"], st["instance_steps"]])
    # one SUM of the statistics and one MAX of the timings over RCCL, after the timed region
    red, elapsed, kernel_ms = reduce_run(dist, red, elapsed, st["solve_kernel_ms"] / max(1, st["solve_launches"]),
                                         device="cuda" if dist is not None and args.dist_backend == "nccl" else None)

    if rank == 0:
        tols = ipm_tolerances(model, N)
        value = world * B * args.steps / elapsed
        n_ipm = n_ipm_cpu if n_ipm_cpu is not None else st["mean_qp_iter"]
        fl_launch = flops_per_iter(nx, nu, N) * n_ipm * B
        achieved = fl_launch / (kernel_ms * 1e-3) / 1e12
        peak = PEAK_TFLOPS[args.precision]
        traffic = load_traffic(model, N, B, args.precision)
        line = {
            "metric": "NMPC steps/sec (batched trajectories), N=20 nx=13 nu=4, 1/2/4/8 MI355X",
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
                                   f"(tol_comp {tols[0]:g}, tol_res {tols[1]:g}) + plant/noise advance",
                       "model": model, "nx": nx, "nu": nu, "horizon_N": N, "batch_per_gpu": B,
                       "global_batch": B * world, "parallelism": f"instance-sharded x{world}, "
                                                                    f"{'gloo' if args.dist_backend == 'gloo' else 'RCCL'} stats reduce",
                       "instances_per_wave": cl.solver.launch_info()["instances_per_wave"]},
            "roofline": {"bound": "mfma", "pipe": "fp64 FMA on VALU" if args.precision == "fp64" else "fp32 FMA on VALU",
                         "kernel": cl.solver.launch_info()["kernel"], "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                         "frac": achieved / peak, "traffic": traffic,
                         "flops_per_launch": fl_launch, "kernel_ms": kernel_ms,
                         "n_ipm": n_ipm, "gpu_mean_qp_iter": st["mean_qp_iter"]},
            "solve_only": {"value": world * B / (kernel_ms * 1e-3), "unit": "QP solves/s",
                           "note": "ipm_kernel alone (mean launch duration from HIP events), all ranks"},
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
