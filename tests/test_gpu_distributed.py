"""BASELINE config 4 in miniature on the one-GPU box: the force model's closed loop sharded over
two ranks (torch.distributed.run, gloo backend — RCCL needs one GPU per rank, and the 8-GPU
run is the driver's), each rank running the device closed loop (batched.ClosedLoop) on its
slice of the global batch, then bench.py's end-of-run reduction. The reduced statistics must
equal a single-process run over the same global batch: instances are keyed by their global id
(sharding.rank_workload, Philox noise by global instance), so sharding changes nothing but the
summation order."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench(args, world, backend="gloo", launcher=None, **env_extra):
    """bench.py as one process (world 1, no launcher) or under torch.distributed.run with `world`
    ranks and the given process-group backend."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), *args]
    if launcher == "self":   # bench.py --gpus N starts its N ranks itself
        cmd += ["--dist-backend", backend]
    elif world > 1 or launcher == "torchrun":
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr", "127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "bench.py"),
               *args, "--dist-backend", backend]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", **env_extra)
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=420)
    assert out.returncode == 0, out.stderr[-3000:]
    return json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])


@pytest.mark.timeout(300)
def test_force_two_ranks_reduce_equals_one_process():
    """Two ranks x 4096 against one process over 8192, both ways the force closed loop can run:
    the lean loop (the default: one wavefront per instance, so sharding changes nothing but the
    summation order of the statistics — 1e-10) and the fused kernel families (NMPC_CL_FAST=0): each
    rank's 4096 instances then run the wavefront family, the single process's 8192 the
    lane-per-component family (fp64 force crossover at B = 8192, nmpc_ipm.hip kernel_kind), which
    agree to the solvers' precision (1e-8 relative; both return the exact QP solutions, by different
    paths), not bit for bit (a family bug that moved a solution showed as 7e-7 relative in round 2)."""
    common = ["--model", "force", "--steps", "4", "--warmup", "2", "--repeats", "2", "--no-cpu-baseline"]
    for env, kernels, rel in (({}, ("cl_fast_kernel", "cl_fast_kernel"), 1e-10),
                              ({"NMPC_CL_FAST": "0"}, ("ipm_kernel", "ipm_lpc_kernel"), 1e-8)):
        two = _bench(common + ["--gpus", "2", "--batch", "4096"], 2, **env)
        one = _bench(common + ["--gpus", "1", "--batch", "8192"], 1, **env)
        assert (two["roofline"]["kernel"], one["roofline"]["kernel"]) == kernels
        assert two["n_gpus"] == 2 and two["config"]["global_batch"] == one["config"]["global_batch"] == 8192
        a, b = two["closed_loop"], one["closed_loop"]
        assert a["instance_steps"] == b["instance_steps"] == 8192 * (2 + 2 * 4)
        assert a["failed_solves"] == b["failed_solves"]
        assert a["mean_cost_per_step"] == pytest.approx(b["mean_cost_per_step"], rel=rel)
        assert a["aed"] == pytest.approx(b["aed"], rel=rel)
        assert two["value"] > 0 and len(two["timing"]["region_ms"]) == 2


@pytest.mark.timeout(300)
def test_bench_gpus_two_starts_two_ranks_itself():
    """`python bench.py --gpus 2` with no launcher (the driver's form) starts its two ranks itself
    (a torch.distributed.run child, before any GPU call in the parent) and relays rank 0's line:
    n_gpus 2, global batch 8192, statistics equal to one process over the same 8192 instances.
    gloo, both ranks on the box's one GPU (RCCL needs a GPU per rank)."""
    common = ["--model", "force", "--steps", "4", "--warmup", "2", "--repeats", "2", "--no-cpu-baseline"]
    two = _bench(common + ["--gpus", "2", "--batch", "4096"], 2, launcher="self")
    one = _bench(common + ["--gpus", "1", "--batch", "8192"], 1)
    assert two["n_gpus"] == 2 and two["config"]["global_batch"] == one["config"]["global_batch"] == 8192
    assert "started by bench.py --gpus 2" in two["config"]["parallelism"]
    a, b = two["closed_loop"], one["closed_loop"]
    assert a["instance_steps"] == b["instance_steps"] == 8192 * (2 + 2 * 4)
    assert a["failed_solves"] == b["failed_solves"]
    assert a["mean_cost_per_step"] == pytest.approx(b["mean_cost_per_step"], rel=1e-10)
    assert a["aed"] == pytest.approx(b["aed"], rel=1e-10)


@pytest.mark.timeout(120)
def test_bench_nccl_refuses_more_ranks_than_gpus():
    """backend nccl with more ranks than visible GPUs exits non-zero with the reason, instead of putting
    two RCCL ranks on one device."""
    import torch
    n = torch.cuda.device_count() + 1
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--model", "force", "--batch", "64",
           "--steps", "1", "--warmup", "1", "--repeats", "1", "--no-cpu-baseline"]
    out = subprocess.run(cmd, cwd=ROOT, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"),
                         capture_output=True, text=True, timeout=100)
    assert out.returncode != 0 and out.stdout.strip() == ""
    assert "needs one GPU per rank" in out.stderr


@pytest.mark.timeout(600)
def test_config4_eight_ranks_reduce_equals_one_process():
    """BASELINE config 4 at its size, rehearsed on the one-GPU box: 65,536 force instances as 8
    ranks x 8,192 (gloo; every rank on the same GPU, each running the lean closed loop on its shard)
    against one process over all 65,536 — the reduced cost / AED / failure /
    step statistics agree to 1e-10 (force_model/controller.py:40-41,54; store_results.py:233-236)."""
    common = ["--model", "force", "--steps", "4", "--warmup", "2", "--repeats", "1", "--no-cpu-baseline"]
    eight = _bench(common + ["--gpus", "8", "--batch", "8192"], 8)
    one = _bench(common + ["--gpus", "1", "--batch", "65536"], 1)
    assert eight["n_gpus"] == 8 and eight["config"]["global_batch"] == one["config"]["global_batch"] == 65536
    assert eight["roofline"]["kernel"] == one["roofline"]["kernel"] == "cl_fast_kernel"
    a, b = eight["closed_loop"], one["closed_loop"]
    assert a["instance_steps"] == b["instance_steps"] == 65536 * (2 + 4)
    assert a["failed_solves"] == b["failed_solves"]
    assert a["mean_cost_per_step"] == pytest.approx(b["mean_cost_per_step"], rel=1e-10)
    assert a["aed"] == pytest.approx(b["aed"], rel=1e-10)


@pytest.mark.timeout(300)
def test_rccl_reduce_on_one_gpu_equals_no_dist():
    """The RCCL leg of BASELINE config 4 on the one-GPU box: bench.py under torch.distributed.run with
    one rank and the "nccl" backend (RCCL on ROCm) initialises a real communicator before any GPU call
    of libnmpc_hip, runs the closed loop in that process and reduces the statistics with all_reduce on
    device tensors (sharding.reduce_run). The reduced cost / AED / failure / step statistics equal a
    run without any process group bit for bit (one rank: the reduction is the identity)."""
    common = ["--model", "force", "--batch", "4096", "--steps", "4", "--warmup", "2", "--repeats", "2",
              "--no-cpu-baseline"]
    rccl = _bench(common, 1, backend="nccl", launcher="torchrun")
    plain = _bench(common, 1)
    assert rccl["config"]["parallelism"] == "instance-sharded x1, RCCL stats reduce (nccl process group)"
    assert plain["config"]["parallelism"] == "instance-sharded x1, single process (no collective)"
    assert rccl["closed_loop"] == plain["closed_loop"]
    assert rccl["closed_loop"]["instance_steps"] == 4096 * (2 + 2 * 4)
