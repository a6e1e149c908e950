"""Instance sharding and the end-of-run reduction of the multi-GPU closed loop.

Every instance's closed loop is independent, so ranks exchange nothing while they run:
  * `rank_workload` — every rank generates the SAME global synthetic batch (batched.workload,
    seeded) and takes its contiguous slice [rank*B, (rank+1)*B); the device noise is keyed
    by the global instance id (`instance_base` + local index), so every instance's
    trajectory is identical for any number of ranks;
  * `reduce_run` — one all_reduce(SUM) of the per-rank statistics [cost, AED numerators,
    failures, instance-steps] and one all_reduce(MAX) of the timed interval and of the mean
    solve-kernel time, at the end (RCCL over xGMI on the GPU box; gloo in the CPU tests).
"""
import numpy as np


def shard(rank, per_rank):
    return slice(rank * per_rank, (rank + 1) * per_rank)


def rank_workload(model, N, per_rank, world, rank, seed=42):
    """(table, offsets, x_init, instance_base) of this rank's shard of the global batch."""
    from .batched import workload
    table, offsets, x = workload(model, N, per_rank * world, seed)
    sl = shard(rank, per_rank)
    return table, offsets[sl].copy(), x[sl].copy(), rank * per_rank


def reduce_run(dist, stats, elapsed, kernel_ms, device=None):
    """SUM-reduce `stats` (1-D float array) and MAX-reduce `elapsed` and `kernel_ms` (scalars, or
    equal-length arrays: one entry per timed region, reduced elementwise) over ranks.
    `dist` is torch.distributed (initialised) or None for a single process; `device` is the
    tensor device the backend needs ("cuda" for RCCL/nccl, None/"cpu" for gloo)."""
    stats = np.asarray(stats, dtype=np.float64)
    el = np.atleast_1d(np.asarray(elapsed, dtype=np.float64))
    km = np.atleast_1d(np.asarray(kernel_ms, dtype=np.float64))
    scalar = np.ndim(elapsed) == 0

    def out(e, k):
        return (float(e[0]), float(k[0])) if scalar else (e, k)

    if dist is None:
        return (stats,) + out(el, km)
    import torch
    t = torch.tensor(stats, dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    m = torch.tensor(np.concatenate([el, km]), dtype=torch.float64, device=device)
    dist.all_reduce(m, op=dist.ReduceOp.MAX)
    m = m.cpu().numpy()
    return (t.cpu().numpy(),) + out(m[:el.size], m[el.size:])
