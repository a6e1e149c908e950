"""Multi-rank host logic of bench.py on CPU: gloo, world_size 2.

Each rank takes its shard of the global synthetic batch (sharding.rank_workload) and computes
per-instance statistics on the host; sharding.reduce_run must reproduce the single-process
totals exactly (SUM of statistics, MAX of timings), and the shards must tile the global batch
with the right global instance bases (the device noise is keyed by them)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from drone_attitude_control_amd.batched import workload
from drone_attitude_control_amd.sharding import rank_workload, reduce_run, shard

MODELS = [("force", 20), ("jerk", 40), ("quad13", 20)]
PER_RANK = 6


def host_stats(table, offsets, x):
    """Deterministic stand-in for a rank's closed-loop statistics."""
    e = x[:, :2] - table[offsets, :2]
    return np.array([np.sum(e ** 2), np.sum(np.abs(e)), float(np.sum(offsets % 7 == 0)), float(len(offsets))])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = {}
        for model, N in MODELS:
            table, offsets, x, base = rank_workload(model, N, PER_RANK, world, rank)
            red, el, km = reduce_run(dist, host_stats(table, offsets, x), elapsed=1.0 + rank, kernel_ms=2.0 * (rank + 1))
            # per-region timings (bench.py --repeats): elementwise MAX over ranks
            _, el_r, km_r = reduce_run(dist, np.zeros(1), np.array([1.0 + rank, 5.0 - rank]),
                                       np.array([0.5 * rank, 1.0]))
            assert np.array_equal(el_r, [1.0 + world - 1, 5.0]) and np.array_equal(km_r, [0.5 * (world - 1), 1.0])
            res[model] = (red, el, km, base, offsets, x)
        out[rank] = res
    finally:
        dist.destroy_process_group()


def test_shards_tile_the_global_batch():
    for model, N in MODELS:
        table, off_g, x_g = workload(model, N, 3 * PER_RANK)
        for r in range(3):
            t, off, x, base = rank_workload(model, N, PER_RANK, 3, r)
            assert base == r * PER_RANK
            assert np.array_equal(off, off_g[shard(r, PER_RANK)]) and np.array_equal(x, x_g[shard(r, PER_RANK)])
            assert np.array_equal(t, table)


def test_single_process_reduce_is_identity():
    s = np.array([1.0, 2.0, 3.0, 4.0])
    red, el, km = reduce_run(None, s, 1.5, 0.5)
    assert np.array_equal(red, s) and el == 1.5 and km == 0.5
    red, el, km = reduce_run(None, s, np.array([1.0, 2.0]), np.array([3.0, 4.0]))
    assert np.array_equal(el, [1.0, 2.0]) and np.array_equal(km, [3.0, 4.0])


@pytest.mark.timeout(300)
def test_gloo_world2_reduce_matches_single_process():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for model, N in MODELS:
        table, off_g, x_g = workload(model, N, world * PER_RANK)
        expect = host_stats(table, off_g, x_g)
        for r in range(world):
            red, el, km, base, off, x = out[r][model]
            assert base == r * PER_RANK
            assert np.allclose(red, expect, rtol=1e-14, atol=0)
            assert el == 2.0 and km == 4.0      # MAX over ranks
        # the two shards concatenate to the global batch
        assert np.array_equal(np.concatenate([out[0][model][4], out[1][model][4]]), off_g)
        assert np.array_equal(np.concatenate([out[0][model][5], out[1][model][5]]), x_g)
