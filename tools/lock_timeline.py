"""Launch timeline of the lean closed loop (tuning aid, needs a GPU): one timed launch of the bench
workload with the iteration log on, then where each instance starts and ends within the launch and
what the latest-finishing ones ran.

    python tools/lock_timeline.py --model quad13 --batch 8192 --steps 20

The log's last two rows hold each instance's start and end in the launch (wall_clock64 ticks, 100 MHz,
low 31 bits); the step rows hold every step's record: 1 + its active-set steps, status and ticks
(lockstep steps record 1 and their ticks, so `slow_steps` counts the rare-path steps, which only
run_instance takes). The per-workgroup figures assume --per-wg instances per workgroup (quad13 B=8192:
32; jerk B=4096: 16). One JSON line."""
import argparse
import json
import os
import sys

import numpy as np

os.environ.setdefault("NMPC_ITER_LOG", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from drone_attitude_control_amd.batched import ClosedLoop, DEFAULT_N  # noqa: E402

TICK_US = 0.01   # 100 MHz


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="quad13")
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--horizon", type=int, default=0)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--launches", type=int, default=3, help="timed launches before the logged one")
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--per-wg", type=int, default=32, help="instances per workgroup (grid: resident workgroups)")
    args = ap.parse_args()
    N = args.horizon or DEFAULT_N[args.model]
    cl = ClosedLoop(args.model, args.batch, N=N, seed=42)
    info = cl.solver.launch_info()
    cl.run(args.warmup)
    for _ in range(args.launches):
        cl.run(args.steps)
    cl.run(args.steps)
    a, b, c = cl.iter_log()
    raw = ((c.astype(np.int64) << 16) | (b.astype(np.int64) << 8) | a.astype(np.int64))
    steps = raw.shape[0] - 2
    start, end = raw[steps], raw[steps + 1]
    t0 = start.min()
    s_us, e_us = (start - t0) * TICK_US, (end - t0) * TICK_US
    tick = c[:steps].astype(np.int64)            # per-step ticks (0: not logged)
    act = a[:steps].astype(np.int64)
    ph2 = (tick > 0).any(axis=0)
    n2 = (tick > 0).sum(axis=0)
    slow = ((act > 1) & (tick > 0)).sum(axis=0)
    order = np.argsort(-e_us)
    top = []
    for i in order[:args.top]:
        top.append({"inst": int(i), "start_us": round(float(s_us[i]), 1), "end_us": round(float(e_us[i]), 1),
                    "run_instance_steps": int(n2[i]), "slow_steps": int(slow[i]),
                    "step_us": [round(float(x) * TICK_US, 1) for x in tick[:, i] if x > 0]})
    q = lambda x: [round(float(v), 1) for v in np.percentile(x, [50, 90, 99, 100])] if x.size else None
    fast = ~ph2
    # per workgroup (the kernels' contiguous ranges): instances with rare-path steps and their step time
    per_wg = args.per_wg
    hard = slow > 0
    ch = (tick * TICK_US).sum(axis=0) * hard
    nwg = (args.batch + per_wg - 1) // per_wg
    wg_n = np.array([hard[g * per_wg:(g + 1) * per_wg].sum() for g in range(nwg)])
    wg_sum = np.array([ch[g * per_wg:(g + 1) * per_wg].sum() for g in range(nwg)])
    wg_max = np.array([ch[g * per_wg:(g + 1) * per_wg].max() for g in range(nwg)])
    wg_end = np.array([e_us[g * per_wg:(g + 1) * per_wg].max() for g in range(nwg)])
    out = {"per_wg": per_wg,
           "wg_hard_instances_p50_p90_max": [int(np.percentile(wg_n, 50)), int(np.percentile(wg_n, 90)), int(wg_n.max())],
           "wg_hard_chain_sum_us_p50_p90_max": q(wg_sum)[:1] + q(wg_sum)[1:2] + q(wg_sum)[3:],
           "wg_hard_chain_max_us_p50_p90_max": q(wg_max)[:1] + q(wg_max)[1:2] + q(wg_max)[3:],
           "wg_end_us_p50_p90_max": q(wg_end)[:1] + q(wg_end)[1:2] + q(wg_end)[3:],
           "slowest_wg": int(np.argmax(wg_end)),
           "slowest_wg_instances": [{"inst": int(i), "slow": int(slow[i]), "chain_us": round(float(ch[i]), 1),
                                     "start_us": round(float(s_us[i]), 1), "end_us": round(float(e_us[i]), 1)}
                                    for g in [int(np.argmax(wg_end))]
                                    for i in range(g * per_wg, min(args.batch, (g + 1) * per_wg)) if hard[i]],
           "hard_instances": int(hard.sum())}
    out.update({"model": args.model, "batch": args.batch, "N": N, "kernel": info["closed_loop_kernel"],
           "order_env": os.environ.get("NMPC_CLF_ORDER", "default"),
           "launch_us": round(float(e_us.max()), 1),
           "end_us_p50_p90_p99_max": {"lockstep_or_fast_only": q(e_us[fast]), "run_instance": q(e_us[ph2])},
           "start_us_p50_p90_p99_max_run_instance": q(s_us[ph2]),
           "run_instance_instances": int(ph2.sum()),
           "run_instance_step_us_p50_p90_p99_max": q(tick[tick > 0] * TICK_US),
           "chain_us_p50_p90_p99_max": q((e_us - s_us)[ph2]),
           "latest": top})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
