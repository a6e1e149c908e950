#!/bin/bash
# The default bench line through a real one-rank RCCL process group (torch.distributed.run), then the jerk
# lockstep variant re-checked against cl_fast_kernel with repeats
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --steps 20 --warmup 3 > gpurun_out/r6ad_bench_rccl.json 2> gpurun_out/r6ad_bench_rccl.err || { tail -20 gpurun_out/r6ad_bench_rccl.err; exit 1; }
python -c "
import json; b=json.load(open('gpurun_out/r6ad_bench_rccl.json')); print(b['config']['parallelism'], '%.1fM' % (b['value'] / 1e6))"
TAG=r6ae VAR=NMPC_CLF_LOCK A=0 B=1 ARGS="--model jerk --batch 4096" bash tools/r6_env_ab.sh
