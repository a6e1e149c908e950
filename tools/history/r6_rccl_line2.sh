#!/bin/bash
# The default bench line through a real one-rank RCCL process group: stdout must hold only the JSON line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --steps 20 --warmup 3 > gpurun_out/r6af_bench_rccl.json 2> gpurun_out/r6af_bench_rccl.err || { tail -20 gpurun_out/r6af_bench_rccl.err; exit 1; }
python -c "
import json; b=json.load(open('gpurun_out/r6af_bench_rccl.json')); print(b['config']['parallelism'], '%.1fM' % (b['value'] / 1e6))"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_distributed.py > gpurun_out/r6af_dist.log 2>&1 || { tail -30 gpurun_out/r6af_dist.log; exit 1; }
tail -1 gpurun_out/r6af_dist.log
