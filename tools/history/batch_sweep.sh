#!/bin/bash
# Kernel time vs batch size (latency- vs throughput-bound diagnosis) for the default kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for B in ${BATCHES:-1024 2048 4096 8192 16384}; do
  timeout -k 10 120 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --batch $B ${BENCH_ARGS:-} > gpurun_out/sweep_$B.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/sweep_$B.json')); print('B=$B kernel %.3f ms  %.0f solves/s' % (d['roofline']['kernel_ms'], d['solve_only']['value']))"
done
