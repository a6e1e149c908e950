#!/bin/bash
# Kernel family A/B (lpc vs wave) for "model N batch" triples given one per argument.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for MB in "$@"; do
  set -- $MB
  for K in lpc wave; do
    NMPC_KERNEL=$K timeout -k 10 120 python bench.py --model $1 --horizon $2 --batch $3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/fam.json 2> gpurun_out/fam.err || { tail -5 gpurun_out/fam.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/fam.json')); print('$1 N=$2 B=$3 $K kernel %.3f ms ipw %d iters %.2f' % (d['roofline']['kernel_ms'], d['config']['instances_per_wave'], d['roofline']['gpu_mean_qp_iter']))"
  done
done
