#!/bin/bash
# Kernel family crossover: solve-kernel time of the lane-per-component (lpc) and the
# wavefront-per-instance (wave) families over models and batch sizes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for MB in ${CASES:-"quad13 20 1024" "quad13 20 2048" "force 20 1024" "force 20 2048" "force 20 4096" "jerk 40 1024" "jerk 40 2048" "jerk 40 4096"}; do
  set -- $MB
  for K in lpc wave; do
    NMPC_KERNEL=$K timeout -k 10 120 python bench.py --model $1 --horizon $2 --batch $3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/fam.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/fam.json')); print('$1 N=$2 B=$3 $K kernel %.3f ms ipw %d' % (d['roofline']['kernel_ms'], d['config']['instances_per_wave']))"
  done
done
