#!/bin/bash
# lockstep vs one-instance-per-wavefront kernel on quad13 (tuning aid): bench lines and step records
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-lk}
: > $OUT/${TAG}_bench.jsonl; : > $OUT/${TAG}_steps.jsonl
for L in 1 0; do
  NMPC_CLF_LOCK=$L timeout -k 10 200 python bench.py --no-cpu-baseline --python-loop-steps 0 --repeats 10 >> $OUT/${TAG}_bench.jsonl 2>> $OUT/${TAG}_err.log || { echo "bench failed"; exit 1; }
  NMPC_CLF_LOCK=$L timeout -k 10 200 python tools/clf_steps.py --model quad13 --batch 8192 --regions 2 >> $OUT/${TAG}_steps.jsonl 2>> $OUT/${TAG}_err.log || { echo "steps failed"; exit 1; }
done
echo probe done
