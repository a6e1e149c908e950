#!/bin/bash
# r7: GPU tests, configs, the quad13 step log, the XCD-placement A/B and its FETCH_SIZE passes (jerk, quad13)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r7d} CONFIGS=1 bash tools/gpu_round.sh || exit 1
timeout -k 10 200 python tools/clf_steps.py --model quad13 --batch 8192 --regions 3 > $OUT/${TAG}_steps.json || exit 1
TAG=${TAG}_xcd A="NMPC_CLF_XCD=0" B="NMPC_CLF_XCD=1" CFGS="--model quad13;--model jerk --batch 4096" REPS=2 bash tools/ab_env.sh || exit 1
export TMPDIR=/tmp
for x in 0 1; do
  for m in "jerk --batch 4096" "quad13"; do
    n=${m%% *}
    NMPC_CLF_XCD=$x timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $PWD/$OUT/fs_${TAG}_${n}_$x -o run -- python3 bench.py --model $m --steps 20 --warmup 20 --repeats 3 --python-loop-steps 0 --no-cpu-baseline > $OUT/fs_${TAG}_${n}_$x.log 2>&1 || { echo "pmc failed"; exit 1; }
  done
done
echo "xcd check done"
