#!/bin/bash
# A/B of an environment knob over the BASELINE configs (tuning aid, GPU box):
#   KNOB=NMPC_WARM_SHIFT VALUES="1 0" [CONFIGS="--model quad13;--model force --batch 1024"] bash tools/ab_env.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for v in ${VALUES}; do
  IFS=';' read -ra CFGS <<< "${CONFIGS:---model quad13;--model jerk --batch 4096;--model force --batch 1024}"
  for a in "${CFGS[@]}"; do
    env $KNOB=$v timeout -k 10 200 python bench.py $a --no-cpu-baseline --repeats ${REPEATS:-5} > $OUT/ab.json 2> $OUT/ab.err || { echo "bench failed: $KNOB=$v $a"; tail -5 $OUT/ab.err; exit 1; }
    python -c "import json; b=json.load(open('$OUT/ab.json')); print('$KNOB=$v', b['config']['model'], b['config']['batch_per_gpu'], '%.3fM' % (b['value']/1e6), 'kernel %.4f' % b['roofline']['kernel_ms'], 'failed', b['closed_loop']['failed_solves'], flush=True)"
  done
done
