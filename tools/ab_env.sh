#!/bin/bash
# Same-box A/B of an environment switch on bench lines: for each config in CFGS (";"-separated bench.py argument
# sets), alternate A and B (REPS times), one JSON line each into gpurun_out/ab_<TAG>.jsonl tagged with the arm.
#   TAG=x A="NMPC_CLF_XCD=0" B="NMPC_CLF_XCD=1" CFGS="--model quad13;--model jerk --batch 4096" REPS=2 bash tools/ab_env.sh
# (ARMS="A B C" with C=... for a third arm)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
: > $OUT/ab_$TAG.jsonl
IFS=';' read -ra CS <<< "$CFGS"
for c in "${CS[@]}"; do
  for r in $(seq ${REPS:-2}); do
    for arm in ${ARMS:-A B}; do
      envs=${!arm}
      line=$(env $envs timeout -k 10 300 python bench.py $c --no-cpu-baseline --python-loop-steps 0 2>> $OUT/ab_$TAG.err) || { echo "bench failed: $arm $c"; tail -20 $OUT/ab_$TAG.err; exit 1; }
      python -c "import json,sys; d=json.loads(sys.argv[1]); d['ab_arm']=sys.argv[2]; d['ab_env']=sys.argv[3]; print(json.dumps(d))" "$line" "$arm" "$envs" >> $OUT/ab_$TAG.jsonl
    done
  done
done
python - "$OUT/ab_$TAG.jsonl" <<'PY'
import json, sys
from collections import defaultdict
r = defaultdict(list)
for l in open(sys.argv[1]):
    d = json.loads(l); r[(d['config']['model'], d['dtype'], d['config']['batch_per_gpu'], d['ab_arm'], d['ab_env'])].append(d['value'] / 1e6)
for k, v in sorted(r.items()): print(k, ' '.join('%.1f' % x for x in v))
PY
