#!/bin/bash
# A/B of lockstep-kernel settings on quad13 (tuning aid): bench lines per env setting, in one process each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-ab}
: > $OUT/${TAG}_ab.jsonl
for cfg in ${CFGS:-"NMPC_CLF_LOCK=0" "NMPC_LOCK_WORKERS=0" "NMPC_LOCK_WORKERS=1" "NMPC_LOCK_WORKERS=2"}; do
  env $cfg timeout -k 10 200 python bench.py --no-cpu-baseline --python-loop-steps 0 --repeats 10 ${BENCH_ARGS:-} > $OUT/${TAG}_one.json 2>> $OUT/${TAG}_err.log || { echo "bench failed: $cfg"; exit 1; }
  python -c "import json; b=json.load(open('$OUT/${TAG}_one.json')); b['ab_cfg']='$cfg'; print(json.dumps(b))" >> $OUT/${TAG}_ab.jsonl
done
python -c "
import json
for l in open('$OUT/${TAG}_ab.jsonl'):
    b=json.loads(l); print(b['ab_cfg'], b['roofline']['kernel'], '%.1fM' % (b['value']/1e6), 'kernel %.4f' % b['roofline']['kernel_ms'], 'iqr %.3f' % b['timing']['iqr_rel'])"
