#!/bin/bash
# Same-box A/B of an environment toggle: VAR=A|B values alternating (order swapped each repeat), 4 repeats
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-eab}
: > gpurun_out/${TAG}_ab.jsonl
for rep in 1 2 3 4; do
  if [ $((rep % 2)) = 1 ]; then ORDER="$A $B"; else ORDER="$B $A"; fi
  for v in $ORDER; do
    env $VAR=$v timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --python-loop-steps 0 $ARGS > gpurun_out/${TAG}_one.json 2> gpurun_out/${TAG}_err.log || { tail -20 gpurun_out/${TAG}_err.log; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/${TAG}_one.json')); print(json.dumps({'$VAR': '$v', 'rep': $rep, 'value': d['value'], 'kernel_ms': d['roofline']['kernel_ms']}))" >> gpurun_out/${TAG}_ab.jsonl
  done
done
python -c "
import json, collections
d = collections.defaultdict(list)
for l in open('gpurun_out/${TAG}_ab.jsonl'):
    r = json.loads(l); d[r['$VAR']].append(r['value'] / 1e6)
for k, v in sorted(d.items()): print('$VAR', k, ['%.1f' % x for x in v], 'mean %.1f' % (sum(v) / len(v)))"
