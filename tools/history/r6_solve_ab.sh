#!/bin/bash
# Same-box A/B of the solve lines: LIB vs default, alternating, 3 repeats; MODELS as "model:batch" words
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-sab}
: > gpurun_out/${TAG}_ab.jsonl
for rep in 1 2 3; do
  for mb in ${MODELS:-jerk:4096 force:8192 quad13:8192}; do
    m=${mb%%:*}; b=${mb##*:}
    for L in default $LIB; do
      if [ "$L" = default ]; then unset NMPC_LIB; SO=drone-attitude-control_amd/lib/libnmpc_hip.so; else export NMPC_LIB=$PWD/drone-attitude-control_amd/lib/exp/libnmpc_hip_$L.so; SO=$NMPC_LIB; fi
      MD5=$(md5sum $SO | cut -c1-12)
      timeout -k 10 200 python bench.py --mode solve --steps 10 --warmup 2 --repeats 3 --no-cpu-baseline --model $m --batch $b > gpurun_out/${TAG}_one.json 2> gpurun_out/${TAG}_err.log || { echo "failed: $L $m"; tail -20 gpurun_out/${TAG}_err.log; exit 1; }
      python -c "
import json; d=json.load(open('gpurun_out/${TAG}_one.json')); r=d['roofline']
print(json.dumps({'lib': '$L', 'md5': '$MD5', 'model': '$m', 'value': d['value'], 'kernel_ms': r['kernel_ms'], 'failed': d['failed_solves']}))" >> gpurun_out/${TAG}_ab.jsonl
    done
  done
done
python -c "
import json, collections
d = collections.defaultdict(list)
for l in open('gpurun_out/${TAG}_ab.jsonl'):
    r = json.loads(l); d[(r['model'], r['lib'])].append(r['value'] / 1e6)
for k, v in sorted(d.items()): print(k, ['%.1f' % x for x in v], 'mean %.1f' % (sum(v) / len(v)))"
