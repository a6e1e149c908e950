#!/bin/bash
# Same-box A/B with the order swapped each repeat: LIB vs default, CONFIGS separated by ';'
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-ab2}
IFS=';' read -ra CFG <<< "${CONFIGS}"
: > gpurun_out/${TAG}_ab.jsonl
for rep in 1 2 3 4; do
  if [ $((rep % 2)) = 1 ]; then ORDER="$LIB default"; else ORDER="default $LIB"; fi
  for c in "${CFG[@]}"; do
    for L in $ORDER; do
      if [ "$L" = default ]; then unset NMPC_LIB; SO=drone-attitude-control_amd/lib/libnmpc_hip.so; else export NMPC_LIB=$PWD/drone-attitude-control_amd/lib/exp/libnmpc_hip_$L.so; SO=$NMPC_LIB; fi
      MD5=$(md5sum $SO | cut -c1-12)   # which build ran (a CPU test run can rebuild the default library)
      timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --python-loop-steps 0 $c > gpurun_out/${TAG}_one.json 2> gpurun_out/${TAG}_err.log || { echo "failed: $L $c"; tail -20 gpurun_out/${TAG}_err.log; exit 1; }
      python -c "
import json; d=json.load(open('gpurun_out/${TAG}_one.json')); r=d['roofline']
print(json.dumps({'lib': '$L', 'md5': '$MD5', 'cfg': '$c', 'rep': $rep, 'value': d['value'], 'kernel_ms': r['kernel_ms']}))" >> gpurun_out/${TAG}_ab.jsonl
    done
  done
done
python -c "
import json, collections
d = collections.defaultdict(list)
for l in open('gpurun_out/${TAG}_ab.jsonl'):
    r = json.loads(l); d[(r['cfg'], r['lib'])].append(r['value'] / 1e6)
for k, v in sorted(d.items()): print(k, ['%.1f' % x for x in v], 'mean %.1f' % (sum(v) / len(v)))"
