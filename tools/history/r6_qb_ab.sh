#!/bin/bash
# Same-box A/B of experimental builds on the closed-loop bench lines: LIBS="qb16 qb32", CONFIGS as bench args
# separated by ';'. Three alternating repeats; one line per run: lib, config, value, kernel ms.
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-ab}
IFS=';' read -ra CFG <<< "${CONFIGS:---model force --batch 1024;--model force --batch 8192}"
: > gpurun_out/${TAG}_ab.jsonl
for rep in 1 2 3; do
  for c in "${CFG[@]}"; do
    for L in default ${LIBS}; do
      if [ "$L" = default ]; then unset NMPC_LIB; SO=drone-attitude-control_amd/lib/libnmpc_hip.so; else export NMPC_LIB=$PWD/drone-attitude-control_amd/lib/exp/libnmpc_hip_$L.so; SO=$NMPC_LIB; fi
      MD5=$(md5sum $SO | cut -c1-12)   # which build ran (a CPU test run can rebuild the default library)
      timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --python-loop-steps 0 $c > gpurun_out/${TAG}_one.json 2> gpurun_out/${TAG}_err.log || { echo "failed: $L $c"; tail -20 gpurun_out/${TAG}_err.log; exit 1; }
      python -c "
import json; d=json.load(open('gpurun_out/${TAG}_one.json')); r=d['roofline']
print(json.dumps({'lib': '$L', 'md5': '$MD5', 'cfg': '$c', 'value': d['value'], 'kernel_ms': r['kernel_ms'], 'kernel': r['kernel']}))" | tee -a gpurun_out/${TAG}_ab.jsonl
    done
  done
done
