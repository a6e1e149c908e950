#!/bin/bash
# Tuning run: for each experimental build lib/exp/libnmpc_hip_<TAG>.so (build.build_experiment)
# and kernel variant, the bench rate and the per-sweep clock cycles (NMPC_SWEEP_CYCLES).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for L in ${LIBS:-U2}; do
  for V in ${VARIANTS:-0}; do
    export NMPC_LIB=drone-attitude-control_amd/lib/exp/libnmpc_hip_$L.so NMPC_VARIANT=$V
    timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/exp_${L}_v$V.json 2> $OUT/exp_${L}_v$V.err || { echo "$L v$V bench failed"; tail -20 $OUT/exp_${L}_v$V.err; exit 1; }
    NMPC_SWEEP_CYCLES=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > /dev/null 2> $OUT/expc_${L}_v$V.err || { echo "$L v$V cycles failed"; tail -20 $OUT/expc_${L}_v$V.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/exp_${L}_v$V.json')); print('$L v$V', round(d['value']), 'steps/s', round(d['roofline']['kernel_ms'],3), 'ms')"
    grep "nmpc cycles" $OUT/expc_${L}_v$V.err | tail -1
  done
done
