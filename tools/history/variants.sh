#!/bin/bash
# Tuning run: GPU tests once, then the bench for every compiled kernel variant of a model.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-var}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -x > $OUT/gputest_$TAG.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gputest_$TAG.log; exit 1; }
  tail -2 $OUT/gputest_$TAG.log
fi
for V in ${VARIANTS:-0 1 2 3}; do
  NMPC_VARIANT=$V timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/bench_${TAG}_v$V.json 2> $OUT/bench_${TAG}_v$V.err || { echo "variant $V failed"; tail -20 $OUT/bench_${TAG}_v$V.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/bench_${TAG}_v$V.json')); print('variant $V', round(d['value']), 'steps/s', round(d['roofline']['kernel_ms'],3), 'ms', d['config']['instances_per_wave'])"
done
