#!/bin/bash
# Round-end measurement on the GPU box: GPU tests, the default bench line (with CPU baseline),
# a rocprofv3 kernel-trace --stats profile of the same bench command, and the PMC passes
# (each counter group in its own run, no tracing mixed in). Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r1}
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -x > $OUT/gputest_$TAG.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gputest_$TAG.log; exit 1; }
tail -1 $OUT/gputest_$TAG.log
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench failed"; tail -30 $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof_$TAG -o run --output-format csv -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof_$TAG.log; exit 1; }
if [ "${SKIP_PMC:-0}" != "1" ]; then
  TAG=$TAG bash tools/pmc.sh || exit 1
fi
echo "profile done"
