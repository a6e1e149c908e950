#!/bin/bash
# GPU-box check: GPU tests, a short bench, and a rocprofv3 kernel-trace profile of the bench.
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-r1}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -x > $OUT/gputest_$TAG.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gputest_$TAG.log; exit 1; }
  tail -3 $OUT/gputest_$TAG.log
fi
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench failed"; tail -30 $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
if [ "${SKIP_PROF:-0}" != "1" ]; then
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof_$TAG.log; exit 1; }
  find $OUT/prof_$TAG -name "*stats*" | head
fi
