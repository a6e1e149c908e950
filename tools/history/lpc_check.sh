#!/bin/bash
# GPU check of the lane-per-component kernels: solver parity tests and the bench per variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-lpc}
export NMPC_KERNEL=${NMPC_KERNEL:-lpc}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_solver.py} -x -q --timeout 120 --timeout-method thread > $OUT/${TAG}_test.log 2>&1 || { echo "tests failed"; tail -40 $OUT/${TAG}_test.log; exit 1; }
  tail -2 $OUT/${TAG}_test.log
fi
for V in ${VARIANTS:-0}; do
  NMPC_VARIANT=$V timeout -k 10 200 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/${TAG}_bench_v$V.json 2> $OUT/${TAG}_bench_v$V.err || { echo "bench v$V failed"; tail -20 $OUT/${TAG}_bench_v$V.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/${TAG}_bench_v$V.json')); print('variant $V', round(d['value']), 'steps/s kernel', round(d['roofline']['kernel_ms'],3), 'ms iters', d['roofline']['gpu_mean_qp_iter'], 'fail', d['closed_loop']['failed_solves'])"
done
