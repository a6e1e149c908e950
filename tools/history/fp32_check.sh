#!/bin/bash
# GPU check of the fp32 lean loop: its closed-loop parity test, the fp32 single-solve errors (printed),
# and the fp32 / fp64 force B=8192 bench lines. Each step time-limited; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-f32}
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_parity.py -k "fp32 or force" -v -s -x --timeout 300 --timeout-method thread > $OUT/${TAG}_parity.log 2>&1 || { echo "parity tests failed"; tail -40 $OUT/${TAG}_parity.log; exit 1; }
grep -h "fp32\|passed\|failed" $OUT/${TAG}_parity.log | tail -8
timeout -k 10 600 python -u -m pytest tests/test_gpu_solver.py -k "fp32" -v -s --timeout 300 --timeout-method thread > $OUT/${TAG}_solver.log 2>&1 || { echo "solver fp32 tests failed"; tail -40 $OUT/${TAG}_solver.log; exit 1; }
grep -h "err\|passed\|failed" $OUT/${TAG}_solver.log | tail -30
: > $OUT/${TAG}_configs.jsonl
for a in "--model force --batch 8192 --precision fp32" "--model force --batch 8192" ${EXTRA_CONFIGS:-}; do
  timeout -k 10 300 python bench.py --python-loop-steps 0 --no-cpu-baseline $a >> $OUT/${TAG}_configs.jsonl 2>> $OUT/${TAG}_configs.err || { echo "config failed: $a"; tail -20 $OUT/${TAG}_configs.err; exit 1; }
done
python -c "
import json
for l in open('$OUT/${TAG}_configs.jsonl'):
    b = json.loads(l); print(b['config']['model'], b['dtype'], b['config']['batch_per_gpu'], b['roofline']['kernel'], '%.3fM' % (b['value'] / 1e6), 'kernel %.4f ms' % b['roofline']['kernel_ms'], 'iqr', round(b['timing']['iqr_rel'],3), 'failed', b['closed_loop']['failed_solves'], 'parked', b['parked_solves'])"
echo "fp32 check done"
