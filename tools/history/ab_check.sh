#!/bin/bash
# GPU check of a lean-loop change: chosen test files (TESTS, default the bench-path parity and the fp32
# solver tests), then bench lines for each env setting in CFGS x each config in CONFIGS (no CPU baseline).
# Each step time-limited; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-abc}
export TMPDIR=/tmp
if [ "${TESTS:-default}" != "none" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_bench_parity.py tests/test_gpu_solver.py} ${TEST_ARGS:-} -v -s -x --timeout 300 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1 || { echo "tests failed"; grep -h "Error\|assert\|FAILED" $OUT/${TAG}_tests.log | tail -30; exit 1; }
  grep -h "max rel err\|closed loop:\|passed\|failed" $OUT/${TAG}_tests.log | tail -25
fi
: > $OUT/${TAG}_ab.jsonl
for cfg in ${CFGS:-"NMPC_NONE=0"}; do
  for a in ${CONFIGS:-"--model=force,--batch=1024" "--model=force,--batch=8192"}; do
    env $cfg timeout -k 10 300 python bench.py --python-loop-steps 0 --no-cpu-baseline ${a//,/ } > $OUT/${TAG}_one.json 2>> $OUT/${TAG}_err.log || { echo "bench failed: $cfg $a"; tail -20 $OUT/${TAG}_err.log; exit 1; }
    python -c "import json; b=json.load(open('$OUT/${TAG}_one.json')); b['ab_cfg']='$cfg'; print(json.dumps(b))" >> $OUT/${TAG}_ab.jsonl
  done
done
python -c "
import json
for l in open('$OUT/${TAG}_ab.jsonl'):
    b=json.loads(l); print(b['ab_cfg'], b['config']['model'], b['dtype'], b['config']['batch_per_gpu'], b['roofline']['kernel'], '%.2fM' % (b['value']/1e6), 'kernel %.4f' % b['roofline']['kernel_ms'], 'iqr %.3f' % b['timing']['iqr_rel'], 'failed', b['closed_loop']['failed_solves'], 'parked', b['parked_solves'])"
echo "ab check done"
