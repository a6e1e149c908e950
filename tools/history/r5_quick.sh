#!/bin/bash
# quick GPU check of a lean-loop change: the bench-path parity tests, the phase timings (timing build) and
# the BASELINE configs' closed-loop rate (no CPU baseline). Each step time-limited; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r5q}
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_parity.py ${TEST_ARGS:-} -v -x --timeout 300 --timeout-method thread > $OUT/${TAG}_parity.log 2>&1 || { echo "parity tests failed"; tail -40 $OUT/${TAG}_parity.log; exit 1; }
tail -1 $OUT/${TAG}_parity.log
: > $OUT/${TAG}_phases.jsonl
for a in "--model force --batch 1024" "--model force --batch 8192" "--model quad13 --batch 8192" "--model jerk --batch 4096"; do
  NMPC_LIB=$PWD/drone-attitude-control_amd/lib/exp/libnmpc_hip_timing.so timeout -k 10 200 python tools/clf_phases.py $a --regions 3 >> $OUT/${TAG}_phases.jsonl 2>> $OUT/${TAG}_phases.err || { echo "phases failed: $a"; tail -5 $OUT/${TAG}_phases.err; exit 1; }
done
: > $OUT/${TAG}_configs.jsonl
for a in "--model quad13 --batch 8192" "--model force --batch 1024" "--model jerk --batch 4096" "--model force --batch 8192"; do
  timeout -k 10 300 python bench.py --python-loop-steps 0 --no-cpu-baseline $a >> $OUT/${TAG}_configs.jsonl 2>> $OUT/${TAG}_configs.err || { echo "config failed: $a"; tail -20 $OUT/${TAG}_configs.err; exit 1; }
done
python -c "
import json
for l in open('$OUT/${TAG}_configs.jsonl'):
    b = json.loads(l); print(b['config']['model'], b['dtype'], b['config']['batch_per_gpu'], '%.3fM' % (b['value'] / 1e6), 'kernel %.4f ms' % b['roofline']['kernel_ms'], 'iqr', round(b['timing']['iqr_rel'],3), 'failed', b['closed_loop']['failed_solves'], 'parked', b['parked_solves'])"
echo "quick done"
