#!/bin/bash
# Round-end evidence on the GPU box: GPU tests, smoke, the default bench line (CPU baseline included),
# every BASELINE config, a rocprofv3 kernel-trace --stats profile of the bench, the PMC passes of the
# headline config. Every GPU step has its own time limit; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r2}
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread > $OUT/gputest_$TAG.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gputest_$TAG.log; exit 1; }
tail -1 $OUT/gputest_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke_$TAG.log; exit 1; }
tail -1 $OUT/smoke_$TAG.log
timeout -k 10 400 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench failed"; tail -30 $OUT/bench_$TAG.err; exit 1; }
python -c "import json; b=json.load(open('$OUT/bench_$TAG.json')); print('bench %.3fM' % (b['value']/1e6), 'kernel %.4f' % b['roofline']['kernel_ms'], 'cpu', b['cpu_baseline']['value'])"
: > $OUT/configs_$TAG.jsonl
for a in "--model force --batch 1024" "--model force --batch 8192 --precision fp32" "--model jerk --batch 4096" "--model quad13"; do
  timeout -k 10 400 python bench.py $a >> $OUT/configs_$TAG.jsonl 2>> $OUT/configs_$TAG.err || { echo "config failed: $a"; exit 1; }
done
python -c "
import json
for l in open('$OUT/configs_$TAG.jsonl'):
    b = json.loads(l); print(b['config']['model'], b['dtype'], b['config']['batch_per_gpu'], '%.3fM' % (b['value'] / 1e6), 'kernel %.4f ms' % b['roofline']['kernel_ms'], 'failed', b['closed_loop']['failed_solves'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof_$TAG -o run --output-format csv -- python3 bench.py --no-cpu-baseline --python-loop-steps 0 > $OUT/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof_$TAG.log; exit 1; }
find $OUT/prof_$TAG -name "*kernel_stats*" | head -3
TAG=$TAG bash tools/pmc.sh || exit 1
echo "final profile done"
