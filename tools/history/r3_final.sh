#!/bin/bash
# Round-3 GPU evidence: GPU tests, smoke, the default bench line, every BASELINE config, a rocprofv3
# kernel-trace --stats profile of the default bench command (its own ms_per_step recorded beside it),
# the PMC passes of the headline config (tools/pmc.sh). Each GPU step has its own time limit; the
# script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r3}
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread > $OUT/${TAG}_gputest.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/${TAG}_gputest.log; exit 1; }
  tail -1 $OUT/${TAG}_gputest.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/${TAG}_smoke.log; exit 1; }
  tail -1 $OUT/${TAG}_smoke.log
fi
timeout -k 10 400 python bench.py > $OUT/${TAG}_bench_quad13.json 2> $OUT/${TAG}_bench.err || { echo "bench failed"; tail -30 $OUT/${TAG}_bench.err; exit 1; }
python -c "import json; b=json.load(open('$OUT/${TAG}_bench_quad13.json')); print('bench %.2fM' % (b['value']/1e6), 'kernel', b['roofline']['kernel'], '%.4f ms' % b['roofline']['kernel_ms'], 'frac %.4f' % b['roofline']['frac'], 'cpu %.3fM' % (b['cpu_baseline']['value']/1e6), 'regions', b['timing']['region_ms'])"
if [ "${CONFIGS:-1}" = "1" ]; then
  : > $OUT/${TAG}_configs.jsonl
  for a in "--model force --batch 1024" "--model force --batch 8192 --precision fp32" "--model jerk --batch 4096" "--model force --batch 8192"; do
    timeout -k 10 400 python bench.py --python-loop-steps 0 $a >> $OUT/${TAG}_configs.jsonl 2>> $OUT/${TAG}_configs.err || { echo "config failed: $a"; exit 1; }
  done
  python -c "
import json
for l in open('$OUT/${TAG}_configs.jsonl'):
    b = json.loads(l); print(b['config']['model'], b['dtype'], b['config']['batch_per_gpu'], '%.3fM' % (b['value'] / 1e6), b['roofline']['kernel'], 'kernel %.4f ms' % b['roofline']['kernel_ms'], 'cpu %.3fM' % (b['cpu_baseline']['value']/1e6), 'failed', b['closed_loop']['failed_solves'])"
fi
if [ "${PROF:-1}" = "1" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof_${TAG} -o run --output-format csv -- python3 bench.py --no-cpu-baseline --python-loop-steps 0 > $OUT/${TAG}_prof_bench.json 2> $OUT/${TAG}_prof.log || { echo "rocprof failed"; tail -30 $OUT/${TAG}_prof.log; exit 1; }
  find $OUT/prof_${TAG} -name "*kernel_stats*" | head -3
  TAG=$TAG bash tools/pmc.sh || exit 1
fi
echo "r3 final done"
