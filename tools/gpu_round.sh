#!/bin/bash
# One GPU-box pass after a change: GPU tests, the default bench line, the quad13 chain statistics
# and (CONFIGS=1) every BASELINE config. Every GPU step has its own time limit; stops at the first
# failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-x}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/gputest_$TAG.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gputest_$TAG.log; exit 1; }
  tail -1 $OUT/gputest_$TAG.log
fi
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo "bench failed"; tail -30 $OUT/bench_$TAG.err; exit 1; }
python -c "import json; b=json.load(open('$OUT/bench_$TAG.json')); print('bench', b['config']['model'], '%.3fM' % (b['value']/1e6), 'kernel %.4f ms' % b['roofline']['kernel_ms'], 'frac %.4f' % b['roofline']['frac'], 'failed', b['closed_loop']['failed_solves'])"
NMPC_ITER_LOG=1 timeout -k 10 200 python tools/chain_stats.py > $OUT/chain_$TAG.json || { echo "chain failed"; exit 1; }
python -c "import json; c=json.load(open('$OUT/chain_$TAG.json')); print('chain mean %.1f p99 %.1f max %.1f' % (c['wave_chain_mean'], c['wave_chain_p99'], c['wave_chain_max']), 'kernel/step %.3f' % c['kernel_ms_per_step'])"
if [ "${CONFIGS:-0}" = "1" ]; then
  : > $OUT/configs_$TAG.jsonl
  for a in "--model force --batch 1024" "--model force --batch 8192 --precision fp32" "--model jerk --batch 4096" "--model quad13"; do
    timeout -k 10 300 python bench.py $a ${CFG_ARGS:-} >> $OUT/configs_$TAG.jsonl 2>> $OUT/configs_$TAG.err || { echo "config failed: $a"; exit 1; }
  done
  python -c "
import json
for l in open('$OUT/configs_$TAG.jsonl'):
    b = json.loads(l); print(b['config']['model'], b['dtype'], b['config']['batch_per_gpu'], '%.3fM' % (b['value'] / 1e6), 'kernel %.4f ms' % b['roofline']['kernel_ms'], 'failed', b['closed_loop']['failed_solves'])"
fi
if [ "${SOLVES:-0}" = "1" ]; then
  : > $OUT/solves_$TAG.jsonl
  for a in "--model quad13" "--model force" "--model jerk --horizon 40 --batch 4096"; do
    timeout -k 10 300 python bench.py --mode solve $a ${CFG_ARGS:-} >> $OUT/solves_$TAG.jsonl 2>> $OUT/solves_$TAG.err || { echo "solve line failed: $a"; exit 1; }
  done
  python -c "
import json
for l in open('$OUT/solves_$TAG.jsonl'):
    b = json.loads(l); print('solve', b['config']['model'], b['config']['batch_per_gpu'], '%.1fM QP/s' % (b['value'] / 1e6), 'kernel %.4f ms' % b['roofline']['kernel_ms'], b.get('fast_counts'))"
fi
echo "round pass done"
