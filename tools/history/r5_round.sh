#!/bin/bash
# Round-4 GPU evidence (profile tags r5*): GPU tests, smoke, the default bench line, every BASELINE
# config, the general-solve line (--mode solve), a rocprofv3 kernel-trace --stats profile of the default
# bench command (its own line recorded beside it), and PMC passes at the bench's launch length for every
# config (tools/pmc_bench.sh). Each GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-r5}
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread ${TEST_ARGS:-} > $OUT/${TAG}_gputest.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/${TAG}_gputest.log; exit 1; }
  tail -1 $OUT/${TAG}_gputest.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/${TAG}_smoke.log; exit 1; }
  tail -1 $OUT/${TAG}_smoke.log
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 400 python bench.py > $OUT/${TAG}_bench_quad13.json 2> $OUT/${TAG}_bench.err || { echo "bench failed"; tail -30 $OUT/${TAG}_bench.err; exit 1; }
  python -c "import json; b=json.load(open('$OUT/${TAG}_bench_quad13.json')); print('bench %.2fM' % (b['value']/1e6), 'kernel', b['roofline']['kernel'], '%.4f ms' % b['roofline']['kernel_ms'], 'frac %.4f' % b['roofline']['frac'], 'cpu %.3fM' % (b['cpu_baseline']['value']/1e6), 'regions', b['timing']['region_ms'], 'parked', b['parked_solves'])"
fi
if [ "${CONFIGS:-1}" = "1" ]; then
  : > $OUT/${TAG}_configs.jsonl
  for a in "--model force --batch 1024" "--model force --batch 8192 --precision fp32" "--model jerk --batch 4096" "--model force --batch 8192"; do
    timeout -k 10 400 python bench.py --python-loop-steps 0 $a >> $OUT/${TAG}_configs.jsonl 2>> $OUT/${TAG}_configs.err || { echo "config failed: $a"; tail -20 $OUT/${TAG}_configs.err; exit 1; }
  done
  python -c "
import json
for l in open('$OUT/${TAG}_configs.jsonl'):
    b = json.loads(l); print(b['config']['model'], b['dtype'], b['config']['batch_per_gpu'], '%.3fM' % (b['value'] / 1e6), b['roofline']['kernel'], 'kernel %.4f ms' % b['roofline']['kernel_ms'], 'cpu %.3fM' % (b['cpu_baseline']['value']/1e6), 'failed', b['closed_loop']['failed_solves'], 'parked', b['parked_solves'])"
fi
if [ "${SOLVE:-1}" = "1" ]; then
  timeout -k 10 400 python bench.py --mode solve --steps 10 --warmup 2 --repeats 5 > $OUT/${TAG}_solve_quad13.json 2> $OUT/${TAG}_solve.err || { echo "solve bench failed"; tail -20 $OUT/${TAG}_solve.err; exit 1; }
  python -c "import json; b=json.load(open('$OUT/${TAG}_solve_quad13.json')); print('solve %.3fM QP/s' % (b['value']/1e6), b['roofline']['kernel'], 'kernel %.4f ms' % b['roofline']['kernel_ms'], 'frac %.4f' % b['roofline']['frac'], 'cpu %.0f' % b['cpu_baseline']['value'])"
fi
if [ "${PROF:-1}" = "1" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof_${TAG} -o run --output-format csv -- python3 bench.py --no-cpu-baseline --python-loop-steps 0 > $OUT/${TAG}_prof_bench.json 2> $OUT/${TAG}_prof.log || { echo "rocprof failed"; tail -30 $OUT/${TAG}_prof.log; exit 1; }
  find $OUT/prof_${TAG} -name "*kernel_stats*" | head -3
fi
if [ "${PMC:-1}" = "1" ]; then
  TAG=${TAG}_quad13_b8192_fp64 KERNEL=cl_lock_kernel BENCH_ARGS="" TRAFFIC=quad13,20,8192,fp64 bash tools/pmc_bench.sh || exit 1
  TAG=${TAG}_force_b1024_fp64 KERNEL=cl_fast_kernel BENCH_ARGS="--model force --batch 1024" TRAFFIC=force,20,1024,fp64 bash tools/pmc_bench.sh || exit 1
  TAG=${TAG}_force_b8192_fp64 KERNEL=cl_fast_kernel BENCH_ARGS="--model force --batch 8192" TRAFFIC=force,20,8192,fp64 bash tools/pmc_bench.sh || exit 1
  TAG=${TAG}_jerk_b4096_fp64 KERNEL=cl_fast_kernel BENCH_ARGS="--model jerk --batch 4096" TRAFFIC=jerk,40,4096,fp64 bash tools/pmc_bench.sh || exit 1
  TAG=${TAG}_force_b8192_fp32 KERNEL=${FP32_KERNEL:-cl_fast_kernel} BENCH_ARGS="--model force --batch 8192 --precision fp32" TRAFFIC=force,20,8192,fp32 bash tools/pmc_bench.sh || exit 1
  TAG=${TAG}_solve_quad13_b8192_fp64 KERNEL=ipm_lpc_kernel MODE=solve STEPS=5 BENCH_ARGS="" TRAFFIC=quad13,20,8192,fp64 bash tools/pmc_bench.sh || exit 1
fi
echo "r5 round done"
