#!/bin/bash
# Round-6 final evidence on one box: the whole GPU suite, smoke, the default bench line, its rocprofv3 kernel
# stats and PMC passes, every BASELINE config line and the solve lines. Output under gpurun_out/${TAG}_*.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r6z}
timeout -k 10 900 python -u -m pytest -q --maxfail=8 --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${TAG}_gpu.log 2>&1 || { tail -30 gpurun_out/${TAG}_gpu.log; exit 1; }
tail -1 gpurun_out/${TAG}_gpu.log
NMPC_LIB=$PWD/drone-attitude-control_amd/lib/exp/libnmpc_hip_clfcheck.so NMPC_CLF_CHECK=1 \
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bench_parity.py tests/test_gpu_closed_loop.py > gpurun_out/${TAG}_check.log 2>&1 || { tail -30 gpurun_out/${TAG}_check.log; exit 1; }
tail -1 gpurun_out/${TAG}_check.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "
import json; b=json.load(open('gpurun_out/${TAG}_bench.json')); r=b['roofline']
print('bench %.1fM'%(b['value']/1e6), r['kernel'], 'kernel_ms %.5f'%r['kernel_ms'], 'frac %.4f'%r['frac'], 'cpu %.2fM'%(b['cpu_baseline']['value']/1e6))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/${TAG}_trace -o run -- python3 bench.py --steps 20 --warmup 3 --python-loop-steps 0 --no-cpu-baseline > gpurun_out/${TAG}_trace_bench.json 2> gpurun_out/${TAG}_trace.err || { tail -20 gpurun_out/${TAG}_trace.err; exit 1; }
TAG=${TAG}q KERNEL=cl_lock_kernel TRAFFIC=quad13,20,8192,fp64 bash tools/pmc_bench.sh || exit 1
TAG=${TAG}f1 KERNEL=cl_fast_kernel BENCH_ARGS="--model force --batch 1024" TRAFFIC=force,20,1024,fp64 bash tools/pmc_bench.sh || exit 1
TAG=${TAG}f3 KERNEL=cl_fast_kernel BENCH_ARGS="--model force --batch 8192 --precision fp32" TRAFFIC=force,20,8192,fp32 bash tools/pmc_bench.sh || exit 1
TAG=${TAG}j KERNEL=cl_fast_kernel BENCH_ARGS="--model jerk --batch 4096" TRAFFIC=jerk,40,4096,fp64 bash tools/pmc_bench.sh || exit 1
TAG=$TAG bash tools/configs_bench.sh || exit 1
: > gpurun_out/${TAG}_solve.jsonl
for a in "" "--model force --batch 8192" "--model jerk --batch 4096"; do
  timeout -k 10 300 python bench.py --mode solve --steps 10 --warmup 2 --repeats 5 $a >> gpurun_out/${TAG}_solve.jsonl 2>> gpurun_out/${TAG}_solve.err || { echo "solve bench failed: $a"; tail -20 gpurun_out/${TAG}_solve.err; exit 1; }
done
echo done
