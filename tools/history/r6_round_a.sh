#!/bin/bash
# Round-6 GPU pass A: the closed-loop tests (opt-in trajectory outputs), the lean-loop parity tests on the
# index-checked build (NMPC_CLF_CHECK), the default bench line, then PMC passes for the closed loop (quad13 /
# jerk, trajectory write-back off) and the fast solve (sf_kernel). Summaries are made on the CPU side.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r6h}
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 python -u -m pytest -q --maxfail=8 --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${TAG}_gpu.log 2>&1 || { tail -30 gpurun_out/${TAG}_gpu.log; exit 1; }
tail -1 gpurun_out/${TAG}_gpu.log
NMPC_LIB=$PWD/drone-attitude-control_amd/lib/exp/libnmpc_hip_clfcheck.so NMPC_CLF_CHECK=1 \
  timeout -k 10 900 $T tests/test_gpu_bench_parity.py tests/test_gpu_closed_loop.py > gpurun_out/${TAG}_check.log 2>&1 || { tail -30 gpurun_out/${TAG}_check.log; exit 1; }
tail -1 gpurun_out/${TAG}_check.log
grep -c "clf check" gpurun_out/${TAG}_check.log || true
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "
import json; b=json.load(open('gpurun_out/${TAG}_bench.json')); r=b['roofline']
print('bench', '%.1fM'%(b['value']/1e6), r['kernel'], 'kernel_ms %.4f'%r.get('kernel_ms', 0), 'frac %.3f'%r['frac'])"
TAG=${TAG}q KERNEL=cl_lock_kernel TRAFFIC=quad13,20,8192,fp64 bash tools/pmc_bench.sh || exit 1
TAG=${TAG}j KERNEL=cl_fast_kernel BENCH_ARGS="--model jerk --batch 4096" TRAFFIC=jerk,40,4096,fp64 bash tools/pmc_bench.sh || exit 1
TAG=${TAG}s KERNEL=sf_kernel MODE=solve TRAFFIC=quad13,20,8192,fp64 bash tools/pmc_bench.sh || exit 1
echo done
