#!/bin/bash
# Round-6 GPU pass B: force PMC passes (write-back off), the kernel-trace stats of the default bench, every
# BASELINE config's bench line, and the force B = 1024 phase / step records (timing build, iter log).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r6k}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/${TAG}_trace -o run -- python3 bench.py --steps 20 --warmup 3 --python-loop-steps 0 > gpurun_out/${TAG}_trace_bench.json 2> gpurun_out/${TAG}_trace.err || { tail -20 gpurun_out/${TAG}_trace.err; exit 1; }
echo trace done
TAG=$TAG bash tools/configs_bench.sh || exit 1
TAG=${TAG}f1 KERNEL=cl_fast_kernel BENCH_ARGS="--model force --batch 1024" TRAFFIC=force,20,1024,fp64 bash tools/pmc_bench.sh || exit 1
TAG=${TAG}f8 KERNEL=cl_fast_kernel BENCH_ARGS="--model force --batch 8192" TRAFFIC=force,20,8192,fp64 bash tools/pmc_bench.sh || exit 1
TAG=${TAG}f3 KERNEL=cl_fast_kernel BENCH_ARGS="--model force --batch 8192 --precision fp32" TRAFFIC=force,20,8192,fp32 bash tools/pmc_bench.sh || exit 1
NMPC_LIB=$PWD/drone-attitude-control_amd/lib/exp/libnmpc_hip_timing.so timeout -k 10 200 python tools/clf_phases.py --model force --batch 1024 --regions 3 > gpurun_out/${TAG}_force_phases.json 2> gpurun_out/${TAG}_force_phases.err || { tail gpurun_out/${TAG}_force_phases.err; exit 1; }
timeout -k 10 200 python tools/clf_steps.py --model force --batch 1024 > gpurun_out/${TAG}_force_steps.json 2> gpurun_out/${TAG}_force_steps.err || { tail gpurun_out/${TAG}_force_steps.err; exit 1; }
echo done
