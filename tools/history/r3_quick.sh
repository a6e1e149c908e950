#!/bin/bash
# quick GPU check of the lean closed loop: timing + oracle agreement (quad13 8192, jerk 4096), then the
# bench-parity and closed-loop GPU tests. Stops after a failure / fault / timeout.
TAG=${1:-q}
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 150 python tools/clf_check.py --model quad13 --batch 8192 --repeats 10 > gpurun_out/${TAG}_clf_q13.log 2>&1; rc=$?; tail -3 gpurun_out/${TAG}_clf_q13.log; [ $rc != 0 ] && exit $rc
timeout -k 10 150 python tools/clf_check.py --model jerk --batch 4096 --repeats 5 > gpurun_out/${TAG}_clf_jerk.log 2>&1; rc=$?; tail -3 gpurun_out/${TAG}_clf_jerk.log; [ $rc != 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_parity.py tests/test_gpu_closed_loop.py -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_par.log 2>&1; rc=$?; tail -5 gpurun_out/${TAG}_par.log
exit $rc
