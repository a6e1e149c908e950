#!/bin/bash
# Round-3 GPU pass: the GPU test suite, then the default bench (driver's command line).
# usage: tools/round3_gpu.sh TAG
# Stops after a fault / abort / timeout (exit codes 124, 134, 137, 139) — nothing more runs on the GPU.
TAG=${1:-r3a}
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) return 0;; esac; return 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputest.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -3 gpurun_out/${TAG}_gputest.log
if fatal $rc; then exit $rc; fi
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc $rc"; tail -c 600 gpurun_out/${TAG}_bench.json
exit $rc
