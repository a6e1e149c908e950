#!/bin/bash
# Solve-kernel time of experimental library builds (lib/exp/libnmpc_hip_<L>.so) vs the default
# build, over batch sizes. LIBS="R80 R40" BATCHES="1024 8192".
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for B in ${BATCHES:-1024 8192}; do
  for L in default ${LIBS}; do
    if [ "$L" = default ]; then unset NMPC_LIB; else export NMPC_LIB=drone-attitude-control_amd/lib/exp/libnmpc_hip_$L.so; fi
    timeout -k 10 120 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --batch $B ${BENCH_ARGS:-} > gpurun_out/ls.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ls.json')); print('$L B=$B kernel %.3f ms iters %.3f' % (d['roofline']['kernel_ms'], d['roofline']['gpu_mean_qp_iter']))"
  done
done
