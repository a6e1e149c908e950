#!/bin/bash
# Per-sweep / per-phase clock cycles (s_memtime) of the solve kernel from the timing experiment
# builds (lib/exp/libnmpc_hip_{swt,pht,fwt}.so, build.build_experiment) at the given batches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for L in ${LIBS:-swt pht fwt}; do
  for B in ${BATCHES:-1024 8192}; do
    NMPC_LIB=drone-attitude-control_amd/lib/exp/libnmpc_hip_$L.so NMPC_SWEEP_CYCLES=1 timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --batch $B ${BENCH_ARGS:-} > gpurun_out/t_${L}_$B.json 2> gpurun_out/t_${L}_$B.err || { tail -5 gpurun_out/t_${L}_$B.err; exit 1; }
    echo "$L B=$B: $(grep 'nmpc cycles' gpurun_out/t_${L}_$B.err | tail -1)"
  done
done
