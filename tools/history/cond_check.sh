#!/bin/bash
# Condensed-family check on the GPU box: parity tests, solve-kernel timing per family, and the
# per-phase cycles of the timing build (lib/exp/libnmpc_hip_ctime.so, NMPC_COND_TIMING).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-cc}
timeout -k 10 200 python -u -m pytest tests/test_gpu_condensed.py -q -s --timeout 120 --timeout-method thread > $OUT/${TAG}_cond.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/${TAG}_cond.log
[ $rc -le 1 ] || exit 1
timeout -k 10 300 python -u tools/family_bench.py --families ${FAMS:-cond} --configs ${CONFIGS:-force20_1024_fp64,force20_8192_fp32,force20_8192_fp64} > $OUT/${TAG}_family.jsonl 2> $OUT/${TAG}_family.err || { echo family failed; tail $OUT/${TAG}_family.err; exit 1; }
NMPC_LIB=drone-attitude-control_amd/lib/exp/libnmpc_hip_ctime.so NMPC_SWEEP_CYCLES=1 timeout -k 10 200 python -u tools/family_bench.py --families cond --reps 1 --configs ${CONFIGS:-force20_1024_fp64,force20_8192_fp32} > /dev/null 2> $OUT/${TAG}_cycles.err || { echo cycles failed; exit 1; }
grep "cond cycles" $OUT/${TAG}_cycles.err | sort -u
