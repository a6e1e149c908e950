#!/bin/bash
# Tuning run: per-sweep clock cycles of the IPM kernel (NMPC_SWEEP_CYCLES) for each variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
for V in ${VARIANTS:-0}; do
  NMPC_SWEEP_CYCLES=1 NMPC_VARIANT=$V timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/cycles_v$V.json 2> $OUT/cycles_v$V.err || { echo "variant $V failed"; tail -20 $OUT/cycles_v$V.err; exit 1; }
  echo "variant $V"; grep "nmpc cycles" $OUT/cycles_v$V.err | tail -2
done
