#!/bin/bash
# rocprofv3 PMC passes over a short bench run (each counter group in its own run; no tracing mixed in)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-pmc}
export TMPDIR=/tmp
# warmup = steps: every solve launch of the run carries the same number of fused closed-loop steps
ARGS="--steps 5 --warmup 5 --repeats 3 --python-loop-steps 0 --no-cpu-baseline ${BENCH_ARGS:-}"
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
         "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE GRBM_COUNT" \
         "SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FLOPS_FP64"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $PWD/$OUT/pmc_${TAG}_$i -o run -- python3 bench.py $ARGS > $OUT/pmc_${TAG}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 $OUT/pmc_${TAG}_$i.log; exit 1; }
done
echo "pmc done"
