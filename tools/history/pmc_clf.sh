#!/bin/bash
# rocprofv3 PMC passes over the lean closed loop (tools/clf_check.py, quad13 B=8192), one counter group
# per run, nothing else traced. Summarise with: python tools/pmc_summary.py TAG --kernel cl_fast_kernel
TAG=${1:-clf}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
ARGS="--model ${MODEL:-quad13} --batch ${BATCH:-8192} --steps 20 --warmup 20 --repeats 3 --oracle 0"
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
         "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FLOPS_FP64 SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $PWD/gpurun_out/pmc_${TAG}_$i -o run -- python3 tools/clf_check.py $ARGS > gpurun_out/pmc_${TAG}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/pmc_${TAG}_$i.log; exit 1; }
done
echo "pmc done"
