#!/bin/bash
# rocprofv3 PMC passes over bench.py at the bench's own launch length (--steps 20, every launch of the
# run 20 steps: warmup 20), one counter group per run, nothing else traced. Then the summary into
# profiles/pmc_traffic.json keyed by (config, kernel, steps per launch).
#   TAG=r5a KERNEL=cl_fast_kernel BENCH_ARGS="--model force --batch 1024" TRAFFIC=force,20,1024,fp64 bash tools/pmc_bench.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-pmc}
STEPS=${STEPS:-20}
MODE=${MODE:-closed_loop}
export TMPDIR=/tmp
if [ "$MODE" = "solve" ]; then
  ARGS="--mode solve --steps $STEPS --warmup 2 --repeats 2 --no-cpu-baseline ${BENCH_ARGS:-}"
else
  ARGS="--steps $STEPS --warmup $STEPS --repeats 3 --python-loop-steps 0 --no-cpu-baseline ${BENCH_ARGS:-}"
fi
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
         "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP32 GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $PWD/$OUT/pmc_${TAG}_$i -o run -- python3 bench.py $ARGS > $OUT/pmc_${TAG}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 $OUT/pmc_${TAG}_$i.log; exit 1; }
done
SPL=$STEPS; [ "$MODE" = "solve" ] && SPL=1
python tools/pmc_summary.py $TAG --kernel ${KERNEL:-cl_fast_kernel} --out gpurun_out/${TAG}_pmc.json \
    ${TRAFFIC:+--traffic $TRAFFIC} --steps-per-launch $SPL --mode $MODE > /dev/null || { echo "pmc summary failed"; exit 1; }
echo "pmc $TAG done"
