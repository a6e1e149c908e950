#!/bin/bash
# the PMC passes of tools/round_evidence.sh alone (its other steps skipped): TAG=... bash tools/pmc_only.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-ev}
OUT=gpurun_out/ev_$TAG; mkdir -p $OUT
export TMPDIR=/tmp
# CFGS: ";"-separated name:args pairs (default: the five configs)
IFS=';' read -ra CS <<< "${CFGS:-quad13:--model quad13;force1024:--model force --batch 1024;force8192f32:--model force --batch 8192 --precision fp32;jerk:--model jerk --batch 4096;quad13f32:--model quad13 --precision fp32}"
for cfg in "${CS[@]}"; do
  name=${cfg%%:*}; args=${cfg#*:}
  echo "[pmc] $name"
  j=0
  for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP32 GRBM_GUI_ACTIVE GRBM_COUNT"; do
    j=$((j+1))
    timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $PWD/gpurun_out/pmc_${TAG}_${name}_$j -o run -- python3 bench.py $args --steps 20 --warmup 20 --repeats 3 --python-loop-steps 0 --no-cpu-baseline > $OUT/pmc_${name}_$j.log 2>&1 || { echo "pmc pass failed: $name $j"; tail -20 $OUT/pmc_${name}_$j.log; exit 1; }
  done
done
echo "[pmc] done"
