#!/bin/bash
# MFMA evidence for the condensed family (cond_ipm_kernel, the dimension-generic path whose Hessian
# block-GEMMs run on v_mfma_f64_16x16x4f64): rocprofv3 PMC passes over tools/family_bench.py
# (force N=20, B=1024 and 8192, fp64), one counter group per run. Summarise with
#   python tools/pmc_summary.py TAG_1024 --kernel cond_ipm_kernel   (and TAG_8192)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=${TAG:-cond}
for B in 1024 8192; do
  i=0
  for C in "SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $PWD/gpurun_out/pmc_${TAG}_${B}_$i -o run -- python3 tools/family_bench.py --families cond --reps 3 --configs force20_${B}_fp64 > gpurun_out/pmc_${TAG}_${B}_$i.log 2>&1 || { echo "pmc pass $B/$i failed"; tail -5 gpurun_out/pmc_${TAG}_${B}_$i.log; exit 1; }
  done
done
echo "pmc cond done"
