#!/bin/bash
# The round's evidence for the final tree, on one MI355X box, into gpurun_out/ev_$TAG/ (copied to profiles/r7/ after):
#   gputest.log        pytest -m gpu (the driver's command)
#   smoke.log          __graft_entry__.smoke()
#   bench.json         python bench.py (the default line: quad13 N=20 B=8192 fp64, CPU baseline included)
#   configs.jsonl      BASELINE configs 2, 3, 5 and the headline dims in fp32 (bench.py --model ...)
#   solves.jsonl       bench.py --mode solve (quad13, force, jerk N=40)
#   gpus2_gloo.json    bench.py --gpus 2 --dist-backend gloo (the self-launched two-rank path on one GPU)
#   steps_quad13.json  the headline's per-step record (tools/clf_steps.py)
#   prof_*/            rocprofv3 --kernel-trace --stats of the default bench (kernel durations)
#   pmc_*              rocprofv3 PMC passes (one counter group per run) at the bench's 20-step launches, per config;
#                      summarised locally by tools/pmc_summary.py into profiles/pmc_traffic.json
# Every GPU step has its own time limit; the script stops at the first failure.
#   TAG=r7z bash tools/round_evidence.sh            (PMC=0: skip the PMC passes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-ev}
OUT=gpurun_out/ev_$TAG; mkdir -p $OUT
export TMPDIR=/tmp
step() { echo "[evidence] $*"; }
step "gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/gputest.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gputest.log; exit 1; }
tail -1 $OUT/gputest.log
step "smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
step "bench (default)"
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
step "configs"
: > $OUT/configs.jsonl
for a in "--model force --batch 1024" "--model force --batch 8192 --precision fp32" "--model jerk --batch 4096" "--model quad13 --precision fp32" "--model quad13"; do
  timeout -k 10 300 python bench.py $a --python-loop-steps 0 >> $OUT/configs.jsonl 2>> $OUT/configs.err || { echo "config failed: $a"; exit 1; }
done
step "solves"
: > $OUT/solves.jsonl
for a in "--model quad13" "--model force" "--model jerk --horizon 40 --batch 4096"; do
  timeout -k 10 300 python bench.py --mode solve $a >> $OUT/solves.jsonl 2>> $OUT/solves.err || { echo "solve failed: $a"; exit 1; }
done
step "two ranks (self-launched, gloo)"
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --model force --batch 4096 --no-cpu-baseline > $OUT/gpus2_gloo.json 2> $OUT/gpus2_gloo.err || { echo "gpus 2 failed"; tail -20 $OUT/gpus2_gloo.err; exit 1; }
step "step log"
timeout -k 10 200 python tools/clf_steps.py --model quad13 --batch 8192 --regions 3 > $OUT/steps_quad13.json || { echo "step log failed"; exit 1; }
step "rocprofv3 kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof_quad13 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --python-loop-steps 0 > $OUT/prof_quad13.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof_quad13.log; exit 1; }
if [ "${PMC:-1}" = "1" ]; then   # (also alone: tools/pmc_only.sh)
  i=0
  for cfg in "quad13:--model quad13" "force1024:--model force --batch 1024" "force8192f32:--model force --batch 8192 --precision fp32" "jerk:--model jerk --batch 4096" "quad13f32:--model quad13 --precision fp32"; do
    name=${cfg%%:*}; args=${cfg#*:}
    step "pmc $name"
    j=0
    for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
             "FETCH_SIZE" "WRITE_SIZE" \
             "SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP32 GRBM_GUI_ACTIVE GRBM_COUNT"; do
      j=$((j+1))
      timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $PWD/gpurun_out/pmc_${TAG}_${name}_$j -o run -- python3 bench.py $args --steps 20 --warmup 20 --repeats 3 --python-loop-steps 0 --no-cpu-baseline > $OUT/pmc_${name}_$j.log 2>&1 || { echo "pmc pass failed: $name $j"; tail -20 $OUT/pmc_${name}_$j.log; exit 1; }
    done
  done
fi
step "done"
