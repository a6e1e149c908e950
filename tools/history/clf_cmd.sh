# Lean closed loop vs the C oracle (tools/clf_check.py) on every shape it runs: small batches against
# modes 1 and 0, then the bench sizes against mode 1, with the per-launch log (NMPC_CLF_DEBUG) on stderr.
export TMPDIR=/tmp; mkdir -p gpurun_out
T=${TAG:-clf}
run() { timeout -k 10 180 python tools/clf_check.py "$@" > gpurun_out/${T}_$2_$4.json 2> gpurun_out/${T}_$2_$4.err; rc=$?; tail -c 700 gpurun_out/${T}_$2_$4.json; echo; return $rc; }
for m in quad13 jerk force; do run --model $m --batch 64 || exit $?; done
NMPC_CLF_DEBUG=1 run --model quad13 --batch 8192 --repeats 10 || exit $?
NMPC_CLF_DEBUG=1 run --model force --batch 1024 --repeats 10 || exit $?
NMPC_CLF_DEBUG=1 run --model jerk --batch 4096 --repeats 10 || exit $?
NMPC_CLF_DEBUG=1 run --model force --batch 8192 --repeats 10 || exit $?
if [ "${VARIANTS:-0}" = "1" ]; then
  NMPC_CLF_VARIANT=1 run --model quad13 --batch 8192 --repeats 10 --oracle 0 || exit $?
  cp gpurun_out/${T}_quad13_8192.json gpurun_out/${T}_quad13_8192_v1.json
  run --model quad13 --batch 8192 --repeats 10 --oracle 0 || exit $?
  for b in 1024 8192; do
    cp gpurun_out/${T}_force_$b.json gpurun_out/${T}_force_${b}_v0.json
    NMPC_CLF_DEBUG=1 NMPC_CLF_VARIANT=1 run --model force --batch $b --repeats 10 || exit $?
    cp gpurun_out/${T}_force_$b.json gpurun_out/${T}_force_${b}_v1.json; cp gpurun_out/${T}_force_$b.err gpurun_out/${T}_force_${b}_v1.err
  done
fi
if [ "${STEPS:-0}" = "1" ]; then
  for a in "force 1024" "quad13 8192" "jerk 4096"; do set -- $a
    timeout -k 10 120 python tools/clf_steps.py --model $1 --batch $2 > gpurun_out/${T}_steps_$1_$2.json 2>&1 || exit $?
  done
fi
