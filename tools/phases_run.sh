set -o pipefail
export NMPC_LIB=$PWD/drone-attitude-control_amd/lib/exp/libnmpc_hip_timing.so
mkdir -p gpurun_out
for a in "--model force --batch 1024" "--model force --batch 8192" "--model quad13 --batch 8192" "--model jerk --batch 4096"; do
  timeout -k 10 200 python tools/clf_phases.py $a --regions 3 >> gpurun_out/r5b_phases.jsonl 2>> gpurun_out/r5b_phases.err || { echo "phases failed: $a"; tail -5 gpurun_out/r5b_phases.err; exit 1; }
done
unset NMPC_LIB
for a in "--model force --batch 1024" "--model quad13 --batch 8192"; do
  timeout -k 10 200 python tools/clf_steps.py $a --regions 2 >> gpurun_out/r5b_steps.jsonl 2>> gpurun_out/r5b_steps.err || { echo "steps failed: $a"; exit 1; }
done
echo phases done
