set -o pipefail
L=$PWD/drone-attitude-control_amd/lib/exp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/gputest_${TAG}.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gputest_${TAG}.log; exit 1; }
tail -1 gpurun_out/gputest_${TAG}.log
TAG=$TAG ARMS="A B C" A="NMPC_LIB=$L/libnmpc_hip_gi.so" B="NMPC_LIB=$L/libnmpc_hip_pdaspre.so" C="NMPC_CLF_XCD=1" CFGS="--model quad13;--model jerk --batch 4096;--model force --batch 1024;--model force --batch 8192 --precision fp32" REPS=2 bash tools/ab_env.sh &&
timeout -k 10 200 python tools/clf_steps.py --model quad13 --batch 8192 --regions 2 > gpurun_out/${TAG}_steps.json
