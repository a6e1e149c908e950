set -o pipefail
L=$PWD/drone-attitude-control_amd/lib/exp
TAG=r7g ARMS="A B C" A="NMPC_LIB=$L/libnmpc_hip_r5.so" B="NMPC_CLF_XCD=1" C="NMPC_LIB=$L/libnmpc_hip_wc.so" CFGS="--model quad13;--model jerk --batch 4096;--model force --batch 1024" REPS=2 bash tools/ab_env.sh &&
NMPC_LIB=$L/libnmpc_hip_r5.so timeout -k 10 200 python tools/clf_steps.py --model quad13 --batch 8192 --regions 2 > gpurun_out/r7g_steps_r5.json &&
timeout -k 10 200 python tools/clf_steps.py --model quad13 --batch 8192 --regions 2 > gpurun_out/r7g_steps_cur.json
