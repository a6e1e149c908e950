set -o pipefail
mkdir -p gpurun_out
L=$PWD/drone-attitude-control_amd/lib/exp/libnmpc_hip_timing.so
NMPC_CLF_LOCK=0 NMPC_LIB=$L timeout -k 10 200 python tools/clf_phases.py --model quad13 --batch 8192 --regions 3 > gpurun_out/${TAG}_phases_fast.json 2> gpurun_out/${TAG}_phases_fast.err &&
NMPC_LIB=$L timeout -k 10 200 python tools/clf_phases.py --model quad13 --batch 8192 --regions 3 > gpurun_out/${TAG}_phases_lock.json 2> gpurun_out/${TAG}_phases_lock.err &&
NMPC_LIB=$L timeout -k 10 200 python tools/clf_phases.py --model force --batch 1024 --regions 3 > gpurun_out/${TAG}_phases_force.json 2> gpurun_out/${TAG}_phases_force.err
