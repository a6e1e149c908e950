set -o pipefail
mkdir -p gpurun_out
NMPC_LIB=$PWD/drone-attitude-control_amd/lib/exp/libnmpc_hip_timing.so timeout -k 10 200 python tools/clf_phases.py --model quad13 --batch 8192 --regions 3 > gpurun_out/lk2_phases.jsonl 2> gpurun_out/lk2_phases.err
