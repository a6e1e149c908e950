#!/bin/bash
# Where the quad13 launch goes now: the phase build (per-instance phase cycles) and the step log (timeline)
set -o pipefail
mkdir -p gpurun_out
NMPC_LIB=$PWD/drone-attitude-control_amd/lib/exp/libnmpc_hip_timing.so timeout -k 10 200 python tools/clf_phases.py --model quad13 --batch 8192 --regions 3 > gpurun_out/${TAG}_q_phases.json 2> gpurun_out/${TAG}_q_phases.err || { tail gpurun_out/${TAG}_q_phases.err; exit 1; }
timeout -k 10 200 python tools/clf_steps.py --model quad13 --batch 8192 > gpurun_out/${TAG}_q_steps.json 2> gpurun_out/${TAG}_q_steps.err || { tail gpurun_out/${TAG}_q_steps.err; exit 1; }
echo done
