set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_solver.py -k "quad13 or full_size or infeasib" > gpurun_out/r6e_t.log 2>&1 || { tail -30 gpurun_out/r6e_t.log; exit 1; }
tail -1 gpurun_out/r6e_t.log
NMPC_LIB=$PWD/drone-attitude-control_amd/lib/exp/libnmpc_hip_sftiming.so NMPC_SF_CYCLES=gpurun_out/sf_cyc4.bin timeout -k 10 200 python bench.py --mode solve --steps 2 --warmup 1 --repeats 1 --no-cpu-baseline > gpurun_out/r6e_sft.json 2>gpurun_out/r6e_sft.err && python tools/sf_phases.py gpurun_out/sf_cyc4.bin 8192 16
for v in 0 1; do NMPC_SF_4X4=$v timeout -k 10 200 python bench.py --mode solve --steps 10 --warmup 2 --repeats 5 --no-cpu-baseline > gpurun_out/r6e_b$v.json && python -c "
import json; b=json.load(open('gpurun_out/r6e_b$v.json')); print('4x4=$v', b['value']/1e6, b['roofline']['kernel_ms'])"; done
