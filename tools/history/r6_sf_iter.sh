#!/bin/bash
# sf_kernel iteration: solver GPU tests, the phase timing of the quad13 solve (timing build), the solve lines
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r6x}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_solver.py > gpurun_out/${TAG}_solver.log 2>&1 || { tail -30 gpurun_out/${TAG}_solver.log; exit 1; }
tail -1 gpurun_out/${TAG}_solver.log
rm -f gpurun_out/${TAG}_cyc.bin
NMPC_LIB=$PWD/drone-attitude-control_amd/lib/exp/libnmpc_hip_sftiming.so NMPC_SF_CYCLES=gpurun_out/${TAG}_cyc.bin timeout -k 10 200 python bench.py --mode solve --steps 2 --warmup 1 --repeats 1 --no-cpu-baseline > gpurun_out/${TAG}_sft.json 2>gpurun_out/${TAG}_sft.err || { tail gpurun_out/${TAG}_sft.err; exit 1; }
python tools/sf_phases.py gpurun_out/${TAG}_cyc.bin 8192 4
: > gpurun_out/${TAG}_solve.jsonl
for a in "" "--model force --batch 8192" "--model jerk --batch 4096"; do
  timeout -k 10 300 python bench.py --mode solve --steps 10 --warmup 2 --repeats 5 $a >> gpurun_out/${TAG}_solve.jsonl 2>> gpurun_out/${TAG}_solve.err || { echo "solve bench failed: $a"; tail -20 gpurun_out/${TAG}_solve.err; exit 1; }
done
python -c "
import json
for l in open('gpurun_out/${TAG}_solve.jsonl'):
    b=json.loads(l); r=b['roofline']; print(b['config']['model'], b['config']['batch_per_gpu'], '%.1fM QP/s'%(b['value']/1e6), r['kernel'], 'kernel %.4f ms'%r['kernel_ms'], 'ms/step %.4f'%b['ms_per_step'], 'frac %.3f %s'%(r['frac'], r['bound']), 'cpu %.3fM'%(b['cpu_baseline']['value']/1e6), 'failed', b['failed_solves'])"
