#!/bin/bash
# fast-solve iteration: the solver GPU tests, the quad13 / force solve lines, and a rocprofv3 kernel-trace of the
# quad13 solve bench (TAG names the outputs)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r6x}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_solver.py > gpurun_out/${TAG}_solver.log 2>&1 || { tail -30 gpurun_out/${TAG}_solver.log; exit 1; }
tail -1 gpurun_out/${TAG}_solver.log
: > gpurun_out/${TAG}_solve.jsonl
for a in "" ${SOLVE_MODELS:-"--model force --batch 8192"}; do
  timeout -k 10 300 python bench.py --mode solve --steps 10 --warmup 2 --repeats 5 $a >> gpurun_out/${TAG}_solve.jsonl 2>> gpurun_out/${TAG}_solve.err || { echo "solve bench failed: $a"; tail -20 gpurun_out/${TAG}_solve.err; exit 1; }
done
python -c "
import json
for l in open('gpurun_out/${TAG}_solve.jsonl'):
    b=json.loads(l); r=b['roofline']; print(b['config']['model'], b['config']['batch_per_gpu'], '%.1fM QP/s'%(b['value']/1e6), r['kernel'], 'kernel %.4f ms'%r['kernel_ms'], 'ms/step %.4f'%b['ms_per_step'], 'frac %.3f %s'%(r['frac'], r['bound']), 'cpu %.3fM'%(b['cpu_baseline']['value']/1e6), 'failed', b['failed_solves'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/prof_${TAG} -o run --output-format csv -- python3 bench.py --mode solve --steps 10 --warmup 2 --repeats 5 --no-cpu-baseline > gpurun_out/${TAG}_prof_solve.json 2> gpurun_out/${TAG}_prof.log || { echo rocprof failed; tail gpurun_out/${TAG}_prof.log; exit 1; }
find gpurun_out/prof_${TAG} -name "*kernel_stats*" -exec head -6 {} \;
