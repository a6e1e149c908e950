set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_solver.py > gpurun_out/r6b_solver.log 2>&1; rc=$?
tail -5 gpurun_out/r6b_solver.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/r6b_solver.log | head -20; exit 1; }
for a in "" "--model force --batch 8192" "--model force --batch 1024" "--model jerk --batch 4096"; do
  timeout -k 10 300 python bench.py --mode solve --steps 10 --warmup 2 --repeats 5 $a >> gpurun_out/r6b_solve.jsonl 2>> gpurun_out/r6b_solve.err || { echo "solve bench failed: $a"; tail -20 gpurun_out/r6b_solve.err; exit 1; }
done
python -c "
import json
for l in open('gpurun_out/r6b_solve.jsonl'):
    b=json.loads(l); r=b['roofline']; print(b['config']['model'], b['config']['batch_per_gpu'], '%.1fM QP/s'%(b['value']/1e6), r['kernel'], 'kernel %.4f ms'%r['kernel_ms'], 'frac %.3f %s'%(r['frac'], r['bound']), 'cpu %.3fM'%(b['cpu_baseline']['value']/1e6), b['cpu_baseline'].get('paths'), 'failed', b['failed_solves'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/gpurun_out/prof_r6b -o run --output-format csv -- python3 bench.py --mode solve --steps 10 --warmup 2 --repeats 5 --no-cpu-baseline > gpurun_out/r6b_prof_solve.json 2> gpurun_out/r6b_prof.log || { echo rocprof failed; tail gpurun_out/r6b_prof.log; exit 1; }
find gpurun_out/prof_r6b -name "*kernel_stats*" -exec head -8 {} \;
