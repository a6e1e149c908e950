#!/bin/bash
# Round-6 GPU pass C: the whole GPU suite, the lean-loop parity tests on the index-checked build, every config's
# bench line, the solve lines, and a same-box A/B of the one-wavefront-per-SIMD force variant (NMPC_CLF_ONE).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r6m}
timeout -k 10 900 python -u -m pytest -q --maxfail=8 --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${TAG}_gpu.log 2>&1 || { tail -30 gpurun_out/${TAG}_gpu.log; exit 1; }
tail -1 gpurun_out/${TAG}_gpu.log
NMPC_LIB=$PWD/drone-attitude-control_amd/lib/exp/libnmpc_hip_clfcheck.so NMPC_CLF_CHECK=1 \
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bench_parity.py tests/test_gpu_closed_loop.py > gpurun_out/${TAG}_check.log 2>&1 || { tail -30 gpurun_out/${TAG}_check.log; exit 1; }
tail -1 gpurun_out/${TAG}_check.log
TAG=$TAG bash tools/configs_bench.sh || exit 1
: > gpurun_out/${TAG}_solve.jsonl
for a in "" "--model force --batch 8192" "--model jerk --batch 4096"; do
  timeout -k 10 300 python bench.py --mode solve --steps 10 --warmup 2 --repeats 5 $a >> gpurun_out/${TAG}_solve.jsonl 2>> gpurun_out/${TAG}_solve.err || { echo "solve bench failed: $a"; tail -20 gpurun_out/${TAG}_solve.err; exit 1; }
done
python -c "
import json
for l in open('gpurun_out/${TAG}_solve.jsonl'):
    b=json.loads(l); r=b['roofline']; print('solve', b['config']['model'], '%.1fM QP/s'%(b['value']/1e6), r['kernel'], 'kernel %.4f ms'%r['kernel_ms'], 'frac %.3f'%r['frac'], 'cpu %.2fM'%(b['cpu_baseline']['value']/1e6))"
: > gpurun_out/${TAG}_one_ab.jsonl
for rep in 1 2 3; do
  for one in 1 0; do
    NMPC_CLF_ONE=$one timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --python-loop-steps 0 --model force --batch 1024 > gpurun_out/${TAG}_one.json 2>> gpurun_out/${TAG}_one.err || { tail gpurun_out/${TAG}_one.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/${TAG}_one.json')); print(json.dumps({'NMPC_CLF_ONE': $one, 'value': d['value'], 'kernel_ms': d['roofline']['kernel_ms']}))" | tee -a gpurun_out/${TAG}_one_ab.jsonl
  done
done
TAG=${TAG}u LIBS="ucg" CONFIGS="--model force --batch 1024;--model force --batch 8192;--model quad13 --batch 8192;--model jerk --batch 4096" bash tools/r6_qb_ab.sh > /dev/null || exit 1
python -c "
import json, collections
d = collections.defaultdict(list)
for l in open('gpurun_out/${TAG}u_ab.jsonl'):
    r = json.loads(l); d[(r['cfg'], r['lib'])].append(r['value'] / 1e6)
for k, v in sorted(d.items()): print(k, ['%.1f' % x for x in v])"
echo done
