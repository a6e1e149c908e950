#!/bin/bash
# Round-3 GPU pass: the GPU test suite, the default bench (driver's command line), optionally the
# other BASELINE configs (CONFIGS=1) and the no-tail probe (PROBE=1).
# usage: [CONFIGS=1] [PROBE=1] [TESTS=0] tools/round3_gpu.sh TAG
# Stops after a fault / abort / timeout (exit codes 124, 134, 137, 139): nothing more runs on the GPU.
TAG=${1:-r3a}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) return 0;; esac; return 1; }
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/${TAG}_gputest.log 2>&1
  rc=$?; echo "pytest rc $rc"; tail -3 gpurun_out/${TAG}_gputest.log
  if fatal $rc; then exit $rc; fi
fi
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc $rc"
python -c "import json; b=json.loads(open('gpurun_out/${TAG}_bench.json').read().splitlines()[-1]); print('bench %.2fM' % (b['value']/1e6), 'kernel %.4f ms' % b['roofline']['kernel_ms'], 'frac', b['roofline']['frac'], 'cpu %.2fM' % (b['cpu_baseline']['value']/1e6), 'failed', b['closed_loop']['failed_solves'], b['timing']['region_ms'])" || true
if fatal $rc; then exit $rc; fi
if [ "${CONFIGS:-0}" = "1" ]; then
  : > gpurun_out/${TAG}_configs.jsonl
  for a in "--model force --batch 1024" "--model force --batch 8192 --precision fp32" "--model jerk --batch 4096" "--model force --batch 8192"; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --python-loop-steps 0 $a >> gpurun_out/${TAG}_configs.jsonl 2>> gpurun_out/${TAG}_configs.err
    rc=$?; if [ $rc != 0 ]; then echo "config failed: $a rc $rc"; exit $rc; fi
  done
  python -c "
import json
for l in open('gpurun_out/${TAG}_configs.jsonl'):
    b = json.loads(l); print(b['config']['model'], b['dtype'], b['config']['batch_per_gpu'], '%.3fM' % (b['value'] / 1e6), 'kernel %.4f ms' % b['roofline']['kernel_ms'], 'frac %.4f' % b['roofline']['frac'], 'cpu %.2fM' % (b['cpu_baseline']['value']/1e6), 'failed', b['closed_loop']['failed_solves'])"
fi
if [ "${PROBE:-0}" = "1" ]; then
  for u in 1 7; do
    NMPC_ITER_LOG=1 timeout -k 10 120 python tools/chain_stats.py --model quad13 --batch 8192 --steps 20 --uniform $u > gpurun_out/${TAG}_uniform$u.json 2>&1
    rc=$?; tail -c 400 gpurun_out/${TAG}_uniform$u.json; echo; if fatal $rc; then exit $rc; fi
  done
  NMPC_ITER_LOG=1 timeout -k 10 120 python tools/chain_stats.py --model quad13 --batch 8192 --steps 20 > gpurun_out/${TAG}_chain.json 2>&1
  rc=$?; tail -c 400 gpurun_out/${TAG}_chain.json; echo
fi
exit 0
