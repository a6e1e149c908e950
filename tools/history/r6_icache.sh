#!/bin/bash
# I-cache counters of the force closed-loop kernel for two builds (default and $LIB)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-ic}
for L in default ${LIB}; do
  if [ "$L" = default ]; then unset NMPC_LIB; else export NMPC_LIB=$PWD/drone-attitude-control_amd/lib/exp/libnmpc_hip_$L.so; fi
  timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $PWD/gpurun_out/${TAG}_$L -o run -- python3 bench.py --steps 20 --warmup 3 --repeats 2 --no-cpu-baseline --python-loop-steps 0 ${BENCH_ARGS} > gpurun_out/${TAG}_$L.log 2>&1 || { tail -5 gpurun_out/${TAG}_$L.log; exit 1; }
  python3 -c "
import csv, collections
v = collections.defaultdict(list)
for r in csv.DictReader(open('gpurun_out/${TAG}_$L/run_counter_collection.csv')):
    if '${KERNEL:-cl_fast_kernel}' in r['Kernel_Name']: v[r['Counter_Name']].append(float(r['Counter_Value']))
print('$L', {k: round(sum(x) / len(x)) for k, x in v.items()})"
done
