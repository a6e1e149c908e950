#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for L in default ${LIB}; do
  if [ "$L" = default ]; then unset NMPC_LIB; else export NMPC_LIB=$PWD/drone-attitude-control_amd/lib/exp/libnmpc_hip_$L.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/tr_$L -o run -- python3 bench.py --steps 20 --warmup 3 --repeats 3 --no-cpu-baseline --python-loop-steps 0 $BENCH_ARGS > gpurun_out/tr_$L.json 2> gpurun_out/tr_$L.err || { tail gpurun_out/tr_$L.err; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/tr_$L/run_kernel_stats.csv')): print('$L', r['Name'][:110], r['Calls'], r['AverageNs'])"
done
