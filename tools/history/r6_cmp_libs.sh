#!/bin/bash
set -o pipefail
for L in default ${LIB}; do
  if [ "$L" = default ]; then unset NMPC_LIB; else export NMPC_LIB=$PWD/drone-attitude-control_amd/lib/exp/libnmpc_hip_$L.so; fi
  for m in "force 8192" "force 1024"; do
    echo -n "$L $m: "; timeout -k 10 120 python tools/r6_cmp_libs.py $m || exit 1
  done
done
