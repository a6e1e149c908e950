#!/bin/bash
# Finish-policy sweep on the GPU box (tuning aid): chain statistics of the quad13 bench loop and the
# bench line for each NMPC_POLISH_* setting. Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-sweep}
MODEL=${MODEL:-quad13}
for cfg in ${CFGS:-"12:12:0.01" "4:12:0.01" "3:4:0.01" "2:3:0.001"}; do
  IFS=: read first steps drop <<< "$cfg"
  export NMPC_POLISH_FIRST=$first NMPC_POLISH_STEPS=$steps NMPC_POLISH_DROP=$drop
  NMPC_ITER_LOG=1 timeout -k 10 200 python tools/chain_stats.py --model $MODEL ${CHAIN_ARGS:-} >> $OUT/chain_$TAG.jsonl || { echo "chain failed $cfg"; exit 1; }
  timeout -k 10 300 python bench.py --model $MODEL --no-cpu-baseline ${BENCH_ARGS:-} >> $OUT/bench_$TAG.jsonl 2>> $OUT/bench_$TAG.err || { echo "bench failed $cfg"; exit 1; }
  python - "$cfg" <<'PY'
import json, sys
c = [json.loads(l) for l in open("gpurun_out/chain_" + __import__("os").environ.get("TAG", "sweep") + ".jsonl")][-1]
b = [json.loads(l) for l in open("gpurun_out/bench_" + __import__("os").environ.get("TAG", "sweep") + ".jsonl")][-1]
print(sys.argv[1], "value %.3fM" % (b["value"] / 1e6), "kernel %.3f ms" % b["roofline"]["kernel_ms"],
      "wave_chain mean %.1f p99 %.1f max %.1f" % (c["wave_chain_mean"], c["wave_chain_p99"], c["wave_chain_max"]),
      "failed", b["closed_loop"]["failed_solves"], flush=True)
PY
done
