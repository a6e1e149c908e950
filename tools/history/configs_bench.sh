#!/bin/bash
# The BASELINE.json configurations other than the headline one, one bench line each
# (configs[1] force B=1024 fp64, configs[2] force B=8192 fp32, configs[4] jerk N=40 B=4096 fp64),
# plus the headline quad13 line. Output: gpurun_out/configs_$TAG.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
TAG=${TAG:-cfg}
: > $OUT/configs_$TAG.jsonl
run() {
  timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 "$@" >> $OUT/configs_$TAG.jsonl 2>> $OUT/configs_$TAG.err || { echo "bench $* failed"; tail -20 $OUT/configs_$TAG.err; exit 1; }
}
run --model force --batch 1024 --precision fp64
run --model force --batch 8192 --precision fp32
run --model jerk --horizon 40 --batch 4096 --precision fp64
run --model quad13 --batch 8192 --precision fp64
python - <<PY
import json
for l in open("$OUT/configs_$TAG.jsonl"):
    d = json.loads(l); c = d["config"]
    print(c["model"], "N=%d" % c["horizon_N"], "B=%d" % c["batch_per_gpu"], d["dtype"], "%.0f steps/s" % d["value"],
          "kernel %.3f ms" % d["roofline"]["kernel_ms"], "frac %.3f" % d["roofline"]["frac"],
          "cpu %.0f" % (d["cpu_baseline"] or {}).get("value", 0), (d["roofline"]["kernel"]))
PY
