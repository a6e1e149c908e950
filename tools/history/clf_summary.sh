# One line per clf_check.py result of a tools/clf_cmd.sh run: python tools/clf_summary.sh TAG
cd "$(dirname "$0")/../gpurun_out" || exit 1
for f in ${1}_*.json; do python - "$f" <<'PY'
import json, sys
f = sys.argv[1]
try:
    d = json.load(open(f))
except Exception:
    sys.exit(0)
if "steps_per_s" not in d:
    sys.exit(0)
m1, m0 = d.get("mode1", {}), d.get("mode0", {})
print(f[:-5], f"{d['steps_per_s'] / 1e6:.2f}M", d.get("launches", [])[:4], "failed", d.get("failed"),
      "m1", m1.get("max_state_err"), m1.get("fail_equal"), "m0", m0.get("max_state_err"), m0.get("fail_equal"))
PY
done
