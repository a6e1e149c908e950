"""Print a compact summary of tools/clf_phases.py output lines (JSON lines on stdin or a file)."""
import json
import sys

D = ["prologue", "explicit+test", "pdas", "gi", "certificate", "outputs", "plant+cost", "record"]
SHOW = ["prologue", "explicit+test", "pdas", "pdas.load_set", "pdas.solve", "pdas.combo", "pdas.check", "gi", "gi.select",
        "gi.solve", "gi.combo", "gi.hupdate", "certificate", "outputs", "plant+cost", "record"]
for l in open(sys.argv[1]) if len(sys.argv) > 1 else sys.stdin:
    d = json.loads(l)
    print(d["model"], d["batch"], "kms", [round(x, 4) for x in d["kernel_ms_per_step"]], "inst p50/p90/p99/max Mcyc",
          [round(x / 1e6, 2) for x in d["instance_cycles_p50_p90_p99_max"]])
    for k in ("all", "slowest_1pct", "worst"):
        v = d[k]
        tot = sum(v[p] for p in D)
        r, g = max(1, v["pdas_rounds"]), max(1, v["gi_iters"])
        print("  ", k, f"tot={tot / 1e6:.1f}M rounds={v['pdas_rounds']:.0f} gi_it={v['gi_iters']:.0f} slow={v['slow_steps']:.0f}",
              " ".join(f"{p}={v[p] / tot * 100:.1f}%" for p in SHOW if p in v))
        print("      per round:", " ".join(f"{p}={v[p] / r:.0f}" for p in ("pdas", "pdas.load_set", "pdas.solve", "pdas.combo", "pdas.check") if p in v),
              "| per gi it:", " ".join(f"{p}={v[p] / g:.0f}" for p in ("gi", "gi.select", "gi.solve", "gi.combo", "gi.hupdate") if p in v))
