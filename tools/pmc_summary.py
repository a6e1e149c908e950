"""Summarise the rocprofv3 PMC passes of tools/pmc.sh for one kernel.

    python tools/pmc_summary.py TAG [--kernel ipm_kernel] [--out profiles/history/r1_pmc_TAG.json]
        [--traffic model,N,batch,precision]

Reads gpurun_out/pmc_<TAG>_<i>/run_counter_collection.csv (one counter group per pass),
averages each counter over the dispatches of the kernel, and writes the per-dispatch means.
With --traffic it also records, in profiles/pmc_traffic.json, the memory-side bytes per
launch that bench.py reports as roofline.traffic:

    traffic = (FETCH_SIZE + WRITE_SIZE) * 1024   [both counters are in KiB]

    traffic = (FETCH_CORR * FETCH_SIZE + WRITE_SIZE) * 1024   [both counters are in KiB]

FETCH_SIZE/WRITE_SIZE count L2 <-> fabric requests, so Infinity-Cache (MALL) hits are
included. MI355X_MICROARCH.md: on gfx950 FETCH_SIZE reports half the bytes of a coalesced
streaming read (calibrated there for 16-B lanes); the same half holds for this engine's 8-B-per-lane
coalesced loads, calibrated on a known byte count — sf_kernel reads x0 + the yref windows, 24.0 MB
per quad13 B = 8192 solve, and FETCH_SIZE reports 12.5 MB (profiles/history/r6j_solve_quad13_sf_pmc.json),
while WRITE_SIZE matches its 23.0 MB of trajectory stores. So FETCH_CORR = 2, WRITE_SIZE as is.

    python tools/pmc_summary.py --rebuild    re-derive every profiles/pmc_traffic.json entry from
                                             its tracked profiles/ source with the correction
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FETCH_CORR = 2.0
TRAFFIC = os.path.join(ROOT, "profiles", "pmc_traffic.json")
NOTE = ("memory-side bytes per solve-kernel launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 from rocprofv3 PMC "
        "passes (tools/pmc_bench.sh, tools/pmc_summary.py; FETCH_SIZE x 2: the gfx950 correction of "
        "MI355X_MICROARCH.md, calibrated for this engine's 8-B coalesced loads on sf_kernel's known read bytes); "
        "includes Infinity-Cache hits; per step = per launch / closed-loop steps per launch; mfma_insts_per_launch "
        "= SQ_INSTS_MFMA; fp64_flops_per_step = 64 x SQ_INSTS_VALU_FLOPS_FP64 per step (executed FP64 flops as "
        "the hardware counts them, idle lanes included)")


def traffic_of(means):
    return (FETCH_CORR * means["FETCH_SIZE"] + means["WRITE_SIZE"]) * 1024.0


def entry(means, model, N, batch, prec, kernel, spl, mode, source):
    t = traffic_of(means)
    return {"model": model, "N": int(N), "batch": int(batch), "precision": prec, "kernel": kernel, "mode": mode,
            "hbm_bytes_per_launch": t, "steps_per_launch": spl, "hbm_bytes_per_step": t / spl,
            "fetch_bytes_raw_per_launch": means["FETCH_SIZE"] * 1024.0,
            "write_bytes_per_launch": means["WRITE_SIZE"] * 1024.0,
            # SQ_INSTS_* count wave-level instructions (x 64 lanes for flops)
            "mfma_insts_per_launch": means.get("SQ_INSTS_MFMA"),
            "fp64_flops_per_step": (64.0 * means["SQ_INSTS_VALU_FLOPS_FP64"] / spl
                                    if "SQ_INSTS_VALU_FLOPS_FP64" in means else None),
            "fp32_flops_per_step": (64.0 * means["SQ_INSTS_VALU_FLOPS_FP32"] / spl
                                    if "SQ_INSTS_VALU_FLOPS_FP32" in means else None),
            # MFMA utilisation inputs: f64 MFMA instructions, the MFMA pipe's busy cycles (summed over SIMDs)
            # and GRBM_GUI_ACTIVE (summed over the 8 XCDs: / 8 = cycles)
            "mfma_f64_insts_per_launch": means.get("SQ_INSTS_VALU_MFMA_F64"),
            "mfma_busy_cycles_per_launch": means.get("SQ_VALU_MFMA_BUSY_CYCLES"),
            "gui_active_per_launch": means.get("GRBM_GUI_ACTIVE"),
            "wait_any_frac": (means["SQ_WAIT_ANY"] / means["SQ_WAVE_CYCLES"]
                              if means.get("SQ_WAVE_CYCLES") and "SQ_WAIT_ANY" in means else None),
            "source": source}


def rebuild():
    d = json.load(open(TRAFFIC))
    out = []
    for e in d["entries"]:
        src = e["source"]
        means = json.load(open(os.path.join(ROOT, src)))["mean_per_dispatch"]
        out.append(entry(means, e["model"], e["N"], e["batch"], e["precision"], e["kernel"], e["steps_per_launch"],
                         e.get("mode", "closed_loop"), src))
    json.dump({"note": NOTE, "entries": out}, open(TRAFFIC, "w"), indent=1)


def collect(tag, kernel):
    vals = defaultdict(lambda: defaultdict(float))   # counter -> dispatch -> value (summed over dims)
    meta = {}
    for f in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", f"pmc_{tag}_*", "*counter_collection.csv"))):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel not in row["Kernel_Name"]:
                    continue
                d = (f, row["Dispatch_Id"])
                vals[row["Counter_Name"]][d] += float(row["Counter_Value"])
                meta = {"kernel": row["Kernel_Name"][:160], "grid": int(row["Grid_Size"]),
                        "workgroup": int(row["Workgroup_Size"]), "vgpr": int(row["VGPR_Count"]),
                        "sgpr": int(row["SGPR_Count"]), "lds_block": int(row["LDS_Block_Size"])}
    means = {c: sum(v.values()) / len(v) for c, v in vals.items() if v}
    ndisp = {c: len(v) for c, v in vals.items()}
    return means, ndisp, meta


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--kernel", default="ipm_kernel")
    ap.add_argument("--out", default=None)
    ap.add_argument("--traffic", default=None, help="model,N,batch,precision")
    ap.add_argument("--steps-per-launch", type=int, default=1,
                    help="closed-loop steps per solve launch (fused closed loop: the bench's --steps)")
    ap.add_argument("--mode", default="closed_loop", help="bench.py --mode of the profiled run")
    ap.add_argument("--rebuild", action="store_true")
    a = ap.parse_args()
    if a.rebuild:
        return rebuild()
    means, ndisp, meta = collect(a.tag, a.kernel)
    if not means:
        raise SystemExit(f"no {a.kernel} dispatches found for tag {a.tag}")
    res = {"tag": a.tag, "kernel": meta, "dispatches_per_counter": ndisp, "mean_per_dispatch": means}
    if "SQ_WAVE_CYCLES" in means and means.get("SQ_WAVES"):
        w = means["SQ_WAVES"]
        res["per_wave"] = {k: v / w for k, v in means.items() if k.startswith("SQ_")}
    if "FETCH_SIZE" in means and "WRITE_SIZE" in means:
        res["traffic_bytes_per_launch"] = traffic_of(means)
    out = a.out or os.path.join(ROOT, "profiles", f"pmc_{a.tag}.json")
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: res[k] for k in res if k != "per_wave"}, indent=1))
    if a.traffic and "traffic_bytes_per_launch" in res:
        model, N, batch, prec = a.traffic.split(",")
        d = json.load(open(TRAFFIC)) if os.path.exists(TRAFFIC) else {"entries": []}
        key = (model, int(N), int(batch), prec, a.kernel, a.steps_per_launch, a.mode)
        d["entries"] = [e for e in d["entries"]
                        if (e["model"], e["N"], e["batch"], e["precision"], e.get("kernel"), e.get("steps_per_launch"),
                            e.get("mode", "closed_loop")) != key]
        d["entries"].append(entry(means, model, N, batch, prec, a.kernel, a.steps_per_launch, a.mode,
                                  os.path.relpath(out, ROOT)))
        d["note"] = NOTE
        with open(TRAFFIC, "w") as fh:
            json.dump(d, fh, indent=1)

if __name__ == "__main__":
    main()
