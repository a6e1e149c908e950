"""Per-kernel register / spill / occupancy summary of one HIP source (hipcc
-Rpass-analysis=kernel-resource-usage), e.g. `python tools/resusage.py nmpc_ipm_lpc.hip`."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "drone-attitude-control_amd", "csrc")


def usage(src, defines=()):
    cmd = ["hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-I", os.path.join(ROOT, "include"),
           *[f"-D{d}" for d in defines], "-c", os.path.join(CSRC, src), "-o", "/dev/null",
           "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark:\s+(.*?)\s*\[-Rpass", line)
        if not m:
            continue
        t = m.group(1)
        if t.startswith("Function Name:"):
            cur = {"name": t.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    return rows


def short(name):
    name = re.sub(r"_ZN4nmpc\d*\w*?(\d+)(ipm_\w+?kernel|cond_ipm_kernel|\w+_kernel)I", r"\2<", name)
    name = re.sub(r"ELj\d+", "", name)
    return name[:70]


if __name__ == "__main__":
    for r in usage(sys.argv[1], sys.argv[2:]):
        print(f"{short(r['name']):72s} VGPR {r.get('VGPRs','?'):>4} AGPR {r.get('AGPRs','?'):>4} "
              f"spillV {r.get('VGPRs Spill','?'):>3} spillS {r.get('SGPRs Spill','?'):>4} "
              f"occ {r.get('Occupancy [waves/SIMD]','?')} LDS {r.get('LDS Size [bytes/block]','?')}")
