"""Build the in-tree HIP library `lib/libnmpc_hip.so` for gfx950 (MI355X).

Explicit hipcc (no JIT cache, no torch extension): the .so lives in the source tree so it
travels to the GPU box with the repository snapshot.
"""
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "lib", "libnmpc_hip.so")
SOURCES = ["nmpc_ipm.hip", "nmpc_ipm_lpc.hip", "nmpc_ipm_lpi.hip", "nmpc_cond.hip", "nmpc_plant.hip", "nmpc_closed_loop.hip",
           "nmpc_cl_fast.hip", "nmpc_solve_fast.hip", "nmpc_api.cpp", "nmpc_cond_host.cpp"]
HEADERS = ["nmpc_internal.h", "nmpc_lpc_geom.h", "nmpc_cl_device.h", os.path.join("..", "..", "include", "nmpc.h")]
ARCH = os.environ.get("NMPC_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-Wno-unused-result", "-Wno-unused-value",
         f"--offload-arch={ARCH}", "-I", os.path.join(ROOT, "include")]


def sources():
    return [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]


def up_to_date():
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    deps = sources() + [os.path.join(CSRC, h) for h in HEADERS] + [__file__]
    return all(os.path.getmtime(d) <= t for d in deps if os.path.exists(d))


def _compile_link(out, defines=(), verbose=False):
    """One object per source, compiled in parallel (each kernel is launched from its own
    translation unit, so no relocatable device code is needed), then one shared link."""
    from concurrent.futures import ThreadPoolExecutor
    objdir = out + ".objs"
    os.makedirs(objdir, exist_ok=True)
    cflags = [f for f in FLAGS if f != "-shared"] + [f"-D{d}" for d in defines]

    def cc(src):
        obj = os.path.join(objdir, os.path.basename(src) + ".o")
        cmd = ["hipcc", *cflags, "-c", src, "-o", obj]
        if verbose:
            print("[nmpc build]", " ".join(cmd), file=sys.stderr)
        subprocess.check_call(cmd)
        return obj

    jobs = max(1, min(len(sources()), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1))))
    # the longest translation units first
    srcs = sorted(sources(), key=lambda p: -os.path.getsize(p))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(cc, srcs))
    tmp = out + ".tmp"
    subprocess.check_call(["hipcc", f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", tmp])
    os.replace(tmp, out)
    for o in objs:
        os.remove(o)
    os.rmdir(objdir)
    return out


def build(force=False, verbose=True):
    if not force and up_to_date():
        return LIB
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    return _compile_link(LIB, verbose=verbose)


def build_experiment(tag, defines):
    """Tuning aid: the same library compiled with extra -D flags into lib/exp/ (select it at
    run time with NMPC_LIB=<path>)."""
    out = os.path.join(PKG, "lib", "exp", f"libnmpc_hip_{tag}.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    return _compile_link(out, defines)


if __name__ == "__main__":
    build(force="--force" in sys.argv)
    print(LIB)
