import os, sys, numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
os.environ["NMPC_ITER_LOG"] = "1"
from drone_attitude_control_amd.batched import ClosedLoop
from drone_attitude_control_amd import sharding
def run(kernel, B=4096, seqs=(2, 4, 4)):
    os.environ["NMPC_KERNEL"] = kernel
    cl = ClosedLoop("force", B, N=20, seed=42)
    logs = []
    for s in seqs:
        cl.run(s)
        f, i, st = cl.iter_log()
        logs.append(np.stack([f, i, st], -1))
    return cl.state(), cl.instance_stats(), np.concatenate(logs, 0)
xs, a, la = run("wave")
xf, b, lb = run("lpc")
d = np.abs(xf - xs).max(axis=1)
dc = np.abs(a[:, 0] - b[:, 0])
w = np.argsort(-dc)[:3]
print("state max", d.max(), "cost diff max", dc.max(), "worst", w.tolist(), dc[w].tolist())
for i in w:
    print(i, "wave", la[:, i].tolist())
    print(i, "lpc ", lb[:, i].tolist())
print("inst0 wave", la[:, 0].tolist())
print("inst0 lpc ", lb[:, 0].tolist())
