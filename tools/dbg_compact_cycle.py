import os, sys
R = "/root/repo"
for p in (R, os.path.join(R, "mycelium-fea-project_amd"), os.path.join(R, "oracle"), os.path.join(R, "tests")):
    sys.path.insert(0, p)
import numpy as np
import fea_oracle as fo
from conftest import load_mesh
from mfea import Engine
nodes, elems = load_mesh("sim_20251117_181147")
xyz = nodes[["x", "y", "z"]].values
top, bot = fo.grip_nodes(xyz, nodes["node_id"].values, 1.5)
e2n = elems[["n1", "n2"]].values
rng = np.random.default_rng(4)
r = rng.standard_normal((len(xyz), 2))
known = np.zeros(len(xyz), bool); known[top] = known[bot] = True
r[known] = 0
def run(nparts, **opt):
    e = Engine(0)
    e.set_parts(nparts, -1)
    for k, v in opt.items(): e.set_option(k, v)
    e.set_mesh(xyz, e2n); e.set_bc(top, bot); e.set_active(None); e.assemble()
    u = e.amg_vcycle(r)
    info = e.amg_info()
    e.close()
    return u, info
u1, i1 = run(1)
uc, ic = run(2, amg_dist=1, amg_dist_cycle=1)
u4, i4 = run(2, amg_dist=1, amg_dist_cycle=0)
print("levels", i1["levels"], ic["levels"], "rows", i1["rows"], ic["rows"], "n_dist", ic["n_dist"], i4["n_dist"])
for name, u in (("compact", uc), ("fourstep", u4)):
    d = np.abs(u - u1).max(axis=1)
    rel = np.linalg.norm(u - u1) / np.linalg.norm(u1)
    bad = np.argsort(d)[-5:]
    print(name, "rel", rel, "worst nodes", bad, d[bad], "u", u[bad], "u1", u1[bad])
