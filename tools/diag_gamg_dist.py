"""Diagnostic (GPU): one distributed GAMG V-cycle vs the one-partition one on
the same operator (mfea_debug_amg_vcycle), level by level
(mfea_debug_amg_vector, natural row order)."""
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (R, os.path.join(R, "mycelium-fea-project_amd"), os.path.join(R, "oracle"), os.path.join(R, "tests")):
    sys.path.insert(0, p)
import fea_oracle as fo  # noqa: E402
from conftest import load_mesh  # noqa: E402
from mfea import Engine  # noqa: E402

nodes, elems = load_mesh("sim_20251117_181147")
xyz = nodes[["x", "y", "z"]].values
top, bot = fo.grip_nodes(xyz, nodes["node_id"].values, 1.5)
e2n = elems[["n1", "n2"]].values
rng = np.random.default_rng(1)
r = rng.standard_normal((len(xyz), 2))
known = np.zeros(len(xyz), bool)
known[top] = known[bot] = True
r[known] = 0


def run(nparts, **opt):
    e = Engine(0)
    e.set_parts(nparts, -1)
    for k, v in opt.items():
        e.set_option(k, v)
    e.set_mesh(xyz, e2n)
    e.set_bc(top, bot)
    e.set_active(None)
    e.assemble()
    u = e.amg_vcycle(r)
    info = e.amg_info()
    vec = {}
    for l in range(info["levels"]):
        for w in range(7):
            try:
                vec[(l, w)] = e.amg_vector(l, w)
            except Exception as ex:  # noqa: BLE001
                vec[(l, w)] = None
    e.close()
    return u, info, vec


u1, i1, v1 = run(1)
print("1 part", i1["rows"], flush=True)
for nparts, opt in ((2, {"amg_rep_rows": 1 << 30}), (3, {"amg_rep_rows": 0})):
    u, info, v = run(nparts, **opt)
    print(nparts, opt, "rows", info["rows"], "n_dist", info["n_dist"],
          "u rel", float(np.linalg.norm(u - u1) / np.linalg.norm(u1)), flush=True)
    for l in range(info["levels"]):
        for w, name in enumerate(["b", "x", "t", "e", "dinv", "g", "Adiag"]):
            a, b = v1.get((l, w)), v.get((l, w))
            if a is None or b is None:
                continue
            d = np.abs(a - b)
            scale = np.abs(a).max() + 1e-300
            bad = np.flatnonzero(d.max(axis=1) > 1e-3 * scale)
            print(f"  L{l} {name}: max|a| {scale:.3e} max|d| {d.max():.3e} bad rows {len(bad)} {bad[:6]}",
                  flush=True)

# detail: level-0 diagonal blocks vs inv(dinv) on the first mismatching rows
e = Engine(0)
e.set_parts(2, -1)
e.set_option("amg_rep_rows", 1 << 30)
e.set_mesh(xyz, e2n)
e.set_bc(top, bot)
e.set_active(None)
e.assemble()
e.amg_vcycle(r)
Ad, Di = e.amg_vector(0, 6), e.amg_vector(0, 4)
A1, D1 = v1[(0, 6)], v1[(0, 4)]
bad = np.flatnonzero(np.abs(Ad - A1).max(axis=1) > 1e-3 * np.abs(A1).max())
for i in bad[:4]:
    print("row", i, "1p Adiag", A1[i], "dist Adiag", Ad[i], "inv(dinv) dist", np.linalg.inv(Di[i].reshape(2, 2)).ravel())
e.close()
