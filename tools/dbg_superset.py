"""Debug: test_gamg_hierarchy_not_kept_for_a_superset's sequence (a hierarchy
built on a reduced set, then the full set: rebuild) repeated; on a failed
second solve, solve again on the same handle and on a fresh one to tell a
corrupted plan from a transient fault.  argv: reps, graph option."""
import sys

sys.path.insert(0, "mycelium-fea-project_amd")
sys.path.insert(0, "oracle")
sys.path.insert(0, "tests")
import numpy as np  # noqa: E402

import fea_oracle as fo  # noqa: E402
from conftest import load_mesh  # noqa: E402
from mfea import Engine, make_opts, PC_GAMG  # noqa: E402

nodes, elems = load_mesh("sim_20251117_181147")
xyz = nodes[["x", "y", "z"]].values
e2n = elems[["n1", "n2"]].values
top, bot = fo.grip_nodes(xyz, nodes["node_id"].values, 1.5)
dy = fo.DISPLACEMENT_MAX * 20 / (fo.N_STEPS - 1)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
graph = int(sys.argv[2]) if len(sys.argv) > 2 else 1
o = make_opts(rtol=1e-13, max_it=200000, precond=PC_GAMG)
fails = 0
for rep in range(reps):
    eng = Engine(0)
    eng.set_option("graph", graph)
    eng.set_mesh(xyz, e2n)
    eng.set_bc(top, bot)
    active = np.random.default_rng(11).random(len(e2n)) > 0.03
    for k, v in (("amg_reuse", 1), ("amg_rebuild_pct", 100000), ("amg_rebuild_rent", 0)):
        eng.set_option(k, v)
    eng.set_active(active)
    eng.assemble()
    r1 = eng.solve(dy, -dy, o)
    eng.set_active(None)
    eng.assemble()
    try:
        st = eng.solve(dy, -dy, o)
        ok = st.status == 0 and st.iters == 29
    except Exception as ex:  # noqa: BLE001
        ok = False
        print(f"rep {rep}: second solve failed: {ex}; safe_omega {eng.get_option('amg_safe_omega')}", flush=True)
    if not ok:
        fails += 1
        for again in range(3):
            try:
                st = eng.solve(dy, -dy, o)
                print(f"   again {again}: status {st.status} iters {st.iters} rebuilt {st.amg_rebuilt}", flush=True)
            except Exception as ex:  # noqa: BLE001
                print(f"   again {again}: failed {ex}", flush=True)
            eng.assemble()
    eng.close()
print(f"graph {graph}: {fails} failed of {reps}", flush=True)
