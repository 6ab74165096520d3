"""Repeat the device floating-row pass (mfea_debug_floating) against SciPy's
connected components on several activities; prints mismatch counts."""
import sys

sys.path.insert(0, "mycelium-fea-project_amd")
sys.path.insert(0, "oracle")
sys.path.insert(0, "tests")
import numpy as np  # noqa: E402
import scipy.sparse as sp  # noqa: E402
from scipy.sparse.csgraph import connected_components  # noqa: E402

import fea_oracle as fo  # noqa: E402
from conftest import load_mesh  # noqa: E402
from mfea import Engine, synth  # noqa: E402


def floating_ref(n, e2n, active, grip):
    a = e2n[active]
    g = sp.coo_matrix((np.ones(len(a)), (a[:, 0], a[:, 1])), shape=(n, n))
    _, lab = connected_components(g, directed=False)
    anchored = np.zeros(lab.max() + 1, bool)
    anchored[lab[grip]] = True
    return ~anchored[lab] & ~grip


reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
nodes, elems = load_mesh("sim_20251117_181147")
cases = [("sim181147", nodes[["x", "y", "z"]].values, elems[["n1", "n2"]].values,
          fo.grip_nodes(nodes[["x", "y", "z"]].values, nodes["node_id"].values, 1.5))]
xyz2, e2n2 = synth.tiled_mesh(1, 5)
cases.append(("C2", xyz2, e2n2, synth.grips(xyz2)))
for name, xyz, e2n, (top, bot) in cases:
    eng = Engine(0)
    eng.set_mesh(xyz, e2n)
    eng.set_bc(top, bot)
    grip = np.zeros(len(xyz), bool)
    grip[np.concatenate([top, bot])] = True
    for frac in (0.0, 0.03, 0.2):
        active = np.random.default_rng(11).random(len(e2n)) >= frac
        ref = floating_ref(len(xyz), np.asarray(e2n), active, grip)
        bad = 0
        for tile in (1024, 512, 2048):
            eng.set_option("cc_tile", tile)
            for _ in range(reps):
                eng.set_active(active)
                fl = eng.floating()
                if not np.array_equal(fl, ref):
                    bad += 1
                    d = np.flatnonzero(fl != ref)
                    print(f"  {name} frac {frac} tile {tile}: {len(d)} nodes differ "
                          f"(device {int(fl[d].sum())} floating / ref {int(ref[d].sum())})", flush=True)
        print(f"{name} frac {frac}: {int(ref.sum())} floating, {bad} mismatches of {3 * reps}", flush=True)
    eng.close()
