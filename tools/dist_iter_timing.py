"""Partitioned GAMG on ONE GPU (mfea_debug_set_parts): per form (option
amg_dist 1 the global hierarchy split over the partitions, 0 block Jacobi
over per-partition hierarchies) and partition count, the step time, its
setup and solve phases and the iteration count, against one partition.

    python3 tools/dist_iter_timing.py [C3_1M|C2_100k|grown] [parts,...]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "mycelium-fea-project_amd"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402

import fea_solver as fs  # noqa: E402
from mfea import PC_GAMG, Engine, make_opts, synth  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3_1M"
parts = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 2, 4]
forms = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [1, 0]
cycle = int(sys.argv[4]) if len(sys.argv) > 4 else 1  # option amg_dist_cycle (1 compact, 0 four-step)
if cfg == "grown":
    from conftest import load_mesh
    import fea_oracle as fo
    nodes, elems = load_mesh("sim_20251117_181147")
    xyz = nodes[["x", "y", "z"]].values
    top, bot = fo.grip_nodes(xyz, nodes["node_id"].values, 1.5)
    e2n = elems[["n1", "n2"]].values
else:
    nx, ny = synth.CONFIGS[cfg]
    xyz, e2n = synth.tiled_mesh(nx, ny, chords=cfg.startswith("C5"))
    top, bot = synth.grips(xyz)
dy = fs.DISPLACEMENT_MAX * 20 / (fs.N_STEPS - 1)
opts = make_opts(rtol=1e-8, max_it=5000, precond=PC_GAMG)
for n in parts:
    for form in (forms if n > 1 else [1]):
        e = Engine(0)
        e.set_parts(n, -1)
        e.set_option("amg_dist", form)
        e.set_option("amg_dist_cycle", cycle)
        e.set_material(fs.E_mod, fs.A, fs.I)
        e.set_mesh(xyz, e2n)
        e.set_bc(top, bot)
        e.set_active(None)
        for _ in range(3):
            e.step(dy, -dy, opts, fs.MAX_STRAIN)
        e.set_option("phase_times", 1)
        res = []
        for _ in range(5):
            _, _, st = e.step(dy, -dy, opts, fs.MAX_STRAIN)
            res.append((st.t_assemble_ms + st.t_rhs_ms + st.t_solve_ms + st.t_post_ms, st.t_setup_ms,
                        st.t_solve_ms, st.iters))
        r = np.median(np.array(res), axis=0)
        it = r[3]
        print(f"{cfg} parts {n} form {('global' + ('' if cycle else ' four-step')) if form == 1 else 'bjacobi'}: step {r[0]:.3f} ms, setup {r[1]:.3f}, "
              f"solve {r[2]:.3f} ms, {int(it)} its, {(r[2] - r[1]) / max(it + 1, 1) * 1e3:.1f} us/iteration",
              flush=True)
        e.close()
