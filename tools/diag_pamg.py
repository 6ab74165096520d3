"""Partitioned GAMG iteration counts by partition count / axis (diagnostic)."""
import sys
import numpy as np
sys.path.insert(0, "mycelium-fea-project_amd"); sys.path.insert(0, "tests")
from mfea import Engine, PC_GAMG, make_opts, synth
eng = Engine(0)
for nx, ny in ((4, 5), (6, 8)):
    xyz, e2n = synth.tiled_mesh(nx, ny)
    top, bot = synth.grips(xyz)
    for npart, axis in ((1, -1), (2, 0), (2, 1), (4, 0), (4, 1), (8, 0), (8, 1)):
        eng.set_parts(npart, axis); eng.set_mesh(xyz, e2n); eng.set_bc(top, bot); eng.set_active(None); eng.assemble()
        st = eng.solve(0.01, -0.01, make_opts(rtol=1e-8, max_it=3000, precond=PC_GAMG))
        print(nx, ny, npart, axis, st.iters, flush=True)
