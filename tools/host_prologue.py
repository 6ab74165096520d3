"""Host time of a step's prologue (MFEA_BUILD_TIMES laps): from solve_amg's
entry to the setup graph's launch, against the assembly kernel it overlaps."""
import os
import sys

os.environ["MFEA_BUILD_TIMES"] = "1"
sys.path.insert(0, "mycelium-fea-project_amd")
from mfea import Engine, make_opts, synth, PC_GAMG  # noqa: E402
import fea_solver as fs  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C2_100k"
nx, ny = synth.CONFIGS[cfg]
xyz, e2n = synth.tiled_mesh(nx, ny, chords=cfg.startswith("C5"))
top, bot = synth.grips(xyz)
eng = Engine(0)
eng.set_material(fs.E_mod, fs.A, fs.I)
eng.set_mesh(xyz, e2n)
eng.set_bc(top, bot)
eng.set_active(None)
for k in range(1, 13):
    d = 1e-4 * k
    eng.step(d, -d, make_opts(rtol=1e-8, precond=PC_GAMG), 1e9)
    print(f"--- step {k}", file=sys.stderr, flush=True)
eng.close()
