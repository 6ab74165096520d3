"""C5 solves at rtol 1e-13 (tests/test_gpu_configs.py's C5 case), one line per
solve: iterations, status, wall time — for a GAMG option sweep.

    python tools/c5_probe.py [--parts N] [--set name=value ...]
"""
import argparse
import json
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mycelium-fea-project_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--parts", type=int, default=1)
    ap.add_argument("--set", nargs="*", default=[])
    ap.add_argument("--rtol", type=float, default=1e-13)
    a = ap.parse_args()
    import fea_solver as fs
    from mfea import PC_GAMG, Engine, make_opts, synth
    xyz, e2n = synth.tiled_mesh(20, 23, chords=True)
    top, bot = synth.grips(xyz)
    dy = fs.DISPLACEMENT_MAX * 20 / (fs.N_STEPS - 1)
    eng = Engine(0)
    for kv in a.set:
        k, v = kv.split("=")
        eng.set_option(k, float(v))
    eng.set_material(fs.E_mod, fs.A, fs.I)
    eng.set_parts(a.parts, -1)
    eng.set_mesh(xyz, e2n)
    eng.set_bc(top, bot)
    eng.set_active(None)
    eng.assemble()
    opts = make_opts(rtol=a.rtol, max_it=2000, precond=PC_GAMG)
    for f in (1, 2, 1):
        t = time.perf_counter()
        st = eng.solve(f * dy, -f * dy, opts)
        print(json.dumps({"f": f, "iters": st.iters, "status": st.status, "relres": st.relres,
                          "ms": round(1e3 * (time.perf_counter() - t), 1),
                          "collapse_level": eng.get_option("amg_collapse_level")}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
