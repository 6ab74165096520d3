"""Same-box A/B of two libmfea.so builds on the benchmark networks.

Each library runs in its own child process (MFEA_LIB=...), alternated over
`--rounds` so box drift hits both alike.  A child builds the mesh once, takes a
warm step, then `--steps` timed steps (device times from mfea_stats, host wall
time), the GAMG iteration time (mfea_profile_iteration) and a hash of U.

    python tools/lib_ab.py --libs abso/libmfea_head.so mycelium-fea-project_amd/libmfea.so
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(cfg, steps):
    sys.path.insert(0, os.path.join(REPO, "mycelium-fea-project_amd"))
    import numpy as np

    import fea_solver as fs
    from mfea import PC_GAMG, Engine, make_opts, synth
    from mfea.synth import CONFIGS
    dy = fs.DISPLACEMENT_MAX * 20 / (fs.N_STEPS - 1)
    opts = make_opts(rtol=1e-8, max_it=2000, precond=PC_GAMG)
    nx, ny = CONFIGS[cfg]
    xyz, e2n = synth.tiled_mesh(nx, ny, chords=cfg.startswith("C5"))
    top, bot = synth.grips(xyz)
    eng = Engine(0)
    eng.set_option("phase_times", 1)  # (the t_*_ms phase split)
    eng.set_material(fs.E_mod, fs.A, fs.I)
    eng.set_mesh(xyz, e2n)
    eng.set_bc(top, bot)
    eng.set_active(None)
    eng.step(dy, -dy, opts, fs.MAX_STRAIN)
    dev, wall, post = [], [], []
    for _ in range(steps):
        eng.set_active(None)
        t = time.perf_counter()
        f, _, st = eng.step(dy, -dy, opts, fs.MAX_STRAIN)
        wall.append(1e3 * (time.perf_counter() - t))
        dev.append(st.t_assemble_ms + st.t_rhs_ms + st.t_solve_ms + st.t_post_ms)
        post.append(st.t_post_ms)
    it_us = 1e3 * eng.profile_iteration(PC_GAMG, reps=30)
    spmv_us = 1e3 * eng.profile_spmv(reps=100)
    U = eng.displacement()
    print(json.dumps({"iters": st.iters, "relres": st.relres, "setup_ms": st.t_setup_ms,
                      "dev_ms_med": float(np.median(dev)), "wall_ms_med": float(np.median(wall)),
                      "post_ms_med": float(np.median(post)), "force": float(f),
                      "iter_us": round(it_us, 2), "spmv_us": round(spmv_us, 2),
                      "U_md5": hashlib.md5(np.ascontiguousarray(U).tobytes()).hexdigest()[:12]}))
    eng.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", nargs="+", required=True)
    ap.add_argument("--configs", nargs="+", default=["C3_1M"])
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--child", default=None)
    a = ap.parse_args()
    if a.child:
        child(a.child, a.steps)
        return
    for cfg in a.configs:
        for rnd in range(a.rounds):
            for lib in a.libs:
                env = dict(os.environ, MFEA_LIB=os.path.abspath(lib))
                out = subprocess.run([sys.executable, __file__, "--libs", lib, "--child", cfg,
                                      "--steps", str(a.steps)], env=env, capture_output=True,
                                     text=True, timeout=300)
                if out.returncode != 0:
                    print(json.dumps({"config": cfg, "lib": lib, "rc": out.returncode,
                                      "err": out.stderr[-2000:]}), flush=True)
                    sys.exit(out.returncode)
                r = json.loads(out.stdout.strip().splitlines()[-1])
                print(json.dumps({"config": cfg, "round": rnd, "lib": os.path.basename(lib), **r}),
                      flush=True)


if __name__ == "__main__":
    main()
