"""Profiling driver for the GAMG-PCG iteration (run under rocprofv3).

Builds the benchmark network, runs one full load step with MFEA_PC_GAMG, then
launches `--reps` iterations in the running state (mfea_profile_iteration:
update + V-cycle + w = A u, all ungated, real stores).  tools/amg_pmc_summary.py
reads the last `reps` iterations out of the trace / counter CSVs.

    rocprofv3 --kernel-trace --stats -d D -o t -- python3 tools/amg_profile.py --config C3_1M
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mycelium-fea-project_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3_1M")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--set", nargs="*", default=[], help="engine options name=value (mfea_set_option)")
    ap.add_argument("--precond", default="gamg", choices=["gamg", "icc", "sor"])
    a = ap.parse_args()
    import fea_solver as fs
    from mfea import PC_GAMG, PC_ICC, PC_SOR, Engine, make_opts, synth
    from mfea.synth import CONFIGS
    nx, ny = CONFIGS[a.config]
    xyz, e2n = synth.tiled_mesh(nx, ny, chords=a.config.startswith("C5"))
    top, bot = synth.grips(xyz)
    eng = Engine(0)
    for kv in a.set:
        k, v = kv.split("=")
        eng.set_option(k, int(v))
    eng.set_material(fs.E_mod, fs.A, fs.I)
    eng.set_mesh(xyz, e2n)
    eng.set_bc(top, bot)
    eng.set_active(None)
    dy = fs.DISPLACEMENT_MAX * 20 / (fs.N_STEPS - 1)
    pc = {"gamg": PC_GAMG, "icc": PC_ICC, "sor": PC_SOR}[a.precond]
    _, _, st = eng.step(dy, -dy, make_opts(rtol=1e-8, max_it=200000, precond=pc), fs.MAX_STRAIN)
    ms = eng.profile_iteration(pc, reps=a.reps)
    print(json.dumps({"config": a.config, "reps": a.reps, "iter_us_hip_events": ms * 1e3,
                      "precond": a.precond, "cg_iters": st.iters, "amg": eng.amg_info()}))
    eng.close()


if __name__ == "__main__":
    main()
