"""Generate the golden fixtures under tests/golden/ — run ONLY in the build container.

Imports the reference Python (``/root/reference/src/fea_solver_no_plotting.py``,
identical numerics to ``src/fea_solver.py``) with bytecode writing disabled,
runs its own ``fea_solver`` on temp copies of reference meshes and packs the
outputs as small ``.npz`` vectors.  The reference source never leaves this
container; only data (meshes, expected outputs) is committed.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Outputs (all under tests/golden/):
  meshes/<name>/{nodes,elements}.csv       copies of reference meshes (data)
  ref/<name>/*.csv                          the reference's own committed goldens
  gen_<name>_<params>.npz                   vectors produced by the reference here
  sys_sim_20251117_181147_step20.npz        K_ff system + direct U_f + PCG counts
"""
from __future__ import annotations

import contextlib
import io
import os
import shutil
import sys
import tempfile

import numpy as np
import pandas as pd

sys.dont_write_bytecode = True
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def rd(path):
    return pd.read_csv(path, float_precision="round_trip")


def copy_mesh(name):
    dst = os.path.join(HERE, "meshes", name)
    os.makedirs(dst, exist_ok=True)
    for f in ("nodes.csv", "elements.csv"):
        shutil.copy(os.path.join(REF, "results", name, f), dst)


def copy_ref_outputs(name, files):
    dst = os.path.join(HERE, "ref", name)
    os.makedirs(dst, exist_ok=True)
    for f in files:
        shutil.copy(os.path.join(REF, "results", name, "fea_results", f), dst)


def run_reference(mod, mesh, n_steps, dmax, grip):
    """Run the reference fea_solver on a temp copy; return its CSV outputs."""
    mod.N_STEPS = n_steps
    mod.DISPLACEMENT_MAX = dmax
    with tempfile.TemporaryDirectory() as td:
        for f in ("nodes.csv", "elements.csv"):
            shutil.copy(os.path.join(REF, "results", mesh, f), td)
        with contextlib.redirect_stdout(io.StringIO()):
            mod.fea_solver(td, tol=grip)
        fr = os.path.join(td, "fea_results")
        out = {
            "force": rd(os.path.join(fr, "force_displacement.csv")).values,
            "stress": rd(os.path.join(fr, "stress_record.csv")).values[:, :-1].astype(np.float64),
            "active": rd(os.path.join(fr, "active_elements.csv")).values[:, :-1].astype(bool),
            "U": rd(os.path.join(fr, "node_displacements.csv")).values[:, :-1].astype(np.float64),
        }
    return out


def main():
    sys.path.insert(0, os.path.join(REF, "src"))
    import fea_solver_no_plotting as ref  # noqa: E402  (reference, never copied)

    defaults = (ref.N_STEPS, ref.DISPLACEMENT_MAX)

    # 1. tiny hand-made meshes + their committed goldens (data files of the reference)
    for name in ("test_I", "test_X", "test_y", "test_t", "test_X_cpp_2", "test_I_cpp", "test_X_cpp"):
        copy_mesh(name)
    for name in ("test_I", "test_X", "test_y"):
        copy_ref_outputs(name, ["force_displacement.csv", "stress_record.csv",
                                "active_elements.csv", "node_displacements.csv"])
    for name in ("test_I_cpp", "test_X_cpp"):
        copy_ref_outputs(name, ["force_displacement.csv", "stress_record.csv",
                                "active_elements.csv", "node_displacements.csv"])

    # 2. real meshes (data)
    for name in ("sim_20251117_181147", "sim_20251117_175809", "sim_20251115_135507"):
        copy_mesh(name)
    copy_ref_outputs("sim_20251117_181147", ["force_displacement.csv"])
    act = rd(os.path.join(REF, "results/sim_20251117_181147/fea_results/active_elements.csv"))
    np.savez_compressed(os.path.join(HERE, "ref", "sim_20251117_181147", "active_packed.npz"),
                        bits=np.packbits(act.values[:, :-1].astype(bool), axis=1),
                        n_elems=act.shape[1] - 1, steps=act["step"].values)

    # 3. vectors produced by the reference here
    jobs = [
        ("test_X", 40, 0.06, 0.5, "golden"),
        ("test_X", 40, 0.02, 1.5, "default"),
        ("test_I", 40, 0.06, 0.5, "golden"),
        ("sim_20251115_135507", 40, 0.02, 0.5, "grip05"),     # 3D mesh (z != 0)
        ("sim_20251117_175809", 40, 0.02, 1.5, "default"),
    ]
    for mesh, ns, dmax, grip, tag in jobs:
        out = run_reference(ref, mesh, ns, dmax, grip)
        nrun = len(out["force"])
        steps_keep = sorted(set([min(1, nrun - 1), nrun // 2, nrun - 1]))
        np.savez_compressed(
            os.path.join(HERE, f"gen_{mesh}_{tag}.npz"),
            n_steps=ns, dmax=dmax, grip=grip,
            force=out["force"], active=np.packbits(out["active"], axis=1), n_elems=out["active"].shape[1],
            stress=out["stress"], U_steps=np.array(steps_keep), U=out["U"][steps_keep])
        print("wrote", mesh, tag, out["force"].shape)

    ref.N_STEPS, ref.DISPLACEMENT_MAX = defaults

    # 4. assembled K at step 0 (all active) to pin assembly.  Meshes are parsed
    # exactly as the reference parses them (pd.read_csv defaults, py:193-194).
    for mesh in ("test_X", "sim_20251117_175809", "sim_20251115_135507"):
        n = pd.read_csv(os.path.join(REF, "results", mesh, "nodes.csv"))
        e = pd.read_csv(os.path.join(REF, "results", mesh, "elements.csv"))
        K = ref.assemble_global_stiffness(n[["x", "y", "z"]].values, e, np.ones(len(e), bool))
        np.savez_compressed(os.path.join(HERE, f"K0_{mesh}.npz"), indptr=K.indptr,
                            indices=K.indices, data=K.data, shape=np.array(K.shape))
        print("K0", mesh, K.nnz)

    # 5. the step-20 linear system of the 22k-DOF mesh (solve parity + iteration counts)
    mesh = "sim_20251117_181147"
    n = pd.read_csv(os.path.join(REF, "results", mesh, "nodes.csv"))
    e = pd.read_csv(os.path.join(REF, "results", mesh, "elements.csv"))
    coords = n[["x", "y", "z"]].values
    K = ref.assemble_global_stiffness(coords, e, np.ones(len(e), bool))
    y = coords[:, 1]
    top = n.loc[np.abs(n["y"] - y.max()) < ref.GRIP_LENGTH, "node_id"].values.astype(int)
    bot = n.loc[np.abs(n["y"] - y.min()) < ref.GRIP_LENGTH, "node_id"].values.astype(int)
    dy = ref.DISPLACEMENT_MAX * 20 / (ref.N_STEPS - 1)
    dd = {}
    for t in top:
        dd.update({3 * t: 0.0, 3 * t + 1: dy, 3 * t + 2: 0.0})
    for b in bot:
        dd.update({3 * b: 0.0, 3 * b + 1: -dy, 3 * b + 2: 0.0})
    known = np.array(list(dd.keys()))
    vals = np.array([dd[k] for k in known])
    U = ref.solve_system(K, known, vals)
    free = np.setdiff1d(np.arange(K.shape[0]), known)
    from scipy.sparse import identity
    from scipy.sparse.linalg import cg
    K_ff = K[free][:, free].tocsr() + 1e-12 * identity(len(free), format="csr")
    b = np.zeros(K.shape[0])[free] - K[free][:, known] @ vals
    Dinv = 1.0 / K_ff.diagonal()
    counts = {}
    for rt in (1e-8, 1e-12):
        it = [0]
        cg(K_ff, b, rtol=rt, atol=0.0, maxiter=100000, M=identity(len(free)).multiply(Dinv).tocsr(),
           callback=lambda xk: it.__setitem__(0, it[0] + 1))
        counts[rt] = it[0]
    np.savez_compressed(os.path.join(HERE, f"sys_{mesh}_step20.npz"), dy=dy, known=known, vals=vals,
                        b_f=b, U=U, free=free, pcg_iters_1e8=counts[1e-8], pcg_iters_1e12=counts[1e-12])
    print("system", mesh, counts)


if __name__ == "__main__":
    main()
