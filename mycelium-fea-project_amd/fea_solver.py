"""Drop-in replacement for the reference's ``src/fea_solver.py`` on MI355X.

Same module constants, same functions, same CLI and the same ``fea_results/``
CSV outputs; the hot path (element stiffness, global assembly, Dirichlet
elimination, the linear solve, reactions and the stress/failure update) runs in
libmfea.so's HIP kernels.  Run it exactly like the reference:

    python mycelium-fea-project_amd/fea_solver.py <results_dir> [options]

Differences by design: the direct SuperLU solve
(src/fea_solver.py:128) is replaced by device PCG preconditioned with a
smoothed-aggregation AMG V-cycle (the reference sweep's `-pc_type gamg`; Jacobi
and block Jacobi on request) run to a tight relative residual (default 1e-13 →
displacement within ~1e-10 relative L2 of the direct solution); PNG plotting
(plot_network, py:137-181) is out of scope.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np
import pandas as pd
import scipy.sparse as sp

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from mfea import _capi  # noqa: E402  (fails loudly when libmfea.so is missing)

# ----------------------------------------------------------------------------
# Material & Simulation Parameters — src/fea_solver.py:14-28 (π = 3.14 as there)
# ----------------------------------------------------------------------------
E_mod = 2500
d = 0.0002
t = 0.000001
A = 3.14 * ((d / 2) ** 2 - (d / 2 - t) ** 2)
I = A * 0.001  # noqa: E741  (reference name)
N_STEPS = 40
DISPLACEMENT_MAX = 0.02
MAX_STRAIN = 0.018
MAX_STRESS = E_mod * MAX_STRAIN
GRIP_LENGTH = 1.5

# solver settings of the device PCG (no counterpart in the direct-solve reference)
RTOL = 1e-13
MAX_IT = 200000
PRECOND = _capi.PC_GAMG  # partitioned runs: the distributed V-cycle of one global hierarchy
REG = 1e-12  # src/fea_solver.py:125

_engine = None
_world_joined = False


def get_engine(device: int | None = None) -> _capi.Engine:
    """Process-wide device handle (device = LOCAL_RANK or 0)."""
    global _engine
    if _engine is None:
        dev = int(os.environ.get("LOCAL_RANK", "0")) if device is None else device
        _engine = _capi.Engine(dev)
    return _engine


def dist_env():
    """(rank, world) of a multi-process launch — ``python -m torch.distributed.run
    --nproc-per-node N fea_solver.py <dir>``, one process per GPU, as the
    reference's ``mpirun -np N fea_petsc_parallel.exe <dir>`` (README.md:18;
    rank/size src/fea_petsc_parallel.cpp:169-171) — else (0, 1)."""
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))


def _join_world(eng, rank, world):
    """Joins this process's handle to the RCCL world: rank 0 makes the
    communicator id, torch.distributed (gloo, launcher plumbing only) carries
    it to the other ranks.  Once per process."""
    global _world_joined
    if _world_joined:
        return
    import torch.distributed as dist
    if not dist.is_initialized():
        dist.init_process_group("gloo")
    obj = [_capi.dist_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    eng.dist_init(rank, world, obj[0])
    _world_joined = True


def gather_records(node_owned, elem_owned, U, stress, active, rank, world):
    """One step's records of the whole mesh on rank 0: every node's U from the
    rank owning the node, every element's stress / activity from the rank
    owning it (its first node's).  The values travel as they are (a -0.0
    displacement stays -0.0 in the CSV, which a sum-reduction would not keep).
    Replaces the reference's VecScatterCreateToZero + MPI_Bcast of U
    (src/fea_petsc_parallel.cpp:373-391); returns None on the other ranks."""
    import torch.distributed as dist
    U3 = np.asarray(U).reshape(-1, 3)
    payload = (np.flatnonzero(node_owned), U3[node_owned], np.flatnonzero(elem_owned),
               np.asarray(stress)[elem_owned], np.asarray(active)[elem_owned])
    out = [None] * world if rank == 0 else None
    dist.gather_object(payload, out, dst=0)
    if rank != 0:
        return None
    Ug, Sg, Ag = np.zeros_like(U3), np.zeros(len(stress)), np.ones(len(active), dtype=bool)
    seen_n, seen_e = np.zeros(len(U3), bool), np.zeros(len(stress), bool)
    for ni, uv, ei, sv, av in out:
        Ug[ni], Sg[ei], Ag[ei] = uv, sv, av
        seen_n[ni] = True
        seen_e[ei] = True
    if not (seen_n.all() and seen_e.all()):
        raise RuntimeError("record gather: a node or element is owned by no rank")
    return Ug.reshape(-1), Sg, Ag


def _opts(rtol=None, max_it=None, precond=None):
    return _capi.make_opts(rtol=RTOL if rtol is None else rtol,
                           max_it=MAX_IT if max_it is None else max_it,
                           precond=PRECOND if precond is None else precond, reg=REG)


def bar_stiffness_bulk(p1s, p2s, E=E_mod, A=A, I=I):  # noqa: E741
    """Element stiffness (N,6,6) and length (N,), src/fea_solver.py:30-68, on device."""
    return get_engine().element_stiffness(p1s, p2s, E, A, I)


def _elem_array(elems):
    if isinstance(elems, pd.DataFrame):
        return elems[["n1", "n2"]].values.astype(np.int64)
    return np.asarray(elems, dtype=np.int64).reshape(-1, 2)


def assemble_global_stiffness(coords, elems, active):
    """Global K as scipy CSR (3N×3N), src/fea_solver.py:74-106, assembled on device.

    Same sparsity pattern as the reference's csr_matrix (explicit zeros kept,
    duplicates summed in element order)."""
    coords = np.asarray(coords, dtype=np.float64)
    e2n = _elem_array(elems)
    eng = _capi.Engine(get_engine_device())
    try:
        eng.set_material(E_mod, A, I)
        eng.set_mesh(coords, e2n)
        eng.set_bc(np.zeros(0, np.int64), np.zeros(0, np.int64))
        eng.set_active(np.asarray(active, dtype=bool))
        eng.assemble()
        indptr, indices, data = eng.export_csr()
    finally:
        eng.close()
    n = 3 * coords.shape[0]
    return sp.csr_matrix((data, indices, indptr), shape=(n, n))


def get_engine_device():
    return int(os.environ.get("LOCAL_RANK", "0"))


def solve_system(K, known_dofs, known_vals):
    """Dirichlet elimination + solve of an arbitrary K, src/fea_solver.py:112-135.

    K_ff + 1e-12·I solved by device Jacobi-PCG (rtol RTOL); raises
    np.linalg.LinAlgError (a SolverFailure) if it does not converge."""
    K = sp.csr_matrix(K)
    U, _ = get_engine().solve_csr(K.indptr, K.indices, K.data, known_dofs, known_vals,
                                  _opts(precond=_capi.PC_JACOBI))
    return U


def _grips(nodes, coords, tol):
    """src/fea_solver.py:207-210."""
    y_min, y_max = coords[:, 1].min(), coords[:, 1].max()
    top = nodes.loc[np.abs(nodes["y"] - y_max) < tol, "node_id"].values.astype(int)
    bot = nodes.loc[np.abs(nodes["y"] - y_min) < tol, "node_id"].values.astype(int)
    return top, bot


def fea_solver(results_dir, tol=GRIP_LENGTH, *, rtol=None, max_it=None, precond=None,
               out_format="python", verbose=True, nparts=1, npy=False):
    """The reference step loop (src/fea_solver.py:186-335) with the hot path on device.

    Reads <results_dir>/nodes.csv + elements.csv, runs N_STEPS load steps and
    writes <results_dir>/fea_results/{stress_record,active_elements,
    node_displacements,force_displacement}.csv, runtime.txt and
    solve_runtime.txt.  Module constants are read at call time, as in the
    reference.  out_format='petsc' writes the fea_petsc.cpp formatting instead
    (src/fea_petsc.cpp:433-516).  npy=True also writes every record as a .npy
    sidecar next to its CSV (the raw per-step array, no step column).

    Multi-GPU: launched as N processes (``torch.distributed.run``, dist_env),
    every rank solves its partition of the mesh (RCCL between the GPUs) and
    rank 0 alone gathers the records and writes the files — the reference's
    MPI variant has every rank write the same files (src/fea_petsc_parallel.cpp:
    491-574).  nparts > 1 in ONE process runs that partitioned solve with its
    partitions all on this device (mfea_debug_set_parts)."""
    start_time = time.time()
    rank, world = dist_env()
    say = print if verbose and rank == 0 else (lambda *a, **k: None)
    say(f"🔧 Running FEA on geometry from {results_dir}")
    fea_dir = os.path.join(results_dir, "fea_results")
    if rank == 0:
        os.makedirs(fea_dir, exist_ok=True)
    nodes = pd.read_csv(os.path.join(results_dir, "nodes.csv"))
    elems = pd.read_csv(os.path.join(results_dir, "elements.csv"))
    coords = nodes[["x", "y", "z"]].values
    n_nodes = len(nodes)
    n_elems = len(elems)
    e2n = _elem_array(elems)
    if n_elems and (e2n.min() < 0 or e2n.max() >= n_nodes):
        # the reference fails here with an IndexError from coords[...] (py:82-83)
        raise IndexError("elements.csv references a node id outside nodes.csv")

    top, bot = _grips(nodes, coords, tol)
    say(f"Top nodes: {len(top)}, Bottom nodes: {len(bot)}")

    eng = get_engine()
    if world > 1:
        _join_world(eng, rank, world)
    else:
        eng.set_parts(nparts)
    eng.set_material(E_mod, A, I)
    eng.set_mesh(coords, e2n)
    eng.set_bc(top, bot)
    eng.set_active(None)
    opts = _opts(rtol, max_it, precond)
    node_owned, elem_owned = eng.ownership() if world > 1 else (None, None)

    stress_record, active_record, disp_record, force_disp_curve, solve_times = [], [], [], [], []
    if rank == 0:
        with open(os.path.join(fea_dir, "solve_runtime.txt"), "w") as f:
            f.write("step, runtime_s\n")
    for step in range(N_STEPS):
        disp_factor = step / (N_STEPS - 1)
        dy_top = +DISPLACEMENT_MAX * disp_factor
        dy_bot = -DISPLACEMENT_MAX * disp_factor
        say(f"➡️  Step {step+1}/{N_STEPS} | dy_top={dy_top:.3f}, dy_bot={dy_bot:.3f}")
        t0 = time.time()
        try:
            total_force, n_active, st = eng.step(dy_top, dy_bot, opts, MAX_STRAIN)
        except np.linalg.LinAlgError:
            say(f"❌ Singular matrix at step {step+1}. Saving partial results and stopping.")
            break
        t1 = time.time()
        solve_times.append(t1 - t0)
        if world > 1:
            rec = gather_records(node_owned, elem_owned, eng.displacement(), eng.stress(), eng.active(),
                                 rank, world)
        else:
            rec = (eng.displacement(), eng.stress(), eng.active())
        if rank == 0:
            with open(os.path.join(fea_dir, "solve_runtime.txt"), "a") as f:
                f.write(f"{step+1}, {t1 - t0:.6f}\n")
            force_disp_curve.append([dy_top - dy_bot, total_force])
            disp_record.append(rec[0])
            stress_record.append(rec[1])
            active_record.append(rec[2])
        if n_active == 0:
            say(f"⚠️  Simulation stopped early at step {step+1}.")
            break

    if rank == 0:
        write_records(fea_dir, n_nodes, n_elems, stress_record, active_record, disp_record,
                      force_disp_curve, out_format, npy=npy)
        say(f"✅ FEA completed. Results saved to {fea_dir}")
        total_time = time.time() - start_time
        with open(os.path.join(fea_dir, "runtime.txt"), "w") as f:
            f.write(f"Total FEA runtime: {total_time:.6f} seconds\n")
        say(f"⏱️ Total runtime: {total_time:.3f} seconds")
    return {"force": np.asarray(force_disp_curve), "stress": np.asarray(stress_record),
            "active": np.asarray(active_record), "U": np.asarray(disp_record)}


def write_records(fea_dir, n_nodes, n_elems, stress_record, active_record, disp_record,
                  force_disp_curve, out_format="python", npy=False):
    """CSV writers, src/fea_solver.py:297-316 (pandas) / src/fea_petsc.cpp:433-516,
    through the native multi-threaded writer (mfea_write_record_csv), which
    reproduces both byte for byte.  The C++ driver writes a record file only
    when it holds at least one step (src/fea_petsc.cpp:435, 457, 477, 508)."""
    petsc = out_format == "petsc"
    style = _capi.CSV_PETSC if petsc else _capi.CSV_PANDAS
    files = (("stress_record.csv", _capi.REC_STRESS, stress_record, n_elems),
             ("active_elements.csv", _capi.REC_ACTIVE, active_record, n_elems),
             ("node_displacements.csv", _capi.REC_DISP, disp_record, 3 * n_nodes),
             ("force_displacement.csv", _capi.REC_FORCE, force_disp_curve, 2))
    for name, kind, rec, ncol in files:
        if petsc and not len(rec):
            continue
        _capi.write_record_csv(os.path.join(fea_dir, name), style, kind, rec, n_cols=ncol)
        if npy:
            _capi.write_record_npy(os.path.join(fea_dir, name[:-4] + ".npy"), kind, rec, n_cols=ncol)


def main(argv=None):
    global N_STEPS, DISPLACEMENT_MAX, MAX_STRAIN, REG
    ap = argparse.ArgumentParser(description="MI355X FEA (drop-in for src/fea_solver.py)")
    ap.add_argument("results_dir")
    ap.add_argument("--grip-length", type=float, default=GRIP_LENGTH)
    ap.add_argument("--disp-max", type=float, default=DISPLACEMENT_MAX)
    ap.add_argument("--n-steps", type=int, default=N_STEPS)
    ap.add_argument("--max-strain", type=float, default=MAX_STRAIN)
    ap.add_argument("--rtol", type=float, default=RTOL)
    ap.add_argument("--max-it", type=int, default=MAX_IT)
    ap.add_argument("--reg", type=float, default=REG)
    ap.add_argument("--pc", choices=["gamg", "jacobi", "bjacobi", "sor", "icc"], default="gamg")
    ap.add_argument("--format", choices=["python", "petsc"], default="python")
    ap.add_argument("--npy", action="store_true", help="also write each record as a .npy sidecar")
    ap.add_argument("--parts", type=int, default=1,
                    help="partitions of the multi-GPU solve, all on this device (one process); "
                         "for one GPU per process launch with torch.distributed.run instead")
    a = ap.parse_args(argv)
    N_STEPS, DISPLACEMENT_MAX, MAX_STRAIN, REG = a.n_steps, a.disp_max, a.max_strain, a.reg
    fea_solver(a.results_dir, tol=a.grip_length, rtol=a.rtol, max_it=a.max_it,
               precond={"gamg": _capi.PC_GAMG, "jacobi": _capi.PC_JACOBI,
                        "bjacobi": _capi.PC_BLOCK_JACOBI, "sor": _capi.PC_SOR, "icc": _capi.PC_ICC}[a.pc],
               out_format=a.format, nparts=a.parts, npy=a.npy)


if __name__ == "__main__":
    if len(sys.argv) < 2:
        print("Usage: python fea_solver.py <results_dir>")
        sys.exit(0)
    main()
