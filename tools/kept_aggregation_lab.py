"""Lab (CPU, SciPy): which part of a GAMG hierarchy kept over element
failures costs the extra iterations?  SciPy smoothed aggregation as
tools/sa_nullspace_lab.py (translations, damped block-Jacobi V(1,1), PCG to
1e-8) on a chord network pulled until elements fail (bench.py's
full_run_failures recipe), on the set after the first failures, with:
  kept-all     every level's aggregation from the intact network (the engine)
  kept-0       level 0's aggregation from the intact network, coarser levels fresh
  split-0      level 0's intact aggregates split into their connected pieces
               on the failed network, coarser levels fresh
  split-all    as kept-all, but every level's aggregates split into pieces
  fresh        every level aggregated on the failed network (a rebuild)

    python3 tools/kept_aggregation_lab.py [nx ny] [step]
"""
import os
import sys

import numpy as np
import scipy.sparse as sp
from scipy.sparse.csgraph import connected_components

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tools"), os.path.join(REPO, "mycelium-fea-project_amd"),
                os.path.join(REPO, "oracle")]
import fea_oracle as fo  # noqa: E402
from mfea import synth  # noqa: E402
from sa_nullspace_lab import aggregate, block_diag_inv, fit, pcg, vcycle  # noqa: E402


def node_graph(A, nd):
    n = A.shape[0] // nd
    c = A.tocoo()
    m = c.data != 0
    G = sp.csr_matrix((np.ones(m.sum()), (c.row[m] // nd, c.col[m] // nd)), shape=(n, n))
    G.setdiag(0)
    G.eliminate_zeros()
    return G


def split(agg, G):
    """aggregates cut into the connected pieces of their rows over G"""
    c = G.tocoo()
    same = agg[c.row] == agg[c.col]
    H = sp.csr_matrix((np.ones(same.sum()), (c.row[same], c.col[same])), shape=G.shape)
    n, lab = connected_components(H, directed=False)
    return lab, n


def hierarchy(A, nd, aggs=None, split_levels=(), max_coarse=64):
    """aggs[l]: a fixed aggregation of level l (None: aggregate this level's
    graph).  split_levels: aggregates of those levels cut into their pieces;
    a piece's coarse row inherits its aggregate's next-level aggregate (the
    kept hierarchy with split aggregates appended)"""
    levels = []
    B = np.tile(np.eye(nd), (A.shape[0] // nd, 1))
    k = nd
    l = 0
    origin = None  # coarse row of this level → the kept aggregation's row it came from
    while True:
        n = A.shape[0] // nd
        Dinv = block_diag_inv(A, nd)
        w = (4.0 / 3.0) / 2.0 if l == 0 else (4.0 / 3.0) / 1.75
        L = {"A": A, "Dinv": Dinv, "w": w, "nd": nd}
        levels.append(L)
        if n <= max_coarse:
            L["coarsest"] = True
            L["Ainv"] = np.linalg.pinv(A.toarray())
            break
        G = node_graph(A, nd)
        if aggs is not None and l < len(aggs) and aggs[l] is not None:
            base = aggs[l] if origin is None else aggs[l][origin]
            agg, na = base, int(base.max()) + 1
        else:
            agg, na = aggregate(G)
            base = None
        if l in split_levels:
            pieces, na = split(agg, G)
            origin = np.zeros(na, np.int64)
            origin[pieces] = agg
            agg = pieces
        else:
            origin = None
        L["agg"] = agg
        Pt, Bc = fit(agg, na, B, nd)
        P = (Pt - w * (Dinv @ (A @ Pt))).tocsr()
        L["P"] = P
        A = (P.T @ A @ P).tocsr()
        B = Bc
        nd = k
        l += 1
    return levels


def planar_system(xyz, e2n, active, top, bot, dy):
    K = fo.assemble_global_stiffness(xyz, e2n, active)
    known, vals = fo.known_dof_map(top, bot, dy, -dy)
    A3, b3, free = fo.free_system(K, known, vals)
    keep = np.flatnonzero(free % 3 < 2)
    return A3[keep][:, keep].tocsr(), b3[keep]


def main():
    nx, ny = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (2, 2)
    want = int(sys.argv[3]) if len(sys.argv) > 3 else None
    xyz, e2n = synth.tiled_mesh(nx, ny, chords=True)
    top, bot = synth.grips(xyz)
    E = len(e2n)
    A0, b0 = planar_system(xyz, e2n, np.ones(E, bool), top, bot, fo.DISPLACEMENT_MAX)
    K = fo.assemble_global_stiffness(xyz, e2n, np.ones(E, bool))
    known, vals = fo.known_dof_map(top, bot, fo.DISPLACEMENT_MAX, -fo.DISPLACEMENT_MAX)
    U = fo.solve_system(K, known, vals)
    scale = 2.1 * fo.MAX_STRAIN / np.abs(fo.element_strain(xyz, e2n, U)).max()
    active = np.ones(E, bool)
    for step in range(fo.N_STEPS):
        dy = fo.DISPLACEMENT_MAX * scale * step / (fo.N_STEPS - 1)
        if (want is None and active.sum() < E) or step == want:
            break
        K = fo.assemble_global_stiffness(xyz, e2n, active)
        known, vals = fo.known_dof_map(top, bot, dy, -dy)
        U = fo.solve_system(K, known, vals)
        with np.errstate(invalid="ignore"):
            active = active & ~(np.abs(fo.element_strain(xyz, e2n, U)) > fo.MAX_STRAIN)
    print(f"{nx}x{ny} chords, step {step}: {E - int(active.sum())} failed", flush=True)
    A, b = planar_system(xyz, e2n, active, top, bot, dy)
    intact = hierarchy(A0, 2)
    aggs = [L.get("agg") for L in intact]
    runs = {
        "kept-all": hierarchy(A, 2, aggs),
        "kept-0": hierarchy(A, 2, aggs[:1]),
        "split-0": hierarchy(A, 2, aggs[:1], split_levels=(0,)),
        "split-all": hierarchy(A, 2, aggs, split_levels=tuple(range(len(aggs)))),
        "fresh": hierarchy(A, 2),
    }
    print("intact network, intact hierarchy:", pcg(A0, b0, lambda r: vcycle(intact, r), max_it=3000)[1])
    for name, lev in runs.items():
        it = pcg(A, b, lambda r: vcycle(lev, r), max_it=3000)[1]
        print(f"  {name:10s} {it:4d} iterations, level rows {[L['A'].shape[0] // L['nd'] for L in lev][:5]}", flush=True)


if __name__ == "__main__":
    main()
