"""Lab (CPU, SciPy): which ORDER makes a whole-matrix IC(0) / SSOR for the
mycelium network both parallel on a GPU and stronger than Jacobi?

The reference's default preconditioner is PETSc PCICC (src/fea_petsc.cpp:331),
IC(0) in the CSV node order, a sequential triangular solve.  Candidates, all
node-block (2×2, planar) factorisations of the WHOLE free system:

  natural   the reference's node order (PETSc's; sequential)
  dfs       depth-first order of the free-node graph (the engine's row order)
  mc        greedy point multicolouring, colour-major (one launch per colour)
  pieces m  the dfs order cut into pieces of m consecutive rows, the pieces
            greedily coloured, colour-major, dfs order inside a piece (one
            lane walks a piece: chains stay in natural order)

IC(0) = incomplete block Cholesky with the pattern of A: M = (D̃+L)D̃⁻¹(D̃+Lᵀ),
L the block lower part (off-diagonals modified on triangles); DIC(0): L = A's
lower part, only D̃ modified; SSOR (ω = 1): D̃ = D.  PCG to rtol 1e-8 on the
unpreconditioned residual (SciPy semantics).

    python3 tools/icc_lab.py [ref | nx ny] [--chords]
"""
import os
import sys
import time

import numpy as np
import scipy.sparse as sp
from scipy.sparse.linalg import splu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mycelium-fea-project_amd"), os.path.join(REPO, "oracle")]
import fea_oracle as fo  # noqa: E402
from mfea import synth  # noqa: E402


def system(args):
    chords = "--chords" in args
    args = [a for a in args if not a.startswith("--")]
    if not args or args[0] == "ref":
        xyz, e2n = synth.load_mesh(os.path.join(REPO, "tests", "golden", "meshes", "sim_20251117_181147"))
        ny = 1
    else:
        nx, ny = int(args[0]), int(args[1])
        xyz, e2n = synth.tiled_mesh(nx, ny, chords=chords)
    top, bot = synth.grips(xyz)
    K = fo.assemble_global_stiffness(xyz, e2n, np.ones(len(e2n), bool))
    dy = fo.DISPLACEMENT_MAX * 20 / (fo.N_STEPS - 1)
    known, vals = fo.known_dof_map(top, bot, dy, -dy)
    A3, b3, free = fo.free_system(K, known, vals)
    planar = free % 3 != 2
    A = A3[planar][:, planar].tocsr()
    b = b3[planar]
    return A, b


def node_graph(A):
    n = A.shape[0] // 2
    B = sp.csr_matrix((np.ones(A.nnz), A.indices // 2, A.indptr), shape=(2 * n, n))
    G = (B[0::2] + B[1::2]).tocsr()
    G.setdiag(0)
    G.eliminate_zeros()
    G.sort_indices()
    return G


def dfs_order(G):
    n = G.shape[0]
    seen = np.zeros(n, bool)
    order = []
    for s in range(n):
        if seen[s]:
            continue
        stack = [s]
        while stack:
            v = stack.pop()
            if seen[v]:
                continue
            seen[v] = True
            order.append(v)
            nb = G.indices[G.indptr[v]:G.indptr[v + 1]]
            for w in nb[::-1]:
                if not seen[w]:
                    stack.append(w)
    return np.array(order)


def greedy_colour(G, order):
    n = G.shape[0]
    col = -np.ones(n, np.int64)
    for v in order:
        used = set(col[G.indices[G.indptr[v]:G.indptr[v + 1]]].tolist())
        c = 0
        while c in used:
            c += 1
        col[v] = c
    return col


def mc_order(G):
    col = greedy_colour(G, np.arange(G.shape[0]))
    return np.lexsort((np.arange(G.shape[0]), col)), col.max() + 1


def piece_order(G, m):
    d = dfs_order(G)
    n = len(d)
    piece = np.empty(n, np.int64)
    piece[d] = np.arange(n) // m
    npc = piece.max() + 1
    # piece graph
    r = np.repeat(np.arange(n), np.diff(G.indptr))
    pr, pc = piece[r], piece[G.indices]
    k = pr != pc
    PG = sp.csr_matrix((np.ones(k.sum()), (pr[k], pc[k])), shape=(npc, npc)).tocsr()
    PG.sum_duplicates()
    pcol = greedy_colour(PG, np.arange(npc))
    pos = np.empty(n, np.int64)
    pos[d] = np.arange(n)
    key_c = pcol[piece]
    return np.lexsort((pos, key_c)), pcol.max() + 1


def permute(A, order):
    p = np.empty(2 * len(order), np.int64)
    p[0::2] = 2 * order
    p[1::2] = 2 * order + 1
    return A[p][:, p].tocsr(), p


def blocks(Ap):
    """{(i, j): 2×2 block} of a 2-DOF block CSR matrix."""
    C = Ap.tocoo()
    out = {}
    for r, c, v in zip(C.row, C.col, C.data):
        key = (r // 2, c // 2)
        blk = out.get(key)
        if blk is None:
            blk = out[key] = np.zeros((2, 2))
        blk[r % 2, c % 2] += v
    return out


def factor(Ap, kind):
    """(Lunit = I + L D̃⁻¹ scalar CSR, D̃⁻¹ block diag) for kind ic / dic / ssor."""
    n = Ap.shape[0] // 2
    B = blocks(Ap)
    lower = [[] for _ in range(n)]  # j < i
    for (i, j) in B:
        if j < i:
            lower[i].append(j)
    for i in range(n):
        lower[i].sort()
    L = {k: v.copy() for k, v in B.items() if k[1] < k[0]}
    Dt_inv = np.zeros((n, 2, 2))
    lower_set = [set(x) for x in lower]
    for i in range(n):
        if kind == "ic":  # off-diagonals: L_ij −= Σ_{k<j, k∈N(i)∩N(j)} L_ik D̃_k⁻¹ L_jkᵀ
            for j in lower[i]:
                for k in lower[i]:
                    if k < j and k in lower_set[j]:
                        L[(i, j)] -= L[(i, k)] @ Dt_inv[k] @ L[(j, k)].T
        T = B[(i, i)].copy()
        if kind != "ssor":
            for k in lower[i]:
                T -= L[(i, k)] @ Dt_inv[k] @ L[(i, k)].T
            if not (T[0, 0] > 0 and np.linalg.det(T) > 0):
                T = B[(i, i)].copy()
        Dt_inv[i] = np.linalg.inv(T)
    rows, cols, vals = [], [], []
    for (i, j), blk in L.items():
        m = blk @ Dt_inv[j]
        for a in range(2):
            for c in range(2):
                rows.append(2 * i + a)
                cols.append(2 * j + c)
                vals.append(m[a, c])
    Lu = sp.csr_matrix((vals, (rows, cols)), shape=(2 * n, 2 * n)) + sp.identity(2 * n, format="csr")
    Db = sp.block_diag(list(Dt_inv), format="csr")
    return Lu.tocsc(), Db


def pcg(A, b, prec, rtol=1e-8, max_it=20000):
    x = np.zeros_like(b)
    r = b.copy()
    nb = np.linalg.norm(b)
    z = prec(r)
    p = z.copy()
    rz = r @ z
    for it in range(1, max_it + 1):
        q = A @ p
        a = rz / (p @ q)
        x += a * p
        r -= a * q
        if np.linalg.norm(r) <= rtol * nb:
            return it
        z = prec(r)
        rz_new = r @ z
        p = z + (rz_new / rz) * p
        rz = rz_new
    return -1


def ic_prec(Ap, kind):
    Lu, Db = factor(Ap, kind)
    lo = splu(Lu, permc_spec="NATURAL", diag_pivot_thresh=0.0, options=dict(SymmetricMode=True))
    up = splu(Lu.T.tocsc(), permc_spec="NATURAL", diag_pivot_thresh=0.0, options=dict(SymmetricMode=True))

    def prec(r):
        return up.solve(Db @ lo.solve(r))
    return prec


def main():
    A, b = system(sys.argv[1:])
    G = node_graph(A)
    n = G.shape[0]
    deg = np.diff(G.indptr)
    print(f"free nodes {n}, mean degree {deg.mean():.2f}, max {deg.max()}")
    Dinv = sp.block_diag([np.linalg.inv(A[2 * i:2 * i + 2, 2 * i:2 * i + 2].toarray()) for i in range(n)], format="csr")
    print(f"jacobi (block)        {pcg(A, b, lambda r: Dinv @ r):6d}")
    orders = {"natural": (np.arange(n), None), "dfs": (dfs_order(G), None), "mc": mc_order(G)}
    for m in (8, 16, 32, 64, 128):
        orders[f"pieces{m}"] = piece_order(G, m)
    for name, (order, ncol) in orders.items():
        Ap, p = permute(A, order)
        bp = b[p]
        res = []
        for kind in ("ic", "dic", "ssor"):
            t = time.time()
            res.append(f"{kind} {pcg(Ap, bp, ic_prec(Ap, kind)):6d}")
        print(f"{name:10s} colours {str(ncol):4s} " + "  ".join(res), flush=True)


if __name__ == "__main__":
    main()
