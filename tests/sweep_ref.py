"""NumPy restatement of the whole-matrix SSOR / IC(0) preconditioners
(csrc/sweep.hip, amg.hpp SweepPlan) — test infrastructure only.

The engine factorises A_0 in the plan's entry order (colour → wave → lane,
a piece's rows on consecutive lanes; the pieces of a colour are independent,
so this is a valid elimination order of the whole matrix).  Here the same order is applied to the oracle's
K_ff, the block factor M = (D̃ + L) D̃⁻¹ (D̃ + Lᵀ) is formed with SciPy, and a
SciPy-semantics PCG runs with it.  PETSc's own ICC runs in the natural node
order (src/fea_petsc.cpp:331); `natural_order` gives that one for comparison.
"""
import ctypes as C

import numpy as np
import scipy.sparse as sp
from scipy.sparse.linalg import splu

P = C.c_void_p
NAMES = ("cwave", "wsteps", "row", "ppos", "dpos", "lo_ptr", "lo_ent", "lo_pos", "up_ptr",
         "up_ent", "up_pos")


def fetch_sweep(shim):
    shim.shim_sweep_array.restype = C.c_int64
    shim.shim_sweep_array.argtypes = [C.c_char_p, P]
    out = {}
    for n in NAMES:
        k = shim.shim_sweep_array(n.encode(), None)
        a = np.zeros(max(k, 1), np.int32)
        shim.shim_sweep_array(n.encode(), a.ctypes.data_as(P))
        out[n] = a[:k]
    out["n_pieces"] = int(shim.shim_sweep_array(b"n_pieces", None))
    return out


def entry_colour(sw):
    """colour of every entry"""
    wave = np.arange(len(sw["row"])) // 64
    return np.searchsorted(sw["cwave"], wave, side="right") - 1


def elimination_order(sw):
    """level-0 rows in the engine's factorisation order (entry order)"""
    r = sw["row"]
    return r[r >= 0]


def block_perm(order, nd):
    return (order[:, None].astype(np.int64) * nd + np.arange(nd)).ravel()


def factor(Ap, nd, kind):
    """(I + L D̃⁻¹ (CSC), D̃⁻¹ block diagonal) of the block matrix Ap in its
    own order; kind "dic" (DIC(0) pivots, non-SPD → D) or "ssor" (D̃ = D)."""
    n = Ap.shape[0] // nd
    C_ = Ap.tocoo()
    bi, bj = C_.row // nd, C_.col // nd
    blocks = {}
    for i, j, a, b, v in zip(bi, bj, C_.row % nd, C_.col % nd, C_.data):
        blk = blocks.get((i, j))
        if blk is None:
            blk = blocks[(i, j)] = np.zeros((nd, nd))
        blk[a, b] += v
    lower = [[] for _ in range(n)]
    for (i, j) in blocks:
        if j < i:
            lower[i].append(j)
    Dt_inv = np.zeros((n, nd, nd))
    for i in range(n):
        D = blocks[(i, i)]
        T = D.copy()
        if kind == "dic":
            for k in lower[i]:
                X = blocks[(i, k)]
                T -= X @ Dt_inv[k] @ X.T
            if not all(np.linalg.det(T[:m, :m]) > 0 for m in range(1, nd + 1)):
                T = D
        Dt_inv[i] = np.linalg.inv(T)
    rows, cols, vals = [], [], []
    for i in range(n):
        for j in lower[i]:
            m = blocks[(i, j)] @ Dt_inv[j]
            for a in range(nd):
                for b in range(nd):
                    rows.append(nd * i + a)
                    cols.append(nd * j + b)
                    vals.append(m[a, b])
    Lu = sp.csr_matrix((vals, (rows, cols)), shape=(nd * n, nd * n)) + sp.identity(nd * n, format="csr")
    return Lu.tocsc(), sp.block_diag(list(Dt_inv), format="csr")


def preconditioner(Ap, nd, kind):
    """r ↦ M⁻¹ r = (I + D̃⁻¹Lᵀ)⁻¹ D̃⁻¹ (I + L D̃⁻¹)⁻¹ r"""
    Lu, Db = factor(Ap, nd, kind)
    opts = dict(SymmetricMode=True)
    lo = splu(Lu, permc_spec="NATURAL", diag_pivot_thresh=0.0, options=opts)
    up = splu(Lu.T.tocsc(), permc_spec="NATURAL", diag_pivot_thresh=0.0, options=opts)
    return lambda r: up.solve(Db @ lo.solve(r))


def pcg(A, b, prec, rtol=1e-8, max_it=100000):
    """SciPy-cg semantics: x₀ = 0, stop on ‖r‖ ≤ rtol‖b‖; returns the count."""
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
            return it, x
        z = prec(r)
        rz, rz_old = r @ z, rz
        p = z + (rz / rz_old) * p
    return -1, x
