"""CPU oracle for the mycelium FEA hot path — TEST INFRASTRUCTURE ONLY.

This module is the *checker*.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it; the product path
(``mycelium-fea-project_amd/``) never does and fails loudly when its HIP library
is missing.

It is a numpy/SciPy restatement of the reference's Python FEA
(``/root/reference/src/fea_solver_no_plotting.py``, identical numerics to
``src/fea_solver.py``).  Every function cites the reference lines it follows.
The hot-path arithmetic of the reference itself lives in third-party SciPy
(``scipy.sparse.csr_matrix`` duplicate summation and ``spsolve`` → SuperLU;
cluster pin scipy 1.8.0, here 1.15.3), so the oracle calls the same SciPy
entry points.

Parity pinning: ``tests/test_oracle_golden.py`` checks this oracle against the
reference's own committed goldens (``results/test_{I,X,y}`` bit-exact,
``sim_20251117_181147`` force/active) and against vectors produced by importing
the reference Python in the build container (``tests/golden/make_golden.py``).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
from scipy.sparse.linalg import spsolve

# ---------------------------------------------------------------------------
# Material & simulation constants — src/fea_solver.py:14-28 (π is 3.14 there)
# ---------------------------------------------------------------------------
E_MOD = 2500.0
D_FIL = 0.0002
T_WALL = 0.000001
AREA = 3.14 * ((D_FIL / 2) ** 2 - (D_FIL / 2 - T_WALL) ** 2)
INERTIA = AREA * 0.001
N_STEPS = 40
DISPLACEMENT_MAX = 0.02
MAX_STRAIN = 0.018
GRIP_LENGTH = 1.5
REG = 1e-12  # src/fea_solver.py:125


def bar_stiffness_bulk(p1s, p2s, E=E_MOD, A=AREA, I=INERTIA):
    """Element stiffness, src/fea_solver.py:30-68.

    Ke = [[S,-S],[-S,S]] with S = (n nᵀ)·k_ax + (I − n nᵀ)·k_b evaluated exactly
    as the reference does: products n_a·n_b, then ·k, then the two parts added.
    """
    v = np.asarray(p2s, dtype=np.float64) - np.asarray(p1s, dtype=np.float64)
    L = np.sqrt((v * v).sum(axis=1))                       # py:38 (x²+y²+z² order)
    Ls = np.where(L < 1e-12, 1e-12, L)                     # py:41
    n = v / Ls[:, None]                                    # py:42
    k_ax = (E * A) / Ls                                    # py:45
    k_b = 12 * E * I / (Ls ** 3)                           # py:58
    TT = n[:, :, None] * n[:, None, :]                     # py:46-47
    P = np.eye(3)[None] - TT                               # py:57
    ax = TT * k_ax[:, None, None]
    bd = P * k_b[:, None, None]
    Ke = np.empty((len(L), 6, 6))
    # axial and bending blocks carry the same sign pattern (py:49-66)
    Ke[:, 0:3, 0:3] = ax + bd
    Ke[:, 3:6, 3:6] = ax + bd
    Ke[:, 0:3, 3:6] = (-TT * k_ax[:, None, None]) + (-P * k_b[:, None, None])
    Ke[:, 3:6, 0:3] = Ke[:, 0:3, 3:6]
    return Ke, L


def assemble_global_stiffness(coords, e2n, active):
    """Global K, src/fea_solver.py:74-106.

    The reference appends 36 COO triplets per active element in element order
    (py:93-103) and lets ``csr_matrix`` sum duplicates (py:105).  Here the same
    triplet stream is built with numpy broadcasting and handed to the same
    SciPy constructor, so duplicate summation order is identical.
    """
    coords = np.asarray(coords, dtype=np.float64)
    e2n = np.asarray(e2n, dtype=np.int64)
    n_dof = 3 * coords.shape[0]
    eidx = np.flatnonzero(np.asarray(active, dtype=bool))
    n1 = e2n[eidx, 0]
    n2 = e2n[eidx, 1]
    Ke, _ = bar_stiffness_bulk(coords[n1], coords[n2])
    dof = np.concatenate([3 * n1[:, None] + np.arange(3), 3 * n2[:, None] + np.arange(3)], axis=1)
    rows = np.repeat(dof, 6, axis=1).ravel()
    cols = np.tile(dof, (1, 6)).ravel()
    return sp.csr_matrix((Ke.ravel(), (rows, cols)), shape=(n_dof, n_dof))


def stiffness_magnitude(p1s, p2s, E=E_MOD, A=AREA, I=INERTIA):
    """|axial term| + |bending term| per Ke entry: the scale of the rounding
    error of Ke.  S = t·k_ax + (δ−t)·k_b cancels catastrophically where
    k_ax ≈ k_b (L ≈ 0.11 mm), so a 1-ulp difference in L³ (NumPy's SIMD pow is
    ≤1 ulp, not correctly rounded) moves S by far more than 1 ulp of S."""
    v = np.asarray(p2s, dtype=np.float64) - np.asarray(p1s, dtype=np.float64)
    L = np.sqrt((v * v).sum(axis=1))
    Ls = np.where(L < 1e-12, 1e-12, L)
    n = v / Ls[:, None]
    TT = n[:, :, None] * n[:, None, :]
    m3 = np.abs(TT * ((E * A) / Ls)[:, None, None]) + \
        np.abs((np.eye(3)[None] - TT) * (12 * E * I / Ls ** 3)[:, None, None])
    return np.block([[m3, m3], [m3, m3]])


def assemble_magnitude(coords, e2n, active):
    """Σ over elements of stiffness_magnitude, in the CSR pattern of K."""
    coords = np.asarray(coords, dtype=np.float64)
    e2n = np.asarray(e2n, dtype=np.int64)
    eidx = np.flatnonzero(np.asarray(active, dtype=bool))
    n1, n2 = e2n[eidx, 0], e2n[eidx, 1]
    M = stiffness_magnitude(coords[n1], coords[n2])
    dof = np.concatenate([3 * n1[:, None] + np.arange(3), 3 * n2[:, None] + np.arange(3)], axis=1)
    rows = np.repeat(dof, 6, axis=1).ravel()
    cols = np.tile(dof, (1, 6)).ravel()
    n = 3 * coords.shape[0]
    return sp.csr_matrix((M.ravel(), (rows, cols)), shape=(n, n))


def known_dof_map(top_nodes, bot_nodes, dy_top, dy_bot):
    """Prescribed DOFs, src/fea_solver.py:223-242.

    A dict filled top-then-bottom: a node in both bands keeps its first
    insertion position but takes the *bottom* value (dict.update semantics).
    """
    d = {}
    for n in top_nodes:
        d.update({3 * n + 0: 0.0, 3 * n + 1: dy_top, 3 * n + 2: 0.0})
    for n in bot_nodes:
        d.update({3 * n + 0: 0.0, 3 * n + 1: dy_bot, 3 * n + 2: 0.0})
    known = np.array(list(d.keys()), dtype=np.int64)
    vals = np.array([d[k] for k in known], dtype=np.float64)
    return known, vals


def solve_system(K, known_dofs, known_vals, reg=REG):
    """Dirichlet elimination + direct solve, src/fea_solver.py:112-135."""
    n_dof = K.shape[0]
    free = np.setdiff1d(np.arange(n_dof), known_dofs)
    Kf = K[free]
    K_ff = Kf[:, free].tocsr()
    K_fk = Kf[:, known_dofs]
    F_f = np.zeros(n_dof)[free] - K_fk @ known_vals
    K_ff = K_ff + reg * sp.identity(K_ff.shape[0], format="csr")
    U_f = spsolve(K_ff, F_f) if len(free) else np.zeros(0)
    U = np.zeros(n_dof)
    U[free] = U_f
    U[known_dofs] = known_vals
    return U


def free_system(K, known_dofs, known_vals, reg=REG):
    """(K_ff + reg·I, b_f, free) exactly as solve_system forms them (py:115-125)."""
    n_dof = K.shape[0]
    free = np.setdiff1d(np.arange(n_dof), known_dofs)
    Kf = K[free]
    K_ff = Kf[:, free].tocsr()
    b = np.zeros(n_dof)[free] - Kf[:, known_dofs] @ known_vals
    return (K_ff + reg * sp.identity(K_ff.shape[0], format="csr")).tocsr(), b, free


def jacobi_pcg(A, b, rtol=1e-8, max_it=100000, x0=None):
    """Reference Jacobi-PCG (SURVEY §8d metric definition).

    x0 = 0; stop when ‖r_k‖₂ ≤ rtol·‖b‖₂ on the recursive (unpreconditioned)
    residual — SciPy ``cg`` semantics.  Returns (x, iterations, ‖r‖/‖b‖).
    Plain textbook PCG; the same recurrences the HIP solver implements.
    """
    n = b.shape[0]
    x = np.zeros(n) if x0 is None else x0.copy()
    dinv = 1.0 / A.diagonal()
    r = b - A @ x
    bn = np.linalg.norm(b)
    if bn == 0.0:
        return np.zeros(n), 0, 0.0
    z = dinv * r
    p = z.copy()
    rho = r @ z
    it = 0
    rn = np.linalg.norm(r)
    while rn > rtol * bn and it < max_it:
        q = A @ p
        alpha = rho / (p @ q)
        x += alpha * p
        r -= alpha * q
        z = dinv * r
        rho_new = r @ z
        p = z + (rho_new / rho) * p
        rho = rho_new
        it += 1
        rn = np.linalg.norm(r)
    return x, it, rn / bn


def grip_nodes(coords, node_ids, tol=GRIP_LENGTH):
    """Top/bottom grip bands, src/fea_solver.py:207-210 (original coords, once)."""
    y = coords[:, 1]
    y_min, y_max = y.min(), y.max()
    top = np.asarray(node_ids)[np.abs(y - y_max) < tol].astype(int)
    bot = np.asarray(node_ids)[np.abs(y - y_min) < tol].astype(int)
    return top, bot


def element_strain(coords, e2n, U):
    """Axial strain of every element, src/fea_solver.py:260-270 (no L clamp).

    The reference's ``np.dot(n, u2 - u1)`` on length-3 vectors is BLAS ddot, an
    FMA chain; the oracle's C helper (cpu_fea.c:cpu_strain) restates it exactly."""
    import ctypes as C
    import cpu_fea
    lib = cpu_fea.lib()
    e2n = np.ascontiguousarray(e2n, dtype=np.int64)
    coords = np.ascontiguousarray(coords, dtype=np.float64)
    U = np.ascontiguousarray(U, dtype=np.float64)
    out = np.empty(e2n.shape[0])
    P = C.c_void_p
    lib.cpu_strain.argtypes = [C.c_int64, P, P, P, P]
    lib.cpu_strain(e2n.shape[0], e2n.ctypes.data_as(P), coords.ctypes.data_as(P),
                   U.ctypes.data_as(P), out.ctypes.data_as(P))
    return out


def run_fea(coords, node_ids, e2n, tol=GRIP_LENGTH, n_steps=N_STEPS,
            disp_max=DISPLACEMENT_MAX, max_strain=MAX_STRAIN, solver="direct", rtol=1e-13):
    """The step loop of ``fea_solver``, src/fea_solver.py:186-295, in memory.

    Returns dict of per-step records: U (steps×3N), stress (steps×E),
    active (steps×E), force (steps×2).  ``solver='pcg'`` swaps spsolve for
    the Jacobi-PCG above (for iteration-count fixtures).
    """
    coords = np.asarray(coords, dtype=np.float64)
    e2n = np.asarray(e2n, dtype=np.int64)
    n_el = e2n.shape[0]
    active = np.ones(n_el, dtype=bool)
    top, bot = grip_nodes(coords, node_ids, tol)
    rec = {"U": [], "stress": [], "active": [], "force": [], "iters": []}
    for step in range(n_steps):
        f = step / (n_steps - 1)
        dy_top = +disp_max * f
        dy_bot = -disp_max * f
        K = assemble_global_stiffness(coords, e2n, active)
        known, vals = known_dof_map(top, bot, dy_top, dy_bot)
        if solver == "direct":
            U = solve_system(K, known, vals)
            rec["iters"].append(-1)
        else:
            A, b, free = free_system(K, known, vals)
            xf, it, _ = jacobi_pcg(A, b, rtol=rtol)
            U = np.zeros(K.shape[0])
            U[free] = xf
            U[known] = vals
            rec["iters"].append(it)
        F = K @ U                                               # py:252
        total_force = F[[3 * n + 1 for n in top]].sum()         # py:253-254
        rec["force"].append([dy_top - dy_bot, total_force])
        strain = element_strain(coords, e2n, U)
        stress = np.where(active, E_MOD * strain, 0.0)          # py:259-272
        with np.errstate(invalid="ignore"):
            fail = active & (np.abs(strain) > max_strain)       # py:273-274
        active = active & ~fail
        rec["stress"].append(stress)
        rec["active"].append(active.copy())
        rec["U"].append(U.copy())
        if active.sum() == 0:                                   # py:283-285
            break
    return {k: np.asarray(v) for k, v in rec.items()}
