"""Lab (CPU, SciPy): would PETSc GAMG's default smoother — Chebyshev on
D⁻¹A over [0.05 λ, 1.05 λ] (its `-mg_levels_ksp_chebyshev_esteig 0,0.05,0,1.05`),
degree 2 — buy back its extra level-0 sweeps on the chord-dense (C5-recipe)
networks?  Same smoothed-aggregation hierarchy as tools/sa_nullspace_lab.py
(translations only), V-cycles with the smoother per level as listed, PCG to
rtol 1e-8.

    python3 tools/smoother_lab.py [nx ny]

Measured (2×2 tiles + chords, 47k DOF): damped block Jacobi V(1,1) 34
iterations; Chebyshev(2,2) on every level 23, on level 0 alone 36; Jacobi
V(2,2) 28.  Chebyshev only pays on every level, and there it costs four
level-0 operator sweeps per cycle against the compact cycle's one (§4.2).
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import sa_nullspace_lab as lab  # noqa: E402
from sa_nullspace_lab import fo, synth  # noqa: E402


def cheb(A, Dinv, b, x, lam, deg, lo=0.05, hi=1.05):
    """deg steps of the Chebyshev iteration for D⁻¹A on [lo·λ, hi·λ]."""
    a, c = lo * lam, hi * lam
    theta, delta = (c + a) / 2, (c - a) / 2
    sigma = theta / delta
    rho = 1 / sigma
    d = (Dinv @ (b - A @ x)) / theta
    x = x + d
    for _ in range(deg - 1):
        rho_new = 1 / (2 * sigma - rho)
        d = rho_new * rho * d + 2 * rho_new / delta * (Dinv @ (b - A @ x))
        x = x + d
        rho = rho_new
    return x


def vcycle(levels, b, l, cfg):
    L = levels[l]
    if L.get("coarsest"):
        return L["Ainv"] @ b
    A, Dinv, w, P = L["A"], L["Dinv"], L["w"], L["P"]
    kind, pre, post = cfg(l)

    def smooth(x, k):
        if kind == "cheb":
            return cheb(A, Dinv, b, x, L["lam"], k)
        for _ in range(k):
            x = x + w * (Dinv @ (b - A @ x))
        return x

    x = smooth(np.zeros_like(b), pre)
    x = x + P @ vcycle(levels, P.T @ (b - A @ x), l + 1, cfg)
    return smooth(x, post)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    nx, ny = (int(args[0]), int(args[1])) if len(args) >= 2 else (2, 2)
    xyz, e2n = synth.tiled_mesh(nx, ny, chords=True)
    top, bot = synth.grips(xyz)
    K = fo.assemble_global_stiffness(xyz, e2n, np.ones(len(e2n), bool))
    dy = fo.DISPLACEMENT_MAX * ny * 20 / (fo.N_STEPS - 1)
    known, vals = fo.known_dof_map(top, bot, dy, -dy)
    A3, b3, free = fo.free_system(K, known, vals)
    planar = free % 3 != 2
    A = A3[planar][:, planar].tocsr()
    b = b3[planar]
    n = A.shape[0] // 2
    B = np.zeros((2 * n, 2))
    B[0::2, 0] = 1.0
    B[1::2, 1] = 1.0
    levels = lab.hierarchy(A, B, None, 2, False)
    rng = np.random.default_rng(0)
    for L in levels:  # λmax(D⁻¹A) by power iteration (PETSc: a few CG steps)
        if L.get("coarsest"):
            continue
        M = L["Dinv"] @ L["A"]
        v = rng.standard_normal(M.shape[0])
        for _ in range(30):
            v = M @ v
            L["lam"] = np.linalg.norm(v)
            v /= L["lam"]
    print(f"{nx}x{ny} tiles + chords: {A.shape[0]} DOF, rows {[L['A'].shape[0] for L in levels]}")
    cases = {
        "jacobi V(1,1) every level": lambda l: ("jac", 1, 1),
        "jacobi V(2,2) every level": lambda l: ("jac", 2, 2),
        "chebyshev(2,2) level 0 only": lambda l: ("cheb", 2, 2) if l == 0 else ("jac", 1, 1),
        "chebyshev(2,2) every level": lambda l: ("cheb", 2, 2),
    }
    for name, cfg in cases.items():
        _, it = lab.pcg(A, b, lambda r: vcycle(levels, r, 0, cfg))
        print(f"  {name:30s} PCG its to 1e-8: {it}")


if __name__ == "__main__":
    main()
