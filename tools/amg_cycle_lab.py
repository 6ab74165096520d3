"""CPU experiment: PCG iteration counts of SA-AMG variants on the benchmark
networks (not product code; the GAMG kernels implement the variant DESIGN.md
§4.2 picks).  Uses the engine's own host plan (aggregates of every level,
through tests/native/host_shim.cpp) and the NumPy numeric setup of
tests/amg_ref.py, then swaps one ingredient at a time:

  base        V(1,1), ω-damped block Jacobi, P_tent = translations (the engine)
  v22         two pre- and two post-smoothing sweeps
  cheb2       Chebyshev degree-2 smoother on D⁻¹A (PETSc GAMG's default)
  cheb2cK     ... on levels ≥ K only (level 0 keeps V(1,1) Jacobi)
  v22cK       two Jacobi sweeps on levels ≥ K only
  cheb2sK / v22sK   ... on level K alone
  cheb2rA_B / v22rA_B   ... on levels A..B
  w / wK      W-cycle (two coarse corrections per level / on levels < K only)
  wfK         W-cycle on levels ≥ K only
  rot         near-nullspace with the in-plane rotation: P_tent columns
              (tx, ty, θ) per aggregate (QR-orthonormalised, PyAMG fit_candidates),
              ND = 3 on every coarse level
  rot_cheb2   both

  python tools/amg_cycle_lab.py --tiles 2 2 --chords [--variants base rot ...]
"""
import argparse
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "tests"), os.path.join(HERE, "..", "oracle"),
                os.path.join(HERE, "..", "mycelium-fea-project_amd")]

import amg_ref  # noqa: E402
from test_amg_cpu import setup_case  # noqa: E402
import ctypes as C  # noqa: E402
from conftest import build_host_shim  # noqa: E402


def shim_lib():
    P = C.c_void_p
    lib = C.CDLL(build_host_shim())
    lib.shim_build.restype = C.c_int
    lib.shim_build.argtypes = [C.c_int64, P, C.c_int64, P, C.c_int, C.c_int64, P, C.c_int64, P,
                               C.c_int, P, C.c_char_p, C.c_int]
    lib.shim_arrays.argtypes = [P] * 6
    lib.shim_sell_values.argtypes = [P, C.c_double, C.c_double, P, P]
    lib.shim_amg.restype = C.c_int
    lib.shim_amg.argtypes = [P, C.c_int, C.c_char_p, C.c_int]
    lib.shim_amg_array.restype = C.c_int64
    lib.shim_amg_array.argtypes = [C.c_int, C.c_char_p, P]
    return lib


def block_diag_inv(A, nd):
    n = A.shape[0] // nd
    Ac = A.tocsr()
    D = np.zeros((n, nd, nd))
    for a in range(nd):
        for b in range(nd):
            D[:, a, b] = Ac[a::nd, b::nd].diagonal()
    return np.linalg.inv(D)


def dapply(Dinv, v):
    nd = Dinv.shape[1]
    return np.einsum("iab,ib->ia", Dinv, v.reshape(-1, nd)).ravel()


def rho_DA(A, Dinv, its=15):
    x = np.random.default_rng(0).standard_normal(A.shape[0])
    lam = 1.0
    for _ in range(its):
        y = dapply(Dinv, A @ x)
        lam = np.linalg.norm(y) / np.linalg.norm(x)
        x = y / np.linalg.norm(y)
    return lam


class Level:
    pass


def build_levels(plan_levels, A0, nd0, coords0, rot, p_omega=4.0 / 3.0):
    """SA hierarchy on the plan's aggregates; rot adds the rotation mode."""
    levs = []
    A, nd = A0.tocsr(), nd0
    X = coords0  # per row (node / aggregate) xy for the rotation candidate
    B = None
    for l, pl in enumerate(plan_levels):
        L = Level()
        L.A, L.nd = A, nd
        L.Dinv = block_diag_inv(A, nd)
        L.rho = rho_DA(A, L.Dinv)
        levs.append(L)
        if pl["coarsest"] or A.shape[0] <= 3 * nd:
            L.coarsest = True
            break
        L.coarsest = False
        agg = pl["agg"]
        nat = pl.get("nat_rows")
        n = A.shape[0] // nd
        assert len(agg) == n, (len(agg), n)
        nc = int(agg.max()) + 1
        if B is None:  # fine candidates
            cols = [np.tile(np.eye(nd), (n, 1))]
            if rot:
                c = X - X.mean(axis=0)
                r = np.zeros((n * nd, 1))
                r[0::nd, 0] = -c[:, 1]
                r[1::nd, 0] = c[:, 0]
                cols.append(r)
            B = np.hstack(cols)
        k = B.shape[1]
        # fit candidates per aggregate: B_agg = Q R, P_tent = Q, B_c = R
        rows, colsP, vals = [], [], []
        Bc = np.zeros((nc * k, k))
        order = np.argsort(agg, kind="stable")
        ag_sorted = agg[order]
        starts = np.searchsorted(ag_sorted, np.arange(nc + 1))
        for J in range(nc):
            nodes = order[starts[J]:starts[J + 1]]
            nodes = nodes[nodes >= 0]
            dofs = (nodes[:, None] * nd + np.arange(nd)).ravel()
            Bl = B[dofs]
            Q, R = np.linalg.qr(Bl)
            kk = Q.shape[1]
            if kk < k:  # aggregate smaller than the candidate count: pad
                Q = np.hstack([Q, np.zeros((Q.shape[0], k - kk))])
                R = np.vstack([R, np.zeros((k - kk, k))])
            rows.append(np.repeat(dofs, k))
            colsP.append(np.tile(J * k + np.arange(k), len(dofs)))
            vals.append(Q.ravel())
            Bc[J * k:(J + 1) * k] = R
        unagg = agg < 0
        Pt = sp.csr_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(colsP))),
                           shape=(n * nd, nc * k))
        # smoothed P: (I − ω/ρ D⁻¹A) P_tent
        DA = sp.csr_matrix(sp.bsr_matrix((L.Dinv, np.arange(n), np.arange(n + 1)), shape=(n * nd, n * nd))) @ A
        P = Pt - (p_omega / L.rho) * (DA @ Pt)
        L.P = P.tocsr()
        A = (L.P.T @ A @ L.P).tocsr()
        # drop exact zeros from padding
        A.eliminate_zeros()
        nd, B = k, Bc
        X = np.array([X[order[starts[J]:starts[J + 1]]].mean(axis=0) for J in range(nc)])
        assert not unagg.any() or True
    return levs


def cheb_coeffs(deg, lo, hi):
    # PyAMG chebyshev_polynomial_coefficients: roots of the shifted Chebyshev
    # polynomial on [lo, hi]; smoother x += p(D⁻¹A) D⁻¹ r
    roots = (hi + lo) / 2 + (hi - lo) / 2 * np.cos(np.pi * (np.arange(deg) + 0.5) / deg)
    scale = np.prod(1 - 1 / roots)  # p(0) = 1 normalisation of 1 - λ q(λ)
    c = np.poly(roots)  # polynomial with those roots
    c = c / c[-1]       # residual polynomial r(λ) = 1 - λ q(λ), r(0) = 1
    q = -c[:-1]          # q coefficients (highest first)
    del scale
    return q


def smooth(L, x, b, kind, sweeps):
    if kind == "jac":
        w = (4.0 / 3.0) / max(L.rho, 1e-300)
        for _ in range(sweeps):
            x = x + w * dapply(L.Dinv, b - L.A @ x)
        return x
    # chebyshev on D⁻¹A, interval [ρ/30, 1.1ρ]
    q = cheb_coeffs(sweeps, L.rho / 30, 1.1 * L.rho)
    r = dapply(L.Dinv, b - L.A @ x)
    y = q[0] * r
    for c in q[1:]:
        y = c * r + dapply(L.Dinv, L.A @ y)
    return x + y


def cycle(levs, b, l, kind, sweeps, gamma, wl=99, k0=0):
    L = levs[l]
    if L.coarsest:
        return np.linalg.solve(L.A.toarray(), b) if L.A.shape[0] <= 4000 else dapply(L.Dinv, b)
    if isinstance(k0, tuple):  # (a, b): levels a..b
        on = k0[0] <= l <= k0[1]
    else:
        on = l >= k0 if k0 >= 0 else l == -k0  # k0 < 0: level −k0 alone
    kl, sl = (kind, sweeps) if on else ("jac", 1)
    x = smooth(L, np.zeros_like(b), b, kl, sl)
    w_here = l < wl if wl >= 0 else l >= -wl  # wl < 0: W on levels ≥ −wl
    for _ in range(gamma if l + 2 < len(levs) and w_here else 1):
        x = x + L.P @ cycle(levs, L.P.T @ (b - L.A @ x), l + 1, kind, sweeps, gamma, wl, k0)
    return smooth(L, x, b, kl, sl)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", type=int, nargs=2, default=[2, 2])
    ap.add_argument("--chords", action="store_true")
    ap.add_argument("--variants", nargs="*", default=["base", "v22", "cheb2", "w", "rot", "rot_cheb2"])
    a = ap.parse_args()
    from mfea import synth
    xyz, e2n = synth.tiled_mesh(*a.tiles, chords=a.chords)
    top, bot = synth.grips(xyz)
    shim = shim_lib()
    levels, Kff, b, nodes0 = setup_case(shim, xyz, e2n, top, bot, np.ones(len(e2n)), 2)
    print(f"DOF {Kff.shape[0]}, plan levels {len(levels)}: rows {[L['n'] for L in levels]}", flush=True)
    t = time.time()
    _, it = amg_ref.pcg(Kff, b, lambda r: amg_ref.vcycle(levels, r), rtol=1e-8)
    print(f"engine (amg_ref)        {it:4d} its  ({time.time() - t:.1f} s)", flush=True)
    coords = xyz[nodes0][:, :2]
    hier = {}
    for v in a.variants:
        rot = v.startswith("rot")
        if rot not in hier:
            hier[rot] = build_levels(levels, Kff, 2, coords, rot)
        levs = hier[rot]
        kind, sweeps, gamma, wl, k0 = "jac", 1, 1, 99, 0
        if "cheb2" in v:
            kind, sweeps = "cheb", 2
        if v.startswith("v22"):
            sweeps = 2
        if v.startswith(("cheb2c", "v22c")):
            k0 = int(v.split("c")[-1])
        if v.startswith(("cheb2s", "v22s")):
            k0 = -int(v.split("s")[-1])
        if v.startswith(("cheb2r", "v22r")):  # e.g. v22r1_2: levels 1..2
            a_, b_ = v.split("r")[-1].split("_")
            k0 = (int(a_), int(b_))
        if v.startswith("w"):
            gamma = 2
            wl = int(v[1:]) if len(v) > 1 and v[1] != "f" else 99
            if v.startswith("wf"):
                wl = -int(v[2:])
        t = time.time()
        _, it = amg_ref.pcg(Kff, b, lambda r: cycle(levs, r, 0, kind, sweeps, gamma, wl, k0), rtol=1e-8)
        print(f"{v:22s} {it:4d} its  levels {len(levs)} rows {[L.A.shape[0] for L in levs][:6]}  "
              f"({time.time() - t:.1f} s)", flush=True)


if __name__ == "__main__":
    main()
