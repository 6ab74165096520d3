"""NumPy restatement of the SA-AMG numeric setup and V-cycle (TEST INFRASTRUCTURE).

Executes the host symbolic plan of ``csrc/amg_symbolic.cpp`` (fetched through
``tests/native/host_shim.cpp``) with the arithmetic of ``csrc/amg.hip``:
A_0 from the assembled SELL slots, exact block-diagonal inverses, the
Gershgorin-bounded smoother weight, the smoothed prolongator and the two
Galerkin products, then the V-cycle and a textbook PCG.  The tests compare
the plan's products against SciPy's ``Pᵀ A P`` and the resulting solve against
the reference's direct solve (``spsolve``, src/fea_solver.py:128).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import scipy.sparse as sp

RHO_FLOOR, RHO_SAFETY = 2.0, 1.45  # amg.hip kRhoFloor / kRhoSafety
RHO_COARSE = 1.75  # capi.hip opt_amg_coarse_rho_ppm: ρ̂ of the levels below 0

_NAMES = ("A.sptr", "A.col", "agg", "P.sptr", "P.col", "pv.ptr", "pv.a", "R.sptr", "R.col", "rp",
          "AP.sptr", "AP.col", "ap.ptr", "ap.a", "ap.b", "ac.ptr", "ac.a", "ac.b",
          "PT.sptr", "PT.col", "pt_row", "pt_ap", "pt_p", "RT.sptr", "RT.col", "rt_pt", "rt_row")


def fetch_plan(shim, active, nd, build=True):
    """build_amg on the shim's last pattern → list of per-level dicts of arrays
    (build=False: the plan the shim built last, e.g. by shim_amg_dist)."""
    if build:
        a = np.ascontiguousarray(active, dtype=np.uint8)
        err = C.create_string_buffer(256)
        nlev = shim.shim_amg(a.ctypes.data_as(C.c_void_p), int(nd), err, 256)
        if nlev < 0:
            raise RuntimeError(err.value.decode())
    else:
        nlev = shim.shim_amg_array(0, b"nlev", None)

    def arr(l, name):
        n = shim.shim_amg_array(l, name.encode(), None)
        out = np.zeros(max(n, 0), dtype=np.int32)
        if n > 0:
            shim.shim_amg_array(l, name.encode(), out.ctypes.data_as(C.c_void_p))
        return out

    levels = []
    for l in range(nlev):
        L = {"n": shim.shim_amg_array(l, b"n", None), "nc": shim.shim_amg_array(l, b"nc", None),
             "coarsest": bool(shim.shim_amg_array(l, b"coarsest", None))}
        for name in _NAMES:
            if name in ("A.sptr", "A.col") or not L["coarsest"]:
                L[name] = arr(l, name)
        for name in ("owner", "aprow"):
            L[name] = arr(l, name)
        levels.append(L)
    levels[0]["row0"] = arr(0, "row0")
    levels[0]["a0.ptr"] = arr(0, "a0.ptr")
    levels[0]["a0.a"] = arr(0, "a0.a")
    return levels


def pos_rows(sptr, n):
    """(row, slot k) of every SELL-64 position (−1 for positions past n)."""
    npos = int(sptr[-1]) * 64
    row = np.full(npos, -1, dtype=np.int64)
    k = np.zeros(npos, dtype=np.int64)
    for s in range(len(sptr) - 1):
        for t in range(sptr[s], sptr[s + 1]):
            r = 64 * s + np.arange(64)
            ok = r < n
            row[t * 64:(t + 1) * 64][ok] = r[ok]
            k[t * 64:(t + 1) * 64] = t - sptr[s]
    return row, k


def seg_sum(vals, ptr):
    """out[q] = Σ vals[ptr[q]:ptr[q+1]] in list order (zeros for empty lists)."""
    npos = len(ptr) - 1
    out = np.zeros((npos,) + vals.shape[1:])
    lens = np.diff(ptr)
    for q in np.flatnonzero(lens):
        acc = np.zeros(vals.shape[1:])
        for t in range(ptr[q], ptr[q + 1]):
            acc = acc + vals[t]
        out[q] = acc
    return out


def _sym(v6, nd):
    if nd == 2:
        return np.stack([np.stack([v6[..., 0], v6[..., 1]], -1), np.stack([v6[..., 1], v6[..., 3]], -1)], -2)
    return np.stack([np.stack([v6[..., 0], v6[..., 1], v6[..., 2]], -1),
                     np.stack([v6[..., 1], v6[..., 3], v6[..., 4]], -1),
                     np.stack([v6[..., 2], v6[..., 4], v6[..., 5]], -1)], -2)


def to_scipy(blocks, sptr, col, n_rows, n_cols, nd, rowmap=None):
    row, _ = pos_rows(sptr, n_rows)
    if rowmap is not None:  # layout rows → the matrix's rows (R̂: rt_row)
        row = np.where(row >= 0, np.asarray(rowmap)[np.maximum(row, 0)], -1)
    ok = (col >= 0) & (row >= 0)
    r, c, b = row[ok], col[ok], blocks[ok]
    rr = (r[:, None, None] * nd + np.arange(nd)[None, :, None]) + 0 * np.arange(nd)[None, None, :]
    cc = (c[:, None, None] * nd + np.arange(nd)[None, None, :]) + 0 * np.arange(nd)[None, :, None]
    return sp.csr_matrix((b.ravel(), (rr.ravel(), cc.ravel())), shape=(n_rows * nd, n_cols * nd))


def _binv(D):
    """Block inverses as amg_dev.hpp binv: a singular (zero) block → zero."""
    out = np.zeros_like(D)
    ok = np.abs(np.linalg.det(D)) > 0
    out[ok] = np.linalg.inv(D[ok])
    return out


def numeric_setup(levels, val, diag, G, N, nd, reg=1e-12, fmask=None, coarse_rho=RHO_COARSE, dmask=None):
    """The per-solve numeric setup of amg.hip on the plan: fills A (blocks),
    dinv, omega, P, AP for every level.  val/diag: the assembled SELL values.
    fmask: per level-0 row, 1 = a floating row whose P_0 row is formed as zero
    (a hierarchy kept over element failures, amg.hip pvals_body).
    coarse_rho: ρ̂ of the levels below 0 (0: the Gershgorin rule, as level 0
    and the engine after a failed solve).
    dmask: per level-0 row, 1 = a row dropped from the tentative prolongator
    (P_tent(i, ·) = 0: no identity block, and its A_ki terms left out of its
    neighbours' P sums) — floating rows and the split-off pieces of kept
    aggregates (amg.hip pvals_body)."""
    L0 = levels[0]
    n0 = L0["n"]
    row, k = pos_rows(L0["A.sptr"], n0)
    npos = len(row)
    A = np.zeros((npos, nd, nd))
    v6 = np.stack([val[c * G:(c + 1) * G] for c in range(6)], -1)        # [G][6]
    offd = seg_sum(_sym(v6, nd)[L0["a0.a"]], L0["a0.ptr"])
    d6 = np.stack([diag[c * N:(c + 1) * N] for c in range(6)], -1).copy()  # [N][6]
    d6[:, [0, 3, 5]] += reg
    isdiag = (k == 0) & (row >= 0)
    A[isdiag] = _sym(d6[L0["row0"][row[isdiag]]], nd)
    offm = (k > 0) & (L0["A.col"] >= 0)
    A[offm] = offd[offm]
    L0["Ab"] = A
    for l, L in enumerate(levels):
        n = L["n"]
        row, k = pos_rows(L["A.sptr"], n)
        Ab = L["Ab"]
        D = Ab[(k == 0) & (row >= 0)]          # rows in order
        Dinv = _binv(D)
        L["dinv"] = Dinv
        ok = (L["A.col"] >= 0) & (row >= 0)
        M = np.abs(np.einsum("pab,pbc->pac", Dinv[row[ok]], Ab[ok])).sum(axis=2)  # [p][a]
        rs = np.zeros((n, nd))
        np.add.at(rs, row[ok], M)
        g = rs.max() if n else 0.0
        # with the over-relaxed coarse levels the engine also fixes level 0 at
        # its exact bound ρ̂_0 = 2 (capi.hip upload_amg, k_amg_a0full)
        if coarse_rho > 0:
            rho = coarse_rho if l > 0 else RHO_FLOOR
        else:
            rho = max(RHO_FLOOR, g / RHO_SAFETY)
        L["omega"] = (4.0 / 3.0) / rho
        L["g"] = g
        L["A"] = to_scipy(Ab, L["A.sptr"], L["A.col"], n, n, nd)
        if L["coarsest"]:
            break
        prow, _ = pos_rows(L["P.sptr"], n)
        items = Ab[L["pv.a"]]
        if l == 0 and dmask is not None:
            items = items * (dmask[L["A.col"][L["pv.a"]]] == 0)[:, None, None]
        S = seg_sum(items, L["pv.ptr"])
        okp = (L["P.col"] >= 0) & (prow >= 0)
        Pb = np.zeros_like(S)
        Pb[okp] = -L["omega"] * np.einsum("pab,pbc->pac", Dinv[prow[okp]], S[okp])
        ident = okp & (L["P.col"] == np.where(prow >= 0, L["agg"][np.maximum(prow, 0)], -9))
        if l == 0 and dmask is not None:
            ident &= dmask[np.maximum(prow, 0)] == 0
        Pb[ident] += np.eye(nd)
        if l == 0 and fmask is not None:
            Pb[okp & (fmask[np.maximum(prow, 0)] != 0)] = 0.0
        L["Pb"] = Pb
        L["P"] = to_scipy(Pb, L["P.sptr"], L["P.col"], n, L["nc"], nd)
        APb = seg_sum(np.einsum("pab,pbc->pac", Ab[L["ap.a"]], Pb[L["ap.b"]]), L["ap.ptr"])
        L["APb"] = APb
        Acb = seg_sum(np.einsum("pba,pbc->pac", Pb[L["ac.a"]], APb[L["ac.b"]]), L["ac.ptr"])
        levels[l + 1]["Ab"] = Acb
    return levels


def compact_transfers(levels):
    """The compact cycle's P̃ = (I − ω D⁻¹ A) P and R̃ = P̃ᵀ (csrc/amg.hip
    k_amg_ptv / k_amg_rtv) from the plan's PT / RT index maps: P̃(i, J) =
    P(i, J) − ω D_i⁻¹ (A·P)(i, J) on A·P's pattern with the level's row labels."""
    for L in levels:
        if L["coarsest"]:
            break
        n, nd = L["n"], L["dinv"].shape[1]
        arow, _ = pos_rows(L["PT.sptr"], n)          # P̃'s own (A·P) row order
        row = np.where(arow >= 0, L["pt_row"][np.maximum(arow, 0)], -1)   # the level's rows
        ok = (L["PT.col"] >= 0) & (row >= 0)
        PTb = np.zeros((len(row), nd, nd))
        pp = L["pt_p"]
        base = np.where((pp >= 0)[:, None, None], L["Pb"][np.maximum(pp, 0)], 0.0)
        DAP = np.einsum("pab,pbc->pac", L["dinv"][np.maximum(row, 0)], L["APb"][np.maximum(L["pt_ap"], 0)])
        PTb[ok] = (base - L["omega"] * DAP)[ok]
        L["PTb"] = PTb
        # as a matrix over the level's rows: relabel A·P rows → level rows
        Pa = to_scipy(PTb, L["PT.sptr"], L["PT.col"], n, L["nc"], nd).tocoo()
        r = L["pt_row"][Pa.row // nd] * nd + Pa.row % nd
        L["Pt"] = sp.csr_matrix((Pa.data, (r, Pa.col)), shape=Pa.shape)
        rok = L["rt_pt"] >= 0
        RTb = np.zeros((len(L["rt_pt"]), nd, nd))
        RTb[rok] = np.transpose(PTb[L["rt_pt"][rok]], (0, 2, 1))
        L["Rt"] = to_scipy(RTb, L["RT.sptr"], L["RT.col"], L["nc"], n, nd, L["rt_row"])
    return levels


def vcycle_compact(levels, b, l=0):
    """The same V(1,1) cycle in two sweeps per level (amg.hpp AmgLevel::PT):
    c = x + ω D⁻¹ (b − A x) with x = ω D⁻¹ b, e = c + P̃ M' (R̃ b)."""
    L = levels[l]
    nd = L["dinv"].shape[1]
    Dinv = L["dinv"]

    def dapply(v, s):
        return s * np.einsum("iab,ib->ia", Dinv, v.reshape(-1, nd)).ravel()

    if L["coarsest"]:
        return dapply(b, 1.0)
    A, w = L["A"], L["omega"]
    x = dapply(b, w)
    c = x + dapply(b - A @ x, w)
    return c + L["Pt"] @ vcycle_compact(levels, L["Rt"] @ b, l + 1)


def vcycle_scaled(levels, r):
    """The compact cycle as the device runs it (csrc/amg.hip k_amg_down /
    k_amg_up): on x_l = s_l D_l⁻¹ b_l alone, with R̂_l = s_{l+1} D_{l+1}⁻¹ R̃_l D_l / ω_l
    (s = ω, 1 on the coarsest level) and Ã_l = ω_l D_l⁻¹ A_l:
    c_l = 2 x_l − Ã_l x_l, x_{l+1} = R̂_l x_l, e_l = c_l + P̃_l e_{l+1}, e = x on the coarsest."""
    def blk(M):
        return sp.block_diag(list(M), format="csr")

    def down_up(l, x):
        L = levels[l]
        if L["coarsest"]:
            return x
        N = levels[l + 1]
        s_n = 1.0 if N["coarsest"] else N["omega"]
        D = blk(np.linalg.inv(L["dinv"]))
        Rhat = (s_n * blk(N["dinv"]) @ L["Rt"] @ D / L["omega"]).tocsr()
        At = (L["omega"] * blk(L["dinv"]) @ L["A"]).tocsr()
        c = 2.0 * x - At @ x
        return c + L["Pt"] @ down_up(l + 1, Rhat @ x)

    if isinstance(r, tuple):  # (level k, x_k): the cycle below level k on its iterate
        return down_up(*r)
    L0 = levels[0]
    nd = L0["dinv"].shape[1]
    s0 = 1.0 if L0["coarsest"] else L0["omega"]
    x0 = s0 * np.einsum("iab,ib->ia", L0["dinv"], r.reshape(-1, nd)).ravel()
    return down_up(0, x0)


def scaled_blocks(levels):
    """Per level the device's compact operators as SELL position blocks:
    R̂ (RT positions), P̃ (PT positions, compact_transfers), Ã (A positions)."""
    for l, L in enumerate(levels[:-1]):
        N = levels[l + 1]
        s_n = 1.0 if N["coarsest"] else N["omega"]
        n, nd = L["n"], L["dinv"].shape[1]
        D = np.linalg.inv(L["dinv"])
        jrow, _ = pos_rows(L["RT.sptr"], L["nc"])
        jrow = np.where(jrow >= 0, L["rt_row"][np.maximum(jrow, 0)], -1)
        col = L["RT.col"]
        ok = (col >= 0) & (jrow >= 0) & (L["rt_pt"] >= 0)
        Rh = np.zeros((len(col), nd, nd))
        PtT = np.transpose(L["PTb"][np.maximum(L["rt_pt"], 0)], (0, 2, 1))
        Rh[ok] = (s_n / L["omega"]) * np.einsum("pab,pbc,pcd->pad", N["dinv"][np.maximum(jrow, 0)], PtT,
                                                 D[np.maximum(col, 0)])[ok]
        L["Rhb"] = Rh
        arow, _ = pos_rows(L["A.sptr"], n)
        L["Atb"] = L["omega"] * np.einsum("pab,pbc->pac", L["dinv"][np.maximum(arow, 0)], L["Ab"])
    return levels


def collapsed_operator(levels, C, k):
    """V_k evaluated from the collapse plan's lists (amg.hip k_amg_tv / k_amg_vv
    in f64): T = V_{k+1} R̂ (identity below the coarsest), V = 2I·diag − Ã + Σ P̃ T.
    C[k]: dict of the plan arrays of level k.  Returns scipy V_k in level rows."""
    nd = levels[0]["dinv"].shape[1]
    vals = {}
    for kk in sorted(C, reverse=True):
        L, c = levels[kk], C[kk]
        Tb = np.zeros((len(c["T.col"]), nd, nd))
        for q in np.flatnonzero(c["T.col"] >= 0):
            acc = np.zeros((nd, nd))
            for t in range(c["tl.ptr"][q], c["tl.ptr"][q + 1]):
                a, b = c["tl.a"][t], c["tl.b"][t]
                acc = acc + (L["Rhb"][b] if a < 0 else vals[kk + 1][a] @ L["Rhb"][b])
            Tb[q] = acc
        Vb = np.zeros((len(c["V.col"]), nd, nd))
        for q in np.flatnonzero(c["V.col"] >= 0):
            acc = 2.0 * np.eye(nd) if c["vdiag"][q] else np.zeros((nd, nd))
            if c["va"][q] >= 0:
                acc = acc - L["Atb"][c["va"][q]]
            for t in range(c["vl.ptr"][q], c["vl.ptr"][q + 1]):
                acc = acc + L["PTb"][c["vl.a"][t]] @ Tb[c["vl.b"][t]]
            Vb[q] = acc
        vals[kk] = Vb
    c = C[k]
    n = levels[k]["n"]
    Va = to_scipy(vals[k], c["V.sptr"], c["V.col"], n, n, nd).tocoo()
    r = c["vrow"][Va.row // nd] * nd + Va.row % nd
    return sp.csr_matrix((Va.data, (r, Va.col)), shape=Va.shape)


def vcycle(levels, b, l=0):
    L = levels[l]
    nd = L["dinv"].shape[1]
    Dinv = L["dinv"]

    def dapply(v, s):
        return s * np.einsum("iab,ib->ia", Dinv, v.reshape(-1, nd)).ravel()

    if L["coarsest"]:
        return dapply(b, 1.0)
    A, P, w = L["A"], L["P"], L["omega"]
    x = dapply(b, w)
    t = b - A @ x
    x = x + P @ vcycle(levels, P.T @ t, l + 1)
    return x + dapply(b - A @ x, w)


def pcg(A, b, M, rtol=1e-8, max_it=1000):
    """Textbook PCG, x0 = 0, stop on ‖r‖ ≤ rtol‖b‖ (SciPy cg semantics)."""
    x = np.zeros_like(b)
    r = b.copy()
    bn = np.linalg.norm(b)
    if bn == 0:
        return x, 0
    z = M(r)
    p = z.copy()
    rho = r @ z
    it = 0
    while np.linalg.norm(r) > rtol * bn and it < max_it:
        q = A @ p
        al = rho / (p @ q)
        x += al * p
        r -= al * q
        z = M(r)
        rn = r @ z
        p = z + (rn / rho) * p
        rho = rn
        it += 1
    return x, it
