"""SA-AMG symbolic plan (csrc/amg_symbolic.cpp), no GPU: the plan's index lists
executed with the arithmetic of csrc/amg.hip (tests/amg_ref.py) must give
A_0 = K_ff + reg·I of the reference (src/fea_solver.py:115-125) and
A_{l+1} = P_lᵀ A_l P_l on every level; the resulting V-cycle must precondition
CG to the direct solve (src/fea_solver.py:128); aggregates must never span two
components of the active free-node graph."""
import ctypes as C

import numpy as np
import pytest
import scipy.sparse as sp
from scipy.sparse.csgraph import connected_components
from scipy.sparse.linalg import spsolve

import amg_ref
import fea_oracle as fo
from conftest import build_host_shim, load_mesh

P = C.c_void_p
EA = fo.E_MOD * fo.AREA
EI12 = (12 * fo.E_MOD) * fo.INERTIA


@pytest.fixture(scope="module")
def shim():
    lib = C.CDLL(build_host_shim())
    lib.shim_build.restype = C.c_int
    lib.shim_build.argtypes = [C.c_int64, P, C.c_int64, P, C.c_int, C.c_int64, P, C.c_int64, P,
                               C.c_int, P, C.c_char_p, C.c_int]
    lib.shim_arrays.argtypes = [P] * 6
    lib.shim_sell_values.argtypes = [P, C.c_double, C.c_double, P, P]
    lib.shim_amg.restype = C.c_int
    lib.shim_amg.argtypes = [P, C.c_int, C.c_char_p, C.c_int]
    lib.shim_floating.restype = C.c_int64
    lib.shim_floating.argtypes = [P, P]
    lib.shim_amg_array.restype = C.c_int64
    lib.shim_amg_array.argtypes = [C.c_int, C.c_char_p, P]
    return lib


def _ptr(a):
    return a.ctypes.data_as(P)


def setup_case(shim, xyz, e2n, top, bot, active, nd):
    """pattern + plan + numeric setup; returns (levels, K_ff in level-0 order, b, perm)."""
    xyz = np.ascontiguousarray(xyz, np.float64)
    e2n = np.ascontiguousarray(e2n, np.int64)
    top = np.ascontiguousarray(top, np.int64)
    bot = np.ascontiguousarray(bot, np.int64)
    N, E = len(xyz), len(e2n)
    sizes = np.zeros(5, np.int64)
    err = C.create_string_buffer(256)
    assert shim.shim_build(N, _ptr(xyz), E, _ptr(e2n), 0, len(top), _ptr(top), len(bot), _ptr(bot),
                           -1, _ptr(sizes), err, 256) == 0, err.value
    nf, G = int(sizes[0]), int(sizes[4])
    perm = np.empty(N, np.int32)
    junk = [np.empty(N, np.int32), np.empty(int(sizes[3]) + 1, np.int32), np.empty(G, np.int32),
            np.empty(G, np.int32), np.empty(N, np.uint8)]
    shim.shim_arrays(_ptr(perm), *[_ptr(j) for j in junk])
    act = np.ascontiguousarray(active, np.uint8)
    val = np.zeros(6 * G)
    diag = np.zeros(6 * N)
    shim.shim_sell_values(_ptr(act), EA, EI12, _ptr(val), _ptr(diag))
    levels = amg_ref.fetch_plan(shim, act, nd)
    amg_ref.numeric_setup(levels, val, diag, G, N, nd)
    # the reference's system, reordered to the plan's rows: level-0 row i is
    # the Pattern's free row row0[i], i.e. original node perm[row0[i]]
    K = fo.assemble_global_stiffness(xyz, e2n, act.astype(bool))
    dy = fo.DISPLACEMENT_MAX * 20 / (fo.N_STEPS - 1)
    known, vals = fo.known_dof_map(top, bot, dy, -dy)
    A3, b3, free = fo.free_system(K, known, vals)
    nodes0 = perm[:nf][levels[0]["row0"]]
    dofs = (nodes0[:, None].astype(np.int64) * 3 + np.arange(nd)).ravel()
    pos = np.searchsorted(free, dofs)
    assert np.array_equal(free[pos], dofs)
    Kff = A3[pos][:, pos].tocsr()
    return levels, Kff, b3[pos], nodes0


def _rel(a, b):
    d = (a - b).tocoo() if sp.issparse(a) else a - b
    na = sp.linalg.norm(b) if sp.issparse(b) else np.linalg.norm(b)
    nd_ = sp.linalg.norm(d) if sp.issparse(d) else np.linalg.norm(d)
    return nd_ / na


def _golden22k():
    nodes, elems = load_mesh("sim_20251117_181147")
    xyz = nodes[["x", "y", "z"]].values
    top, bot = fo.grip_nodes(xyz, nodes["node_id"].values, fo.GRIP_LENGTH)
    return xyz, elems[["n1", "n2"]].values, top, bot


def test_plan_products_match_scipy_galerkin(shim):
    xyz, e2n, top, bot = _golden22k()
    levels, Kff, b, _ = setup_case(shim, xyz, e2n, top, bot, np.ones(len(e2n)), 2)
    assert len(levels) >= 3
    # A_0 = K_ff + reg·I exactly as the reference forms it (planar: x, y DOFs)
    assert _rel(levels[0]["A"], Kff) <= 1e-15
    for l in range(len(levels) - 1):
        L, Nx = levels[l], levels[l + 1]
        Ac = (L["P"].T @ L["A"] @ L["P"]).tocsr()
        assert _rel(Nx["A"], Ac) <= 1e-13, l
        assert Nx["n"] == L["nc"] < L["n"]
    # the coarsest level is block diagonal: its block inverse is the exact solve
    C_ = levels[-1]["A"].tocoo()
    assert np.all(C_.row // 2 == C_.col // 2)


def test_vcycle_pcg_reaches_direct_solve(shim):
    xyz, e2n, top, bot = _golden22k()
    levels, Kff, b, _ = setup_case(shim, xyz, e2n, top, bot, np.ones(len(e2n)), 2)
    ref = spsolve(Kff.tocsc(), b)
    x, it = amg_ref.pcg(Kff, b, lambda r: amg_ref.vcycle(levels, r), rtol=1e-13)
    assert np.linalg.norm(x - ref) / np.linalg.norm(ref) <= 1e-10
    _, it8 = amg_ref.pcg(Kff, b, lambda r: amg_ref.vcycle(levels, r), rtol=1e-8)
    # Jacobi-PCG needs 1,644 iterations on this system (tests/golden, SciPy)
    assert it8 <= 40, it8


def test_vcycle_is_symmetric_positive_definite(shim):
    xyz, e2n, top, bot = _golden22k()
    levels, Kff, _, _ = setup_case(shim, xyz, e2n, top, bot, np.ones(len(e2n)), 2)
    rng = np.random.default_rng(7)
    n = Kff.shape[0]
    X = rng.standard_normal((n, 6))
    MX = np.stack([amg_ref.vcycle(levels, X[:, k]) for k in range(6)], 1)
    G = X.T @ MX
    assert np.abs(G - G.T).max() <= 1e-9 * np.abs(G).max()
    assert np.all(np.linalg.eigvalsh(0.5 * (G + G.T)) > 0)


def test_3d_mesh_plan(shim):
    nodes, elems = load_mesh("sim_20251115_135507")
    xyz = nodes[["x", "y", "z"]].values
    assert np.any(xyz[:, 2] != 0)
    top, bot = fo.grip_nodes(xyz, nodes["node_id"].values, 0.5)
    e2n = elems[["n1", "n2"]].values
    levels, Kff, b, _ = setup_case(shim, xyz, e2n, top, bot, np.ones(len(e2n)), 3)
    assert _rel(levels[0]["A"], Kff) <= 1e-15
    for l in range(len(levels) - 1):
        L = levels[l]
        assert _rel(levels[l + 1]["A"], (L["P"].T @ L["A"] @ L["P"]).tocsr()) <= 1e-13
    ref = spsolve(Kff.tocsc(), b)
    x, _ = amg_ref.pcg(Kff, b, lambda r: amg_ref.vcycle(levels, r), rtol=1e-13)
    assert np.linalg.norm(x - ref) / np.linalg.norm(ref) <= 1e-10


def test_aggregates_respect_components_after_failures(shim):
    """Deactivate a band of elements (as strain failures do): aggregates stay
    inside components of the ACTIVE free graph, so an unloaded component keeps
    exactly zero iterates (the direct solve's answer there)."""
    xyz, e2n, top, bot = _golden22k()
    mid = xyz[:, 1].mean()
    y1, y2 = xyz[e2n[:, 0], 1], xyz[e2n[:, 1], 1]
    active = ~(((y1 - mid) * (y2 - mid) <= 0) & (np.abs(xyz[e2n[:, 0], 0] - xyz[:, 0].mean()) < 0.8))
    levels, Kff, b, perm = setup_case(shim, xyz, e2n, top, bot, active, 2)
    L0 = levels[0]
    n = L0["n"]
    G = sp.csr_matrix((np.ones(Kff.nnz), (Kff.tocoo().row // 2, Kff.tocoo().col // 2)), shape=(n, n))
    ncomp, lab = connected_components(G, directed=False)
    agg = L0["agg"]
    for a in np.unique(agg[agg >= 0]):
        assert len(np.unique(lab[agg == a])) == 1
    # a component with zero load stays exactly zero through the V-cycle
    z = amg_ref.vcycle(levels, b)
    bn = np.abs(b.reshape(-1, 2)).sum(1)
    for c in range(ncomp):
        m = lab == c
        if not np.any(bn[m]):
            assert not np.any(z.reshape(-1, 2)[m]), c
    ref = spsolve(Kff.tocsc(), b)
    x, _ = amg_ref.pcg(Kff, b, lambda r: amg_ref.vcycle(levels, r), rtol=1e-13)
    assert np.linalg.norm(x - ref) / np.linalg.norm(ref) <= 1e-10


def test_kept_hierarchy_over_failures(shim):
    """The hierarchy of the intact network kept over element failures (capi.hip
    ensure_amg, option amg_reuse): the plan of the intact set, the values of
    the failed one, and P_0's rows of floating pieces (no path to a grip,
    floating_free_rows) formed as zero.  The V-cycle stays SPD on the loaded
    part, PCG reaches the direct solve, and every floating row stays EXACTLY
    zero, as spsolve leaves it."""
    xyz, e2n, top, bot = _golden22k()
    rng = np.random.default_rng(3)
    active = (rng.random(len(e2n)) > 0.05).astype(np.uint8)
    # the failed set's K / b in the intact plan's level-0 order
    levels_f, Kff, b, nodes0 = setup_case(shim, xyz, e2n, top, bot, active, 2)
    # floating rows: the host routine against scipy's connected components
    nf = levels_f[0]["n"]
    fl = np.zeros(nf, np.uint8)
    n_fl = shim.shim_floating(_ptr(np.ascontiguousarray(active)), _ptr(fl))
    n = len(xyz)
    a = e2n[active.astype(bool)]
    _, lab = connected_components(sp.coo_matrix((np.ones(len(a)), (a[:, 0], a[:, 1])), shape=(n, n)),
                                  directed=False)
    anchored = np.zeros(lab.max() + 1, bool)
    anchored[lab[np.concatenate([top, bot])]] = True
    perm = np.empty(n, np.int32)
    _, G_, nsl = _pattern_sizes(shim, xyz, e2n, top, bot)
    junk = [np.empty(n, np.int32), np.empty(nsl + 1, np.int32), np.empty(G_, np.int32),
            np.empty(G_, np.int32), np.empty(n, np.uint8)]
    shim.shim_arrays(_ptr(perm), *[_ptr(j) for j in junk])
    assert np.array_equal(fl.astype(bool), ~anchored[lab[perm[:nf]]])
    assert n_fl > 10
    # the intact set's plan, the failed set's values
    val = np.zeros(6 * G_)
    diag = np.zeros(6 * n)
    shim.shim_sell_values(_ptr(active), EA, EI12, _ptr(val), _ptr(diag))
    levels = amg_ref.fetch_plan(shim, np.ones(len(e2n), np.uint8), 2)
    fm = fl[levels[0]["row0"]]
    amg_ref.numeric_setup(levels, val, diag, G_, n, 2, fmask=fm)
    # K / b in THIS plan's level-0 order
    Kf = fo.assemble_global_stiffness(xyz, e2n, active.astype(bool))
    dy = fo.DISPLACEMENT_MAX * 20 / (fo.N_STEPS - 1)
    known, vals = fo.known_dof_map(top, bot, dy, -dy)
    A3, b3, free = fo.free_system(Kf, known, vals)
    nodes = perm[:nf][levels[0]["row0"]]
    dofs = (nodes[:, None].astype(np.int64) * 3 + np.arange(2)).ravel()
    pos = np.searchsorted(free, dofs)
    K2, b2 = A3[pos][:, pos].tocsr(), b3[pos]
    assert _rel(levels[0]["A"], K2) <= 1e-15
    ref = spsolve(K2.tocsc(), b2)
    x, it = amg_ref.pcg(K2, b2, lambda r: amg_ref.vcycle(levels, r), rtol=1e-13, max_it=2000)
    assert np.linalg.norm(x - ref) / np.linalg.norm(ref) <= 1e-10
    fr = np.repeat(fm.astype(bool), 2)
    assert np.all(x[fr] == 0.0) and np.all(ref[fr] == 0.0)
    _, it8 = amg_ref.pcg(K2, b2, lambda r: amg_ref.vcycle(levels, r), rtol=1e-8, max_it=2000)
    assert it8 <= 60, it8
    print(f"kept hierarchy: {it8} iterations to 1e-8, {n_fl} floating rows")


def _pattern_sizes(shim, xyz, e2n, top, bot):
    xyz = np.ascontiguousarray(xyz, np.float64)
    e2n = np.ascontiguousarray(e2n, np.int64)
    top = np.ascontiguousarray(top, np.int64)
    bot = np.ascontiguousarray(bot, np.int64)
    sizes = np.zeros(5, np.int64)
    err = C.create_string_buffer(256)
    assert shim.shim_build(len(xyz), _ptr(xyz), len(e2n), _ptr(e2n), 0, len(top), _ptr(top), len(bot),
                           _ptr(bot), -1, _ptr(sizes), err, 256) == 0
    return int(sizes[0]), int(sizes[4]), int(sizes[3])


def test_compact_cycle_transfers_and_cycle(shim):
    """The compact cycle's plan (PT / RT patterns and index maps, csrc/amg_symbolic.cpp):
    P̃ = (I − ω D⁻¹ A) P and R̃ = P̃ᵀ exactly as SciPy forms them, and the two-sweep
    cycle equal to the four-step V(1,1) cycle (the same preconditioner)."""
    xyz, e2n, top, bot = _golden22k()
    levels, Kff, b, _ = setup_case(shim, xyz, e2n, top, bot, np.ones(len(e2n)), 2)
    amg_ref.compact_transfers(levels)
    for L in levels[:-1]:
        n, nd = L["n"], 2
        Dinv = sp.block_diag(list(L["dinv"]), format="csr")
        ref = (L["P"] - L["omega"] * (Dinv @ L["A"] @ L["P"])).tocsr()
        assert _rel(L["Pt"], ref) <= 1e-13
        assert _rel(L["Rt"], L["Pt"].T.tocsr()) == 0.0
        # every P block sits inside A·P's pattern: pt_p covers all of P's entries
        assert np.count_nonzero(L["pt_p"] >= 0) == np.count_nonzero(L["P.col"] >= 0)
    rng = np.random.default_rng(3)
    for _ in range(3):
        r = rng.standard_normal(Kff.shape[0])
        u4, u2 = amg_ref.vcycle(levels, r), amg_ref.vcycle_compact(levels, r)
        assert np.linalg.norm(u4 - u2) <= 1e-12 * np.linalg.norm(u4)
        us = amg_ref.vcycle_scaled(levels, r)   # the device's form: x only, R̂ and Ã
        assert np.linalg.norm(u4 - us) <= 1e-12 * np.linalg.norm(u4)


def test_spatial_labels_keep_the_hierarchy(shim):
    """Z-order row labels (amg.hpp AmgLayout): the same aggregates, so the same
    Galerkin products and the same PCG iteration count as depth-first labels,
    with the labels a permutation of the depth-first ones."""
    xyz, e2n, top, bot = _golden22k()
    shim.shim_amg_layout.argtypes = [C.c_int]
    shim.shim_amg_spatial.restype = C.c_int
    out = {}
    try:
        for sp_ in (0, 1):
            shim.shim_amg_layout(sp_)
            levels, Kff, b, nodes0 = setup_case(shim, xyz, e2n, top, bot, np.ones(len(e2n)), 2)
            assert shim.shim_amg_spatial() == sp_
            for l in range(len(levels) - 1):
                L, Nx = levels[l], levels[l + 1]
                assert _rel(Nx["A"], (L["P"].T @ L["A"] @ L["P"]).tocsr()) <= 1e-13
            _, it = amg_ref.pcg(Kff, b, lambda r: amg_ref.vcycle(levels, r), rtol=1e-8)
            out[sp_] = (it, [L["n"] for L in levels], np.sort(nodes0))
    finally:
        shim.shim_amg_layout(0)
    assert out[0][0] == out[1][0] and out[0][1] == out[1][1]
    assert np.array_equal(out[0][2], out[1][2])


def test_collapsed_cycle_equals_the_recursion(shim):
    """The compact cycle below level kc as one operator (amg_collapse.cpp): V_kc
    evaluated from the plan's product lists applies exactly the recursive
    compact cycle from level kc (2I − Ã, R̂, P̃ of every level below)."""
    xyz, e2n, top, bot = _golden22k()
    levels, Kff, b, _ = setup_case(shim, xyz, e2n, top, bot, np.ones(len(e2n)), 2)
    amg_ref.compact_transfers(levels)
    amg_ref.scaled_blocks(levels)
    shim.shim_amg_collapse.restype = C.c_int
    shim.shim_amg_collapse.argtypes = [C.c_int64, C.c_int64, C.c_int, C.c_char_p, C.c_int]
    shim.shim_coll_array.restype = C.c_int64
    shim.shim_coll_array.argtypes = [C.c_int, C.c_char_p, P]
    err = C.create_string_buffer(256)
    nlev = len(levels)
    for min_level in (nlev - 2, 1):
        kc = shim.shim_amg_collapse(1 << 40, 1 << 40, min_level, err, 256)
        assert kc == max(1, min_level), (kc, err.value)
        plan = {}
        for k in range(kc, nlev - 1):
            d = {}
            for name in ("T.sptr", "T.col", "tl.ptr", "tl.a", "tl.b", "V.sptr", "V.col", "vrow", "vl.ptr",
                         "vl.a", "vl.b", "va", "vdiag"):
                m = shim.shim_coll_array(k, name.encode(), None)
                a = np.zeros(max(m, 0), np.int32)
                if m > 0:
                    shim.shim_coll_array(k, name.encode(), a.ctypes.data_as(P))
                d[name] = a
            plan[k] = d
        V = amg_ref.collapsed_operator(levels, plan, kc)
        rng = np.random.default_rng(kc)
        for _ in range(2):
            x = rng.standard_normal(V.shape[0])
            ref = amg_ref.vcycle_scaled(levels, (kc, x))
            assert np.linalg.norm(V @ x - ref) <= 1e-12 * np.linalg.norm(ref), kc
    # a budget no level fits: no collapse
    assert shim.shim_amg_collapse(16, 1 << 40, 1, err, 256) == 0


@pytest.mark.parametrize("mesh", ["golden22k", "C2_1x5", "C5_2x2"])
def test_coarse_levels_spectral_radius_below_two(shim, mesh):
    """The coarse smoothers run at ω = 4 / (3 · 1.75) (capi.hip
    opt_amg_coarse_rho_ppm), over-relaxed against the Gershgorin-safe rule, so
    the V-cycle stays SPD only while ω·λmax(D_l⁻¹A_l) < 2, i.e. λmax < 2.625.
    Level 0 has λmax ≤ 2 exactly (A = Σ_e [[S,−S],[−S,S]] ≤ 2 D); the Galerkin
    levels measure ≤ 2 as well on the reference network, the tiled benchmark
    recipe and the chord (C5) recipe — 24 % under the limit — while their
    Gershgorin bounds reach 3.2.  (A solve that fails anyway falls back to the
    Gershgorin rule, test_gpu_amg.py::test_coarse_overrelaxation_fallback.)"""
    from mfea import synth
    if mesh == "golden22k":
        xyz, e2n, top, bot = _golden22k()
    else:
        nx, ny, ch = {"C2_1x5": (1, 5, False), "C5_2x2": (2, 2, True)}[mesh]
        xyz, e2n = synth.tiled_mesh(nx, ny, chords=ch)
        top, bot = synth.grips(xyz)
    levels, _, _, _ = setup_case(shim, xyz, e2n, top, bot, np.ones(len(e2n)), 2)
    rng = np.random.default_rng(3)
    for l, L in enumerate(levels):
        if L["coarsest"]:
            break
        M = (sp.block_diag(list(L["dinv"]), format="csr") @ L["A"]).tocsr()
        v = rng.standard_normal(M.shape[0])
        for _ in range(60):
            v = M @ v
            lam = np.linalg.norm(v)
            v /= lam
        assert lam <= 2.05, (mesh, l, lam, L["g"])
        if l > 0:
            assert L["omega"] * lam < 1.6, (mesh, l, L["omega"], lam)


def test_auto_form_choice_is_collective(shim):
    """with amg_dist −1 each rank times both GAMG forms of a
    partitioned solve and picks the faster; ranks on different forms issue
    different exchanges and hang.  capi.hip max-all-reduces each time over the
    ranks before the choice (max_over_ranks), so the choice (amg.hpp
    amg_auto_pending / amg_auto_choice) sees the same inputs everywhere.
    Two mocked ranks whose own timings disagree: local choices differ, the
    choices on the reduced timings agree."""
    shim.shim_amg_auto_pending.restype = C.c_int
    shim.shim_amg_auto_pending.argtypes = [C.c_double, C.c_double]
    shim.shim_amg_auto_choice.restype = C.c_int
    shim.shim_amg_auto_choice.argtypes = [C.c_double, C.c_double]
    # timing order: the global form first, then block Jacobi, then decide
    assert shim.shim_amg_auto_pending(-1.0, -1.0) == 1
    assert shim.shim_amg_auto_pending(-1.0, 2e-3) == 0
    assert shim.shim_amg_auto_pending(1e-3, 2e-3) == -1
    ranks = [(0.9e-3, 1.0e-3), (1.1e-3, 1.0e-3)]  # (block Jacobi, global) per rank
    local = [shim.shim_amg_auto_choice(*t) for t in ranks]
    assert local[0] != local[1]                     # what a per-rank choice would do
    tmax = tuple(max(t[k] for t in ranks) for k in range(2))
    assert [shim.shim_amg_auto_choice(*tmax) for _ in ranks] == [1, 1]
    assert shim.shim_amg_auto_choice(1e-3, 1e-3) == 1   # ties: the global hierarchy


def test_merged_levels_equal_the_compositions(shim):
    """Levels 0 and 1 merged around the level-2 collapse (amg.hpp AmgMerge,
    amg_collapse.cpp build_amg_merge): the DQ and U values the plan's lists
    give (amg.hip k_amg_mprod, here in f64) are exactly 2R̂₀ − Ã₁R̂₀, R̂₁R̂₀,
    P̃₀ and P̃₀P̃₁ — so the 3-launch cycle applies the same preconditioner."""
    xyz, e2n, top, bot = _golden22k()
    levels, Kff, b, _ = setup_case(shim, xyz, e2n, top, bot, np.ones(len(e2n)), 2)
    amg_ref.compact_transfers(levels)
    amg_ref.scaled_blocks(levels)
    nlev = len(levels)
    assert nlev >= 4
    shim.shim_amg_collapse.restype = C.c_int
    shim.shim_amg_collapse.argtypes = [C.c_int64, C.c_int64, C.c_int, C.c_char_p, C.c_int]
    shim.shim_amg_merge.restype = C.c_int
    shim.shim_amg_merge.argtypes = [C.c_char_p, C.c_int]
    shim.shim_merge_array.restype = C.c_int64
    shim.shim_merge_array.argtypes = [C.c_char_p, P]
    err = C.create_string_buffer(256)
    assert shim.shim_amg_collapse(1 << 40, 1 << 40, 2, err, 256) == 2, err.value
    assert shim.shim_amg_merge(err, 256) == 1, err.value

    def arr(name):
        m = shim.shim_merge_array(name.encode(), None)
        a = np.zeros(max(m, 0), np.int32)
        if m > 0:
            shim.shim_merge_array(name.encode(), a.ctypes.data_as(P))
        return a

    n0, n1, n2 = levels[0]["n"], levels[1]["n"], levels[2]["n"]
    assert shim.shim_merge_array(b"n1", None) == n1 and shim.shim_merge_array(b"n2", None) == n2
    split = shim.shim_merge_array(b"dq_split", None)
    L0, L1 = levels[0], levels[1]
    nd = L0["dinv"].shape[1]

    def evaluate(col, ext, ptr, la, lb, X, Y, E, f, sgn):
        out = np.zeros((len(col), nd, nd))
        for q in np.flatnonzero(col >= 0):
            acc = np.zeros((nd, nd))
            for t in range(ptr[q], ptr[q + 1]):
                acc = acc + X(q)[la[t]] @ Y[lb[t]]
            base = f * E[ext[q]] if ext[q] >= 0 else np.zeros((nd, nd))
            out[q] = base + sgn(q) * acc
        return out

    # DQ: c_1 rows (positions < split: Ã_1 × R̂_0, + 2 R̂_0), then x_2 rows (R̂_1 × R̂_0)
    dcol = arr("DQ.col")
    DQb = evaluate(dcol, arr("dq_ext"), arr("dq.ptr"), arr("dq.a"), arr("dq.b"),
                   lambda q: L1["Atb"] if q < split else L1["Rhb"], L0["Rhb"], L0["Rhb"], 2.0,
                   lambda q: -1.0 if q < split else 1.0)
    dst = arr("dq_dst")
    dq = amg_ref.to_scipy(DQb, arr("DQ.sptr"), dcol, len(dst), n0, nd).tocoo()
    rows = dst[dq.row // nd]
    keep_c1, keep_q = rows < n1, (rows >= n1) & (rows < n1 + n2)
    C1 = sp.csr_matrix((dq.data[keep_c1], (rows[keep_c1] * nd + dq.row[keep_c1] % nd, dq.col[keep_c1])),
                       shape=(n1 * nd, n0 * nd))
    Qm = sp.csr_matrix((dq.data[keep_q], ((rows[keep_q] - n1) * nd + dq.row[keep_q] % nd, dq.col[keep_q])),
                       shape=(n2 * nd, n0 * nd))
    R0 = amg_ref.to_scipy(L0["Rhb"], L0["RT.sptr"], L0["RT.col"], n1, n0, nd, L0["rt_row"])
    R1 = amg_ref.to_scipy(L1["Rhb"], L1["RT.sptr"], L1["RT.col"], n2, n1, nd, L1["rt_row"])
    A1 = amg_ref.to_scipy(L1["Atb"], L1["A.sptr"], L1["A.col"], n1, n1, nd)
    ref_c1 = (2.0 * R0 - A1 @ R0).toarray()
    assert np.abs(C1.toarray() - ref_c1).max() <= 1e-12 * np.abs(ref_c1).max()
    ref_q = (R1 @ R0).toarray()
    assert np.abs(Qm.toarray() - ref_q).max() <= 1e-12 * np.abs(ref_q).max()
    # U: P̃_0's row order; columns c_1 at [0, n1), e_2 at [n1 + n2, n1 + 2 n2)
    ucol = arr("U.col")
    Ub = evaluate(ucol, arr("u_ext"), arr("u.ptr"), arr("u.a"), arr("u.b"), lambda q: L0["PTb"], L1["PTb"],
                  L0["PTb"], 1.0, lambda q: 1.0)
    Ua = amg_ref.to_scipy(Ub, arr("U.sptr"), ucol, n0, n1 + 2 * n2, nd).tocoo()
    r = L0["pt_row"][Ua.row // nd] * nd + Ua.row % nd
    c = Ua.col // nd
    lo, hi = c < n1, c >= n1 + n2
    Pm = sp.csr_matrix((Ua.data[lo], (r[lo], Ua.col[lo])), shape=(n0 * nd, n1 * nd)).toarray()
    Wm = sp.csr_matrix((Ua.data[hi], (r[hi], Ua.col[hi] - (n1 + n2) * nd)), shape=(n0 * nd, n2 * nd)).toarray()
    assert np.abs(Pm - L0["Pt"].toarray()).max() <= 1e-12 * np.abs(Pm).max()
    ref_w = (L0["Pt"] @ L1["Pt"]).toarray()
    assert np.abs(Wm - ref_w).max() <= 1e-12 * np.abs(ref_w).max()
    # indices stay inside what the device arrays hold
    assert dst.max() <= n1 + 2 * n2 and ucol.max() < n1 + 2 * n2 and dcol.max() < n0
