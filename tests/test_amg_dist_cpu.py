"""Distributed SA-AMG (csrc/amg_symbolic.cpp + csrc/amg_dist.cpp), no GPU.

The multi-GPU GAMG builds ONE global hierarchy on every rank and splits the
rows of its large levels over the ranks (amg.hpp AmgRank).  Checked here with
the NumPy restatement of the device arithmetic (tests/amg_ref.py):

* the hierarchy equals the one-partition hierarchy: the same level sizes and
  the same PCG iteration count to 1e-8 (the reference's solve,
  src/fea_solver.py:128, is the target either way);
* every rank's rows are one contiguous range per level, covering each level
  exactly once;
* the exchange plans are complete: a V-cycle run rank by rank — every rank
  with its own arrays, NaN wherever it holds no value, values moving only
  through the plans (each transfer checked against the sender's list) —
  gives the global V-cycle's output on every rank's rows, with no NaN;
* every value the numeric setup of a rank's rows reads is its own or arrives
  through the setup plans.
"""
import ctypes as C

import numpy as np
import pytest
import scipy.sparse as sp

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
    lib.shim_amg_array.restype = C.c_int64
    lib.shim_amg_array.argtypes = [C.c_int, C.c_char_p, P]
    lib.shim_amg_dist.restype = C.c_int
    lib.shim_amg_dist.argtypes = [P, C.c_int, C.c_int, P, C.c_int64, C.c_char_p, C.c_int]
    lib.shim_node_owner.restype = C.c_int
    lib.shim_node_owner.argtypes = [C.c_int64, P, C.c_int64, P, C.c_int64, P, C.c_int64, P, C.c_int, C.c_int,
                                    C.c_double, P]
    lib.shim_amg_rank.restype = C.c_int
    lib.shim_amg_rank.argtypes = [C.c_int, C.c_char_p, C.c_int]
    lib.shim_rank_array.restype = C.c_int64
    lib.shim_rank_array.argtypes = [C.c_char_p, C.c_int, P]
    lib.shim_level0_blocks.restype = C.c_int
    lib.shim_level0_blocks.argtypes = [C.c_int64, P, C.c_int64, P, C.c_int64, P, C.c_int64, P, C.c_int, C.c_int,
                                       C.c_double, P, C.c_int, C.c_double, C.c_double, C.c_double, P,
                                       C.c_char_p, C.c_int]
    return lib


def _p(a):
    return a.ctypes.data_as(P)


def _case(shim, xyz, e2n, top, bot, world, rep_rows, nd=2, active=None):
    """pattern, node owners, the (distributed) plan with its numeric setup, the
    reference system in level-0 order, and every rank's share."""
    xyz = np.ascontiguousarray(xyz, np.float64)
    e2n = np.ascontiguousarray(e2n, np.int64)
    top = np.ascontiguousarray(top, np.int64)
    bot = np.ascontiguousarray(bot, np.int64)
    N, E = len(xyz), len(e2n)
    sizes = np.zeros(5, np.int64)
    err = C.create_string_buffer(256)
    assert shim.shim_build(N, _p(xyz), E, _p(e2n), 0, len(top), _p(top), len(bot), _p(bot), -1, _p(sizes),
                           err, 256) == 0, err.value
    nf, G = int(sizes[0]), int(sizes[4])
    perm = np.empty(N, np.int32)
    junk = [np.empty(N, np.int32), np.empty(int(sizes[3]) + 1, np.int32), np.empty(G, np.int32),
            np.empty(G, np.int32), np.empty(N, np.uint8)]
    shim.shim_arrays(_p(perm), *[_p(j) for j in junk])
    act = np.ascontiguousarray(np.ones(E) if active is None else active, np.uint8)
    val, diag = np.zeros(6 * G), np.zeros(6 * N)
    shim.shim_sell_values(_p(act), EA, EI12, _p(val), _p(diag))
    owner = np.zeros(N, np.int32)
    shim.shim_node_owner(N, _p(xyz), E, _p(e2n), len(top), _p(top), len(bot), _p(bot), world, -1, 0.35, _p(owner))
    assert shim.shim_amg_dist(_p(act), nd, world, _p(owner), rep_rows, err, 256) > 0, err.value
    levels = amg_ref.fetch_plan(shim, act, nd, build=False)
    amg_ref.numeric_setup(levels, val, diag, G, N, nd)
    n_dist = shim.shim_amg_array(0, b"n_dist", None)
    K = fo.assemble_global_stiffness(xyz, e2n, act.astype(bool))
    known, vals = fo.known_dof_map(top, bot, 0.01, -0.01)
    A3, b3, free = fo.free_system(K, known, vals)
    nodes0 = perm[:nf][levels[0]["row0"]]
    dofs = (nodes0[:, None].astype(np.int64) * 3 + np.arange(nd)).ravel()
    pos = np.searchsorted(free, dofs)
    ranks = [_rank(shim, r, len(levels), n_dist) for r in range(world)]
    return levels, A3[pos][:, pos].tocsr(), b3[pos], n_dist, ranks


def _rank(shim, r, nlev, n_dist):
    err = C.create_string_buffer(256)
    assert shim.shim_amg_rank(r, err, 256) == n_dist, err.value

    def arr(name, l=0):
        n = shim.shim_rank_array(name.encode(), l, None)
        out = np.zeros(max(n, 0), np.int64)
        if n > 0:
            shim.shim_rank_array(name.encode(), l, _p(out))
        return out

    rk = {k: arr(k) for k in ("lo", "hi", "aplo", "aphi", "rlo", "rhi")}
    fields = ("peers", "soff", "scnt", "roff", "rcnt", "sidx", "ridx")
    for kind in ("xa", "xr", "xp", "sp", "sap"):
        rk[kind] = [{f: arr(f"{kind}.{f}", l) for f in fields} for l in range(n_dist)]
    for kind in ("xg", "sg", "xc", "spt", "sd"):
        rk[kind] = {f: arr(f"{kind}.{f}") for f in fields}
    for k in ("rtlo", "rthi", "compact"):
        rk[k] = int(arr(k)[0])
    return rk


def _xchg(ranks, plans, arrays):
    """Move values through one exchange: arrays[r] is rank r's array (items on
    axis 0); every received segment must be the sender's send segment."""
    W = len(ranks)
    for r in range(W):
        x = plans[r]
        for i, p in enumerate(x["peers"]):
            items = x["ridx"][x["roff"][i]:x["roff"][i] + x["rcnt"][i]]
            y = plans[p]
            k = int(np.flatnonzero(y["peers"] == r)[0])
            sent = y["sidx"][y["soff"][k]:y["soff"][k] + y["scnt"][k]]
            assert np.array_equal(sent, items)
            arrays[r][items] = arrays[p][items]


def _dist_vcycle(levels, ranks, n_dist, rvec, nd):
    """The schedule of capi.hip enqueue_gamg_vcycle, rank by rank."""
    W, nlev = len(ranks), len(levels)
    V = [[{k: np.full((L["n"], nd), np.nan) for k in "bxte"} for L in levels] for _ in range(W)]

    def rows(l, r):
        return slice(int(ranks[r]["lo"][l]), int(ranks[r]["hi"][l]))

    def mv(M, rs, v):  # rows rs (node rows) of M times v (n × nd)
        return (M[rs.start * nd:rs.stop * nd] @ v.reshape(-1)).reshape(-1, nd)

    r2 = rvec.reshape(-1, nd)
    for r in range(W):
        rs = rows(0, r)
        V[r][0]["b"][rs] = r2[rs]
        V[r][0]["x"][rs] = levels[0]["omega"] * np.einsum("iab,ib->ia", levels[0]["dinv"][rs], r2[rs])
    top = min(n_dist, nlev - 1)
    for l in range(top):
        L = levels[l]
        _xchg(ranks, [rk["xa"][l] for rk in ranks], [V[r][l]["x"] for r in range(W)])
        for r in range(W):
            rs = rows(l, r)
            V[r][l]["t"][rs] = V[r][l]["b"][rs] - mv(L["A"], rs, V[r][l]["x"])
        _xchg(ranks, [rk["xr"][l] for rk in ranks], [V[r][l]["t"] for r in range(W)])
        N = levels[l + 1]
        sc = 1.0 if N["coarsest"] else N["omega"]
        for r in range(W):
            cs = slice(int(ranks[r]["rlo"][l]), int(ranks[r]["rhi"][l]))
            bc = (L["P"].T.tocsr()[cs.start * nd:cs.stop * nd] @ V[r][l]["t"].reshape(-1)).reshape(-1, nd)
            V[r][l + 1]["b"][cs] = bc
            V[r][l + 1]["x"][cs] = sc * np.einsum("iab,ib->ia", N["dinv"][cs], bc)
    if n_dist < nlev:
        _xchg(ranks, [rk["xg"] for rk in ranks], [V[r][n_dist]["b"] for r in range(W)])
        for r in range(W):
            b = V[r][n_dist]["b"]
            assert not np.isnan(b).any()
            e = amg_ref.vcycle(levels, b.reshape(-1), n_dist).reshape(-1, nd)
            V[r][n_dist]["x" if levels[n_dist]["coarsest"] else "e"][:] = e
    for l in range(top - 1, -1, -1):
        L, N = levels[l], levels[l + 1]
        out = "x" if N["coarsest"] else "e"
        if l + 1 < n_dist:
            _xchg(ranks, [rk["xp"][l] for rk in ranks], [V[r][l + 1][out] for r in range(W)])
        for r in range(W):
            rs = rows(l, r)
            V[r][l]["x"][rs] = V[r][l]["x"][rs] + mv(L["P"], rs, V[r][l + 1][out])
        _xchg(ranks, [rk["xa"][l] for rk in ranks], [V[r][l]["x"] for r in range(W)])
        for r in range(W):
            rs = rows(l, r)
            y = V[r][l]["b"][rs] - mv(L["A"], rs, V[r][l]["x"])
            V[r][l]["e"][rs] = V[r][l]["x"][rs] + L["omega"] * np.einsum("iab,ib->ia", L["dinv"][rs], y)
    u = np.full((levels[0]["n"], nd), np.nan)
    for r in range(W):
        rs = rows(0, r)
        u[rs] = V[r][0]["e"][rs]
    return u.reshape(-1)


def _golden22k():
    nodes, elems = load_mesh("sim_20251117_181147")
    xyz = nodes[["x", "y", "z"]].values
    top, bot = fo.grip_nodes(xyz, nodes["node_id"].values, fo.GRIP_LENGTH)
    return xyz, elems[["n1", "n2"]].values, top, bot


@pytest.mark.parametrize("world,rep_rows", [(2, 500), (3, 300), (4, 60), (8, 500)])
def test_distributed_vcycle_equals_global(shim, world, rep_rows):
    xyz, e2n, top, bot = _golden22k()
    levels, Kff, b, n_dist, ranks = _case(shim, xyz, e2n, top, bot, world, rep_rows)
    assert n_dist >= 2  # at least one split level below level 0
    nlev = len(levels)
    # contiguous owner ranges covering every split level once
    for l in range(min(n_dist + 1, nlev)):
        own = levels[l]["owner"]
        assert len(own) == levels[l]["n"] and np.all(np.diff(own) >= 0)
    for l in range(nlev):
        spans = sorted((int(rk["lo"][l]), int(rk["hi"][l])) for rk in ranks)
        if l < n_dist:
            assert spans[0][0] == 0 and spans[-1][1] == levels[l]["n"]
            assert all(a[1] == b_[0] for a, b_ in zip(spans, spans[1:]))
        else:
            assert all(s == (0, levels[l]["n"]) for s in spans)
    rng = np.random.default_rng(world)
    r = rng.standard_normal(b.size)
    ud = _dist_vcycle(levels, ranks, n_dist, r, 2)
    ug = amg_ref.vcycle(levels, r)
    assert not np.isnan(ud).any()
    assert np.allclose(ud, ug, rtol=1e-12, atol=1e-12 * np.abs(ug).max())


@pytest.mark.parametrize("world", [2, 4, 8])
def test_distributed_setup_reads_only_owned_or_received(shim, world):
    xyz, e2n, top, bot = _golden22k()
    levels, _, _, n_dist, ranks = _case(shim, xyz, e2n, top, bot, world, 60)
    nlev = len(levels)
    for rk in ranks:
        for l in range(min(n_dist, nlev - 1)):
            L, N = levels[l], levels[l + 1]
            prow, _ = amg_ref.pos_rows(L["P.sptr"], L["n"])
            aprow, _ = amg_ref.pos_rows(L["AP.sptr"], L["n"])
            rrow, _ = amg_ref.pos_rows(L["R.sptr"], N["n"])
            crow, _ = amg_ref.pos_rows(N["A.sptr"], N["n"])
            lo, hi = rk["lo"][l], rk["hi"][l]
            p_ok = ((prow >= lo) & (prow < hi))
            p_ok[rk["sp"][l]["ridx"]] = True
            ap_ok = (aprow >= rk["aplo"][l]) & (aprow < rk["aphi"][l])
            ap_ok[rk["sap"][l]["ridx"]] = True
            mine_ap = np.flatnonzero((aprow >= rk["aplo"][l]) & (aprow < rk["aphi"][l]) & (L["AP.col"] >= 0))
            for q in mine_ap:
                assert p_ok[L["ap.b"][L["ap.ptr"][q]:L["ap.ptr"][q + 1]]].all()
            mine_r = np.flatnonzero((rrow >= rk["rlo"][l]) & (rrow < rk["rhi"][l]) & (L["R.col"] >= 0))
            assert p_ok[L["rp"][mine_r]].all()
            mine_c = np.flatnonzero((crow >= rk["rlo"][l]) & (crow < rk["rhi"][l]) & (N["A.col"] >= 0))
            for q in mine_c:
                s = slice(L["ac.ptr"][q], L["ac.ptr"][q + 1])
                assert p_ok[L["ac.a"][s]].all() and ap_ok[L["ac.b"][s]].all()
        if n_dist < nlev:  # the replicated level: own rows formed, the rest gathered
            G = levels[n_dist]
            grow, _ = amg_ref.pos_rows(G["A.sptr"], G["n"])
            ok = (grow >= rk["rlo"][n_dist - 1]) & (grow < rk["rhi"][n_dist - 1])
            ok[rk["sg"]["ridx"]] = True
            assert ok[(G["A.col"] >= 0) & (grow >= 0)].all()


def test_distributed_hierarchy_is_the_one_partition_hierarchy(shim):
    """Same aggregates → same level sizes and the same PCG iteration count as
    one partition (17 on this network at rtol 1e-8, tests/test_amg_cpu.py)."""
    xyz, e2n, top, bot = _golden22k()
    out = []
    for world in (1, 4):
        levels, Kff, b, n_dist, _ = _case(shim, xyz, e2n, top, bot, world, 500)
        _, it = amg_ref.pcg(Kff, b, lambda r: amg_ref.vcycle(levels, r), rtol=1e-8)
        out.append(([L["n"] for L in levels], it, n_dist))
    assert out[0][0] == out[1][0] and out[0][1] == out[1][1], out
    assert out[1][2] >= 2


@pytest.mark.parametrize("world", [2, 3, 4])
def test_rank_level0_from_partition_pattern(shim, world):
    """Each rank forms A_0's rows from ITS partition's assembled slots
    (build_amg_level0, the device's a0 lists): equal to the global A_0
    (K_ff + reg·I, src/fea_solver.py:115-125) row for row."""
    xyz, e2n, top, bot = _golden22k()
    levels, _, _, n_dist, ranks = _case(shim, xyz, e2n, top, bot, world, 500)
    x = np.ascontiguousarray(xyz, np.float64)
    e = np.ascontiguousarray(e2n, np.int64)
    t = np.ascontiguousarray(top, np.int64)
    b = np.ascontiguousarray(bot, np.int64)
    act = np.ones(len(e), np.uint8)
    Ab = levels[0]["Ab"]
    npos = Ab.shape[0]
    got = np.full((npos, 4), np.nan)
    err = C.create_string_buffer(256)
    for r in range(world):
        assert shim.shim_level0_blocks(len(x), _p(x), len(e), _p(e), len(t), _p(t), len(b), _p(b), world, r, 0.35,
                                       _p(act), 2, EA, EI12, 1e-12, _p(got), err, 256) == 0, err.value
    row, _ = amg_ref.pos_rows(levels[0]["A.sptr"], levels[0]["n"])
    valid = (row >= 0) & (levels[0]["A.col"] >= 0)
    ref = Ab.reshape(npos, 4)[valid]
    mine = got[valid]
    assert not np.isnan(mine).any()
    assert np.allclose(mine, ref, rtol=1e-14, atol=1e-14 * np.abs(ref).max())


def _compact_dist_vcycle(levels, ranks, rvec, nd):
    """The compact schedule of capi.hip enqueue_gamg_vcycle (AmgRank::compact:
    level 0 split, every level below replicated), rank by rank with NaN
    wherever a rank holds no value: x_0 on its rows, the xc halo, down_0 (its
    Ã_0 rows → c_0, its R̂_0 rows → x_1), the x_1 all-gather (xg), the
    replicated cycle from level 1, up_0 on its P̃_0 rows."""
    W = len(ranks)
    L0, N = levels[0], levels[1]
    blk = lambda M: sp.block_diag(list(M), format="csr")  # noqa: E731
    s_n = 1.0 if N["coarsest"] else N["omega"]
    Rhat = (s_n * blk(N["dinv"]) @ L0["Rt"] @ blk(np.linalg.inv(L0["dinv"])) / L0["omega"]).tocsr()
    At = (L0["omega"] * blk(L0["dinv"]) @ L0["A"]).tocsr()
    r2 = rvec.reshape(-1, nd)
    x0 = [np.full(r2.shape, np.nan) for _ in range(W)]
    x1 = [np.full((N["n"], nd), np.nan) for _ in range(W)]
    c0 = [np.full(r2.shape, np.nan) for _ in range(W)]
    for r, rk in enumerate(ranks):
        rs = slice(int(rk["lo"][0]), int(rk["hi"][0]))
        x0[r][rs] = L0["omega"] * np.einsum("iab,ib->ia", L0["dinv"][rs], r2[rs])
    _xchg(ranks, [rk["xc"] for rk in ranks], x0)

    def rows_of(M, idx, v):  # rows idx (node rows) of M times v; NaN if a read value is missing
        d = (idx[:, None] * nd + np.arange(nd)).ravel()
        sub = M[d]
        vv = v.reshape(-1)
        cols = np.unique(sub.indices)
        assert not np.isnan(vv[cols]).any(), "a read value neither owned nor received"
        return (sub @ np.nan_to_num(vv)).reshape(-1, nd)

    for r, rk in enumerate(ranks):
        own = np.arange(int(rk["lo"][0]), int(rk["hi"][0]))
        c0[r][own] = 2.0 * x0[r][own] - rows_of(At, own, x0[r])
        rows1 = L0["rt_row"][int(rk["rtlo"]):int(rk["rthi"])]
        x1[r][rows1] = rows_of(Rhat, rows1, x0[r])
    _xchg(ranks, [rk["xg"] for rk in ranks], x1)
    u = np.full(r2.shape, np.nan)
    for r, rk in enumerate(ranks):
        assert not np.isnan(x1[r]).any()
        e1 = amg_ref.vcycle_scaled(levels, (1, x1[r].reshape(-1))).reshape(-1, nd)
        rows0 = L0["pt_row"][int(rk["aplo"][0]):int(rk["aphi"][0])]
        u[rows0] = c0[r][rows0] + rows_of(L0["Pt"], rows0, e1)
    return u.reshape(-1)


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_compact_distributed_vcycle_equals_global(shim, world):
    """The compact distributed cycle (level 0 split over the ranks, every level
    below replicated: capi.hip enqueue_gamg_vcycle's AmgRank::compact branch)
    gives the one-partition compact cycle's output on every rank's rows,
    every value it reads owned or received through xc / xg; its R̂_0 rows
    cover level 1 once; its setup reads only owned or received P̃_0 blocks
    (spt) and level-0 diagonal blocks (sd)."""
    xyz, e2n, top, bot = _golden22k()
    levels, Kff, b, n_dist, ranks = _case(shim, xyz, e2n, top, bot, world, 1 << 40)
    assert n_dist == 1 and all(rk["compact"] for rk in ranks)
    amg_ref.compact_transfers(levels)
    L0, N = levels[0], levels[1]
    spans = sorted((rk["rtlo"], rk["rthi"]) for rk in ranks)
    assert spans[0][0] == 0 and spans[-1][1] == N["n"]
    assert all(a[1] == b_[0] for a, b_ in zip(spans, spans[1:]))
    for rk_i, rk in enumerate(ranks):  # R̂_0 rows of rank r produce level-1 rows r owns
        rows1 = L0["rt_row"][rk["rtlo"]:rk["rthi"]]
        assert np.all(N["owner"][rows1] == rk_i)
    rng = np.random.default_rng(world)
    r = rng.standard_normal(b.size)
    ud = _compact_dist_vcycle(levels, ranks, r, 2)
    ug = amg_ref.vcycle_scaled(levels, r)
    assert not np.isnan(ud).any()
    assert np.allclose(ud, ug, rtol=1e-12, atol=1e-12 * np.abs(ug).max())
    # the R̂_0 setup: P̃_0 positions and diagonal blocks read, owned or received
    ptrow, _ = amg_ref.pos_rows(L0["PT.sptr"], L0["n"])
    rtrow, _ = amg_ref.pos_rows(L0["RT.sptr"], N["n"])
    arow, ak = amg_ref.pos_rows(L0["A.sptr"], L0["n"])
    for rk in ranks:
        pt_ok = (ptrow >= rk["aplo"][0]) & (ptrow < rk["aphi"][0])
        pt_ok[rk["spt"]["ridx"]] = True
        d_ok = (arow >= rk["lo"][0]) & (arow < rk["hi"][0]) & (ak == 0)
        d_ok[rk["sd"]["ridx"]] = True
        mine = np.flatnonzero((rtrow >= rk["rtlo"]) & (rtrow < rk["rthi"]) & (L0["RT.col"] >= 0))
        assert pt_ok[L0["rt_pt"][mine]].all()
        cols = L0["RT.col"][mine]
        dpos = np.array([np.flatnonzero((arow == c) & (ak == 0))[0] for c in np.unique(cols)])
        assert d_ok[dpos].all()
