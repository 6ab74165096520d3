"""CPU checks of the chain-piece sweep plan (amg.hpp SweepPlan, built by
amg_symbolic.cpp build_sweep for MFEA_PC_SOR / MFEA_PC_ICC) through the host
shim, and of the preconditioner it defines through the NumPy restatement
(tests/sweep_ref.py):
  * the plan covers every coupling of A_0 exactly once — predecessor /
    successor inside a piece, or a cross coupling to a piece of an earlier
    (lo) or later (up) colour — so nothing is dropped (the round-4 block
    Jacobi dropped every coupling between 256-row blocks);
  * IC(0) in the plan's order needs no more iterations than in the natural
    order PETSc uses (within 10 %), and at most 0.6× point-Jacobi PCG's."""
import ctypes as C

import numpy as np
import pytest

import sweep_ref
from conftest import build_host_shim, load_mesh
from test_amg_cpu import EA, EI12, _ptr  # noqa: F401  (shared constants)

import fea_oracle as fo  # noqa: E402  (checker only)

P = C.c_void_p


@pytest.fixture(scope="module")
def shim():
    lib = C.CDLL(build_host_shim())
    lib.shim_build.restype = C.c_int
    lib.shim_build.argtypes = [C.c_int64, P, C.c_int64, P, C.c_int, C.c_int64, P, C.c_int64, P,
                               C.c_int, P, C.c_char_p, C.c_int]
    lib.shim_arrays.argtypes = [P] * 6
    lib.shim_amg_levels.restype = C.c_int
    lib.shim_amg_levels.argtypes = [P, C.c_int, C.c_int, C.c_char_p, C.c_int]
    lib.shim_amg_array.restype = C.c_int64
    lib.shim_amg_array.argtypes = [C.c_int, C.c_char_p, P]
    lib.shim_sweep.restype = C.c_int
    lib.shim_sweep.argtypes = [C.c_int, C.c_char_p, C.c_int]
    return lib


def _arr(shim, name):
    k = shim.shim_amg_array(0, name.encode(), None)
    a = np.zeros(max(k, 1), np.int32)
    shim.shim_amg_array(0, name.encode(), _ptr(a))
    return a[:k]


def one_level_case(shim, xyz, e2n, top, bot, active, nd, piece_len=16):
    """the one-level plan + sweep plan; K_ff and b in level-0 row order"""
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
    assert shim.shim_amg_levels(_ptr(act), nd, 1, err, 256) == 1, err.value
    ncol = shim.shim_sweep(piece_len, err, 256)
    assert ncol > 0, err.value
    sw = sweep_ref.fetch_sweep(shim)
    row0 = _arr(shim, "row0")
    K = fo.assemble_global_stiffness(xyz, e2n, act.astype(bool))
    dy = fo.DISPLACEMENT_MAX * 20 / (fo.N_STEPS - 1)
    known, vals = fo.known_dof_map(top, bot, dy, -dy)
    A3, b3, free = fo.free_system(K, known, vals)
    nodes0 = perm[:nf][row0]
    dofs = (nodes0[:, None].astype(np.int64) * 3 + np.arange(nd)).ravel()
    pos = np.searchsorted(free, dofs)
    assert np.array_equal(free[pos], dofs)
    return sw, ncol, A3[pos][:, pos].tocsr(), b3[pos], nodes0


def _golden22k():
    nodes, elems = load_mesh("sim_20251117_181147")
    xyz = nodes[["x", "y", "z"]].values
    top, bot = fo.grip_nodes(xyz, nodes["node_id"].values, fo.GRIP_LENGTH)
    return xyz, elems[["n1", "n2"]].values, top, bot


def _cases():
    from mfea import synth
    xyz, e2n, top, bot = _golden22k()
    yield "sim181147", xyz, e2n, top, bot, np.ones(len(e2n), bool)
    rng = np.random.default_rng(3)
    yield "sim181147_failed", xyz, e2n, top, bot, rng.random(len(e2n)) > 0.05
    xyz, e2n = synth.tiled_mesh(2, 2, chords=True)
    top, bot = synth.grips(xyz)
    yield "C5_2x2", xyz, e2n, top, bot, np.ones(len(e2n), bool)


@pytest.mark.parametrize("case", ["sim181147", "sim181147_failed", "C5_2x2"])
@pytest.mark.parametrize("piece_len", [1, 16, 64])
def test_plan_covers_every_coupling_once(shim, case, piece_len):
    name, xyz, e2n, top, bot, active = next(c for c in _cases() if c[0] == case)
    sw, ncol, K, b, _ = one_level_case(shim, xyz, e2n, top, bot, active, 2, piece_len)
    sptr, col = _arr(shim, "A.sptr"), _arr(shim, "A.col")
    n = K.shape[0] // 2
    row = sw["row"]
    valid = row >= 0
    assert np.array_equal(np.sort(row[valid]), np.arange(n))
    ent = np.empty(n, np.int64)
    ent[row[valid]] = np.nonzero(valid)[0]
    colour = sweep_ref.entry_colour(sw)
    assert colour.max() + 1 == ncol <= 32
    # wave layout: pieces packed from lane 0, padding only at a wave's end
    r = row.reshape(-1, 64)
    assert np.all(np.diff((r >= 0).astype(int), axis=1) <= 0)
    assert len(sw["wsteps"]) == len(r)
    pos_row = lambda q: 64 * np.searchsorted(sptr, q // 64, side="right") - 64 + q % 64  # noqa: E731
    for i in range(n):
        e = ent[i]
        s0 = i >> 6
        base = sptr[s0] * 64 + (i & 63)
        qs = base + 64 * np.arange(sptr[s0 + 1] - sptr[s0])
        nb = {int(col[q]): int(q) for q in qs[1:] if col[q] >= 0 and col[q] != i}
        assert sw["dpos"][e] == base and col[base] == i
        got = {}
        if sw["ppos"][e] >= 0:   # predecessor: the previous lane of the wave
            assert e % 64 > 0 and row[e - 1] >= 0
            got[int(row[e - 1])] = int(sw["ppos"][e])
        if e % 64 < 63 and row[e + 1] >= 0 and sw["ppos"][e + 1] >= 0:
            got[int(row[e + 1])] = -1        # successor: its block is the successor's ppos
        for lst, cmp in (("lo", np.less), ("up", np.greater)):
            a, z = sw[lst + "_ptr"][e], sw[lst + "_ptr"][e + 1]
            for t in range(a, z):
                je = sw[lst + "_ent"][t]
                assert cmp(colour[je], colour[e])
                j = int(row[je])
                assert j not in got
                got[j] = int(sw[lst + "_pos"][t])
        assert set(got) == set(nb), i
        for j, q in got.items():
            if q >= 0:
                assert q == nb[j] and pos_row(q) == i
    # no two pieces of one colour couple: checked above through the lo / up
    # colour order; pieces of one row each make a point colouring
    if piece_len == 1:
        assert np.all(sw["ppos"] < 0)
    # scan steps cover every piece: ⌈log₂ length⌉ of the wave's longest
    starts = (row >= 0) & (sw["ppos"] < 0)
    pid = np.cumsum(starts) - 1
    lens = np.bincount(pid[row >= 0])
    wave_of = np.nonzero(starts)[0] // 64
    for wv, L in zip(wave_of, lens):
        assert (1 << sw["wsteps"][wv]) >= L


@pytest.mark.parametrize("case", ["sim181147", "C5_2x2"])
def test_icc_order_as_strong_as_natural(shim, case):
    """IC(0) / SSOR in the plan's order against the natural order (PETSc's),
    block Jacobi and point Jacobi, PCG to rtol 1e-8 on the same system."""
    name, xyz, e2n, top, bot, active = next(c for c in _cases() if c[0] == case)
    sw, ncol, K, b, nodes0 = one_level_case(shim, xyz, e2n, top, bot, active, 2, 64)
    order = sweep_ref.elimination_order(sw)
    p = sweep_ref.block_perm(order, 2)
    Kp, bp = K[p][:, p].tocsr(), b[p]
    it_icc, x = sweep_ref.pcg(Kp, bp, sweep_ref.preconditioner(Kp, 2, "dic"))
    it_sor, _ = sweep_ref.pcg(Kp, bp, sweep_ref.preconditioner(Kp, 2, "ssor"))
    # the natural order: original node order (level-0 rows sorted by node id)
    pn = sweep_ref.block_perm(np.argsort(nodes0), 2)
    Kn, bn = K[pn][:, pn].tocsr(), b[pn]
    it_nat, _ = sweep_ref.pcg(Kn, bn, sweep_ref.preconditioner(Kn, 2, "dic"))
    dinv = 1.0 / K.diagonal()
    it_jac, _ = sweep_ref.pcg(K, b, lambda r: dinv * r)
    assert it_icc > 0 and it_sor > 0 and it_nat > 0 and it_jac > 0
    assert it_icc <= 1.10 * it_nat, (it_icc, it_nat)
    assert it_icc <= 0.6 * it_jac, (it_icc, it_jac)
    assert it_sor < it_jac
    assert np.linalg.norm(Kp @ x - bp) <= 1e-8 * np.linalg.norm(bp) * 1.0001
    print(f"{case}: colours {ncol}, pieces {sw['n_pieces']}, icc {it_icc} (natural {it_nat}), "
          f"sor {it_sor}, jacobi {it_jac}")
