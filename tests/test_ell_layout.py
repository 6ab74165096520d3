"""CPU checks of the wave-local CG operator layout (symbolic.cpp build_ell):
every free-neighbour slot lands in exactly one lane, groups never straddle a
wave, in-wave sources point at the neighbour's owner lane, halo slots sit in
slot 0 with a symmetric partner, and an emulation of the kernel's SpMV over
the lanes equals the SELL SpMV."""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

from conftest import build_host_shim
import test_host_cpu as T

P = C.c_void_p
NONE, HALO = 0xFF, 0xFE


@pytest.fixture(scope="module")
def lib():
    lib = C.CDLL(build_host_shim())
    lib.shim_build.restype = C.c_int
    lib.shim_build.argtypes = [C.c_int64, P, C.c_int64, P, C.c_int, C.c_int64, P, C.c_int64, P,
                               C.c_int, P, C.c_char_p, C.c_int]
    lib.shim_arrays.argtypes = [P] * 6
    lib.shim_ell.restype = C.c_int64
    lib.shim_ell.argtypes = [P] * 7 + [C.c_char_p, C.c_int]
    return lib


def ell(lib, pat):
    err = C.create_string_buffer(256)
    n = lib.shim_ell(None, None, None, None, None, None, None, err, 256)
    assert n >= 0, err.value
    nf = pat["n_free"]
    out = {"n": int(n), "lane_row": np.empty(n, np.int32), "row_lane": np.empty(nf, np.int32),
           "info": np.empty(n, np.int32), "code": np.empty(n, np.uint32),
           "partner": np.empty(n, np.int32), "src_pos": np.empty(3 * n, np.int32),
           "nbr_lane": np.empty(3 * n, np.int32)}
    if n:
        lib.shim_ell(*(T.ptr(out[k]) for k in ("lane_row", "row_lane", "info", "code", "partner",
                                                "src_pos", "nbr_lane")), err, 256)
    out["src_pos"] = out["src_pos"].reshape(3, n)
    out["nbr_lane"] = out["nbr_lane"].reshape(3, n)
    return out


def sell_slots(pat):
    """(row, pos, col) of every free row's free-neighbour slot."""
    nf, sp, rl, sc = pat["n_free"], pat["slice_ptr"], pat["row_len"], pat["s_col"]
    rows, poss = [], []
    for i in range(nf):
        s, l = divmod(i, 64)
        for k in range(rl[i]):
            pos = (sp[s] + k) * 64 + l
            if sc[pos] < nf:
                rows.append(i)
                poss.append(pos)
    rows, poss = np.array(rows, np.int64), np.array(poss, np.int64)
    return rows, poss, sc[poss] if len(poss) else poss


def check_layout(pat, L):
    nf, n = pat["n_free"], L["n"]
    assert n % 64 == 0
    if nf == 0:
        assert n == 0
        return
    lr, rl_, info, code, partner = L["lane_row"], L["row_lane"], L["info"], L["code"], L["partner"]
    assert (lr[rl_] == np.arange(nf)).all()
    owners = np.flatnonzero(lr >= 0)
    assert len(owners) == nf
    for l0 in owners:
        g = info[l0] + 1
        assert l0 // 64 == (l0 + g - 1) // 64, "group straddles a wave"
        for t in range(1, g):
            assert info[l0 + t] == -t and lr[l0 + t] == -1
    # slot coverage
    rows, poss, cols = sell_slots(pat)
    sp = L["src_pos"]
    got = np.sort(sp[sp >= 0])
    assert (got == np.sort(poss)).all(), "every free-neighbour slot exactly once"
    owner_of = np.empty(n, np.int64)
    for l in range(n):
        owner_of[l] = l + info[l] if info[l] < 0 else l
    col_of = dict(zip(poss.tolist(), cols.tolist()))
    row_of = dict(zip(poss.tolist(), rows.tolist()))
    for k in range(3):
        srcs = (code >> (8 * k)) & 0xFF
        for l in np.flatnonzero(sp[k] >= 0):
            pos = int(sp[k, l])
            i, j = row_of[pos], col_of[pos]
            assert lr[owner_of[l]] == i
            assert L["nbr_lane"][k, l] == rl_[j]
            same = rl_[j] // 64 == l // 64
            if same:
                assert srcs[l] == rl_[j] % 64
            else:
                assert k == 0 and srcs[l] == HALO
        assert (srcs[sp[k] < 0] == NONE).all()
    halo = (code & 0xFF) == HALO
    assert (partner[~halo] == -1).all()
    hl = np.flatnonzero(halo)
    assert (partner[hl] >= 0).all() and (partner[partner[hl]] == hl).all()
    assert halo[partner[hl]].all()


def ell_spmv(pat, L, val, u_row, diag):
    """Emulates the kernel's SpMV over the lanes: y_owner = D u + Σ own slots +
    Σ helpers (in order).  val: per SELL position 3×3 blocks; diag per row."""
    n, nf = L["n"], pat["n_free"]
    lr, info, sp = L["lane_row"], L["info"], L["src_pos"]
    u_lane = np.zeros((n, 3))
    u_lane[lr >= 0] = u_row[lr[lr >= 0]]
    y = np.zeros((n, 3))
    for l in range(n):
        if lr[l] >= 0:
            y[l] = diag[lr[l]] @ u_lane[l]
        for k in range(3):
            pos = sp[k, l]
            if pos >= 0:
                y[l] += val[pos] @ u_lane[L["nbr_lane"][k, l]]
    out = np.zeros((nf, 3))
    for l0 in np.flatnonzero(lr >= 0):
        acc = y[l0].copy()
        for t in range(1, info[l0] + 1):
            acc += y[l0 + t]
        out[lr[l0]] = acc
    return out


def sell_spmv(pat, val, u_row, diag):
    rows, poss, cols = sell_slots(pat)
    y = np.einsum("nab,nb->na", diag, u_row)
    np.add.at(y, rows, np.einsum("nab,nb->na", val[poss], u_row[cols]))
    return y


def meshes():
    from mfea import synth
    xyz, e2n = synth.tiled_mesh(1, 2)
    top, bot = synth.grips(xyz)
    yield "tiled1x2", xyz, e2n, top, bot
    nodes, elems = T.load_mesh("test_X")
    xyz = nodes[["x", "y", "z"]].to_numpy()
    yield "test_X", xyz, elems[["n1", "n2"]].to_numpy(), [], []
    rng = np.random.default_rng(7)
    # a star: one node of degree 40 (many helpers, several waves)
    n = 200
    xyz = rng.normal(size=(n, 3))
    e2n = np.array([(0, i) for i in range(1, 41)] + [(i, i + 1) for i in range(41, n - 1)] +
                   [(5, 150), (5, 150), (60, 190)])
    yield "star", xyz, e2n, [n - 1], [41]


@pytest.mark.parametrize("case", list(range(3)))
def test_ell_layout_and_spmv(lib, case):
    name, xyz, e2n, top, bot = list(meshes())[case]
    pat = T.build(lib, xyz, e2n, top, bot, window=-1)
    L = ell(lib, pat)
    check_layout(pat, L)
    nf = pat["n_free"]
    rng = np.random.default_rng(case)
    G = len(pat["s_col"])
    val = rng.normal(size=(G, 3, 3))
    diag = rng.normal(size=(nf, 3, 3))
    u = rng.normal(size=(nf, 3))
    y_ell = ell_spmv(pat, L, val, u, diag)
    y_sell = sell_spmv(pat, val, u, diag)
    np.testing.assert_allclose(y_ell, y_sell, rtol=1e-12, atol=1e-12)


def test_ell_halo_fraction_tiled(lib):
    """On the DFS-ordered tiled network most slots resolve inside the wave."""
    from mfea import synth
    xyz, e2n = synth.tiled_mesh(1, 2)
    top, bot = synth.grips(xyz)
    pat = T.build(lib, xyz, e2n, top, bot, window=-1)
    L = ell(lib, pat)
    used = L["src_pos"] >= 0
    halo = ((L["code"] & 0xFF) == HALO).sum()
    assert halo / used.sum() < 0.2
    assert L["n"] < 1.15 * pat["n_free"]
