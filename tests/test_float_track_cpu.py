"""The floating-row tracker (csrc/amg_symbolic.cpp FloatTracker), no GPU: kept
current over element failures by searches from the failed elements' ends, it
must give the same floating free rows as the whole-graph union-find
(floating_free_rows) on the activity after every failure — the rows the kept
GAMG hierarchy masks so that unloaded pieces stay at exactly zero, as the
reference's direct solve leaves them (src/fea_solver.py:128, 268-295)."""
import ctypes as C

import numpy as np
import pytest

import fea_oracle as fo
from conftest import build_host_shim, load_mesh

P = C.c_void_p


@pytest.fixture(scope="module")
def shim():
    lib = C.CDLL(build_host_shim())
    lib.shim_build.restype = C.c_int
    lib.shim_build.argtypes = [C.c_int64, P, C.c_int64, P, C.c_int, C.c_int64, P, C.c_int64, P,
                               C.c_int, P, C.c_char_p, C.c_int]
    lib.shim_floating.restype = C.c_int64
    lib.shim_floating.argtypes = [P, P]
    lib.shim_float_track.restype = C.c_int64
    lib.shim_float_track.argtypes = [P, C.c_int64, P, P, P]
    return lib


def _ptr(a):
    return a.ctypes.data_as(P)


def build(shim, xyz, e2n, top, bot):
    xyz = np.ascontiguousarray(xyz, np.float64)
    e2n = np.ascontiguousarray(e2n, np.int64)
    top = np.ascontiguousarray(top, np.int64)
    bot = np.ascontiguousarray(bot, np.int64)
    sizes = np.zeros(5, np.int64)
    err = C.create_string_buffer(256)
    assert shim.shim_build(len(xyz), _ptr(xyz), len(e2n), _ptr(e2n), 0, len(top), _ptr(top), len(bot),
                           _ptr(bot), -1, _ptr(sizes), err, 256) == 0, err.value
    return int(sizes[0])


def whole_pass(shim, active, nf):
    out = np.zeros(max(nf, 1), np.uint8)
    shim.shim_floating(_ptr(np.ascontiguousarray(active, np.uint8)), _ptr(out))
    return out[:nf]


def tracked(shim, active, fails, nf):
    act = np.ascontiguousarray(active, np.uint8).copy()
    ids = np.ascontiguousarray(fails, np.int32)
    fl = np.zeros(max(nf, 1), np.uint8)
    new = np.zeros(max(nf, 1), np.int32)
    n = shim.shim_float_track(_ptr(act), len(ids), _ptr(ids), _ptr(fl), _ptr(new))
    return act, fl[:nf], new[:n]


def _golden22k():
    nodes, elems = load_mesh("sim_20251117_181147")
    xyz = nodes[["x", "y", "z"]].values
    top, bot = fo.grip_nodes(xyz, nodes["node_id"].values, fo.GRIP_LENGTH)
    return xyz, elems[["n1", "n2"]].values, top, bot


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_tracker_matches_whole_graph_pass_over_failures(shim, seed):
    xyz, e2n, top, bot = _golden22k()
    nf = build(shim, xyz, e2n, top, bot)
    E = len(e2n)
    rng = np.random.default_rng(seed)
    order = rng.permutation(E)[: E // 6]
    start = np.ones(E, np.uint8)
    before = whole_pass(shim, start, nf)
    for k in (1, 10, 100, 400, 1250):  # prefixes of one failure sequence
        act, fl, new = tracked(shim, start, order[:k], nf)
        ref = whole_pass(shim, act, nf)
        assert np.array_equal(fl, ref), (k, int(fl.sum()), int(ref.sum()))
        # every newly floating row listed exactly once
        assert len(np.unique(new)) == len(new)
        assert np.array_equal(np.sort(new), np.flatnonzero(ref & ~before))


def test_tracker_whole_network_cut_off_from_the_grips(shim):
    """Every element at a grip fails: the loaded component loses all its grips
    to one-node pieces and the whole rest floats (the tracker's rest pass)."""
    xyz, e2n, top, bot = _golden22k()
    nf = build(shim, xyz, e2n, top, bot)
    grip = np.zeros(len(xyz), bool)
    grip[top] = grip[bot] = True
    cut = np.flatnonzero(grip[e2n[:, 0]] | grip[e2n[:, 1]])
    start = np.ones(len(e2n), np.uint8)
    act, fl, new = tracked(shim, start, cut, nf)
    ref = whole_pass(shim, act, nf)
    assert ref.all() and np.array_equal(fl, ref)
    before = whole_pass(shim, start, nf)
    assert np.array_equal(np.sort(new), np.flatnonzero(ref & ~before))


def test_tracker_from_a_partly_failed_start(shim):
    """The whole-graph pass of a set that already lost elements, then more
    failures (a kept hierarchy whose tracker was re-initialised)."""
    xyz, e2n, top, bot = _golden22k()
    nf = build(shim, xyz, e2n, top, bot)
    rng = np.random.default_rng(7)
    start = (rng.random(len(e2n)) > 0.05).astype(np.uint8)
    live = np.flatnonzero(start)
    fails = rng.permutation(live)[:800]
    act, fl, _ = tracked(shim, start, fails, nf)
    assert np.array_equal(fl, whole_pass(shim, act, nf))
