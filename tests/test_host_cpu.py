"""Host logic of the engine, no GPU: the symbolic phase (free/known permutation,
SELL-64 node-block layout), the CSR export, the C ABI surface, the CPU
baseline, the synthetic generator and the CSV writers."""
import ctypes as C
import glob
import os
import re

import numpy as np
import pytest
import scipy.sparse as sp

import fea_oracle as fo
from conftest import GOLDEN, PKG, REPO, build_host_shim, load_mesh, read_rt

P = C.c_void_p


@pytest.fixture(scope="module")
def shim():
    lib = C.CDLL(build_host_shim())
    lib.shim_build.restype = C.c_int
    lib.shim_build.argtypes = [C.c_int64, P, C.c_int64, P, C.c_int, C.c_int64, P, C.c_int64, P,
                               C.c_int, P, C.c_char_p, C.c_int]
    lib.shim_arrays.argtypes = [P] * 6
    lib.shim_export.restype = C.c_int64
    lib.shim_export.argtypes = [P, C.c_double, C.c_double, P, P, P]
    return lib


def ptr(a):
    return a.ctypes.data_as(P)


def build(shim, xyz, e2n, top=(), bot=(), skip=False, window=512):
    xyz = np.ascontiguousarray(xyz, np.float64)
    e2n = np.ascontiguousarray(e2n, np.int64)
    top = np.ascontiguousarray(top, np.int64)
    bot = np.ascontiguousarray(bot, np.int64)
    sizes = np.zeros(5, np.int64)
    err = C.create_string_buffer(256)
    rc = shim.shim_build(len(xyz), ptr(xyz), len(e2n), ptr(e2n), int(skip), len(top), ptr(top),
                         len(bot), ptr(bot), window, ptr(sizes), err, 256)
    if rc:
        raise ValueError(err.value.decode())
    N = len(xyz)
    out = {"n_free": int(sizes[0]), "n_top": int(sizes[1]), "n_known": int(sizes[2]),
           "perm": np.empty(N, np.int32), "row_len": np.empty(N, np.int32),
           "slice_ptr": np.empty(int(sizes[3]) + 1, np.int32),
           "s_col": np.empty(int(sizes[4]), np.int32), "s_elem": np.empty(int(sizes[4]), np.int32),
           "code": np.empty(N, np.uint8)}
    shim.shim_arrays(ptr(out["perm"]), ptr(out["row_len"]), ptr(out["slice_ptr"]),
                     ptr(out["s_col"]), ptr(out["s_elem"]), ptr(out["code"]))
    return out


def export(shim, n_nodes, active):
    a = np.ascontiguousarray(active, np.uint8)
    EA = fo.E_MOD * fo.AREA
    EI12 = (12 * fo.E_MOD) * fo.INERTIA
    nnz = shim.shim_export(ptr(a), EA, EI12, None, None, None)
    ip = np.empty(3 * n_nodes + 1, np.int64)
    ix = np.empty(nnz, np.int32)
    dv = np.empty(nnz)
    shim.shim_export(ptr(a), EA, EI12, ptr(ip), ptr(ix), ptr(dv))
    return sp.csr_matrix((dv, ix, ip), shape=(3 * n_nodes, 3 * n_nodes))


def _mesh(name):
    nodes, elems = load_mesh(name)
    return nodes, nodes[["x", "y", "z"]].values, elems[["n1", "n2"]].values


# ---------------------------------------------------------------------------
def test_permutation_free_first_then_top_then_bottom(shim):
    nodes, xyz, e2n = _mesh("sim_20251117_181147")
    top, bot = fo.grip_nodes(xyz, nodes["node_id"].values, 1.5)
    p = build(shim, xyz, e2n, top, bot)
    perm = p["perm"]
    assert sorted(perm.tolist()) == list(range(len(xyz)))
    known = set(top.tolist()) | set(bot.tolist())
    assert p["n_free"] == len(xyz) - len(known)
    assert not (set(perm[: p["n_free"]].tolist()) & known)
    assert perm[p["n_free"]: p["n_free"] + p["n_top"]].tolist() == list(top)
    # bottom value overrides top (src/fea_solver.py:226-242)
    inv = np.empty_like(perm)
    inv[perm] = np.arange(len(perm))
    for n in set(top.tolist()) & set(bot.tolist()):
        assert p["code"][inv[n]] == 2
    for n in set(top.tolist()) - set(bot.tolist()):
        assert p["code"][inv[n]] == 1


def test_sell_slots_hold_incident_elements_in_id_order(shim):
    nodes, xyz, e2n = _mesh("sim_20251117_175809")
    top, bot = fo.grip_nodes(xyz, nodes["node_id"].values, 1.5)
    p = build(shim, xyz, e2n, top, bot)
    perm, inv = p["perm"], np.empty_like(p["perm"])
    inv[perm] = np.arange(len(perm))
    inc = [[] for _ in range(len(xyz))]
    for e, (a, b) in enumerate(e2n):
        if a != b:
            inc[a].append(e)
            inc[b].append(e)
    ns = len(p["slice_ptr"]) - 1
    for s in range(ns):
        rows = range(64 * s, min(64 * s + 64, len(xyz)))
        width = p["slice_ptr"][s + 1] - p["slice_ptr"][s]
        assert width == max(p["row_len"][r] for r in rows)
        for r in rows:
            n = perm[r]
            assert p["row_len"][r] == len(inc[n])
            for k in range(width):
                idx = (p["slice_ptr"][s] + k) * 64 + (r - 64 * s)
                if k < p["row_len"][r]:
                    e = inc[n][k]
                    assert p["s_elem"][idx] == e
                    other = e2n[e, 1] if e2n[e, 0] == n else e2n[e, 0]
                    assert p["s_col"][idx] == inv[other]
                else:
                    assert p["s_elem"][idx] == -1 and p["s_col"][idx] == -1


@pytest.mark.parametrize("mesh", ["test_X", "sim_20251117_175809", "sim_20251115_135507"])
def test_export_csr_matches_reference_pattern(shim, mesh):
    nodes, xyz, e2n = _mesh(mesh)
    z = np.load(os.path.join(GOLDEN, f"K0_{mesh}.npz"))
    build(shim, xyz, e2n)
    K = export(shim, len(xyz), np.ones(len(e2n), np.uint8))
    assert np.array_equal(K.indptr, z["indptr"])
    assert np.array_equal(K.indices, z["indices"])
    bound = 16 * np.finfo(float).eps * fo.assemble_magnitude(xyz, e2n, np.ones(len(e2n), bool)).data
    assert np.all(np.abs(K.data - z["data"]) <= bound)


def test_export_csr_with_inactive_elements(shim):
    nodes, xyz, e2n = _mesh("sim_20251117_181147")
    active = (np.arange(len(e2n)) % 3) != 0
    build(shim, xyz, e2n)
    K = export(shim, len(xyz), active.astype(np.uint8))
    Kr = fo.assemble_global_stiffness(xyz, e2n, active)
    assert np.array_equal(K.indptr, Kr.indptr)
    assert np.array_equal(K.indices, Kr.indices)
    bound = 16 * np.finfo(float).eps * fo.assemble_magnitude(xyz, e2n, active).data
    assert np.all(np.abs(K.data - Kr.data) <= bound)


def test_out_of_range_elements_rejected_or_skipped(shim):
    """test_X_cpp_2: elements reference nodes 7–14 but only 0–6 exist.  The
    Python reference raises (src/fea_solver.py:82-83); the PETSc code skips
    them (src/fea_petsc.cpp:241) — MFEA_MESH_SKIP_INVALID."""
    nodes, xyz, e2n = _mesh("test_X_cpp_2")
    with pytest.raises(ValueError, match="out of range"):
        build(shim, xyz, e2n)
    p = build(shim, xyz, e2n, skip=True)
    valid = (e2n < len(xyz)).all(axis=1)
    assert p["row_len"].sum() == 2 * valid.sum()


def test_self_loop_elements_are_excluded():
    pass  # covered by the C++ builder (deg excludes a == b); kept as a marker


# ---------------------------------------------------------------------------
def test_library_exports_every_declared_symbol():
    header = "".join(open(f).read() for f in glob.glob(os.path.join(REPO, "include", "*.h")))
    declared = set(re.findall(r"^\s*(?:int|void)\s+(mfea_\w+)\s*\(", header, re.M))
    assert len(declared) >= 20
    lib = C.CDLL(os.path.join(PKG, "libmfea.so"))
    for name in declared:
        assert hasattr(lib, name), name
    from mfea import _capi
    assert declared == set(_capi.EXPORTED)
    assert _capi.abi_version() == 8


def test_create_without_gpu_fails_cleanly():
    from mfea import _capi
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except ImportError:
        pass
    with pytest.raises(_capi.MfeaError) as ei:
        _capi.Engine(0)
    assert ei.value.code == _capi.EDEVICE


# ---------------------------------------------------------------------------
def test_cpu_baseline_matches_direct_solve():
    import cpu_fea
    z = np.load(os.path.join(GOLDEN, "sys_sim_20251117_181147_step20.npz"))
    nodes, xyz, e2n = _mesh("sim_20251117_181147")
    top, bot = fo.grip_nodes(xyz, nodes["node_id"].values, 1.5)
    c = cpu_fea.CpuFea(xyz, e2n, top, bot, fo.E_MOD, fo.AREA, fo.INERTIA)
    dy = float(z["dy"])
    r = c.step(dy, -dy, rtol=1e-8, threads=4)
    assert abs(r["iters"] - int(z["pcg_iters_1e8"])) <= 3
    c.active[:] = 1
    r = c.step(dy, -dy, rtol=1e-13, threads=4)
    assert np.linalg.norm(r["U"] - z["U"]) / np.linalg.norm(z["U"]) <= 1e-10
    K = fo.assemble_global_stiffness(xyz, e2n, np.ones(len(e2n), bool))
    F = (K @ z["U"])[[3 * t + 1 for t in top]].sum()
    assert abs(r["force"] - F) <= 1e-9 * abs(F)


def test_synthetic_generator_sizes():
    from mfea import synth
    for (nx, ny), (nn, ne) in {(1, 4): (29500, 30301), (4, 4): (118000, 121252)}.items():
        xyz, e2n = synth.tiled_mesh(nx, ny)
        assert (len(xyz), len(e2n)) == (nn, ne)
    xyz, e2n = synth.tiled_mesh(1, 5)
    assert 3 * len(xyz) == 110625


def test_petsc_writer_reproduces_cpp_golden_text(tmp_path):
    """fea_solver.py --format petsc (csrc/records.cpp's ostream dialect) writes
    fea_petsc.cpp's text byte for byte (src/fea_petsc.cpp:433-516)."""
    import fea_solver as fs
    ref = os.path.join(GOLDEN, "ref", "test_I_cpp")
    st = read_rt(os.path.join(ref, "stress_record.csv")).values[:, :-1]
    ac = read_rt(os.path.join(ref, "active_elements.csv")).values[:, :-1]
    U = read_rt(os.path.join(ref, "node_displacements.csv")).values[:, :-1]
    F = read_rt(os.path.join(ref, "force_displacement.csv")).values
    fs.write_records(str(tmp_path), 4, 3, list(st), list(ac.astype(bool)), list(U), list(F), out_format="petsc")
    for f in ("stress_record.csv", "active_elements.csv", "node_displacements.csv",
              "force_displacement.csv"):
        assert (tmp_path / f).read_text() == open(os.path.join(ref, f)).read(), f


def test_python_writer_reproduces_golden_text(tmp_path):
    import fea_solver as fs
    ref = os.path.join(GOLDEN, "ref", "test_X")
    st = read_rt(os.path.join(ref, "stress_record.csv")).values[:, :-1]
    ac = read_rt(os.path.join(ref, "active_elements.csv")).values[:, :-1].astype(bool)
    U = read_rt(os.path.join(ref, "node_displacements.csv")).values[:, :-1]
    F = read_rt(os.path.join(ref, "force_displacement.csv")).values
    fs.write_records(str(tmp_path), 15, 14, list(st), list(ac), list(U), list(F))
    for f in ("stress_record.csv", "active_elements.csv", "node_displacements.csv",
              "force_displacement.csv"):
        assert (tmp_path / f).read_text() == open(os.path.join(ref, f)).read(), f
