"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the
reference's golden vectors.  Tolerances (north_star): displacement within
1e-10 relative L2 of the converged direct solve; node indexing bit-exact;
assembly values within 4 ulp of the reference's csr_matrix.
"""
import os
import shutil

import numpy as np
import pandas as pd
import pytest
import scipy.sparse as sp

from conftest import GOLDEN, load_gen, load_mesh, read_rt

pytestmark = pytest.mark.gpu

import fea_oracle as fo  # noqa: E402  (checker only)


def rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    nb = np.linalg.norm(b)
    return np.linalg.norm(a - b) / (nb if nb > 0 else 1.0)


def ulp_diff(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    sc = np.maximum(np.spacing(np.abs(a)), np.spacing(np.abs(b)))
    return np.max(np.abs(a - b) / np.where(sc > 0, sc, 1e-300)) if a.size else 0.0


# ---------------------------------------------------------------------------
# element stiffness (src/fea_solver.py:30-68)
# ---------------------------------------------------------------------------
def test_element_stiffness_matches_oracle(engine):
    rng = np.random.default_rng(7)
    p1 = rng.normal(size=(20000, 3))
    p2 = p1 + rng.normal(size=(20000, 3)) * rng.uniform(1e-3, 0.2, size=(20000, 1))
    p2[:50] = p1[:50]                    # zero-length → L_safe clamp
    p2[50:100, 2] = p1[50:100, 2]        # planar elements
    Ke, L = engine.element_stiffness(p1, p2, fo.E_MOD, fo.AREA, fo.INERTIA)
    Ko, Lo = fo.bar_stiffness_bulk(p1, p2)
    assert np.array_equal(L, Lo)
    # Only L³ may differ (double-double cube vs NumPy's ≤1-ulp pow); the bound is
    # 4ε × (|axial term| + |bending term|) per entry — the rounding-error scale
    # of S = t·k_ax + (δ−t)·k_b, which cancels where k_ax ≈ k_b.
    M = fo.stiffness_magnitude(p1, p2)
    assert np.all(np.abs(Ke - Ko) <= 4 * np.finfo(float).eps * M)
    assert np.mean(Ke == Ko) > 0.9


def _assembly_terms(xyz, e2n, active):
    """Per stored K entry: Σ|terms| (the rounding scale) and the number of
    element terms summed into it (1 for a single-element off-diagonal block)."""
    mag = fo.assemble_magnitude(xyz, e2n, active)
    e2n = np.asarray(e2n, np.int64)
    eidx = np.flatnonzero(np.asarray(active, bool))
    n1, n2 = e2n[eidx, 0], e2n[eidx, 1]
    dof = np.concatenate([3 * n1[:, None] + np.arange(3), 3 * n2[:, None] + np.arange(3)], axis=1)
    rows = np.repeat(dof, 6, axis=1).ravel()
    cols = np.tile(dof, (1, 6)).ravel()
    n = 3 * len(xyz)
    cnt = sp.csr_matrix((np.ones(rows.size), (rows, cols)), shape=(n, n))
    return mag.data, cnt.data


def check_assembly(dv, Kref, xyz, e2n, active):
    """K values against the reference's csr_matrix, by how the entry is formed:
    * one element term (off-diagonal blocks without a multi-edge): the
      element's own rounding, ≤ 4ε·(|axial| + |bending|) — and ≤ 4 ulp of the
      value itself wherever that sum does not cancel (|v| ≥ ½ Σ|terms|; where
      S = t·k_ax + (δ−t)·k_b cancels, a 1-ulp difference in L³ between
      NumPy's pow and the device's cube is many ulps of the small result);
    * k ≥ 2 terms (diagonals, multi-edges): summed in scipy's duplicate order,
      which its unstable sort leaves undefined above 16 row entries, so the
      bound is the sequential-sum one, (k + 3)·ε·Σ|terms|."""
    mag, k = _assembly_terms(xyz, e2n, active)
    eps = np.finfo(float).eps
    d = np.abs(dv - Kref.data)
    one = k == 1
    assert np.all(d[one] <= 4 * eps * mag[one])
    wc = one & (np.abs(Kref.data) >= 0.5 * mag)
    ulp = np.spacing(np.abs(Kref.data[wc]))
    assert np.all(d[wc] <= 4 * ulp), np.max(d[wc] / ulp)
    assert np.all(d[~one] <= (k[~one] + 3) * eps * mag[~one])


def stress_from_U(xyz, e2n, U, active_prev):
    """E·ε of every element active at step start (0 otherwise), with the
    oracle's restatement of the reference's strain arithmetic
    (src/fea_solver.py:263-272; oracle/cpu_fea.c cpu_strain)."""
    strain = fo.element_strain(xyz, e2n, U)
    return np.where(active_prev, fo.E_MOD * strain, 0.0), strain


def force_close(F, Fr):
    """Reaction sums; near-zero curves (fully clamped meshes) are rounding noise."""
    F, Fr = np.asarray(F), np.asarray(Fr)
    return np.all(np.abs(F - Fr) <= 1e-9 * np.max(np.abs(Fr)) + 1e-18)


def check_stress_records(xyz, e2n, U, S, A):
    """Stress and failure records bit for bit equal to the reference's strain
    arithmetic applied to the displacements the device produced (the stress
    kernel checked apart from the solve, whose U is bound by 1e-10)."""
    prev = np.ones(len(e2n), bool)
    for s in range(U.shape[0]):
        Sr, strain = stress_from_U(xyz, e2n, U[s], prev)
        assert np.array_equal(S[s], Sr), s
        with np.errstate(invalid="ignore"):
            nxt = prev & ~(np.abs(strain) > fo.MAX_STRAIN)
        assert np.array_equal(A[s], nxt), s
        prev = nxt


# ---------------------------------------------------------------------------
# assembly (src/fea_solver.py:74-106) — pattern identical, values ≤ 4 ulp
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("mesh", ["test_X", "sim_20251117_175809", "sim_20251115_135507"])
def test_assembly_matches_reference_K(engine, mesh):
    nodes, elems = load_mesh(mesh)
    z = np.load(os.path.join(GOLDEN, f"K0_{mesh}.npz"))
    Kref = sp.csr_matrix((z["data"], z["indices"], z["indptr"]), shape=tuple(z["shape"]))
    xyz, e2n = nodes[["x", "y", "z"]].values, elems[["n1", "n2"]].values
    engine.set_mesh(xyz, e2n)
    engine.set_bc([], [])
    engine.set_active(None)
    engine.assemble()
    ip, ix, dv = engine.export_csr()
    assert np.array_equal(ip, Kref.indptr)
    assert np.array_equal(ix, Kref.indices)
    check_assembly(dv, Kref, xyz, e2n, np.ones(len(e2n), bool))
    assert np.mean(dv == Kref.data) > 0.9


def test_assembly_with_inactive_elements(engine):
    nodes, elems = load_mesh("sim_20251117_175809")
    xyz = nodes[["x", "y", "z"]].values
    e2n = elems[["n1", "n2"]].values
    rng = np.random.default_rng(3)
    active = rng.random(len(e2n)) > 0.3
    Kref = fo.assemble_global_stiffness(xyz, e2n, active)
    engine.set_mesh(xyz, e2n)
    engine.set_bc([], [])
    engine.set_active(active)
    engine.assemble()
    ip, ix, dv = engine.export_csr()
    assert np.array_equal(ip, Kref.indptr)
    assert np.array_equal(ix, Kref.indices)
    check_assembly(dv, Kref, xyz, e2n, active)


# ---------------------------------------------------------------------------
# element-centric colour assembly (option asm_kernel 1, kernels.hip
# k_assemble_colour): off-diagonal blocks bit for bit the row gather's (the
# same S_e bits), diagonal blocks summed in colour order within the
# sequential-sum bound of the reference's csr_matrix, as the row gather's are
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("mesh", ["test_X", "sim_20251117_175809", "sim_20251115_135507"])
def test_colour_assembly_matches_row_gather(engine, mesh):
    nodes, elems = load_mesh(mesh)
    xyz, e2n = nodes[["x", "y", "z"]].values, elems[["n1", "n2"]].values
    active = np.random.default_rng(5).random(len(e2n)) > 0.2
    Kref = fo.assemble_global_stiffness(xyz, e2n, active)
    engine.set_mesh(xyz, e2n)
    engine.set_bc([], [])
    engine.set_active(active)
    engine.assemble()
    ip0, ix0, dv0 = engine.export_csr()
    engine.set_option("asm_kernel", 1)
    engine.assemble()
    ip, ix, dv = engine.export_csr()
    assert 0 < engine.get_option("asm_colours") <= 64
    assert np.array_equal(ip, ip0) and np.array_equal(ix, ix0)
    rows = np.repeat(np.arange(len(ip) - 1), np.diff(ip))
    off = rows // 3 != ix // 3
    assert np.array_equal(dv[off], dv0[off])
    check_assembly(dv, Kref, xyz, e2n, active)
    engine.assemble()  # deterministic: colours in order, no atomics
    assert np.array_equal(engine.export_csr()[2], dv)
    engine.set_option("asm_kernel", 2)  # element pass + row pass: the row gather's bits
    engine.assemble()
    assert np.array_equal(engine.export_csr()[2], dv0)


@pytest.mark.parametrize("precond", [0, 2])
def test_colour_assembly_solve_matches_direct(engine, precond):
    from mfea import make_opts
    sysz = np.load(os.path.join(GOLDEN, "sys_sim_20251117_181147_step20.npz"))
    _sim181147(engine)
    engine.set_option("asm_kernel", 1)
    engine.assemble()
    st = engine.solve(float(sysz["dy"]), -float(sysz["dy"]),
                      make_opts(rtol=1e-13, max_it=200000, precond=precond))
    assert st.status == 0
    assert rel(engine.displacement(), sysz["U"]) <= 1e-10


def test_colour_assembly_steps_match_row_gather(engine):
    """A loading run with failures: the same failed sets and reactions as the
    row gather (GAMG, whose RHS then runs as its own kernel)."""
    from mfea import make_opts
    nodes, elems = load_mesh("sim_20251117_175809")
    xyz = nodes[["x", "y", "z"]].values
    top, bot = fo.grip_nodes(xyz, nodes["node_id"].values, 1.5)
    out = []
    for kern in (0, 1, 2):
        engine.set_option("asm_kernel", kern)
        engine.set_mesh(xyz, elems[["n1", "n2"]].values)
        engine.set_bc(top, bot)
        engine.set_active(None)
        f, n = [], []
        for k in range(1, 25):
            d = 0.004 * k
            fk, nk, st = engine.step(d, -d, make_opts(rtol=1e-12, precond=2), 0.018)
            assert st.status == 0
            f.append(fk)
            n.append(nk)
        out.append((np.array(f), np.array(n)))
    assert np.array_equal(out[0][1], out[1][1])
    assert np.all(np.abs(out[0][0] - out[1][0]) <= 1e-8 * np.max(np.abs(out[0][0])))
    assert np.array_equal(out[0][1], out[2][1])
    assert np.all(np.abs(out[0][0] - out[2][0]) <= 1e-8 * np.max(np.abs(out[0][0])))


def test_set_active_is_ordered_with_the_next_assembly(engine):
    """The activity's upload runs on the handle's (non-blocking) stream: a
    null-stream fill could still be landing while the next assembly read it —
    a K from a mix of two activities, once in ≈ 100 sequences (capi.hip
    hmemcpy / hmemset).  The same K every time, the reference's bits."""
    nodes, elems = load_mesh("sim_20251117_181147")
    xyz, e2n = nodes[["x", "y", "z"]].values, elems[["n1", "n2"]].values
    engine.set_mesh(xyz, e2n)
    engine.set_bc([], [])
    reduced = np.random.default_rng(11).random(len(e2n)) > 0.03
    ref = None
    for _ in range(40):
        engine.set_active(reduced)
        engine.assemble()
        engine.set_active(None)
        engine.assemble()
        dv = engine.export_csr()[2]
        ref = dv if ref is None else ref
        assert np.array_equal(dv, ref)
    K = fo.assemble_global_stiffness(xyz, e2n, np.ones(len(e2n), bool))
    check_assembly(ref, K, xyz, e2n, np.ones(len(e2n), bool))


def test_speculative_post_matches_waited_post(engine):
    """Options spec_post / batch_graph: the post behind the solve's planned
    batch (eager, or captured with the batch in one graph).  A run
    whose tolerance alternates (the planned batch now too short — its post's
    failures undone, the solve goes on — now too long) gives the same forces,
    activity and stresses, bit for bit, as the post after the solve's wait."""
    from mfea import make_opts
    nodes, elems = load_mesh("sim_20251117_175809")
    xyz = nodes[["x", "y", "z"]].values
    top, bot = fo.grip_nodes(xyz, nodes["node_id"].values, 1.5)
    runs = []
    # batch: the batch + post as one graph; head: the assembly in the setup graph
    # combo: the batch and the post behind the setup in one graph
    for spec, batch, head, combo in ((0, 0, 0, 0), (1, 0, 0, 0), (1, 1, 0, 0), (1, 1, 0, 1), (1, 1, 1, 1)):
        engine.set_option("spec_post", spec)
        engine.set_option("batch_graph", batch)
        engine.set_option("step_graph", head)
        engine.set_option("combo_graph", combo)
        engine.set_mesh(xyz, elems[["n1", "n2"]].values)
        engine.set_bc(top, bot)
        engine.set_active(None)
        rec = []
        for k in range(1, 25):
            d = 0.004 * k
            f, n, st = engine.step(d, -d, make_opts(rtol=1e-5 if k % 3 else 1e-12, precond=2), 0.018)
            assert st.status == 0
            rec.append((f, n, st.iters, engine.stress().copy(), engine.active().copy()))
        runs.append(rec)
    assert sum(r[1] < runs[0][0][1] for r in runs[0]) > 0  # elements failed
    for other in runs[1:]:
        for a, b in zip(runs[0], other):
            assert a[0] == b[0] and a[1] == b[1] and a[2] == b[2]
            assert np.array_equal(a[3], b[3]) and np.array_equal(a[4], b[4])


# ---------------------------------------------------------------------------
# solve (src/fea_solver.py:112-135): ≤ 1e-10 relative L2 vs the direct solve
# ---------------------------------------------------------------------------
def _sim181147(engine):
    nodes, elems = load_mesh("sim_20251117_181147")
    xyz = nodes[["x", "y", "z"]].values
    top, bot = fo.grip_nodes(xyz, nodes["node_id"].values, 1.5)
    engine.set_mesh(xyz, elems[["n1", "n2"]].values)
    engine.set_bc(top, bot)
    engine.set_active(None)
    return xyz


@pytest.mark.parametrize("precond", [0, 1])
def test_solve_matches_direct(engine, precond):
    from mfea import make_opts
    sysz = np.load(os.path.join(GOLDEN, "sys_sim_20251117_181147_step20.npz"))
    _sim181147(engine)
    engine.assemble()
    st = engine.solve(float(sysz["dy"]), -float(sysz["dy"]),
                      make_opts(rtol=1e-13, max_it=200000, precond=precond))
    U = engine.displacement()
    assert st.status == 0
    assert rel(U, sysz["U"]) <= 1e-10
    if precond == 0:
        # Jacobi-PCG iteration count to 1e-8 = SciPy cg's (1644) within a few
        st8 = engine.solve(float(sysz["dy"]), -float(sysz["dy"]), make_opts(rtol=1e-8))
        assert abs(st8.iters - int(sysz["pcg_iters_1e8"])) <= 3


def test_solve_deterministic(engine):
    from mfea import make_opts
    _sim181147(engine)
    engine.assemble()
    engine.solve(0.01, -0.01, make_opts(rtol=1e-10))
    U1 = engine.displacement()
    engine.assemble()
    engine.solve(0.01, -0.01, make_opts(rtol=1e-10))
    assert np.array_equal(U1, engine.displacement())


def test_solve_csr_generic(engine):
    """solve_system with a caller-supplied K (the reference's own API)."""
    from mfea import make_opts
    nodes, elems = load_mesh("sim_20251117_175809")
    xyz = nodes[["x", "y", "z"]].values
    K = fo.assemble_global_stiffness(xyz, elems[["n1", "n2"]].values, np.ones(len(elems), bool))
    top, bot = fo.grip_nodes(xyz, nodes["node_id"].values, 1.5)
    known, vals = fo.known_dof_map(top, bot, 0.01, -0.01)
    Uref = fo.solve_system(K, known, vals)
    U, st = engine.solve_csr(K.indptr, K.indices, K.data, known, vals,
                             make_opts(rtol=1e-13, max_it=200000))
    assert st.status == 0
    assert rel(U, Uref) <= 1e-10
    assert np.array_equal(U[known], vals)


def test_fully_clamped_mesh_has_empty_solve(engine):
    """test_I at GRIP_LENGTH 1.5: every node is a grip node, n_free = 0."""
    from mfea import make_opts
    nodes, elems = load_mesh("test_I")
    xyz = nodes[["x", "y", "z"]].values
    top, bot = fo.grip_nodes(xyz, nodes["node_id"].values, 1.5)
    engine.set_mesh(xyz, elems[["n1", "n2"]].values)
    engine.set_bc(top, bot)
    engine.set_active(None)
    f, n_act, st = engine.step(0.01, -0.01, make_opts(rtol=1e-13), 0.018)
    K = fo.assemble_global_stiffness(xyz, elems[["n1", "n2"]].values, np.ones(3, bool))
    known, vals = fo.known_dof_map(top, bot, 0.01, -0.01)
    Uref = fo.solve_system(K, known, vals)
    assert st.n_free == 0 and st.iters == 0
    assert np.array_equal(engine.displacement(), Uref)
    Fref = (K @ Uref)[[3 * n + 1 for n in top]].sum()
    assert abs(f - Fref) <= 1e-12 * max(1.0, abs(Fref))


# ---------------------------------------------------------------------------
# full drop-in runs against the reference's committed goldens
# ---------------------------------------------------------------------------
def _run_dropin(tmp_path, mesh, n_steps, dmax, grip, **kw):
    import fea_solver as fs
    d = tmp_path / mesh
    shutil.copytree(os.path.join(GOLDEN, "meshes", mesh), d)
    saved = (fs.N_STEPS, fs.DISPLACEMENT_MAX)
    fs.N_STEPS, fs.DISPLACEMENT_MAX = n_steps, dmax
    try:
        fs.fea_solver(str(d), tol=grip, verbose=False, **kw)
    finally:
        fs.N_STEPS, fs.DISPLACEMENT_MAX = saved
    return d / "fea_results"


@pytest.mark.parametrize("mesh,n_steps", [("test_I", 40), ("test_X", 40), ("test_y", 100)])
def test_dropin_reproduces_committed_goldens(tmp_path, mesh, n_steps):
    out = _run_dropin(tmp_path, mesh, n_steps, 0.06, 0.5)
    ref = os.path.join(GOLDEN, "ref", mesh)
    for f in ("force_displacement.csv", "stress_record.csv", "node_displacements.csv",
              "active_elements.csv"):
        a, b = read_rt(out / f), read_rt(os.path.join(ref, f))
        assert list(a.columns) == list(b.columns), f
        assert a.shape == b.shape, f
    U = read_rt(out / "node_displacements.csv").values[:, :-1]
    Ur = read_rt(os.path.join(ref, "node_displacements.csv")).values[:, :-1]
    for s in range(U.shape[0]):
        assert rel(U[s], Ur[s]) <= 1e-10
    F = read_rt(out / "force_displacement.csv").values
    Fr = read_rt(os.path.join(ref, "force_displacement.csv")).values
    assert np.array_equal(F[:, 0], Fr[:, 0])
    assert rel(F[:, 1], Fr[:, 1]) <= 1e-10
    A = read_rt(out / "active_elements.csv")
    Ar = read_rt(os.path.join(ref, "active_elements.csv"))
    assert A.equals(Ar)
    nodes, elems = load_mesh(mesh)
    S = read_rt(out / "stress_record.csv").values[:, :-1]
    check_stress_records(nodes[["x", "y", "z"]].values, elems[["n1", "n2"]].values, U, S,
                         A.values[:, :-1].astype(bool))


def test_dropin_petsc_format_matches_cpp_golden(tmp_path):
    out = _run_dropin(tmp_path, "test_I_cpp", 40, 0.06, 0.5, out_format="petsc")
    ref = os.path.join(GOLDEN, "ref", "test_I_cpp")
    for f in ("force_displacement.csv", "stress_record.csv", "node_displacements.csv",
              "active_elements.csv"):
        a = (out / f).read_text().splitlines()
        b = open(os.path.join(ref, f)).read().splitlines()
        assert a[0] == b[0] and len(a) == len(b), f
    a = read_rt(out / "node_displacements.csv").values
    b = read_rt(os.path.join(ref, "node_displacements.csv")).values
    assert np.allclose(a, b, rtol=1e-10, atol=1e-14)


@pytest.mark.parametrize("gen,mesh", [
    ("gen_sim_20251117_175809_default.npz", "sim_20251117_175809"),
    ("gen_sim_20251115_135507_grip05.npz", "sim_20251115_135507"),   # 3D mesh (z ≠ 0)
    ("gen_test_X_default.npz", "test_X"),
])
def test_dropin_matches_reference_vectors(tmp_path, gen, mesh):
    g = load_gen(gen)
    res = _run_dropin(tmp_path, mesh, int(g["n_steps"]), float(g["dmax"]), float(g["grip"]))
    F = read_rt(res / "force_displacement.csv").values
    assert F.shape == g["force"].shape
    assert force_close(F[:, 1], g["force"][:, 1])
    A = read_rt(res / "active_elements.csv").values[:, :-1].astype(bool)
    assert np.array_equal(A, g["active"])
    U = read_rt(res / "node_displacements.csv").values[:, :-1]
    for k, s in enumerate(g["U_steps"]):
        assert rel(U[s], g["U"][k]) <= 1e-10
    nodes, elems = load_mesh(mesh)
    S = read_rt(res / "stress_record.csv").values[:, :-1]
    check_stress_records(nodes[["x", "y", "z"]].values, elems[["n1", "n2"]].values, U, S, A)


def test_sim181147_force_and_failures_match_committed_golden(tmp_path):
    """The reference's own 22k-DOF run (results/sim_20251117_181147/fea_results)."""
    res = _run_dropin(tmp_path, "sim_20251117_181147", 40, 0.02, 1.5)
    F = read_rt(res / "force_displacement.csv").values
    Fr = read_rt(os.path.join(GOLDEN, "ref", "sim_20251117_181147", "force_displacement.csv")).values
    assert rel(F[:, 1], Fr[:, 1]) <= 1e-9
    z = np.load(os.path.join(GOLDEN, "ref", "sim_20251117_181147", "active_packed.npz"))
    Ar = np.unpackbits(z["bits"], axis=1)[:, : int(z["n_elems"])].astype(bool)
    A = read_rt(res / "active_elements.csv").values[:, :-1].astype(bool)
    assert np.array_equal(A, Ar)
    nodes, elems = load_mesh("sim_20251117_181147")
    U = read_rt(res / "node_displacements.csv").values[:, :-1]
    S = read_rt(res / "stress_record.csv").values[:, :-1]
    check_stress_records(nodes[["x", "y", "z"]].values, elems[["n1", "n2"]].values, U, S, A)


# ---------------------------------------------------------------------------
# full-size properties (C2 synthetic, 110k DOF)
# ---------------------------------------------------------------------------
def test_c2_properties(engine):
    from mfea import make_opts, synth
    xyz, e2n = synth.tiled_mesh(1, 5)
    top, bot = synth.grips(xyz)
    engine.set_mesh(xyz, e2n)
    engine.set_bc(top, bot)
    engine.set_active(None)
    engine.assemble()
    st1 = engine.solve(0.005, -0.005, make_opts(rtol=1e-12, max_it=200000))
    U1 = engine.displacement()
    st2 = engine.solve(0.010, -0.010, make_opts(rtol=1e-12, max_it=200000))
    U2 = engine.displacement()
    assert st1.status == 0 and st2.status == 0
    assert np.all(U1[2::3] == 0.0)                   # planar: z decouples exactly
    assert rel(U2, 2 * U1) <= 1e-9                   # linearity in the load
    # true residual of the free system, checked with the CPU oracle's K
    K = fo.assemble_global_stiffness(xyz, e2n, np.ones(len(e2n), bool))
    known, vals = fo.known_dof_map(top, bot, 0.010, -0.010)
    A, b, free = fo.free_system(K, known, vals)
    assert np.linalg.norm(A @ U2[free] - b) <= 1e-10 * np.linalg.norm(b)


# ---------------------------------------------------------------------------
# the two CG iteration kernels: wave-local lanes (default) and SELL (reference
# layout); same algorithm, so same iterates up to summation order
# ---------------------------------------------------------------------------
def _solve_with(engine, kernel, dy, opts):
    from mfea._capi import CG_KERNEL
    with engine.options(cg_kernel=CG_KERNEL[kernel]):  # "lanes" | "sell" (else chosen by density)
        st = engine.solve(dy, -dy, opts)
        assert engine.info()["cg_lanes"] == (kernel == "lanes")
        return st, engine.displacement()


@pytest.mark.parametrize("precond", [0, 1])
def test_lane_kernel_matches_sell_and_direct(engine, precond):
    from mfea import make_opts
    sysz = np.load(os.path.join(GOLDEN, "sys_sim_20251117_181147_step20.npz"))
    _sim181147(engine)
    engine.assemble()
    dy = float(sysz["dy"])
    st_l, U_l = _solve_with(engine, "lanes", dy, make_opts(rtol=1e-13, max_it=200000, precond=precond))
    st_s, U_s = _solve_with(engine, "sell", dy, make_opts(rtol=1e-13, max_it=200000, precond=precond))
    assert st_l.status == 0 and st_s.status == 0
    assert rel(U_l, sysz["U"]) <= 1e-10 and rel(U_s, sysz["U"]) <= 1e-10
    s8l, _ = _solve_with(engine, "lanes", dy, make_opts(rtol=1e-8, precond=precond))
    s8s, _ = _solve_with(engine, "sell", dy, make_opts(rtol=1e-8, precond=precond))
    assert abs(s8l.iters - s8s.iters) <= 3
    if precond == 0:
        assert abs(s8l.iters - int(sysz["pcg_iters_1e8"])) <= 3


def _direct(xyz, e2n, top, bot, dy):
    K = fo.assemble_global_stiffness(xyz, e2n, np.ones(len(e2n), bool))
    known, vals = fo.known_dof_map(top, bot, dy, -dy)
    return fo.solve_system(K, known, vals)


def _true_relres(xyz, e2n, top, bot, dy, U):
    K = fo.assemble_global_stiffness(xyz, e2n, np.ones(len(e2n), bool))
    known, vals = fo.known_dof_map(top, bot, dy, -dy)
    A, b, free = fo.free_system(K, known, vals)
    return np.linalg.norm(A @ U[free] - b) / np.linalg.norm(b)


def test_lane_kernel_high_degree_and_multiedges(engine):
    """A hub of degree 40 (helper lanes spanning most of a wave), duplicated
    elements, shortcuts, and a chain across several waves; hyphal lengths
    (0.05 mm) keep the system well conditioned (cond ≈ 2e6), so both kernels
    must reach the direct solve."""
    from mfea import make_opts
    n = 400
    xyz = np.zeros((n, 3))
    ang = 2 * np.pi * np.arange(1, 41) / 40
    xyz[1:41, 0] = 0.05 * np.cos(ang)
    xyz[1:41, 1] = 0.05 * np.sin(ang)
    i = np.arange(41, n)
    xyz[41:, 0] = 0.01 * np.sin(i)
    xyz[41:, 1] = 0.06 + 0.05 * (i - 41)
    e2n = [(0, i) for i in range(1, 41)] + [(i, i + 1) for i in range(41, n - 1)]
    e2n += [(5, 41), (5, 41), (60, 62), (7, 45), (41, 43), (20, 200)]
    e2n = np.array(e2n)
    top = np.arange(380, 400)
    bot = np.arange(41, 46)
    engine.set_mesh(xyz, e2n)
    engine.set_bc(top, bot)
    engine.set_active(None)
    engine.assemble()
    assert engine.info()["n_lanes"] > engine.info()["n_free_nodes"] + 10   # helper lanes
    opts = make_opts(rtol=1e-13, max_it=200000)
    st_l, U_l = _solve_with(engine, "lanes", 0.01, opts)
    st_s, U_s = _solve_with(engine, "sell", 0.01, opts)
    assert st_l.status == 0 and st_s.status == 0
    Uref = _direct(xyz, e2n, top, bot, 0.01)
    assert rel(U_l, Uref) <= 1e-10 and rel(U_s, Uref) <= 1e-10
    assert _true_relres(xyz, e2n, top, bot, 0.01, U_l) <= 1e-12
    assert abs(st_l.iters - st_s.iters) <= 3


def test_lane_kernel_natural_order_many_halos():
    """Natural (export) row order: most neighbours are out of wave, so most
    slots go through pushed halo records and groups grow helper lanes."""
    from mfea import Engine, make_opts, synth
    xyz, e2n = synth.tiled_mesh(1, 1)
    top, bot = synth.grips(xyz)
    engine = Engine(0)
    try:
        engine.set_option("order", 0)
        engine.set_option("cg_kernel", 1)  # dense in lanes: default would pick SELL
        engine.set_mesh(xyz, e2n)
        engine.set_bc(top, bot)
        engine.set_active(None)
        engine.assemble()
        info = engine.info()
        assert info["cg_lanes"] == 1 and info["n_halo"] > info["n_free_nodes"] // 4
        Uref = _direct(xyz, e2n, top, bot, 0.01)
        st, U = _solve_with(engine, "lanes", 0.01, make_opts(rtol=1e-13, max_it=200000))
        assert st.status == 0
        assert rel(U, Uref) <= 1e-10
    finally:
        engine.close()


@pytest.mark.parametrize("precond", [0, 1])
def test_planar_lanes_bitwise_equal_3dof_lanes(engine, precond):
    """On a planar mesh the 2-DOF lanes drop z components that are exactly 0
    in every iterate: U must equal the 3-DOF lanes' U bit for bit."""
    from mfea import make_opts
    _sim181147(engine)
    engine.assemble()
    opts = make_opts(rtol=1e-10, max_it=200000, precond=precond)
    st2, U2 = _solve_with(engine, "lanes", 0.01, opts)
    with engine.options(lane_dof=3):   # rebuilds the layout with 3 DOFs per node
        engine.assemble()
        st3, U3 = _solve_with(engine, "lanes", 0.01, opts)
    engine.assemble()
    assert st2.status == 0 and st3.status == 0 and st2.iters == st3.iters
    assert np.array_equal(U2, U3)
    assert np.all(U2[2::3] == 0.0)


# ---------------------------------------------------------------------------
# launch geometries of the lane kernel (ell.hip): block size 64/128/256 and the
# halo record layout (compact / per lane) forced on a small system — same
# iterates up to summation order, each geometry bitwise reproducible
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("bs,hc,precond,maxg", [
    (64, "1", 0, 0), (128, "0", 0, 0), (256, "1", 0, 0), (128, "1", 1, 0), (256, "0", 1, 0),
    (512, "1", 0, 0), (512, "0", 1, 0),
    # grid capped: every wave makes several passes (as at C3)
    (64, "1", 0, 5), (256, "0", 1, 3), (128, "1", 1, 2), (512, "1", 0, 2)])
def test_lane_geometries_match_direct(bs, hc, precond, maxg):
    """hc: compact halo records (large systems) or one record per lane; maxg
    caps the grid so every wave makes several passes."""
    from mfea import Engine, make_opts
    sysz = np.load(os.path.join(GOLDEN, "sys_sim_20251117_181147_step20.npz"))
    eng = Engine(0)
    try:
        eng.set_option("ell_block", bs)
        eng.set_option("ell_compact", int(hc))
        eng.set_option("ell_maxg", maxg)
        eng.set_option("cg_kernel", 1)
        _sim181147(eng)
        eng.assemble()
        dy = float(sysz["dy"])
        st = eng.solve(dy, -dy, make_opts(rtol=1e-13, max_it=200000, precond=precond))
        U = eng.displacement()
        assert st.status == 0 and rel(U, sysz["U"]) <= 1e-10
        eng.solve(dy, -dy, make_opts(rtol=1e-13, max_it=200000, precond=precond))
        assert np.array_equal(U, eng.displacement())
        if precond == 0:
            s8 = eng.solve(dy, -dy, make_opts(rtol=1e-8))
            assert abs(s8.iters - int(sysz["pcg_iters_1e8"])) <= 3
        # one full step with failures on the geometry: same records as the default
        f, n, _ = eng.step(dy, -dy, make_opts(rtol=1e-13, max_it=200000, precond=precond), 0.018)
        assert n == eng.active().sum()
    finally:
        eng.close()


def test_dense_network_runs_sell_kernel_and_matches_direct(engine):
    """Dense-filament networks (the C5 recipe: intra-tile chords, mean degree
    ≈ 7.5) need > 2 lanes per free row; the engine then runs the SELL kernel."""
    from mfea import make_opts, synth
    xyz, e2n = synth.tiled_mesh(1, 1, chords=True)
    top, bot = synth.grips(xyz)
    engine.set_mesh(xyz, e2n)
    engine.set_bc(top, bot)
    engine.set_active(None)
    engine.assemble()
    info = engine.info()
    assert info["n_lanes"] > 2 * info["n_free_nodes"] and info["cg_lanes"] == 0
    st = engine.solve(0.01, -0.01, make_opts(rtol=1e-13, max_it=200000))
    assert st.status == 0
    assert rel(engine.displacement(), _direct(xyz, e2n, top, bot, 0.01)) <= 1e-10
