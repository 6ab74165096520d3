"""Every BASELINE.json HIP configuration at its own workload, through the C ABI.

  C2_100k   1×5 tiles of results/sim_20251117_181147 (110,625 DOF), 1 GPU
  C3_1M     6×8 tiles (1,062,000 DOF), 1 GPU
  C4_1M_8p  the C3 network cut into 8 partitions (the multi-GPU plan, kernels
            and exchange schedule on one device — mfea_debug_set_parts)
  C5_10M    20×23 tiles + chords (10,177,500 DOF), 1 and 8 partitions

C2-C4: U within 1e-10 relative L2 of the oracle's direct solve of the same
system (src/fea_solver.py:112-135: K_ff + 1e-12 I, spsolve) at rtol 1e-13, for
GAMG and Jacobi-PCG, plus the true residual of the free system.  C5 is too
large for a direct solve here, so it is pinned by size-independent
properties: the true residual of the free system — K U formed element by
element from the oracle's own element matrices (src/fea_solver.py:30-68) —
at most 1e-10 ‖b‖, U_z ≡ 0 on the planar network, and linearity in the grip
displacement (U(2 dy) = 2 U(dy)).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

import fea_oracle as fo  # noqa: E402  (checker only)

DY = fo.DISPLACEMENT_MAX * 20 / (fo.N_STEPS - 1)  # the bench's load step 20


def rel(a, b):
    return np.linalg.norm(np.asarray(a) - np.asarray(b)) / np.linalg.norm(b)


def _opts(pc, rtol=1e-13):
    from mfea import PC_GAMG, PC_JACOBI, make_opts
    return make_opts(rtol=rtol, max_it=200000 if pc == "jacobi" else 2000,
                     precond=PC_JACOBI if pc == "jacobi" else PC_GAMG)


_CASES = {"C2_100k": (1, 5, False), "C3_1M": (6, 8, False)}
_cache = {}


def _direct(name):
    """mesh, grips and the oracle's direct solve of load step 20 (cached)."""
    if name not in _cache:
        from mfea import synth
        nx, ny, chords = _CASES[name]
        xyz, e2n = synth.tiled_mesh(nx, ny, chords=chords)
        top, bot = synth.grips(xyz)
        K = fo.assemble_global_stiffness(xyz, e2n, np.ones(len(e2n), bool))
        known, vals = fo.known_dof_map(top, bot, DY, -DY)
        A, b, free = fo.free_system(K, known, vals)
        _cache[name] = (xyz, e2n, top, bot, A, b, free, fo.solve_system(K, known, vals))
    return _cache[name]


def _load(eng, xyz, e2n, top, bot, nparts=1):
    eng.set_parts(nparts, -1)
    eng.set_mesh(xyz, e2n)
    eng.set_bc(top, bot)
    eng.set_active(None)
    eng.assemble()


@pytest.mark.parametrize("pc", ["gamg", "jacobi"])
@pytest.mark.parametrize("name,nparts", [("C2_100k", 1), ("C3_1M", 1), ("C4_1M_8p", 8)],
                         ids=["C2_100k", "C3_1M", "C4_1M_8p"])
def test_config_matches_direct(engine, name, nparts, pc):
    xyz, e2n, top, bot, A, b, free, Uref = _direct("C3_1M" if name.startswith("C4") else name)
    try:
        _load(engine, xyz, e2n, top, bot, nparts)
        assert engine.info()["n_parts"] == nparts
        st = engine.solve(DY, -DY, _opts(pc))
        U = engine.displacement()
    finally:
        engine.set_parts(1)
    assert st.status == 0, (name, pc)
    assert rel(U, Uref) <= 1e-10, (name, pc, rel(U, Uref))
    assert np.linalg.norm(A @ U[free] - b) <= 1e-12 * np.linalg.norm(b), (name, pc)
    assert np.all(U[2::3] == 0.0)  # planar: z decouples exactly


def test_C4_1M_8p_gamg_iterations_match_one_partition(engine):
    """The multi-GPU GAMG needs the one-partition iteration count (±3) at the
    metric's rtol 1e-8 on the C3 network cut 8 ways."""
    xyz, e2n, top, bot = _direct("C3_1M")[:4]
    its = []
    try:
        for n in (1, 8):
            _load(engine, xyz, e2n, top, bot, n)
            st = engine.solve(DY, -DY, _opts("gamg", 1e-8))
            assert st.status == 0
            its.append(st.iters)
    finally:
        engine.set_parts(1)
    assert abs(its[1] - its[0]) <= 3, its


def _element_matvec(xyz, e2n, U, chunk=1 << 20):
    """K U with K = Σ_e Ke (all elements active), element by element from the
    oracle's bar_stiffness_bulk (src/fea_solver.py:30-68) — no global matrix."""
    F = np.zeros(U.size)
    for s in range(0, len(e2n), chunk):
        e = e2n[s:s + chunk]
        Ke, _ = fo.bar_stiffness_bulk(xyz[e[:, 0]], xyz[e[:, 1]], fo.E_MOD, fo.AREA, fo.INERTIA)
        dofs = np.concatenate([3 * e[:, :1] + np.arange(3), 3 * e[:, 1:] + np.arange(3)], axis=1)
        Fe = np.einsum("eij,ej->ei", Ke, U[dofs])
        F += np.bincount(dofs.ravel(), weights=Fe.ravel(), minlength=U.size)
    return F


@pytest.fixture(scope="module")
def c5():
    from mfea import synth
    xyz, e2n = synth.tiled_mesh(20, 23, chords=True)
    top, bot = synth.grips(xyz)
    known, vals = fo.known_dof_map(top, bot, DY, -DY)
    free = np.setdiff1d(np.arange(3 * len(xyz)), known)
    Xk = np.zeros(3 * len(xyz))
    Xk[known] = vals
    bnorm = np.linalg.norm(_element_matvec(xyz, e2n, Xk)[free])  # ‖b_f‖ = ‖K_fk x_k‖
    return xyz, e2n, top, bot, free, bnorm


@pytest.mark.parametrize("nparts", [1, 8], ids=["C5_10M_1p", "C5_10M_8p"])
def test_C5_10M_dense_properties(engine, c5, nparts):
    xyz, e2n, top, bot, free, bnorm = c5
    assert 3 * len(xyz) == 10_177_500
    try:
        _load(engine, xyz, e2n, top, bot, nparts)
        st = engine.solve(DY, -DY, _opts("gamg"))
        U = engine.displacement()
        st2 = engine.solve(2 * DY, -2 * DY, _opts("gamg"))
        U2 = engine.displacement()
    finally:
        engine.set_parts(1)
    assert st.status == 0 and st2.status == 0
    # (K U)_f + reg U_f = K_ff U_f + K_fk x_k + reg U_f = A U_f − b = residual
    r = _element_matvec(xyz, e2n, U)[free] + fo.REG * U[free]
    assert np.linalg.norm(r) <= 1e-10 * bnorm, np.linalg.norm(r) / bnorm
    assert np.all(U[2::3] == 0.0)
    assert rel(U2, 2 * U) <= 1e-10
