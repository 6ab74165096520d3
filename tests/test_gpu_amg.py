"""GPU parity of the SA-AMG preconditioned CG (MFEA_PC_GAMG, csrc/amg.hip):
displacements within 1e-10 relative L2 of the reference's direct solve
(src/fea_solver.py:128) at rtol 1e-13, iteration counts equal to the NumPy
restatement of the same hierarchy (tests/amg_ref.py) within ±2, bitwise
reproducible solves, and the rebuild of the hierarchy when elements fail."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_mesh

pytestmark = pytest.mark.gpu

import fea_oracle as fo  # noqa: E402  (checker only)


def rel(a, b):
    nb = np.linalg.norm(b)
    return np.linalg.norm(np.asarray(a) - np.asarray(b)) / (nb if nb > 0 else 1.0)


def _opts(rtol, **kw):
    from mfea import PC_GAMG, make_opts
    return make_opts(rtol=rtol, max_it=2000, precond=PC_GAMG, **kw)


def _sim181147(engine):
    nodes, elems = load_mesh("sim_20251117_181147")
    xyz = nodes[["x", "y", "z"]].values
    top, bot = fo.grip_nodes(xyz, nodes["node_id"].values, 1.5)
    e2n = elems[["n1", "n2"]].values
    engine.set_mesh(xyz, e2n)
    engine.set_bc(top, bot)
    engine.set_active(None)
    return xyz, e2n, top, bot


def test_gamg_matches_direct_and_restatement(engine):
    sysz = np.load(os.path.join(GOLDEN, "sys_sim_20251117_181147_step20.npz"))
    _sim181147(engine)
    engine.assemble()
    dy = float(sysz["dy"])
    st = engine.solve(dy, -dy, _opts(1e-13))
    assert st.status == 0 and st.amg_levels >= 3
    assert rel(engine.displacement(), sysz["U"]) <= 1e-10
    st8 = engine.solve(dy, -dy, _opts(1e-8))
    # the NumPy restatement of this hierarchy needs 17 (tests/test_amg_cpu.py);
    # Jacobi-PCG needs 1,644 (SciPy cg, tests/golden)
    assert abs(st8.iters - 17) <= 2, st8.iters
    info = engine.amg_info()
    assert info["rows"][0] == engine.info()["n_free_nodes"] and info["nd"] == 2


def test_gamg_deterministic_and_no_rebuild(engine):
    _sim181147(engine)
    engine.assemble()
    st1 = engine.solve(0.01, -0.01, _opts(1e-10))
    U1 = engine.displacement()
    engine.assemble()
    st2 = engine.solve(0.01, -0.01, _opts(1e-10))
    assert np.array_equal(U1, engine.displacement())
    assert st1.iters == st2.iters and st2.amg_rebuilt == 0
    engine.set_active(None)   # same (all-active) set: the plan is kept
    engine.assemble()
    assert engine.solve(0.01, -0.01, _opts(1e-10)).amg_rebuilt == 0


@pytest.mark.parametrize("reuse", [0, 1])
def test_gamg_rebuilds_after_failures_and_matches_direct(engine, reuse):
    """Steps with element failures: every step's U matches the direct solve of
    that step's K.  amg_reuse 0: the hierarchy is rebuilt for every new active
    set; 1 (default): the intact set's hierarchy is kept (floating pieces
    masked) unless the iterations degrade."""
    xyz, e2n, top, bot = _sim181147(engine)
    active = np.ones(len(e2n), bool)
    rebuilt, reused = [], []
    with engine.options(amg_reuse=reuse):
        for step in (10, 25, 39):
            dy = fo.DISPLACEMENT_MAX * step / (fo.N_STEPS - 1)
            engine.set_active(active)
            f, n_act, st = engine.step(dy, -dy, _opts(1e-13), fo.MAX_STRAIN)
            rebuilt.append(st.amg_rebuilt)
            reused.append(engine.get_option("amg_reused"))
            K = fo.assemble_global_stiffness(xyz, e2n, active)
            known, vals = fo.known_dof_map(top, bot, dy, -dy)
            Uref = fo.solve_system(K, known, vals)
            assert rel(engine.displacement(), Uref) <= 1e-10, step
            active = engine.active()
    assert n_act < len(e2n)          # failures happened
    if reuse:
        assert reused[-1] == 1 or rebuilt[-1] == 1
    else:
        assert sum(rebuilt[1:]) >= 1     # a later step rebuilt the plan
        assert not any(reused)


def _floating_nodes(xyz, e2n, active, top, bot):
    """Nodes with no path of active elements to a grip node (scipy csgraph)."""
    import scipy.sparse as sp
    from scipy.sparse.csgraph import connected_components
    n = len(xyz)
    a = e2n[active]
    g = sp.coo_matrix((np.ones(len(a)), (a[:, 0], a[:, 1])), shape=(n, n))
    _, lab = connected_components(g, directed=False)
    anchored = np.zeros(lab.max() + 1, bool)
    anchored[lab[np.concatenate([top, bot])]] = True
    return ~anchored[lab]


def test_gamg_kept_hierarchy_floating_pieces_exactly_zero(engine):
    """Knock out 6 % of the elements (seeded): pieces cut off from both grips
    appear.  The intact set's hierarchy is kept (amg_reuse 1, no rebuild
    forced): U matches the direct solve and is EXACTLY zero on every floating
    node, as spsolve gives (zero load there); the kept hierarchy also survives
    the reverse change back to the intact set."""
    xyz, e2n, top, bot = _sim181147(engine)
    dy = fo.DISPLACEMENT_MAX * 20 / (fo.N_STEPS - 1)
    with engine.options(amg_reuse=1, amg_rebuild_pct=100000, amg_rebuild_rent=0):
        engine.set_active(None)
        engine.assemble()
        st0 = engine.solve(dy, -dy, _opts(1e-13))
        rng = np.random.default_rng(7)
        active = rng.random(len(e2n)) > 0.06
        fl = _floating_nodes(xyz, e2n, active, top, bot)
        free_fl = fl.copy()
        free_fl[np.concatenate([top, bot])] = False
        assert free_fl.sum() > 20
        engine.set_active(active)
        engine.assemble()
        st = engine.solve(dy, -dy, _opts(1e-13))
        assert st.amg_rebuilt == 0 and engine.get_option("amg_reused") == 1
        U = engine.displacement().reshape(-1, 3)
        K = fo.assemble_global_stiffness(xyz, e2n, active)
        known, vals = fo.known_dof_map(top, bot, dy, -dy)
        Uref = fo.solve_system(K, known, vals)
        assert rel(U.ravel(), Uref) <= 1e-10
        assert np.all(U[free_fl] == 0.0)
        assert np.all(Uref.reshape(-1, 3)[free_fl] == 0.0)
        engine.set_active(None)
        engine.assemble()
        st1 = engine.solve(dy, -dy, _opts(1e-13))
        assert st1.amg_rebuilt == 0 and st1.iters == st0.iters
        K = fo.assemble_global_stiffness(xyz, e2n, np.ones(len(e2n), bool))
        assert rel(engine.displacement(), fo.solve_system(K, known, vals)) <= 1e-10


@pytest.mark.parametrize("frac", [0.0, 0.01, 0.06, 0.3, 0.7, 1.0])
def test_device_floating_rows_match_scipy_components(engine, frac):
    """The floating mask's connected components on the device (kernels.hip
    launch_floating: CAS root hooking, deterministic roots) against SciPy's
    csgraph on the same activity: the free nodes with no active path to a
    grip, exactly; run twice, bitwise the same."""
    xyz, e2n, top, bot = _sim181147(engine)
    grip = np.zeros(len(xyz), bool)
    grip[np.concatenate([top, bot])] = True
    rng = np.random.default_rng(int(frac * 1000) + 3)
    active = rng.random(len(e2n)) >= frac
    engine.set_active(active)
    fl = engine.floating()
    ref = _floating_nodes(xyz, e2n, active, top, bot) & ~grip
    assert np.array_equal(fl, ref), (int(fl.sum()), int(ref.sum()))
    assert np.array_equal(engine.floating(), fl)
    engine.set_active(None)


def test_device_floating_rows_tiled_network(engine):
    """The same on the 1×5-tile C2 network (110 k DOF) with 20 % of the
    elements out: many components, hooks racing across the whole grid."""
    from mfea import synth
    xyz, e2n = synth.tiled_mesh(1, 5)
    top, bot = synth.grips(xyz)
    engine.set_mesh(xyz, e2n)
    engine.set_bc(top, bot)
    grip = np.zeros(len(xyz), bool)
    grip[np.concatenate([top, bot])] = True
    active = np.random.default_rng(5).random(len(e2n)) >= 0.2
    engine.set_active(active)
    ref = _floating_nodes(xyz, e2n, active, top, bot) & ~grip
    assert ref.sum() > 100
    assert np.array_equal(engine.floating(), ref)
    engine.set_active(None)


def test_gamg_failures_through_post_keep_floating_exactly_zero(engine):
    """The reference loop with failures driven by the post kernel alone (no
    set_active between steps, src/fea_solver.py:216-295), pulled to 3× the
    displacement so that pieces float: the hierarchy is kept (the floating
    set moved by the failed ids, capi.hip local_failures / push_fmask), and
    every step's U matches the direct solve of the set it ran on and is
    EXACTLY zero on every floating free node."""
    xyz, e2n, top, bot = _sim181147(engine)
    grip = np.zeros(len(xyz), bool)
    grip[np.concatenate([top, bot])] = True
    seen_float = 0
    with engine.options(amg_reuse=1, amg_rebuild_pct=100000, amg_rebuild_rent=0):
        engine.set_active(None)
        active = np.ones(len(e2n), bool)
        for step in range(fo.N_STEPS):
            dy = 3 * fo.DISPLACEMENT_MAX * step / (fo.N_STEPS - 1)
            f, n_act, st = engine.step(dy, -dy, _opts(1e-13), fo.MAX_STRAIN)
            assert st.status == 0, step
            if step > 0 and n_act > 0 and step % 3 == 0:
                fl = _floating_nodes(xyz, e2n, active, top, bot) & ~grip
                U = engine.displacement().reshape(-1, 3)
                K = fo.assemble_global_stiffness(xyz, e2n, active)
                known, vals = fo.known_dof_map(top, bot, dy, -dy)
                Uref = fo.solve_system(K, known, vals)
                assert rel(U.ravel(), Uref) <= 1e-10, step
                assert np.all(U[fl] == 0.0), step
                seen_float = max(seen_float, int(fl.sum()))
            nxt = engine.active().astype(bool)
            assert int(nxt.sum()) == n_act and not np.any(nxt & ~active)
            active = nxt
            if n_act == 0:
                break
        assert engine.get_option("amg_reused") == 1
    assert active.sum() < len(e2n) and seen_float > 0


def test_gamg_hierarchy_not_kept_for_a_superset(engine):
    """A hierarchy built on a REDUCED active set holds only that set's
    elements in A_0's slot lists; elements coming back (set_active(None))
    must rebuild it — a kept one would solve a system missing their
    couplings.  U then matches the direct solve of the intact K."""
    xyz, e2n, top, bot = _sim181147(engine)
    dy = fo.DISPLACEMENT_MAX * 20 / (fo.N_STEPS - 1)
    known, vals = fo.known_dof_map(top, bot, dy, -dy)
    rng = np.random.default_rng(11)
    active = rng.random(len(e2n)) > 0.03
    with engine.options(amg_reuse=1, amg_rebuild_pct=100000, amg_rebuild_rent=0):
        engine.set_active(active)
        engine.assemble()
        assert engine.solve(dy, -dy, _opts(1e-13)).status == 0
        engine.set_active(None)
        engine.assemble()
        st = engine.solve(dy, -dy, _opts(1e-13))
        assert st.status == 0 and st.amg_rebuilt == 1
        assert engine.get_option("amg_reused") == 0
        K = fo.assemble_global_stiffness(xyz, e2n, np.ones(len(e2n), bool))
        assert rel(engine.displacement(), fo.solve_system(K, known, vals)) <= 1e-10


def test_small_max_it_keeps_overrelaxed_weights(engine):
    """A caller's deliberately small max_it is not the coarse weights' fault:
    the solve reports EMAXIT (LinAlgError in the drop-in) and the handle keeps
    the over-relaxed smoothers for the next solve."""
    from mfea import PC_GAMG, make_opts
    _sim181147(engine)
    engine.assemble()
    assert engine.get_option("amg_safe_omega") == 0
    with pytest.raises(np.linalg.LinAlgError):
        engine.solve(0.01, -0.01, make_opts(rtol=1e-13, max_it=3, precond=PC_GAMG))
    assert engine.get_option("amg_safe_omega") == 0
    assert engine.solve(0.01, -0.01, _opts(1e-13)).status == 0
    assert engine.get_option("amg_safe_omega") == 0


def test_gamg_3d_mesh_matches_direct(engine):
    nodes, elems = load_mesh("sim_20251115_135507")
    xyz = nodes[["x", "y", "z"]].values
    top, bot = fo.grip_nodes(xyz, nodes["node_id"].values, 0.5)
    e2n = elems[["n1", "n2"]].values
    engine.set_mesh(xyz, e2n)
    engine.set_bc(top, bot)
    engine.set_active(None)
    engine.assemble()
    st = engine.solve(0.01, -0.01, _opts(1e-13))
    assert st.status == 0 and engine.amg_info()["nd"] == 3
    K = fo.assemble_global_stiffness(xyz, e2n, np.ones(len(e2n), bool))
    known, vals = fo.known_dof_map(top, bot, 0.01, -0.01)
    assert rel(engine.displacement(), fo.solve_system(K, known, vals)) <= 1e-10


def test_gamg_profile_iteration(engine):
    from mfea import PC_GAMG
    _sim181147(engine)
    engine.assemble()
    engine.solve(0.01, -0.01, _opts(1e-8))
    ms = engine.profile_iteration(PC_GAMG, reps=20)
    assert 0 < ms < 5.0


# ---------------------------------------------------------------------------
# benchmark sizes: C3 = 6×8 tiles (1.06 M DOF), the C5 chord recipe
# on 2×2 tiles; U against the oracle's direct solve of the same system
# ---------------------------------------------------------------------------
def _big_case(engine, nx, ny, chords):
    from mfea import synth
    xyz, e2n = synth.tiled_mesh(nx, ny, chords=chords)
    top, bot = synth.grips(xyz)
    engine.set_mesh(xyz, e2n)
    engine.set_bc(top, bot)
    engine.set_active(None)
    engine.assemble()
    dy = fo.DISPLACEMENT_MAX * 20 / (fo.N_STEPS - 1)
    K = fo.assemble_global_stiffness(xyz, e2n, np.ones(len(e2n), bool))
    known, vals = fo.known_dof_map(top, bot, dy, -dy)
    A, b, free = fo.free_system(K, known, vals)
    Uref = fo.solve_system(K, known, vals)
    return dy, A, b, free, Uref


@pytest.mark.parametrize("nx,ny,chords", [(6, 8, False), (2, 2, True)])
def test_benchmark_sizes_match_direct(engine, nx, ny, chords):
    from mfea import PC_JACOBI, make_opts
    dy, A, b, free, Uref = _big_case(engine, nx, ny, chords)
    for pc in ("gamg", "jacobi"):
        opts = _opts(1e-13) if pc == "gamg" else make_opts(rtol=1e-13, max_it=200000, precond=PC_JACOBI)
        st = engine.solve(dy, -dy, opts)
        U = engine.displacement()
        assert st.status == 0, pc
        assert rel(U, Uref) <= 1e-10, (pc, rel(U, Uref))
        assert np.linalg.norm(A @ U[free] - b) <= 1e-12 * np.linalg.norm(b), pc
        if chords is False:
            assert np.all(U[2::3] == 0.0)  # planar: z decouples exactly


# ---------------------------------------------------------------------------
# V-cycle kernel variants (csrc/amg.hip): lanes per row of the restriction and
# of the coarse operators.  Every variant converges to the direct solve.
# ---------------------------------------------------------------------------
def _variant_solves(engine, option, values, nx=1, ny=5, cycle=0):
    from mfea import synth
    xyz, e2n = synth.tiled_mesh(nx, ny)
    top, bot = synth.grips(xyz)
    dy = fo.DISPLACEMENT_MAX * 20 / (fo.N_STEPS - 1)
    out = {}
    # every level in its own kernels; the session engine gets its options back
    with engine.options(amg_tail_rows=0, amg_cycle=cycle, amg_collapse=0, **{option: values[0]}):
        engine.set_mesh(xyz, e2n)
        engine.set_bc(top, bot)
        engine.set_active(None)
        engine.assemble()
        for v in values:
            engine.set_option(option, v)
            st = engine.solve(dy, -dy, _opts(1e-13))
            assert st.status == 0, (option, v)
            out[v] = (engine.displacement(), st.iters)
    K = fo.assemble_global_stiffness(xyz, e2n, np.ones(len(e2n), bool))
    known, vals = fo.known_dof_map(top, bot, dy, -dy)
    return out, fo.solve_system(K, known, vals)


@pytest.mark.parametrize("option,values", [("amg_restrict_lanes", [1, 2, 4, 8, 16]), ("amg_op_lanes", [1, 2, 4]),
                                           ("amg_up_lanes", [1, 2, 4])])
def test_vcycle_lane_splits_match_direct(engine, option, values):
    # four-step form and the compact one (every level's sweeps: no collapse)
    for cycle in (0, 1):
        _lane_splits(engine, option, values, cycle)


def _lane_splits(engine, option, values, cycle):
    out, Uref = _variant_solves(engine, option, values, cycle=cycle)
    for v, (U, _) in out.items():
        assert rel(U, Uref) <= 1e-10, (option, cycle, v, rel(U, Uref))


def test_tail_lds_and_global_bitwise_equal(engine):
    """The single-workgroup tail with its vectors in LDS (k_amg_tail_lds) and
    in global memory (k_amg_tail) run the same arithmetic: U bit for bit."""
    from mfea import synth
    xyz, e2n = synth.tiled_mesh(1, 5)
    top, bot = synth.grips(xyz)
    dy = fo.DISPLACEMENT_MAX * 20 / (fo.N_STEPS - 1)
    out = {}
    with engine.options(amg_tail_rows=2048, amg_tail_lds=1, amg_cycle=0):
        engine.set_mesh(xyz, e2n)
        engine.set_bc(top, bot)
        engine.set_active(None)
        engine.assemble()
        rows = engine.amg_info()["rows"]
        # the tail runs only if some level below level 0 fits in it
        assert len(rows) >= 3 and any(r <= 2048 for r in rows[1:]), rows
        for v in (1, 0):
            engine.set_option("amg_tail_lds", v)
            st = engine.solve(dy, -dy, _opts(1e-10))
            assert st.status == 0
            out[v] = (engine.displacement(), st.iters)
    assert out[0][1] == out[1][1] and np.array_equal(out[0][0], out[1][0])


def test_converged_solve_leaves_no_stale_chunks(engine):
    """A solve that converges in fewer chunks than the previous one planned
    must not let the extra queued chunks touch x (cg.hip k_cg_advance poisons
    the slot every queued chunk gates on): a loose solve after a tight one
    equals the loose solve on a fresh handle bit for bit, and its reported
    relres is the residual of the U it returns."""
    from mfea import Engine
    sysz = np.load(os.path.join(GOLDEN, "sys_sim_20251117_181147_step20.npz"))
    dy = float(sysz["dy"])
    xyz, e2n, top, bot = _sim181147(engine)
    engine.assemble()
    assert engine.solve(dy, -dy, _opts(1e-13)).status == 0   # plans ~30+ iterations next
    st = engine.solve(dy, -dy, _opts(1e-6))
    U = engine.displacement()
    with Engine(0) as fresh:
        fresh.set_mesh(xyz, e2n)
        fresh.set_bc(top, bot)
        fresh.set_active(None)
        fresh.assemble()
        # under-planned (a looser solve first): chunks are queued one at a
        # time once the plan is used up, so no chunk runs after convergence
        assert fresh.solve(dy, -dy, _opts(1e-2)).iters < st.iters
        st_f = fresh.solve(dy, -dy, _opts(1e-6))
        U_f = fresh.displacement()
    assert st.iters == st_f.iters
    assert np.array_equal(U, U_f)
    K = fo.assemble_global_stiffness(xyz, e2n, np.ones(len(e2n), bool))
    known, vals = fo.known_dof_map(top, bot, dy, -dy)
    A, b, free = fo.free_system(K, known, vals)
    true_rel = np.linalg.norm(b - A @ U[free]) / np.linalg.norm(b)
    assert abs(true_rel - st.relres) <= 0.05 * st.relres, (true_rel, st.relres)


# meshes of the cycle-variant tests below
def _mesh_case(engine, mesh):
    from mfea import synth
    if mesh == "sim135507_3d":
        nodes, elems = load_mesh("sim_20251115_135507")
        xyz = nodes[["x", "y", "z"]].values
        top, bot = fo.grip_nodes(xyz, nodes["node_id"].values, 0.5)
        e2n = elems[["n1", "n2"]].values
    else:
        nx, ny, chords = {"C2_1x5": (1, 5, False), "C3_6x8": (6, 8, False), "C5_2x2": (2, 2, True)}[mesh]
        xyz, e2n = synth.tiled_mesh(nx, ny, chords=chords)
        top, bot = synth.grips(xyz)
    engine.set_mesh(xyz, e2n)
    engine.set_bc(top, bot)
    engine.set_active(None)
    engine.assemble()
    return xyz, e2n, top, bot


# ---------------------------------------------------------------------------
# the compact cycle (amg_cycle 1: two sweeps per level with P̃ = (I − ωD⁻¹A)P,
# R̃ = P̃ᵀ; tests/test_amg_cpu.py pins it against the four-step cycle): the
# direct solve's U, and the four-step cycle's iteration count (the same
# preconditioner up to f32 rounding)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("mesh", ["C2_1x5", "C3_6x8", "C5_2x2", "sim135507_3d"])
def test_compact_cycle_matches_direct(engine, mesh):
    dy = fo.DISPLACEMENT_MAX * 20 / (fo.N_STEPS - 1)
    its = {}
    with engine.options(amg_cycle=0, amg_collapse=0):
        xyz, e2n, top, bot = _mesh_case(engine, mesh)
        for cyc in (0, 1):   # four-step, compact (every level's sweeps)
            engine.set_option("amg_cycle", cyc)
            its[cyc] = engine.solve(dy, -dy, _opts(1e-8)).iters
            st = engine.solve(dy, -dy, _opts(1e-13))
            assert st.status == 0, cyc
            U = engine.displacement()
            K = fo.assemble_global_stiffness(xyz, e2n, np.ones(len(e2n), bool))
            known, vals = fo.known_dof_map(top, bot, dy, -dy)
            A, b, free = fo.free_system(K, known, vals)
            assert rel(U, fo.solve_system(K, known, vals)) <= 1e-10, (cyc, mesh)
            assert np.linalg.norm(A @ U[free] - b) <= 1e-12 * np.linalg.norm(b)
    assert abs(its[0] - its[1]) <= 1, its


def test_compact_cycle_failure_steps(engine):
    xyz, e2n, top, bot = _sim181147(engine)
    active = np.ones(len(e2n), bool)
    with engine.options(amg_cycle=1):
        for step in (10, 25, 39):
            dy = fo.DISPLACEMENT_MAX * step / (fo.N_STEPS - 1)
            engine.set_active(active)
            f, n_act, st = engine.step(dy, -dy, _opts(1e-13), fo.MAX_STRAIN)
            K = fo.assemble_global_stiffness(xyz, e2n, active)
            known, vals = fo.known_dof_map(top, bot, dy, -dy)
            assert rel(engine.displacement(), fo.solve_system(K, known, vals)) <= 1e-10, step
            active = engine.active()


def test_solve_after_layout_rebuild_assembles(engine):
    """A layout option rebuilds the operator (empty until assembled); the next
    mfea_solve assembles the current active set itself instead of solving a
    zero operator."""
    xyz, e2n, top, bot = _sim181147(engine)
    engine.assemble()
    dy = 0.01
    K = fo.assemble_global_stiffness(xyz, e2n, np.ones(len(e2n), bool))
    known, vals = fo.known_dof_map(top, bot, dy, -dy)
    Uref = fo.solve_system(K, known, vals)
    with engine.options(amg_tail_rows=1024):
        st = engine.solve(dy, -dy, _opts(1e-13))   # rebuilt by the option, not re-assembled by the caller
        assert st.status == 0 and st.iters > 0
        assert rel(engine.displacement(), Uref) <= 1e-10



# ---------------------------------------------------------------------------
# the collapsed compact cycle (amg_collapse: the cycle below level kc as one
# explicit operator V_kc = (2I − Ã) + P̃ V R̂, formed every setup;
# tests/test_amg_cpu.py pins V against the recursion): the direct solve's U
# and the uncollapsed cycle's iteration count, for the automatic level and
# every forced one
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("mesh", ["C2_1x5", "C3_6x8", "C5_2x2", "sim135507_3d"])
def test_collapsed_cycle_matches_direct(engine, mesh):
    dy = fo.DISPLACEMENT_MAX * 20 / (fo.N_STEPS - 1)
    with engine.options(amg_cycle=1, amg_collapse=0):
        xyz, e2n, top, bot = _mesh_case(engine, mesh)
        it0 = engine.solve(dy, -dy, _opts(1e-8)).iters
        nlev = len(engine.amg_info()["rows"])
        K = fo.assemble_global_stiffness(xyz, e2n, np.ones(len(e2n), bool))
        known, vals = fo.known_dof_map(top, bot, dy, -dy)
        A, b, free = fo.free_system(K, known, vals)
        Uref = fo.solve_system(K, known, vals)
        seen = set()
        for coll in [-1] + list(range(1, nlev - 1)):
            engine.set_option("amg_collapse", coll)   # a rebuild: solve re-assembles
            engine.set_option("amg_collapse_mb", 1 << 20 if coll > 0 else 32)
            engine.set_option("amg_collapse_pairs", (1 << 31) - 2 if coll > 0 else 8000000)
            it = engine.solve(dy, -dy, _opts(1e-8)).iters
            kc = engine.get_option("amg_collapse_level")
            assert kc >= 1 and (coll < 0 or kc == coll), (coll, kc)
            seen.add(kc)
            assert abs(it - it0) <= 1, (coll, it, it0)
            st = engine.solve(dy, -dy, _opts(1e-13))
            assert st.status == 0
            U = engine.displacement()
            assert rel(U, Uref) <= 1e-10, (mesh, coll)
            assert np.linalg.norm(A @ U[free] - b) <= 1e-12 * np.linalg.norm(b)
        engine.set_option("amg_collapse_mb", 32)
        engine.set_option("amg_collapse_pairs", 8000000)
    assert len(seen) >= 1


@pytest.mark.parametrize("mesh", ["C2_1x5", "C3_6x8", "C5_2x2", "sim135507_3d"])
def test_fused_setup_bitwise_equals_separate_launches(engine, mesh):
    """The compact operators formed inside the Galerkin chain's launches
    (k_amg_fuse_p / k_amg_fuse_ac) run the same arithmetic as their own
    launches: U and the iteration count bit for bit, collapsed or not."""
    dy = fo.DISPLACEMENT_MAX * 20 / (fo.N_STEPS - 1)
    # spatial 1: Z-ordered level 0, whose fused setup forms A_0, D⁻¹, Ã_0 and
    # P_0 in one row pass (k_amg_a0full) against the separate launches
    for coll, spatial in ((0, -1), (-1, -1), (-1, 1)):
        with engine.options(amg_cycle=1, amg_collapse=coll, amg_spatial=spatial):
            _mesh_case(engine, mesh)
            out = {}
            for v in (0, 1):
                engine.set_option("amg_fuse_setup", v)
                st = engine.solve(dy, -dy, _opts(1e-10))
                assert st.status == 0
                out[v] = (engine.displacement(), st.iters)
            engine.set_option("amg_fuse_setup", 1)
        assert out[0][1] == out[1][1] and np.array_equal(out[0][0], out[1][0]), (mesh, coll, spatial)


def test_default_options_table_matches_library():
    """mfea._capi.DEFAULT_OPTIONS documents the library's option defaults (a
    fresh handle: the session engine's options are test-scoped)."""
    from mfea import Engine
    from mfea._capi import DEFAULT_OPTIONS
    eng = Engine(0)
    try:
        got = {k: eng.get_option(k) for k in DEFAULT_OPTIONS}
    finally:
        eng.close()
    assert got == DEFAULT_OPTIONS


def test_coarse_overrelaxation_fallback(engine):
    """The coarse smoothers' over-relaxed weight (amg_coarse_rho_ppm) is
    measured, not proven, safe (tests/test_amg_cpu.py::
    test_coarse_levels_spectral_radius_below_two).  A weight that breaks the
    cycle — here ρ̂ = 0.2, ω = 6.7 — makes the solve fail; the engine then
    re-forms the hierarchy with the Gershgorin-safe weights and solves again:
    the same U as the default, and the handle stays on the safe weights."""
    sysz = np.load(os.path.join(GOLDEN, "sys_sim_20251117_181147_step20.npz"))
    dy = float(sysz["dy"])
    with engine.options(amg_coarse_rho_ppm=200000):
        _sim181147(engine)
        engine.assemble()
        assert engine.get_option("amg_safe_omega") == 0
        st = engine.solve(dy, -dy, _opts(1e-13))
        assert st.status == 0
        assert engine.get_option("amg_safe_omega") == 1
        assert rel(engine.displacement(), sysz["U"]) <= 1e-10
    assert engine.get_option("amg_safe_omega") == 0  # a new weight, a new chance


def test_level0_blocks_per_position_are_bitwise_the_row_pass(engine):
    """Option amg_a0_slot: level 0's blocks and D⁻¹ formed one thread per SELL
    position (k_amg_a0slot) give the row pass's (k_amg_a0dinv) solves bit for
    bit — on the reference network and on a C2-shaped tiled one."""
    from mfea import PC_GAMG, make_opts, synth
    dy = fo.DISPLACEMENT_MAX * 20 / (fo.N_STEPS - 1)
    xyz, e2n = synth.tiled_mesh(1, 5)
    top, bot = synth.grips(xyz)
    for mesh in ("ref", "tiled"):
        runs = []
        for slot in (0, 1):
            with engine.options(amg_a0_slot=slot):
                if mesh == "ref":
                    _sim181147(engine)
                else:
                    engine.set_mesh(xyz, e2n)
                    engine.set_bc(top, bot)
                    engine.set_active(None)
                out = []
                for k in (1, 2):
                    f, n, st = engine.step(k * dy, -k * dy, make_opts(rtol=1e-10, max_it=20000, precond=PC_GAMG), 0.018)
                    assert st.status == 0
                    out.append((f, st.iters, engine.displacement().copy()))
                runs.append(out)
        for a, b in zip(*runs):
            assert a[0] == b[0] and a[1] == b[1] and np.array_equal(a[2], b[2]), mesh


@pytest.mark.parametrize("precond", ["gamg", "icc"])
def test_setup_entry_in_the_graph_is_bitwise_the_eager_entry(engine, precond):
    """Option setup_entry: the solve's entry launches (level-0 b, the first
    preconditioner application, w, update 0) replayed inside the setup's
    graph give the eager launches' iterates bit for bit, step after step."""
    from mfea import PC_GAMG, PC_ICC, make_opts
    _sim181147(engine)
    pc = PC_GAMG if precond == "gamg" else PC_ICC
    dy = fo.DISPLACEMENT_MAX * 20 / (fo.N_STEPS - 1)
    runs = []
    for entry in (0, 1):
        engine.set_option("setup_entry", entry)
        engine.set_active(None)
        out = []
        for k in (1, 2, 3):
            f, n, st = engine.step(k * dy, -k * dy, make_opts(rtol=1e-10, max_it=20000, precond=pc), 0.018)
            out.append((f, st.iters, engine.displacement().copy()))
        runs.append(out)
    for a, b in zip(*runs):
        assert a[0] == b[0] and a[1] == b[1] and np.array_equal(a[2], b[2])
