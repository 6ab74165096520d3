"""GPU parity of the multi-GPU partitioned solve (partition.hpp).

The partitions run on ONE device here (mfea_debug_set_parts): the same
partition plan, lane kernels (DIST variants) and exchange schedule as the
one-process-per-GPU RCCL path, with device copies standing in for the RCCL
group.  Bars: the displacement within 1e-10 relative L2 of the direct solve,
Jacobi-PCG iteration counts within ±3 of SciPy's, and the drop-in CSV records
equal to the reference's golden vectors, for 2-4 partitions along x and y,
planar (2 DOF lanes) and 3-D (3 DOF lanes) meshes, with element failures
crossing partition boundaries.
"""
import os
import shutil

import numpy as np
import pytest

from conftest import GOLDEN, load_gen, load_mesh, read_rt
from test_gpu_parity import check_stress_records, force_close, rel

pytestmark = pytest.mark.gpu

import fea_oracle as fo  # noqa: E402  (checker only)


@pytest.fixture(scope="module")
def peng():
    from mfea import Engine
    eng = Engine(0)
    yield eng
    eng.close()


def _sim181147(eng, nparts, axis=-1):
    nodes, elems = load_mesh("sim_20251117_181147")
    xyz = nodes[["x", "y", "z"]].values
    top, bot = fo.grip_nodes(xyz, nodes["node_id"].values, 1.5)
    eng.set_parts(nparts, axis)
    eng.set_mesh(xyz, elems[["n1", "n2"]].values)
    eng.set_bc(top, bot)
    eng.set_active(None)
    return xyz, elems[["n1", "n2"]].values, top, bot


@pytest.mark.parametrize("nparts,axis,precond", [(2, -1, 0), (3, 0, 0), (4, 1, 0), (3, -1, 1)])
def test_partitioned_solve_matches_direct(peng, nparts, axis, precond):
    from mfea import make_opts
    sysz = np.load(os.path.join(GOLDEN, "sys_sim_20251117_181147_step20.npz"))
    _sim181147(peng, nparts, axis)
    info = peng.info()
    assert info["n_parts"] == nparts and info["n_pairs"] > 0 and info["n_ghost"] > 0
    peng.assemble()
    dy = float(sysz["dy"])
    st = peng.solve(dy, -dy, make_opts(rtol=1e-13, max_it=200000, precond=precond))
    U = peng.displacement()
    assert st.status == 0
    assert rel(U, sysz["U"]) <= 1e-10
    if precond == 0:
        st8 = peng.solve(dy, -dy, make_opts(rtol=1e-8))
        assert abs(st8.iters - int(sysz["pcg_iters_1e8"])) <= 3


def _its_one_partition(engine, xyz, e2n, top, bot, dy, rtol=1e-8):
    from mfea import PC_GAMG, make_opts
    engine.set_parts(1)
    engine.set_mesh(xyz, e2n)
    engine.set_bc(top, bot)
    engine.set_active(None)
    engine.assemble()
    st = engine.solve(dy, -dy, make_opts(rtol=rtol, max_it=2000, precond=PC_GAMG))
    assert st.status == 0
    return st.iters, engine.displacement()


@pytest.mark.parametrize("nparts,axis", [(2, -1), (3, 0), (4, 1), (4, -1)])
def test_partitioned_gamg_matches_direct(peng, engine, nparts, axis):
    """The distributed V-cycle of ONE global hierarchy (option "amg_dist" 1):
    U to 1e-10 of the direct solve, and the one-partition
    iteration count (±3) at rtol 1e-8 although every strip boundary cuts
    through this network's hyphae."""
    from mfea import PC_GAMG, make_opts
    sysz = np.load(os.path.join(GOLDEN, "sys_sim_20251117_181147_step20.npz"))
    dy = float(sysz["dy"])
    with peng.options(amg_dist=1):
        xyz, e2n, top, bot = _sim181147(peng, nparts, axis)
        peng.assemble()
        st = peng.solve(dy, -dy, make_opts(rtol=1e-13, max_it=2000, precond=PC_GAMG))
        assert st.status == 0 and st.amg_levels >= 3
        assert rel(peng.displacement(), sysz["U"]) <= 1e-10
        assert peng.amg_info()["n_dist"] >= 1
        st8 = peng.solve(dy, -dy, make_opts(rtol=1e-8, max_it=2000, precond=PC_GAMG))
    it1, _ = _its_one_partition(engine, xyz, e2n, top, bot, dy)
    assert abs(st8.iters - it1) <= 3, (st8.iters, it1)


@pytest.mark.parametrize("rep_rows", [0, 300, 1 << 30])
def test_partitioned_gamg_split_depths(peng, rep_rows):
    """Every level split (0: the coarsest solve is local too), the default
    split, and level 0 alone split: the same U to 1e-10 of the direct solve."""
    from mfea import PC_GAMG, make_opts
    sysz = np.load(os.path.join(GOLDEN, "sys_sim_20251117_181147_step20.npz"))
    dy = float(sysz["dy"])
    with peng.options(amg_rep_rows=rep_rows, amg_dist=1, amg_dist_cycle=0):
        _sim181147(peng, 3)
        peng.assemble()
        st = peng.solve(dy, -dy, make_opts(rtol=1e-13, max_it=2000, precond=PC_GAMG))
        info = peng.amg_info()
        U = peng.displacement()
    assert st.status == 0
    if rep_rows == 0:
        assert info["n_dist"] == info["levels"]
    if rep_rows == 1 << 30:
        assert info["n_dist"] == 1
    assert rel(U, sysz["U"]) <= 1e-10


@pytest.mark.parametrize("nparts", [2, 3, 8])
def test_partitioned_compact_cycle_matches_four_step_and_one_partition(peng, engine, nparts):
    """The distributed V-cycle in its compact form (option amg_dist_cycle 1:
    level 0 split, the levels below replicated and collapsed as on one
    partition; capi.hip enqueue_gamg_vcycle) against the four-step form and
    the one-partition hierarchy: U to 1e-10 of the direct solve and within
    1e-12·‖U‖ of the four-step form at rtol 1e-14, the one-partition
    iteration count at 1e-8 (±1), and one cycle's output equal to the
    one-partition compact cycle's up to f32 rounding."""
    from mfea import PC_GAMG, make_opts
    sysz = np.load(os.path.join(GOLDEN, "sys_sim_20251117_181147_step20.npz"))
    dy = float(sysz["dy"])
    out = {}
    for cyc in (1, 0):
        with peng.options(amg_dist=1, amg_dist_cycle=cyc):
            xyz, e2n, top, bot = _sim181147(peng, nparts)
            peng.assemble()
            st = peng.solve(dy, -dy, make_opts(rtol=1e-14, max_it=2000, precond=PC_GAMG))
            assert st.status == 0, cyc
            U = peng.displacement()
            st8 = peng.solve(dy, -dy, make_opts(rtol=1e-8, max_it=2000, precond=PC_GAMG))
            info = peng.amg_info()
            # a random residual on the loaded rows (zero on the grips and on
            # the pieces cut off from them, as every CG residual is there:
            # their near-singular coarse blocks would amplify anything else)
            import scipy.sparse as sps
            from scipy.sparse.csgraph import connected_components
            rng = np.random.default_rng(4)
            r = rng.standard_normal((len(xyz), 2))
            g = sps.coo_matrix((np.ones(len(e2n)), (e2n[:, 0], e2n[:, 1])), shape=(len(xyz),) * 2)
            _, lab = connected_components(g, directed=False)
            anchored = np.zeros(lab.max() + 1, bool)
            anchored[lab[np.concatenate([top, bot])]] = True
            known = ~anchored[lab]
            known[np.concatenate([top, bot])] = True
            r[known] = 0
            u = peng.amg_vcycle(r)
        out[cyc] = (U, st8.iters, info, u)
        assert rel(U, sysz["U"]) <= 1e-10, cyc
    assert out[1][2]["n_dist"] == 1
    assert np.linalg.norm(out[1][0] - out[0][0]) <= 1e-12 * np.linalg.norm(out[0][0]) * 100
    it1, _ = _its_one_partition(engine, xyz, e2n, top, bot, dy)
    assert abs(out[1][1] - it1) <= 1, (out[1][1], it1)
    u1 = engine.amg_vcycle(r)
    assert rel(out[1][3], u1) <= 1e-5


@pytest.mark.parametrize("nparts,amg_dist", [(2, 1), (3, 1), (2, 0), (4, 0)])
def test_partitioned_gamg_preconditioned_norm(peng, engine, nparts, amg_dist):
    """PETSc's default KSPCG test (‖M⁻¹r‖ ≤ rtol·‖M⁻¹b‖, src/fea_petsc.cpp:
    336-341) on the partitioned GAMG forms: the stopping ratio is formed from
    the rank-gathered ‖M⁻¹b‖ (k_amg_cg_update<DIST>).  The global hierarchy
    (amg_dist 1) is the one-partition preconditioner, so it stops on the
    one-partition iteration (±1) with the same ratio; block Jacobi (0) stops
    below rtol; a tight rtol reaches the direct solve either way."""
    from mfea import NORM_PRECONDITIONED, PC_GAMG, make_opts
    sysz = np.load(os.path.join(GOLDEN, "sys_sim_20251117_181147_step20.npz"))
    dy = float(sysz["dy"])
    pre = make_opts(rtol=1e-5, max_it=5000, precond=PC_GAMG, norm=NORM_PRECONDITIONED)
    tight = make_opts(rtol=1e-14, max_it=5000, precond=PC_GAMG, norm=NORM_PRECONDITIONED)
    with peng.options(amg_dist=amg_dist):
        xyz, e2n, top, bot = _sim181147(peng, nparts)
        peng.assemble()
        st = peng.solve(dy, -dy, pre)
        assert st.status == 0 and 0 < st.relres <= 1e-5 and st.iters > 0
        assert peng.solve(dy, -dy, tight).status == 0
        assert rel(peng.displacement(), sysz["U"]) <= 1e-10
    if amg_dist == 1:
        engine.set_parts(1)
        engine.set_mesh(xyz, e2n)
        engine.set_bc(top, bot)
        engine.set_active(None)
        engine.assemble()
        st1 = engine.solve(dy, -dy, pre)
        assert st1.status == 0 and abs(st.iters - st1.iters) <= 1, (st.iters, st1.iters)
        if st.iters == st1.iters:
            # the f32 V-cycle sums split levels in another order: ‖M⁻¹r‖ moves
            # in the 6th digit (measured 2.4e-6 relative at 2 parts)
            assert abs(st.relres - st1.relres) <= 1e-4 * st1.relres


@pytest.mark.parametrize("nparts,axis", [(2, -1), (3, 0), (4, 1)])
def test_partitioned_block_jacobi_gamg_matches_direct(peng, nparts, axis):
    """Option "amg_dist" 0: block Jacobi over per-partition hierarchies inside
    the global CG (amg.hpp AmgHalo).  This network has no sparse gap for the
    strip boundaries to follow, so the dropped couplings cost iterations
    (≈ 190-310 at 1e-8 vs 17 on one partition); U still to 1e-10."""
    from mfea import PC_GAMG, make_opts
    sysz = np.load(os.path.join(GOLDEN, "sys_sim_20251117_181147_step20.npz"))
    with peng.options(amg_dist=0):
        _sim181147(peng, nparts, axis)
        peng.assemble()
        dy = float(sysz["dy"])
        st = peng.solve(dy, -dy, make_opts(rtol=1e-13, max_it=2000, precond=PC_GAMG))
        assert st.status == 0 and st.amg_levels >= 3
        assert rel(peng.displacement(), sysz["U"]) <= 1e-10
        st8 = peng.solve(dy, -dy, make_opts(rtol=1e-8, max_it=2000, precond=PC_GAMG))
    assert st8.iters <= int(sysz["pcg_iters_1e8"]) // 4, st8.iters


def test_partitioned_gamg_auto_mode_picks_the_faster(peng, engine):
    """Option "amg_dist" -1 (the default): the first solve of an active set
    runs the global hierarchy, the second block Jacobi, the third the faster
    — on this network (no gaps for the cuts to follow) the global one, with
    the one-partition iteration count."""
    from mfea import PC_GAMG, make_opts
    sysz = np.load(os.path.join(GOLDEN, "sys_sim_20251117_181147_step20.npz"))
    dy = float(sysz["dy"])
    assert peng.get_option("amg_dist") == -1
    xyz, e2n, top, bot = _sim181147(peng, 3)
    peng.assemble()
    its = [peng.solve(dy, -dy, make_opts(rtol=1e-8, max_it=2000, precond=PC_GAMG)).iters for _ in range(3)]
    it1, _ = _its_one_partition(engine, xyz, e2n, top, bot, dy)
    assert abs(its[0] - it1) <= 3 and its[1] > 4 * it1, (its, it1)
    assert its[2] == its[0], its
    assert rel(peng.displacement(), sysz["U"]) <= 1e-6


def test_partitioned_gamg_grown_network_8_parts(peng, engine):
    """A network grown by the native producer (165k DOF, no tiling gaps) on 8
    partitions: the one-partition iteration count (±3) and the same U."""
    from mfea import PC_GAMG, grow_network, make_opts, scaled_grow_params, synth
    xyz, e2n = grow_network(scaled_grow_params(3))
    top, bot = synth.grips(xyz)
    it1, U1 = _its_one_partition(engine, xyz, e2n, top, bot, 0.01)
    peng.set_parts(8, -1)
    peng.set_mesh(xyz, e2n)
    peng.set_bc(top, bot)
    peng.set_active(None)
    peng.assemble()
    with peng.options(amg_dist=1):
        st = peng.solve(0.01, -0.01, make_opts(rtol=1e-8, max_it=2000, precond=PC_GAMG))
    assert st.status == 0 and peng.info()["n_parts"] == 8
    assert abs(st.iters - it1) <= 3, (st.iters, it1)
    assert rel(peng.displacement(), U1) <= 1e-6


@pytest.mark.parametrize("nparts,axis", [(2, 0), (4, 0), (2, 1), (4, -1), (8, -1)])
def test_partitioned_gamg_iterations_on_tiled_network(peng, engine, nparts, axis):
    """A tiled network (4×4 tiles, 340k DOF): the strip boundaries fall in the
    gaps between tiles (partition.hpp min-cut placement; axis -1 = the px × py
    grid with the fewest cut elements) and the partitioned hierarchy converges
    in the one-partition iteration count (±2).  (Forced 1-D strips one tile
    row tall — 4 along y here — need ≈ 200: DESIGN.md §5.)"""
    from mfea import PC_GAMG, make_opts, synth
    xyz, e2n = synth.tiled_mesh(4, 4)
    top, bot = synth.grips(xyz)
    its, Us = [], []
    for eng, n in ((engine, 1), (peng, nparts)):
        eng.set_parts(n, axis)
        eng.set_mesh(xyz, e2n)
        eng.set_bc(top, bot)
        eng.set_active(None)
        eng.assemble()
        st = eng.solve(0.01, -0.01, make_opts(rtol=1e-8, max_it=2000, precond=PC_GAMG))
        assert st.status == 0
        its.append(st.iters)
        Us.append(eng.displacement())
    engine.set_parts(1)
    assert abs(its[1] - its[0]) <= 2, its
    assert rel(Us[1], Us[0]) <= 1e-6


@pytest.mark.parametrize("precond,amg_dist", [(0, -1), (2, 1), (2, 0)])
def test_partitioned_graph_replay_equals_eager(peng, precond, amg_dist):
    """The chunk (kernels + exchanges) as a hipGraph replay and as eager
    launches: the same operations in the same order, bit-equal U (GAMG: the
    distributed V-cycle and block Jacobi)."""
    from mfea import make_opts
    _sim181147(peng, 3)
    peng.assemble()
    opts = make_opts(rtol=1e-10, max_it=200000, precond=precond)
    out = []
    for g in (1, 0):
        with peng.options(dist_graph=g, amg_dist=amg_dist):
            st = peng.solve(0.01, -0.01, opts)
            out.append((st.iters, peng.displacement()))
    assert out[0][0] == out[1][0]
    assert np.array_equal(out[0][1], out[1][1])


def test_partitioned_gamg_step_with_failures(peng):
    """Load steps with element failures on 3 partitions under GAMG: each
    step's U against the direct solve of that step's K (the hierarchy of every
    partition follows its own active elements)."""
    from mfea import PC_GAMG, make_opts
    xyz, e2n, top, bot = _sim181147(peng, 3)
    active = np.ones(len(e2n), bool)
    for step in (10, 25, 39):
        dy = fo.DISPLACEMENT_MAX * step / (fo.N_STEPS - 1)
        peng.set_active(active)
        f, n_act, st = peng.step(dy, -dy, make_opts(rtol=1e-13, max_it=2000, precond=PC_GAMG), fo.MAX_STRAIN)
        K = fo.assemble_global_stiffness(xyz, e2n, active)
        known, vals = fo.known_dof_map(top, bot, dy, -dy)
        assert rel(peng.displacement(), fo.solve_system(K, known, vals)) <= 1e-10, step
        active = peng.active()
    assert n_act < len(e2n)


def test_partitioned_global_activity_follows_failures(peng):
    """The global activity the partitioned GAMG plan reads moves by the
    failed-element ids each post exchanges (no E-byte reduction): after steps
    with failures and no mfea_set_active in between it equals the gathered
    device activity, and the solves still match the direct solve."""
    from mfea import PC_GAMG, make_opts
    xyz, e2n, top, bot = _sim181147(peng, 4)
    peng.set_active(None)
    active = np.ones(len(e2n), bool)
    seen_failures = False
    for step in (20, 30, 39):
        dy = fo.DISPLACEMENT_MAX * step / (fo.N_STEPS - 1)
        f, n_act, st = peng.step(dy, -dy, make_opts(rtol=1e-13, max_it=2000, precond=PC_GAMG), fo.MAX_STRAIN)
        K = fo.assemble_global_stiffness(xyz, e2n, active)
        known, vals = fo.known_dof_map(top, bot, dy, -dy)
        assert rel(peng.displacement(), fo.solve_system(K, known, vals)) <= 1e-10, step
        active = peng.active()
        seen_failures |= n_act < len(e2n)
        assert np.array_equal(peng.global_active(), active), step
    assert seen_failures


def test_partitioned_solve_deterministic(peng):
    from mfea import make_opts
    _sim181147(peng, 3)
    peng.assemble()
    peng.solve(0.01, -0.01, make_opts(rtol=1e-10))
    U1 = peng.displacement()
    peng.assemble()
    peng.solve(0.01, -0.01, make_opts(rtol=1e-10))
    assert np.array_equal(U1, peng.displacement())


def test_partitioned_step_matches_single_partition(peng, engine):
    """One full load step (assembly → PCG → reaction, stress, failures) of the
    C2-shaped network (1×5 tiles, 110k DOF) on 4 partitions vs 1."""
    from mfea import make_opts, synth
    xyz, e2n = synth.tiled_mesh(1, 5)
    top, bot = synth.grips(xyz)
    out = []
    for eng, npart in ((engine, 1), (peng, 4)):
        eng.set_parts(npart)
        eng.set_mesh(xyz, e2n)
        eng.set_bc(top, bot)
        eng.set_active(None)
        f, n_act, st = eng.step(0.0102564, -0.0102564, make_opts(rtol=1e-13, max_it=200000), 0.018)
        out.append((f, n_act, st.iters, eng.displacement(), eng.stress(), eng.active()))
    engine.set_parts(1)
    (f1, n1, it1, U1, S1, A1), (f4, n4, it4, U4, S4, A4) = out
    assert abs(it1 - it4) <= 3
    assert rel(U4, U1) <= 1e-10
    # the reaction is a sum of K·U over the grip rows with heavy cancellation
    # (|f| ≈ 1e-5 of Σ|terms|): relative agreement is ~1e5 × the U error
    assert abs(f4 - f1) <= 1e-8 * abs(f1)
    assert n4 == n1 and np.array_equal(A4, A1)
    assert rel(S4, S1) <= 1e-8


def _run_dropin(tmp_path, mesh, n_steps, dmax, grip, nparts):
    import fea_solver as fs
    d = tmp_path / mesh
    shutil.copytree(os.path.join(GOLDEN, "meshes", mesh), d)
    saved = (fs.N_STEPS, fs.DISPLACEMENT_MAX)
    fs.N_STEPS, fs.DISPLACEMENT_MAX = n_steps, dmax
    try:
        fs.fea_solver(str(d), tol=grip, verbose=False, nparts=nparts)
    finally:
        fs.N_STEPS, fs.DISPLACEMENT_MAX = saved
        fs.get_engine().set_parts(1)
    return d / "fea_results"


@pytest.mark.parametrize("gen,mesh,nparts", [
    ("gen_sim_20251117_175809_default.npz", "sim_20251117_175809", 3),
    ("gen_sim_20251115_135507_grip05.npz", "sim_20251115_135507", 2),   # 3D mesh (z ≠ 0)
])
def test_partitioned_dropin_matches_reference_vectors(tmp_path, gen, mesh, nparts):
    g = load_gen(gen)
    res = _run_dropin(tmp_path, mesh, int(g["n_steps"]), float(g["dmax"]), float(g["grip"]), nparts)
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


def test_partitioned_failures_match_committed_golden(tmp_path):
    """The reference's 22k-DOF run with element failures, on 2 partitions."""
    res = _run_dropin(tmp_path, "sim_20251117_181147", 40, 0.02, 1.5, 2)
    F = read_rt(res / "force_displacement.csv").values
    Fr = read_rt(os.path.join(GOLDEN, "ref", "sim_20251117_181147", "force_displacement.csv")).values
    assert rel(F[:, 1], Fr[:, 1]) <= 1e-9
    z = np.load(os.path.join(GOLDEN, "ref", "sim_20251117_181147", "active_packed.npz"))
    Ar = np.unpackbits(z["bits"], axis=1)[:, : int(z["n_elems"])].astype(bool)
    A = read_rt(res / "active_elements.csv").values[:, :-1].astype(bool)
    assert np.array_equal(A, Ar)


def test_dropin_partitioned_csvs_match_one_partition(tmp_path):
    """The drop-in's records on 3 partitions (the multi-GPU plan, one device)
    equal the one-partition records: same files, same columns, the same
    failures; U and stress to 1e-10, the force (a sum with heavy
    cancellation) to 1e-8."""
    import pandas as pd
    out = []
    for n in (1, 3):
        d = tmp_path / f"p{n}"
        d.mkdir()
        res = _run_dropin(d, "sim_20251117_175809", 40, 0.02, 1.5, n)
        out.append({f: pd.read_csv(res / f, float_precision="round_trip")
                    for f in ("force_displacement.csv", "stress_record.csv", "active_elements.csv",
                              "node_displacements.csv")})
    a, b = out
    for f in a:
        assert list(a[f].columns) == list(b[f].columns) and a[f].shape == b[f].shape, f
    assert a["active_elements.csv"].equals(b["active_elements.csv"])
    # stress = E·n·(u2 − u1)/L: a difference of nearly equal displacements,
    # so its relative agreement is ~1e3 × U's
    for f, tol in (("node_displacements.csv", 1e-10), ("stress_record.csv", 1e-7)):
        A, B = a[f].values[:, :-1], b[f].values[:, :-1]
        for k in range(1, len(A)):
            assert rel(B[k], A[k]) <= tol, (f, k)
    Fa, Fb = a["force_displacement.csv"].values, b["force_displacement.csv"].values
    assert np.array_equal(Fa[:, 0], Fb[:, 0])
    assert np.abs(Fb[:, 1] - Fa[:, 1]).max() <= 1e-8 * np.abs(Fa[:, 1]).max()


def test_partitioned_coarse_overrelaxation_fallback(peng):
    """The over-relaxed coarse smoothers' fallback on a partitioned handle
    (both GAMG forms): a breaking weight (ρ̂ = 0.2) makes the solve fail, every
    partition re-forms its levels with the Gershgorin-safe weights, and the
    solve still meets the direct solve."""
    from mfea import PC_GAMG, make_opts
    sysz = np.load(os.path.join(GOLDEN, "sys_sim_20251117_181147_step20.npz"))
    dy = float(sysz["dy"])
    for dist in (1, 0):
        with peng.options(amg_coarse_rho_ppm=200000, amg_dist=dist):
            _sim181147(peng, 4, -1)
            peng.assemble()
            st = peng.solve(dy, -dy, make_opts(rtol=1e-13, max_it=2000, precond=PC_GAMG))
            assert st.status == 0 and peng.get_option("amg_safe_omega") == 1, dist
            assert rel(peng.displacement(), sysz["U"]) <= 1e-10, dist
