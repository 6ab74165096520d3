"""The producer's networks through the FEA hot path (SURVEY §8f3 → §8a).

* The reference-scale network the producer writes for seed 42 (byte-identical
  to the reference's results/sim_20251122_155110, tests/test_grow_cpu.py)
  through the drop-in `fea_solver` — 40 load steps with failures — against the
  oracle's run of the reference algorithm (src/fea_solver.py:186-295): U and
  force within 1e-10 relative L2, identical failure records.
* A 9× larger grown dish (scale 3) solved with GAMG and Jacobi-PCG against
  the direct solve (src/fea_solver.py:128) within 1e-10.
"""
import os

import numpy as np
import pandas as pd
import pytest

pytestmark = pytest.mark.gpu

import fea_oracle as fo  # noqa: E402  (checker only)


def rel(a, b):
    nb = np.linalg.norm(b)
    return np.linalg.norm(np.asarray(a) - np.asarray(b)) / (nb if nb > 0 else 1.0)


def test_grown_reference_network_dropin_matches_oracle(tmp_path):
    import mfea
    import fea_solver as fs
    d = tmp_path / "sim_grown"
    mfea.grow_network(out_dir=str(d))
    nodes = pd.read_csv(d / "nodes.csv")
    elems = pd.read_csv(d / "elements.csv")
    res = fs.fea_solver(str(d), tol=1.5, verbose=False, rtol=1e-13)
    ref = fo.run_fea(nodes[["x", "y", "z"]].values, nodes["node_id"].values, elems[["n1", "n2"]].values,
                     tol=1.5)
    assert res["U"].shape == ref["U"].shape
    assert rel(res["U"], ref["U"]) <= 1e-10
    assert rel(res["force"], ref["force"]) <= 1e-10
    assert np.array_equal(res["active"], ref["active"])
    assert (d / "fea_results" / "force_displacement.csv").exists()


def test_grown_large_network_solves_match_direct(engine):
    import mfea
    from mfea import PC_GAMG, PC_JACOBI, make_opts
    xyz, e2n = mfea.grow_network(mfea.scaled_grow_params(3.0))
    from mfea import synth
    top, bot = synth.grips(xyz)
    engine.set_mesh(xyz, e2n)
    engine.set_bc(top, bot)
    engine.set_active(None)
    engine.assemble()
    dy = fo.DISPLACEMENT_MAX * 20 / (fo.N_STEPS - 1)
    K = fo.assemble_global_stiffness(xyz, e2n, np.ones(len(e2n), bool))
    known, vals = fo.known_dof_map(top, bot, dy, -dy)
    Uref = fo.solve_system(K, known, vals)
    for pc, max_it in ((PC_GAMG, 2000), (PC_JACOBI, 400000)):
        st = engine.solve(dy, -dy, make_opts(rtol=1e-13, max_it=max_it, precond=pc))
        assert st.status == 0, pc
        assert rel(engine.displacement(), Uref) <= 1e-10, (pc, rel(engine.displacement(), Uref))
    assert 3 * len(xyz) > 150000
