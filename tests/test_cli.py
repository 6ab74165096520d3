"""The command-line drop-in for the reference's PETSc executables
(mycelium-fea-project_amd/mfea_petsc ↔ src/fea_petsc.cpp main()).

CPU part: argument handling and failure paths need no device (usage, unknown
options, unreadable CSVs, no GPU).  GPU part: the C++ driver's records on the
reference's committed PETSc goldens (results/test_I_cpp) and on the 22k-DOF
network against the committed Python golden (force within 1e-9)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, PKG, read_rt

EXE = os.path.join(PKG, "mfea_petsc")


def run(*args, timeout=300):
    return subprocess.run([EXE, *map(str, args)], capture_output=True, text=True, timeout=timeout)


def test_cli_usage_and_bad_options():
    assert os.path.exists(EXE), "build with make -C mycelium-fea-project_amd"
    r = run()
    assert r.returncode == 1 and "Usage:" in r.stdout
    r = run("x", "-pc_type", "lu")
    assert r.returncode == 1 and "not supported" in r.stderr
    r = run("x", "-ksp_type", "gmres")
    assert r.returncode == 1 and "cg only" in r.stderr
    r = run("x", "-bogus", "1")
    assert r.returncode == 1 and "unknown option" in r.stderr
    r = run("x", "-pc_type", "gamg", "-ksp_norm_type", "natural")
    assert r.returncode == 1 and "not supported" in r.stderr


def test_cli_unreadable_input(tmp_path):
    r = run(tmp_path / "missing")
    assert r.returncode == 1
    assert "Error reading input CSVs: Failed to open nodes file" in r.stdout


def test_cli_without_gpu_fails_cleanly(tmp_path):
    from mfea import Engine, MfeaError
    try:
        Engine(0).close()
        pytest.skip("GPU present")
    except MfeaError:
        pass
    d = tmp_path / "test_I"
    shutil.copytree(os.path.join(GOLDEN, "meshes", "test_I"), d)
    r = run(d)
    assert r.returncode == 1 and "mfea_create" in r.stderr


@pytest.mark.gpu
def test_cli_reproduces_petsc_golden(tmp_path):
    """results/test_I_cpp (PETSc output, 12 significant digits): same files,
    headers and step count; values to the printed precision."""
    d = tmp_path / "test_I_cpp"
    shutil.copytree(os.path.join(GOLDEN, "meshes", "test_I_cpp"), d)
    r = run(d, "-n_steps", 40, "-disp_max", 0.06, "-grip_length", 0.5, "-ksp_rtol", 1e-13,
            "-ksp_norm_type", "unpreconditioned", "-pc_type", "jacobi")
    assert r.returncode == 0, r.stderr
    assert "KSP converged reason: " in r.stdout and "Time taken by myLongRunningFunction" in r.stdout
    ref = os.path.join(GOLDEN, "ref", "test_I_cpp")
    for f in ("force_displacement.csv", "stress_record.csv", "node_displacements.csv",
              "active_elements.csv"):
        a = (d / "fea_results" / f).read_text().splitlines()
        b = open(os.path.join(ref, f)).read().splitlines()
        assert a[0] == b[0] and len(a) == len(b), f
        A = read_rt(d / "fea_results" / f).values
        B = read_rt(os.path.join(ref, f)).values
        assert np.allclose(A, B, rtol=1e-10, atol=1e-14), f
    assert (d / "fea_results" / "runtime.txt").read_text().startswith("FEA run finished")


@pytest.mark.gpu
@pytest.mark.parametrize("pc", ["jacobi", "gamg", "icc", "sor", None])
def test_cli_sim181147_force_matches_python_golden(tmp_path, pc):
    """None: no -pc_type — the reference source's default PCICC
    (src/fea_petsc.cpp:331), here DIC(0)."""
    d = tmp_path / "sim"
    shutil.copytree(os.path.join(GOLDEN, "meshes", "sim_20251117_181147"), d)
    r = run(d, "-ksp_rtol", 1e-13, "-ksp_norm_type", "unpreconditioned", *(["-pc_type", pc] if pc else []),
            "-ksp_max_it", 200000)
    assert r.returncode == 0, r.stderr
    expect = {"jacobi": "jacobi", "gamg": "gamg",
              "icc": "icc (DIC(0) of the whole matrix, chain-piece multicolour order)",
              "sor": "sor (SSOR of the whole matrix, chain-piece multicolour order)"}[pc or "icc"]
    assert f"PC Object: type {expect}\n" in r.stdout
    assert "256-row" not in r.stdout
    F = read_rt(d / "fea_results" / "force_displacement.csv").values
    Fr = read_rt(os.path.join(GOLDEN, "ref", "sim_20251117_181147", "force_displacement.csv")).values
    assert F.shape == Fr.shape
    # 12 printed digits bound the comparison
    assert np.linalg.norm(F[:, 1] - Fr[:, 1]) / np.linalg.norm(Fr[:, 1]) <= 1e-9
    z = np.load(os.path.join(GOLDEN, "ref", "sim_20251117_181147", "active_packed.npz"))
    Ar = np.unpackbits(z["bits"], axis=1)[:, : int(z["n_elems"])].astype(bool)
    A = read_rt(d / "fea_results" / "active_elements.csv").values[:, :-1].astype(bool)
    assert np.array_equal(A, Ar)


@pytest.mark.gpu
def test_cli_skips_out_of_range_elements_like_petsc(tmp_path):
    """results/test_X_cpp_2 references nodes 7-14 of a 7-node file: the PETSc
    driver skips those elements (src/fea_petsc.cpp:241) instead of failing."""
    d = tmp_path / "bad"
    shutil.copytree(os.path.join(GOLDEN, "meshes", "test_X_cpp_2"), d)
    r = run(d, "-grip_length", 0.5)
    assert r.returncode == 0, r.stderr
    assert (d / "fea_results" / "force_displacement.csv").exists()
