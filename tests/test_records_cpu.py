"""The native record writer (mfea_write_record_csv, records.cpp) — host only, no GPU.

Its output must be byte-identical to the reference's writers:
src/fea_solver.py:297-316 (pandas DataFrame.to_csv) and src/fea_petsc.cpp:433-516
(ostream << setprecision(12)).  Checked against pandas itself on random and
adversarial values (subnormals, powers of ten around the repr switch points,
integers, ±0, ±inf, NaN) and against the reference's committed golden files."""
import os

import numpy as np
import pandas as pd
import pytest

from conftest import GOLDEN, read_rt
from mfea import _capi


def _pandas_text(tmp_path, kind, rows, n_cols):
    """What the reference's pandas writer produces (src/fea_solver.py:298-316)."""
    p = tmp_path / "pandas.csv"
    if kind == _capi.REC_FORCE:
        pd.DataFrame(rows, columns=["total_displacement", "total_force"]).to_csv(p, index=False)
    else:
        cols = np.arange(n_cols) if kind == _capi.REC_DISP else [f"elem_{i}" for i in range(n_cols)]
        df = pd.DataFrame(rows, columns=cols)
        df["step"] = np.arange(1, len(rows) + 1)
        df.to_csv(p, index=False)
    return p.read_text()


def _native_text(tmp_path, style, kind, rows, n_cols, threads=4):
    p = tmp_path / "native.csv"
    _capi.write_record_csv(str(p), style, kind, rows, n_cols=n_cols, threads=threads)
    return p.read_text()


def _adversarial(rng, n):
    pow10 = 10.0 ** np.arange(-330, 309, dtype=np.float64)
    special = np.array([0.0, -0.0, 1.0, -1.0, 0.1, 1e-4, 9.999e-5, 1e-5, 1e15, 1e16, 9.999999e15,
                        123456789012345678.0, 5e-324, -5e-324, 2.2250738585072014e-308,
                        1.7976931348623157e308, np.inf, -np.inf, np.nan, 0.5, 100.0, 1234.5,
                        0.30000000000000004, 2.0 ** 53, 2.0 ** 53 + 2])
    with np.errstate(over="ignore"):
        big = -pow10 * 3  # overflows to -inf at the top end (on purpose)
    parts = [special, pow10, big, np.nextafter(pow10, np.inf), np.nextafter(pow10, 0),
             rng.normal(size=n) * 10.0 ** rng.integers(-20, 20, size=n),
             rng.integers(-10 ** 6, 10 ** 6, size=n).astype(np.float64),
             np.frombuffer(rng.bytes(8 * n), dtype=np.float64)]
    return np.concatenate(parts)


@pytest.mark.parametrize("threads", [1, 7])
def test_float_cells_match_pandas_to_csv(tmp_path, threads):
    rng = np.random.default_rng(3)
    v = _adversarial(rng, 20000)
    v = v[: (len(v) // 4) * 4]
    rows = v.reshape(4, -1)
    for kind in (_capi.REC_STRESS, _capi.REC_DISP):
        want = _pandas_text(tmp_path, kind, rows, rows.shape[1])
        got = _native_text(tmp_path, _capi.CSV_PANDAS, kind, rows, rows.shape[1], threads)
        assert got == want


def test_active_and_force_match_pandas(tmp_path):
    rng = np.random.default_rng(5)
    act = rng.random((6, 9000)) < 0.7
    assert _native_text(tmp_path, _capi.CSV_PANDAS, _capi.REC_ACTIVE, act, 9000) == \
        _pandas_text(tmp_path, _capi.REC_ACTIVE, act, 9000)
    fd = np.column_stack([np.linspace(0, 0.04, 40), rng.normal(size=40) * 1e-6])
    assert _native_text(tmp_path, _capi.CSV_PANDAS, _capi.REC_FORCE, fd, 2) == \
        _pandas_text(tmp_path, _capi.REC_FORCE, fd, 2)


def test_empty_records_match_pandas(tmp_path):
    for kind, n in ((_capi.REC_STRESS, 5), (_capi.REC_DISP, 12), (_capi.REC_FORCE, 2)):
        assert _native_text(tmp_path, _capi.CSV_PANDAS, kind, [], n) == \
            _pandas_text(tmp_path, kind, np.zeros((0, n)), n)


def test_petsc_style_matches_ostream_precision12(tmp_path):
    """src/fea_petsc.cpp:449: std::setprecision(12) — "%.12g" with libstdc++."""
    rng = np.random.default_rng(11)
    v = _adversarial(rng, 2000)
    v = v[: (len(v) // 3) * 3]
    got = _native_text(tmp_path, _capi.CSV_PETSC, _capi.REC_DISP, v[None, :], len(v))
    lines = got.splitlines()
    n = len(v) // 3
    hdr = [f"node_{i}_x" for i in range(n)] + [f"node_{i}_y" for i in range(n)] + \
        [f"node_{i}_z" for i in range(n)]
    assert lines[0] == ",".join(hdr) + ",step"
    want = [("%.12g" % x) for x in v]
    want = ["-nan" if (s == "nan" and np.signbit(x)) else s for s, x in zip(want, v)]
    assert lines[1] == ",".join(want) + ",1"


@pytest.mark.parametrize("mesh", ["test_X", "test_I", "test_y"])
def test_native_writer_reproduces_golden_files(tmp_path, mesh):
    """The reference's own committed outputs, re-written from their values."""
    import fea_solver as fs
    ref = os.path.join(GOLDEN, "ref", mesh)
    st = read_rt(os.path.join(ref, "stress_record.csv")).values[:, :-1]
    ac = read_rt(os.path.join(ref, "active_elements.csv")).values[:, :-1].astype(bool)
    U = read_rt(os.path.join(ref, "node_displacements.csv")).values[:, :-1]
    F = read_rt(os.path.join(ref, "force_displacement.csv")).values
    fs.write_records(str(tmp_path), U.shape[1] // 3, st.shape[1], list(st), list(ac), list(U), list(F))
    for f in ("stress_record.csv", "active_elements.csv", "node_displacements.csv",
              "force_displacement.csv"):
        assert (tmp_path / f).read_text() == open(os.path.join(ref, f)).read(), f


def test_petsc_writer_reproduces_cpp_golden(tmp_path):
    import fea_solver as fs
    ref = os.path.join(GOLDEN, "ref", "test_I_cpp")
    st = read_rt(os.path.join(ref, "stress_record.csv")).values[:, :-1]
    ac = read_rt(os.path.join(ref, "active_elements.csv")).values[:, :-1]
    U = read_rt(os.path.join(ref, "node_displacements.csv")).values[:, :-1]
    F = read_rt(os.path.join(ref, "force_displacement.csv")).values
    fs.write_records(str(tmp_path), 4, 3, list(st), list(ac.astype(bool)), list(U), list(F),
                     out_format="petsc")
    for f in ("stress_record.csv", "active_elements.csv", "node_displacements.csv",
              "force_displacement.csv"):
        assert (tmp_path / f).read_text() == open(os.path.join(ref, f)).read(), f


def test_writer_errors_are_reported(tmp_path):
    with pytest.raises(_capi.MfeaError, match="2 columns"):
        _capi.write_record_csv(str(tmp_path / "f.csv"), _capi.CSV_PANDAS, _capi.REC_FORCE,
                               np.zeros((2, 3)))
    with pytest.raises(_capi.MfeaError, match="cannot open"):
        _capi.write_record_csv(str(tmp_path / "no" / "f.csv"), _capi.CSV_PANDAS, _capi.REC_STRESS,
                               np.zeros((1, 3)))


def test_npy_sidecar_roundtrip(tmp_path):
    """mfea_write_record_npy: np.load(allow_pickle=False) returns the record
    array itself (float64 bit for bit incl. NaN / ±0 / subnormals, bool for the
    activity), for every kind and for an empty record."""
    rng = np.random.default_rng(5)
    vals = _adversarial(rng, 3 * 257)[:3 * 257].reshape(3, 257)
    for kind, rec in ((_capi.REC_STRESS, vals), (_capi.REC_DISP, vals[:, :255]),
                      (_capi.REC_FORCE, vals[:, :2])):
        p = tmp_path / f"k{kind}.npy"
        _capi.write_record_npy(str(p), kind, rec)
        got = np.load(p, allow_pickle=False)
        assert got.dtype == np.float64 and got.shape == rec.shape
        assert np.array_equal(got.view(np.uint64), np.ascontiguousarray(rec).view(np.uint64))
    act = rng.random((4, 1000)) < 0.7
    p = tmp_path / "act.npy"
    _capi.write_record_npy(str(p), _capi.REC_ACTIVE, act)
    got = np.load(p, allow_pickle=False)
    assert got.dtype == np.bool_ and np.array_equal(got, act)
    p = tmp_path / "empty.npy"
    _capi.write_record_npy(str(p), _capi.REC_STRESS, [], n_cols=7)
    assert np.load(p, allow_pickle=False).shape == (0, 7)
    # the header is 64-byte aligned, as numpy writes it
    raw = (tmp_path / "act.npy").read_bytes()
    assert raw[:8] == b"\x93NUMPY\x01\x00" and (10 + int.from_bytes(raw[8:10], "little")) % 64 == 0
