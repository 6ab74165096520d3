"""CSV formats of the reference outputs.

Python style (pandas ``to_csv``): written by ``fea_solver.write_records``.
PETSc style: ``std::setprecision(12)`` through an ostream
(src/fea_petsc.cpp:433-516) — ``%.12g`` formatting, active as 1/0, the
mislabelled ``node_i_x…node_i_y…node_i_z`` header over interleaved values.
"""
from __future__ import annotations

import os

import numpy as np


def _g12(v) -> str:
    s = "%.12g" % v
    if s in ("nan", "-nan"):
        return "-nan" if np.signbit(v) else "nan"
    return s


def write_petsc_records(fea_dir, n_nodes, n_elems, stress_record, active_record, disp_record,
                        force_disp_curve):
    hdr_e = ",".join(f"elem_{e}" for e in range(n_elems))
    if stress_record:
        with open(os.path.join(fea_dir, "stress_record.csv"), "w") as f:
            f.write(hdr_e + ",step\n")
            for s, row in enumerate(stress_record):
                f.write(",".join(_g12(v) for v in row) + f",{s + 1}\n")
    if active_record:
        with open(os.path.join(fea_dir, "active_elements.csv"), "w") as f:
            f.write(hdr_e + ",step\n")
            for s, row in enumerate(active_record):
                f.write(",".join("1" if v else "0" for v in row) + f",{s + 1}\n")
    if disp_record:
        with open(os.path.join(fea_dir, "node_displacements.csv"), "w") as f:
            hdr = [f"node_{i}_x" for i in range(n_nodes)] + [f"node_{i}_y" for i in range(n_nodes)] \
                + [f"node_{i}_z" for i in range(n_nodes)]
            f.write(",".join(hdr) + ",step\n")
            for s, row in enumerate(disp_record):
                f.write(",".join(_g12(v) for v in row) + f",{s + 1}\n")
    if force_disp_curve:
        with open(os.path.join(fea_dir, "force_displacement.csv"), "w") as f:
            f.write("total_displacement,total_force\n")
            for a, b in force_disp_curve:
                f.write(f"{_g12(a)},{_g12(b)}\n")
