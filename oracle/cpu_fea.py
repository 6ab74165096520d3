"""ctypes wrapper of oracle/cpu_fea.c — TEST/BASELINE INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libcpu_fea.so")
SRC = os.path.join(HERE, "cpu_fea.c")


def build(force=False):
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        subprocess.check_call(["gcc", "-O3", "-march=x86-64-v3", "-ffp-contract=off", "-fopenmp", "-shared", "-fPIC",
                               SRC, "-o", LIB, "-lm"])
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = C.CDLL(LIB)
        P = C.c_void_p
        _lib.cpu_set_material.argtypes = [C.c_double] * 3
        _lib.cpu_mesh_create.restype = P
        _lib.cpu_mesh_create.argtypes = [C.c_int64, P, C.c_int64, P, C.c_int64, P, C.c_int64, P]
        _lib.cpu_mesh_destroy.argtypes = [P]
        _lib.cpu_fea_step.restype = C.c_int
        _lib.cpu_fea_step.argtypes = [P, P, C.c_double, C.c_double, C.c_double, C.c_int, C.c_double,
                                      C.c_double, C.c_int, P, P, P, P, P]
    return _lib


class CpuFea:
    """One mesh on the host; step() runs assemble + RHS + Jacobi-PCG + post."""

    def __init__(self, xyz, e2n, top, bot, E, A, I):
        L = lib()
        self.xyz = np.ascontiguousarray(xyz, dtype=np.float64)
        self.e2n = np.ascontiguousarray(e2n, dtype=np.int64)
        self.top = np.ascontiguousarray(top, dtype=np.int64)
        self.bot = np.ascontiguousarray(bot, dtype=np.int64)
        L.cpu_set_material(E, A, I)
        p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
        self.m = L.cpu_mesh_create(len(self.xyz), p(self.xyz), len(self.e2n), p(self.e2n),
                                   len(self.top), p(self.top), len(self.bot), p(self.bot))
        self.active = np.ones(len(self.e2n), dtype=np.uint8)

    def step(self, dy_top, dy_bot, rtol=1e-8, max_it=100000, reg=1e-12, max_strain=0.018,
             threads=0):
        L = lib()
        U = np.empty(3 * len(self.xyz))
        stress = np.empty(len(self.e2n))
        F = C.c_double()
        rr = C.c_double()
        times = np.zeros(4)
        p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
        it = L.cpu_fea_step(self.m, p(self.active), dy_top, dy_bot, rtol, max_it, reg, max_strain,
                            threads, p(U), p(stress), C.byref(F), C.byref(rr), p(times))
        return {"iters": it, "U": U, "stress": stress, "force": F.value, "relres": rr.value,
                "times": times, "active": self.active.astype(bool).copy()}

    def close(self):
        if self.m:
            lib().cpu_mesh_destroy(self.m)
            self.m = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
