"""ctypes binding of libmfea.so (include/mfea.h).

The HIP library is the product path: if it is missing this module raises
ImportError at import time — there is no CPU fallback.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# mfea_set_option defaults (include/mfea_debug.h)
DEFAULT_OPTIONS = {"graph": 1, "phase_times": 0, "dist_graph": 1, "order": -1, "lane_dof": 0, "cg_kernel": 0,
                   "ell_block": 256, "ell_maxg": 0, "ell_compact": 1, "amg_tail_rows": 2048,
                   "amg_max_levels": 32, "amg_restrict_lanes": 0, "amg_op_lanes": 0,
                   "amg_tail_lds": 1, "dist_timeout_ms": 60000, "part_slack_pct": 35, "amg_dist": -1,
                   "amg_rep_rows": 32768, "amg_dist_cycle": 1, "dist_sums": 1, "amg_cycle": 1, "amg_fuse_setup": 1,
                   "amg_up_lanes": 0, "amg_spatial": -1, "amg_collapse": -1, "amg_collapse_mb": 32,
                   "amg_collapse_pairs": 8000000, "amg_theta_ppm": 0, "amg_reuse": 1, "amg_rebuild_pct": 800, "amg_rebuild_rent": 100,
                   "amg_coarse_rho_ppm": 1750000, "sweep_piece": 64, "cc_tile": 1024,
                   "asm_kernel": 0, "spec_post": 1, "setup_entry": 1,
                   "batch_graph": 1, "step_graph": 0,
                   "graph_start": 1, "combo_graph": 1, "amg_a0_slot": 1}
CG_KERNEL = {"auto": 0, "lanes": 1, "sell": 2}

LIB_PATH = os.environ.get("MFEA_LIB", os.path.join(os.path.dirname(_HERE), "libmfea.so"))

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"mfea: HIP library not found at {LIB_PATH}; build it with "
        f"`make -C mycelium-fea-project_amd` (or __graft_entry__.build())")
_lib = C.CDLL(LIB_PATH)

# error codes (mfea.h)
OK, EINVAL, EDEVICE, ESTATE, EMAXIT, EBREAKDOWN, ENOMEM, ECOMM = 0, -1, -2, -3, -4, -5, -6, -7
PC_JACOBI, PC_BLOCK_JACOBI, PC_GAMG, PC_SOR, PC_ICC = 0, 1, 2, 3, 4
NORM_UNPRECONDITIONED, NORM_PRECONDITIONED = 0, 1
MESH_SKIP_INVALID = 1


class SolveOpts(C.Structure):
    _fields_ = [("rtol", C.c_double), ("atol", C.c_double), ("max_it", C.c_int32),
                ("precond", C.c_int32), ("norm", C.c_int32), ("chunk", C.c_int32),
                ("reg", C.c_double)]


class Stats(C.Structure):
    _fields_ = [("iters", C.c_int32), ("status", C.c_int32), ("relres", C.c_double),
                ("bnorm", C.c_double), ("n_free", C.c_int64), ("t_assemble_ms", C.c_double),
                ("t_rhs_ms", C.c_double), ("t_solve_ms", C.c_double), ("t_post_ms", C.c_double),
                ("t_setup_ms", C.c_double), ("amg_levels", C.c_int32), ("amg_rebuilt", C.c_int32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class Info(C.Structure):
    _fields_ = [("n_nodes", C.c_int64), ("n_elems", C.c_int64), ("n_free_nodes", C.c_int64),
                ("n_top", C.c_int64), ("n_known", C.c_int64), ("n_slices", C.c_int64),
                ("n_slots", C.c_int64), ("free_incidences", C.c_int64), ("planar", C.c_int32),
                ("cg_lanes", C.c_int32), ("n_lanes", C.c_int64), ("n_halo", C.c_int64),
                ("n_parts", C.c_int32), ("part", C.c_int32), ("n_pairs", C.c_int64),
                ("n_ghost", C.c_int64), ("halo_compact", C.c_int32), ("block_size", C.c_int32),
                ("grid", C.c_int64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class GrowParams(C.Structure):
    """mfea_grow_params (include/mfea.h) — src/mycelium_sim_2D.cpp:17-33."""
    _fields_ = [("seed", C.c_uint64),
                ("h0", C.c_double), ("dt", C.c_double), ("lambda_angle", C.c_double),
                ("P_branch", C.c_double), ("c_g", C.c_double), ("D", C.c_double),
                ("M_cap", C.c_double), ("omega0", C.c_double),
                ("t_steps", C.c_int32), ("h0_per_point", C.c_int32),
                ("anastomosis_tol", C.c_double), ("wall_thickness", C.c_double),
                ("dish_size", C.c_double), ("substrate_width", C.c_double), ("substrate_E", C.c_double),
                ("inoc_nx", C.c_int32), ("inoc_ny", C.c_int32), ("inoc_dist", C.c_double),
                ("voxel_size", C.c_double), ("snapshot_every", C.c_int32), ("snapshot_dir", C.c_char_p),
                ("verbose", C.c_int32), ("threads", C.c_int32)]


_P = C.c_void_p
_sig = {
    "mfea_get_info": (C.c_int, [_P, C.POINTER(Info)]),
    "mfea_profile_iteration": (C.c_int, [_P, C.c_int, C.c_int, C.POINTER(C.c_double)]),
    "mfea_profile_spmv": (C.c_int, [_P, C.c_int, C.POINTER(C.c_double)]),
    "mfea_abi_version": (C.c_int, []),
    "mfea_last_error": (C.c_int, [C.c_char_p, C.c_size_t]),
    "mfea_create": (C.c_int, [C.c_int, C.POINTER(_P)]),
    "mfea_destroy": (C.c_int, [_P]),
    "mfea_set_material": (C.c_int, [_P, C.c_double, C.c_double, C.c_double]),
    "mfea_set_mesh": (C.c_int, [_P, C.c_int64, _P, C.c_int64, _P, C.c_uint32]),
    "mfea_set_bc": (C.c_int, [_P, C.c_int64, _P, C.c_int64, _P]),
    "mfea_set_active": (C.c_int, [_P, _P]),
    "mfea_assemble": (C.c_int, [_P]),
    "mfea_solve": (C.c_int, [_P, C.c_double, C.c_double, C.POINTER(SolveOpts), C.POINTER(Stats)]),
    "mfea_post": (C.c_int, [_P, C.c_double, C.POINTER(C.c_double), C.POINTER(C.c_int64)]),
    "mfea_step": (C.c_int, [_P, C.c_double, C.c_double, C.POINTER(SolveOpts), C.c_double,
                            C.POINTER(C.c_double), C.POINTER(C.c_int64), C.POINTER(Stats)]),
    "mfea_get_displacement": (C.c_int, [_P, _P]),
    "mfea_get_stress": (C.c_int, [_P, _P]),
    "mfea_get_active": (C.c_int, [_P, _P]),
    "mfea_element_stiffness": (C.c_int, [_P, C.c_int64, _P, _P, C.c_double, C.c_double,
                                         C.c_double, _P, _P]),
    "mfea_export_csr": (C.c_int, [_P, C.POINTER(C.c_int64), _P, _P, _P]),
    "mfea_solve_csr": (C.c_int, [_P, C.c_int64, _P, _P, _P, C.c_int64, _P, _P,
                                 C.POINTER(SolveOpts), _P, C.POINTER(Stats)]),
    "mfea_dist_unique_id": (C.c_int, [_P]),
    "mfea_dist_init": (C.c_int, [_P, C.c_int, C.c_int, _P]),
    "mfea_set_partition_axis": (C.c_int, [_P, C.c_int]),
    "mfea_get_ownership": (C.c_int, [_P, _P, _P]),
    "mfea_gather_results": (C.c_int, [_P, _P, _P, _P]),
    "mfea_write_record_npy": (C.c_int, [C.c_char_p, C.c_int, C.c_int64, C.c_int64, _P, _P]),
    "mfea_write_record_csv": (C.c_int, [C.c_char_p, C.c_int, C.c_int, C.c_int64, C.c_int64, _P, _P,
                                        C.c_int]),
    "mfea_grow_default_params": (None, [C.POINTER(GrowParams)]),
    "mfea_grow": (C.c_int, [C.POINTER(GrowParams), C.POINTER(_P)]),
    "mfea_grow_info": (C.c_int, [_P, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "mfea_grow_mesh": (C.c_int, [_P, _P, _P]),
    "mfea_grow_write": (C.c_int, [_P, C.c_char_p]),
    "mfea_grow_free": (None, [_P]),
    # include/mfea_debug.h
    "mfea_debug_trace_iteration": (C.c_int, [_P, C.c_int, _P, C.c_int64, C.POINTER(C.c_int64)]),
    "mfea_debug_set_parts": (C.c_int, [_P, C.c_int, C.c_int]),
    "mfea_debug_global_active": (C.c_int, [_P, C.c_void_p]),
    "mfea_debug_floating": (C.c_int, [_P, C.c_void_p]),
    "mfea_set_option": (C.c_int, [_P, C.c_char_p, C.c_int64]),
    "mfea_get_option": (C.c_int, [_P, C.c_char_p, C.POINTER(C.c_int64)]),
    "mfea_debug_amg_vcycle": (C.c_int, [_P, _P, _P]),
    "mfea_debug_amg_vector": (C.c_int, [_P, C.c_int, C.c_int, _P, C.c_int64, C.POINTER(C.c_int64)]),
    "mfea_debug_amg_info": (C.c_int, [_P, C.POINTER(C.c_int), _P, _P, _P, C.c_int,
                                      C.POINTER(C.c_int64), C.POINTER(C.c_int), C.POINTER(C.c_int), _P]),
}
for _name, (_res, _args) in _sig.items():
    _f = getattr(_lib, _name)
    _f.restype = _res
    _f.argtypes = _args

EXPORTED = tuple(_sig)


class MfeaError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"mfea error {code}: {msg}")
        self.code = code


class SolverFailure(np.linalg.LinAlgError):
    """PCG did not converge (max_it) or broke down.  Subclasses LinAlgError so
    the reference driver's ``except np.linalg.LinAlgError`` (src/fea_solver.py:247)
    catches it."""

    def __init__(self, code, msg, stats=None):
        super().__init__(f"mfea solver failure {code}: {msg}")
        self.code = code
        self.stats = stats


def last_error() -> str:
    buf = C.create_string_buffer(1024)
    _lib.mfea_last_error(buf, len(buf))
    return buf.value.decode(errors="replace")


def _check(rc, stats=None):
    if rc == OK:
        return
    if rc in (EMAXIT, EBREAKDOWN):
        raise SolverFailure(rc, last_error(), stats)
    raise MfeaError(rc, last_error())


def _ptr(a):
    return a.ctypes.data_as(_P) if a is not None and a.size else None


def abi_version() -> int:
    return _lib.mfea_abi_version()


def dist_unique_id() -> bytes:
    """The 128-byte RCCL unique id (rank 0 makes it, the launcher broadcasts it)."""
    buf = (C.c_uint8 * 128)()
    _check(_lib.mfea_dist_unique_id(buf))
    return bytes(buf)


CSV_PANDAS, CSV_PETSC = 0, 1
REC_STRESS, REC_ACTIVE, REC_DISP, REC_FORCE = 0, 1, 2, 3


def write_record_csv(path, style, kind, records, n_cols=None, threads=None):
    """One end-of-run record file through the native writer (mfea_write_record_csv):
    byte-identical to the reference's pandas / ostream writers.  records: list
    of per-step rows (or a 2-D array)."""
    flags = kind == REC_ACTIVE
    dt = np.uint8 if flags else np.float64
    if len(records):
        a = np.ascontiguousarray(np.asarray(records), dtype=dt).reshape(len(records), -1)
    else:
        a = np.zeros((0, n_cols or 0), dtype=dt)
    nr, nc = a.shape
    if threads is None:
        threads = min(16, os.cpu_count() or 1)
    p = a.ctypes.data_as(_P) if a.size else None
    _check(_lib.mfea_write_record_csv(os.fsencode(path), int(style), int(kind), nr, nc,
                                      None if flags else p, p if flags else None, int(threads)))


def write_record_npy(path, kind, records, n_cols=None):
    """The record as a .npy sidecar through the native writer
    (mfea_write_record_npy): float64 rows, or bool rows for REC_ACTIVE."""
    flags = kind == REC_ACTIVE
    dt = np.uint8 if flags else np.float64
    if len(records):
        a = np.ascontiguousarray(np.asarray(records), dtype=dt).reshape(len(records), -1)
    else:
        a = np.zeros((0, n_cols or 0), dtype=dt)
    nr, nc = a.shape
    p = a.ctypes.data_as(_P) if a.size else None
    _check(_lib.mfea_write_record_npy(os.fsencode(path), int(kind), nr, nc,
                                      None if flags else p, p if flags else None))


def grow_params(**kw) -> GrowParams:
    """The reference simulator's parameters (mfea_grow_default_params), with
    fields overridden by keyword."""
    p = GrowParams()
    _lib.mfea_grow_default_params(C.byref(p))
    for k, v in kw.items():
        if k not in dict(GrowParams._fields_):
            raise TypeError(f"unknown growth parameter {k!r}")
        setattr(p, k, os.fsencode(v) if k == "snapshot_dir" and v is not None else v)
    return p


def scaled_grow_params(scale=1.0, **kw) -> GrowParams:
    """A scale-times larger dish (host/mfea_grow.cpp --scale): inoculum grid
    5·scale × 5·scale at the reference's spacing, substrate and Omega0 scaled
    by the area, everything else the reference's."""
    p = grow_params()
    if scale != 1.0:
        p.dish_size *= scale
        p.substrate_width *= scale
        p.substrate_E *= scale * scale
        p.omega0 *= scale * scale
        p.inoc_nx = p.inoc_ny = int(5 * scale + 0.5)
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def grow_network(params: GrowParams | None = None, out_dir=None):
    """Run the native producer (mfea_grow).  Returns (xyz, e2n) as the
    reference's nodes.csv / elements.csv would read back (6 significant
    digits), and writes those files (+ mycelium_growth_stats.csv) to out_dir
    if given."""
    p = params if params is not None else grow_params()
    g = _P()
    _check(_lib.mfea_grow(C.byref(p), C.byref(g)))
    try:
        nn, ne, nh = C.c_int64(), C.c_int64(), C.c_int64()
        _check(_lib.mfea_grow_info(g, C.byref(nn), C.byref(ne), C.byref(nh)))
        xyz = np.empty((nn.value, 3), np.float64)
        e2n = np.empty((ne.value, 2), np.int32)
        _check(_lib.mfea_grow_mesh(g, _ptr(xyz), _ptr(e2n)))
        if out_dir is not None:
            os.makedirs(out_dir, exist_ok=True)
            _check(_lib.mfea_grow_write(g, os.fsencode(out_dir)))
    finally:
        _lib.mfea_grow_free(g)
    return xyz, e2n.astype(np.int64)


def make_opts(rtol=1e-8, atol=0.0, max_it=100000, precond=PC_JACOBI, norm=NORM_UNPRECONDITIONED,
              chunk=0, reg=1e-12) -> SolveOpts:
    return SolveOpts(rtol, atol, int(max_it), int(precond), int(norm), int(chunk), reg)


class Engine:
    """One device handle (mfea_handle).  Host arrays are copied on every call."""

    def __init__(self, device: int = 0):
        h = _P()
        _check(_lib.mfea_create(int(device), C.byref(h)))
        self._h = h
        self.n_nodes = 0
        self.n_elems = 0

    def close(self):
        if getattr(self, "_h", None):
            _lib.mfea_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---- partitioning -------------------------------------------------------
    def dist_init(self, rank: int, world: int, unique_id: bytes):
        """Join an RCCL world (one process per GPU); call before set_mesh."""
        if len(unique_id) != 128:
            raise ValueError("unique_id must be 128 bytes")
        buf = (C.c_uint8 * 128).from_buffer_copy(unique_id)
        _check(_lib.mfea_dist_init(self._h, int(rank), int(world), buf))

    def set_partition_axis(self, axis: int = -1):
        _check(_lib.mfea_set_partition_axis(self._h, int(axis)))

    def global_active(self) -> np.ndarray:
        """The host's global element activity the partitioned plan reads
        (mfea_debug_global_active)."""
        out = np.zeros(self.n_elems, np.uint8)
        _check(_lib.mfea_debug_global_active(self._h, out.ctypes.data_as(C.c_void_p)))
        return out.astype(bool)

    def floating(self) -> np.ndarray:
        """Free nodes cut off from both grips by the current activity, from the
        device's connected components (mfea_debug_floating)."""
        out = np.zeros(self.n_nodes, np.uint8)
        _check(_lib.mfea_debug_floating(self._h, out.ctypes.data_as(C.c_void_p)))
        return out.astype(bool)

    def set_parts(self, nparts: int, axis: int = -1):
        """nparts partitions of the multi-GPU solve held by this handle on one
        device (mfea_debug_set_parts: the partitioned path, testable on one GPU)."""
        _check(_lib.mfea_debug_set_parts(self._h, int(nparts), int(axis)))

    def set_option(self, name: str, value: int):
        """mfea_set_option (include/mfea_debug.h): tuning / comparison knobs."""
        _check(_lib.mfea_set_option(self._h, name.encode(), int(value)))

    def get_option(self, name: str) -> int:
        """mfea_get_option: the option's current value."""
        v = C.c_int64()
        _check(_lib.mfea_get_option(self._h, name.encode(), C.byref(v)))
        return v.value

    @contextlib.contextmanager
    def options(self, **kw):
        """Set options for a block, then restore the values they had before."""
        prev = {k: self.get_option(k) for k in kw}
        try:
            for k, v in kw.items():
                self.set_option(k, v)
            yield self
        finally:
            for k, v in prev.items():
                self.set_option(k, v)

    # ---- setup --------------------------------------------------------------
    def set_material(self, E, A, I):
        _check(_lib.mfea_set_material(self._h, float(E), float(A), float(I)))

    def set_mesh(self, xyz, e2n, skip_invalid=False):
        xyz = np.ascontiguousarray(xyz, dtype=np.float64).reshape(-1, 3)
        e2n = np.ascontiguousarray(e2n, dtype=np.int64).reshape(-1, 2)
        self._xyz, self._e2n = xyz, e2n
        _check(_lib.mfea_set_mesh(self._h, xyz.shape[0], _ptr(xyz), e2n.shape[0], _ptr(e2n),
                                  MESH_SKIP_INVALID if skip_invalid else 0))
        self.n_nodes, self.n_elems = xyz.shape[0], e2n.shape[0]

    def set_bc(self, top, bot):
        top = np.ascontiguousarray(top, dtype=np.int64).ravel()
        bot = np.ascontiguousarray(bot, dtype=np.int64).ravel()
        _check(_lib.mfea_set_bc(self._h, top.size, _ptr(top), bot.size, _ptr(bot)))

    def set_active(self, active=None):
        if active is None:
            _check(_lib.mfea_set_active(self._h, None))
        else:
            a = np.ascontiguousarray(active, dtype=np.uint8).ravel()
            if a.size != self.n_elems:
                raise ValueError("active must have one entry per element")
            _check(_lib.mfea_set_active(self._h, _ptr(a)))

    # ---- hot path -----------------------------------------------------------
    def assemble(self):
        _check(_lib.mfea_assemble(self._h))

    def solve(self, dy_top, dy_bot, opts: SolveOpts | None = None) -> Stats:
        st = Stats()
        o = opts if opts is not None else make_opts()
        _check(_lib.mfea_solve(self._h, float(dy_top), float(dy_bot), C.byref(o), C.byref(st)), st)
        return st

    def post(self, max_strain):
        f = C.c_double()
        n = C.c_int64()
        _check(_lib.mfea_post(self._h, float(max_strain), C.byref(f), C.byref(n)))
        return f.value, n.value

    def step(self, dy_top, dy_bot, opts: SolveOpts | None, max_strain):
        st = Stats()
        f = C.c_double()
        n = C.c_int64()
        o = opts if opts is not None else make_opts()
        _check(_lib.mfea_step(self._h, float(dy_top), float(dy_bot), C.byref(o), float(max_strain),
                              C.byref(f), C.byref(n), C.byref(st)), st)
        return f.value, n.value, st

    # ---- results --------------------------------------------------------------
    def displacement(self):
        U = np.empty(3 * self.n_nodes)
        _check(_lib.mfea_get_displacement(self._h, _ptr(U)))
        return U

    def stress(self):
        s = np.empty(self.n_elems)
        if self.n_elems:
            _check(_lib.mfea_get_stress(self._h, _ptr(s)))
        return s

    def active(self):
        a = np.empty(self.n_elems, dtype=np.uint8)
        if self.n_elems:
            _check(_lib.mfea_get_active(self._h, _ptr(a)))
        return a.astype(bool)

    def ownership(self):
        """(node_owned, elem_owned) bool arrays: what this handle reports
        (mfea_get_ownership; one partition: everything)."""
        n = np.empty(self.n_nodes, dtype=np.uint8)
        e = np.empty(self.n_elems, dtype=np.uint8)
        _check(_lib.mfea_get_ownership(self._h, _ptr(n), _ptr(e)))
        return n.astype(bool), e.astype(bool)

    def gather_results(self):
        """mfea_gather_results: (U, stress, active) of the whole mesh on rank
        0 of an RCCL world (None elsewhere); collective."""
        U = np.empty(3 * self.n_nodes)
        S = np.empty(self.n_elems)
        A = np.empty(self.n_elems, dtype=np.uint8)
        _check(_lib.mfea_gather_results(self._h, _ptr(U), _ptr(S), _ptr(A)))
        return U, S, A.astype(bool)

    def info(self) -> dict:
        inf = Info()
        _check(_lib.mfea_get_info(self._h, C.byref(inf)))
        return inf.as_dict()

    def profile_iteration(self, precond=PC_JACOBI, reps=50) -> float:
        """Average duration (ms) of the fused SpMV + CG iteration kernel."""
        ms = C.c_double()
        _check(_lib.mfea_profile_iteration(self._h, int(precond), int(reps), C.byref(ms)))
        return ms.value

    def profile_spmv(self, reps=100) -> float:
        """GAMG: average duration (ms) of the w = A_0 u kernel (mfea_profile_spmv)."""
        ms = C.c_double()
        _check(_lib.mfea_profile_spmv(self._h, int(reps), C.byref(ms)))
        return ms.value

    def trace_iteration(self, precond=PC_JACOBI, cap=1 << 16):
        """Per-wave s_memrealtime stamps (100 MHz) of one CG iteration launch:
        (waves, 4) = entry, partials reduced, SpMV done, stores drained."""
        out = np.zeros(4 * cap, dtype=np.uint64)
        nw = C.c_int64()
        _check(_lib.mfea_debug_trace_iteration(self._h, int(precond), out.ctypes.data, out.size,
                                               C.byref(nw)))
        return out[:4 * nw.value].reshape(-1, 4)

    def amg_info(self) -> dict:
        """The MFEA_PC_GAMG hierarchy for the current active set: rows and
        stored blocks per level, index-list entries of the numeric setup."""
        cap = 64
        nl = C.c_int()
        rows = np.zeros(cap, dtype=np.int64)
        blocks = np.zeros(cap, dtype=np.int64)
        pblocks = np.zeros(cap, dtype=np.int64)
        items = C.c_int64()
        nd = C.c_int()
        ndist = C.c_int()
        ptblocks = np.zeros(cap, dtype=np.int64)
        _check(_lib.mfea_debug_amg_info(self._h, C.byref(nl), rows.ctypes.data, blocks.ctypes.data,
                                        pblocks.ctypes.data, cap, C.byref(items), C.byref(nd), C.byref(ndist),
                                        ptblocks.ctypes.data))
        n = nl.value
        return {"levels": n, "rows": rows[:n].tolist(), "blocks": blocks[:n].tolist(),
                "pblocks": pblocks[:n].tolist(), "ptblocks": ptblocks[:n].tolist(),
                "pair_items": items.value, "nd": nd.value, "n_dist": ndist.value,
                "cycle": self.get_option("amg_cycle"),
                "collapse_level": self.get_option("amg_collapse_level"),
                "collapse_blocks": self.get_option("amg_collapse_blocks"),
                "merged": self.get_option("amg_merged"),
                "merge_dq_blocks": self.get_option("amg_merge_dq_blocks"),
                "merge_u_blocks": self.get_option("amg_merge_u_blocks")}

    def amg_vcycle(self, r):
        """mfea_debug_amg_vcycle: one GAMG V-cycle u = M r (n_nodes × ND, original
        node order; call after assemble)."""
        r = np.ascontiguousarray(r, dtype=np.float64)
        u = np.empty_like(r)
        _check(_lib.mfea_debug_amg_vcycle(self._h, _ptr(r), _ptr(u)))
        return u

    def amg_vector(self, level, which):
        """mfea_debug_amg_vector: a V-cycle vector (0 b, 1 x, 2 t, 3 e) of a
        level after amg_vcycle, in the level's natural row order."""
        n = C.c_int64()
        _check(_lib.mfea_debug_amg_vector(self._h, int(level), int(which), None, 0, C.byref(n)))
        nd = self.amg_info()["nd"]
        w = nd * nd if which in (4, 6) else nd
        out = np.zeros(n.value * w)
        _check(_lib.mfea_debug_amg_vector(self._h, int(level), int(which), _ptr(out), out.size, C.byref(n)))
        return out.reshape(n.value, w)

    # ---- reference-API helpers ------------------------------------------------
    def element_stiffness(self, p1s, p2s, E, A, I):
        p1 = np.ascontiguousarray(p1s, dtype=np.float64).reshape(-1, 3)
        p2 = np.ascontiguousarray(p2s, dtype=np.float64).reshape(-1, 3)
        n = p1.shape[0]
        Ke = np.empty((n, 6, 6))
        L = np.empty(n)
        _check(_lib.mfea_element_stiffness(self._h, n, _ptr(p1), _ptr(p2), float(E), float(A),
                                           float(I), _ptr(Ke), _ptr(L)))
        return Ke, L

    def export_csr(self):
        nnz = C.c_int64(0)
        _check(_lib.mfea_export_csr(self._h, C.byref(nnz), None, None, None))
        indptr = np.empty(3 * self.n_nodes + 1, dtype=np.int64)
        indices = np.empty(nnz.value, dtype=np.int32)
        data = np.empty(nnz.value)
        _check(_lib.mfea_export_csr(self._h, C.byref(nnz), indptr.ctypes.data_as(_P),
                                    indices.ctypes.data_as(_P), data.ctypes.data_as(_P)))
        return indptr, indices, data

    def solve_csr(self, indptr, indices, data, known_dofs, known_vals, opts=None):
        indptr = np.ascontiguousarray(indptr, dtype=np.int64)
        indices = np.ascontiguousarray(indices, dtype=np.int32)
        data = np.ascontiguousarray(data, dtype=np.float64)
        kd = np.ascontiguousarray(known_dofs, dtype=np.int64).ravel()
        kv = np.ascontiguousarray(known_vals, dtype=np.float64).ravel()
        n = indptr.size - 1
        U = np.empty(n)
        st = Stats()
        o = opts if opts is not None else make_opts()
        _check(_lib.mfea_solve_csr(self._h, n, indptr.ctypes.data_as(_P), _ptr(indices), _ptr(data),
                                   kd.size, _ptr(kd), _ptr(kv), C.byref(o), _ptr(U), C.byref(st)), st)
        return U, st
