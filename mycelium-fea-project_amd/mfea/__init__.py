"""mfea — MI355X-native engine for the mycelium FEA hot path (assembly + PCG).

Host layer over libmfea.so (include/mfea.h).  The drop-in module mirroring the
reference's ``src/fea_solver.py`` API is ``fea_solver`` next to this package.
"""
from ._capi import (Engine, MfeaError, SolverFailure, SolveOpts, Stats, abi_version,  # noqa: F401
                    make_opts, PC_JACOBI, PC_BLOCK_JACOBI, PC_GAMG, PC_SOR, PC_ICC, NORM_PRECONDITIONED,
                    NORM_UNPRECONDITIONED, LIB_PATH, dist_unique_id,
                    GrowParams, grow_params, scaled_grow_params, grow_network)
