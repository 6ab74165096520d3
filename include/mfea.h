/*
 * mfea.h — C ABI of the MI355X-native mycelium FEA engine (libmfea.so).
 *
 * The reference has no FFI: its hot path is Python calling NumPy/SciPy
 * (src/fea_solver.py) or a C++ main() calling PETSc (src/fea_petsc.cpp).
 * Each entry point below replaces one piece of that path; the reference
 * interface it stands in for is cited beside it.  Plain pointers and sizes
 * only (no torch types).  All functions return 0 on success and a negative
 * MFEA_E* code on failure; mfea_last_error() returns the message of the most
 * recent failure on the calling thread.
 *
 * Ownership: host arrays passed in are caller-owned and copied (or written)
 * synchronously before the call returns.  Device buffers belong to the handle.
 * Threading: one host thread per handle; a handle is not re-entrant.
 * Node/element indices are 0-based rows of nodes.csv / elements.csv
 * (src/fea_petsc.cpp:39-40 — node index = row order).
 */
#ifndef MFEA_H
#define MFEA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 8: MFEA_PC_SOR / MFEA_PC_ICC factorise the whole matrix (were block Jacobi
 *    over 256-row blocks); every preconditioner honours mfea_solve_opts.norm */
#define MFEA_ABI_VERSION 8

/* error / status codes */
#define MFEA_OK 0
#define MFEA_EINVAL -1      /* bad argument (e.g. node id out of range)                */
#define MFEA_EDEVICE -2     /* HIP runtime error                                       */
#define MFEA_ESTATE -3      /* call out of order (no mesh, no BCs, ...)                */
#define MFEA_EMAXIT -4      /* PCG hit max_it (PETSc KSP_DIVERGED_ITS)                  */
#define MFEA_EBREAKDOWN -5  /* PCG breakdown: p·Ap <= 0 or non-finite (KSP_DIVERGED_*) */
#define MFEA_ENOMEM -6
#define MFEA_ECOMM -7       /* RCCL failure (multi-GPU)                                */

/* mesh flags (mfea_set_mesh) */
#define MFEA_MESH_SKIP_INVALID 1u /* skip elements with out-of-range node ids, as
                                     src/fea_petsc.cpp:241 does; default: reject,
                                     as src/fea_solver.py:82-83 would (IndexError) */

/* solver selection (mfea_solve_opts.precond) */
#define MFEA_PC_JACOBI 0        /* PCJACOBI — diagonal of K_ff + reg·I              */
#define MFEA_PC_BLOCK_JACOBI 1  /* 3×3 node-block Jacobi (exact inverse per block)   */
#define MFEA_PC_GAMG 2          /* smoothed-aggregation AMG V-cycle, the counterpart of
                                   the reference sweep's `-pc_type gamg`
                                   (src/fea_petsc_solverAndPC.cpp:330-391).  Partitioned
                                   handles: ONE global hierarchy whose large levels are
                                   split over the ranks (the one-partition iteration
                                   count) or block Jacobi over per-partition ones — per
                                   active set the faster of the two, measured
                                   (mfea_debug.h option "amg_dist") */

#define MFEA_PC_SOR 3           /* `-pc_type sor`: SSOR (ω = 1, PETSc's default) on the
                                   node blocks of the WHOLE K_ff + reg·I, every coupling
                                   kept, factorised in a chain-piece multicolour order
                                   (hyphal chains of ≤ 64 rows keep their natural order;
                                   the pieces of one colour are independent and each
                                   piece's recurrence is a scan across a wave's lanes;
                                   csrc/sweep.hip); one partition */
#define MFEA_PC_ICC 4           /* `-pc_type icc` (the reference source's default PCICC,
                                   src/fea_petsc.cpp:331; also `ilu`, the same factor on
                                   an SPD matrix): DIC(0) — incomplete block Cholesky of
                                   the whole K_ff + reg·I with A's off-diagonal blocks and
                                   f64 pivots D̃_i = D_i − Σ_{j<i} A_ij D̃_j⁻¹ A_ijᵀ — in
                                   the same chain-piece multicolour order as MFEA_PC_SOR */

/* Every preconditioner stops on the norm mfea_solve_opts.norm selects. */
/* stopping norm (mfea_solve_opts.norm) */
#define MFEA_NORM_UNPRECONDITIONED 0 /* ‖r‖₂ ≤ rtol·‖b‖₂  (SciPy cg; the metric)      */
#define MFEA_NORM_PRECONDITIONED 1   /* ‖z‖₂ ≤ rtol·‖M⁻¹b‖₂ (PETSc KSPCG default)     */

typedef struct mfea_handle mfea_handle;

typedef struct {
  double rtol;      /* relative tolerance; PETSc default 1e-5, metric 1e-8, parity 1e-13 */
  double atol;      /* absolute tolerance on the chosen norm (PETSc default 1e-50)       */
  int32_t max_it;   /* PETSc default 10000                                              */
  int32_t precond;  /* MFEA_PC_*                                                         */
  int32_t norm;     /* MFEA_NORM_*                                                       */
  int32_t chunk;    /* iterations per captured hipGraph replay (0 = library default)     */
  double reg;       /* diagonal regularisation of K_ff, src/fea_solver.py:125 (1e-12)    */
} mfea_solve_opts;

typedef struct {
  int32_t iters;     /* PCG iterations executed                                        */
  int32_t status;    /* 0 converged, MFEA_EMAXIT, MFEA_EBREAKDOWN                       */
  double relres;     /* final ‖r‖/‖b‖ (recursive residual)                               */
  double bnorm;      /* ‖b_f‖₂                                                          */
  int64_t n_free;    /* free DOFs                                                       */
  double t_assemble_ms, t_rhs_ms, t_solve_ms, t_post_ms; /* device time (HIP events),
                        recorded only with option "phase_times" 1 (0 otherwise): an
                        event between two kernels idles the GPU for several µs      */
  double t_setup_ms; /* MFEA_PC_GAMG: numeric hierarchy setup (inside t_solve_ms)     */
  int32_t amg_levels; /* MFEA_PC_GAMG: levels of the hierarchy (0 otherwise)         */
  int32_t amg_rebuilt; /* 1 if this solve rebuilt the symbolic hierarchy (new active set) */
} mfea_stats;

/* ---- lifecycle ------------------------------------------------------------ */
int mfea_abi_version(void);
int mfea_last_error(char* buf, size_t n);
/* One handle drives one device.  Multi-GPU = one process (one handle) per GPU,
 * joined by mfea_dist_init. */
int mfea_create(int device, mfea_handle** out);
int mfea_destroy(mfea_handle* h);

/* Material constants, src/fea_solver.py:14-20 / src/fea_petsc.cpp:23-27. */
int mfea_set_material(mfea_handle* h, double E, double A, double I);

/* ---- mesh + boundary conditions (symbolic, once per mesh) ------------------ */
/* Replaces the CSV→array hand-off of fea_solver (src/fea_solver.py:193-201) and
 * read_nodes_csv/read_elems_csv (src/fea_petsc.cpp:42-82, 179-200).
 * xyz: n_nodes×3 row-major f64; e2n: n_elems×2 int64.  Builds the node-block
 * sliced-ELL pattern, the free/known permutation and uploads the mesh. */
int mfea_set_mesh(mfea_handle* h, int64_t n_nodes, const double* xyz, int64_t n_elems,
                  const int64_t* e2n, uint32_t flags);
/* Grip node sets, src/fea_solver.py:207-210 / src/fea_petsc.cpp:203-213.
 * All 3 DOFs of every grip node are prescribed (x=0, y=dy, z=0); a node in
 * both bands takes the bottom value (src/fea_solver.py:226-242 dict order,
 * src/fea_petsc.cpp:292-294 last INSERT wins).  Rebuilds the permutation. */
int mfea_set_bc(mfea_handle* h, int64_t n_top, const int64_t* top, int64_t n_bot,
                const int64_t* bot);
/* Element activity (E bytes, nonzero = active); NULL = all active
 * (src/fea_solver.py:201, src/fea_petsc.cpp:200). */
int mfea_set_active(mfea_handle* h, const uint8_t* active);

/* ---- the hot path ---------------------------------------------------------- */
/* Element stiffness + global assembly on device for the current active set.
 * Replaces bar_stiffness_bulk + assemble_global_stiffness
 * (src/fea_solver.py:30-106) and element_stiffness_6x6 + the MatSetValue loop
 * (src/fea_petsc.cpp:88-140, 229-263). */
int mfea_assemble(mfea_handle* h);
/* Dirichlet elimination, RHS and preconditioned CG on device.
 * Replaces solve_system (src/fea_solver.py:112-135) and MatZeroRowsColumnsIS +
 * diag regularisation + KSPSolve (src/fea_petsc.cpp:286-357).
 * Solves the operator of the last mfea_assemble; a handle (re)built since
 * (mfea_set_mesh / mfea_set_bc, or a layout option of mfea_set_option) is
 * assembled for its current active set first.
 * Returns MFEA_EMAXIT / MFEA_EBREAKDOWN on solver failure (stats still filled);
 * the Python shim maps them to np.linalg.LinAlgError (src/fea_solver.py:250-254). */
int mfea_solve(mfea_handle* h, double dy_top, double dy_bot, const mfea_solve_opts* opts,
               mfea_stats* st);
/* Reaction + stress/failure on device.  Replaces src/fea_solver.py:256-284 and
 * src/fea_petsc.cpp:360-406: total_force = Σ_{top} (K·U)[3n+1] on the
 * unregularised K; stress = E·ε for elements active at step start (0 else);
 * elements with |ε| > max_strain are deactivated for the next step. */
int mfea_post(mfea_handle* h, double max_strain, double* total_force, int64_t* n_active);
/* One full load step = assemble + solve + post (the bench "step"). */
int mfea_step(mfea_handle* h, double dy_top, double dy_bot, const mfea_solve_opts* opts,
              double max_strain, double* total_force, int64_t* n_active, mfea_stats* st);

/* ---- results (device → host, original node/element order) ----------------- */
int mfea_get_displacement(mfea_handle* h, double* U /* 3·n_nodes, interleaved xyz */);
int mfea_get_stress(mfea_handle* h, double* stress /* n_elems */);
int mfea_get_active(mfea_handle* h, uint8_t* active /* n_elems */);

/* ---- reference-API helpers ------------------------------------------------- */
/* bar_stiffness_bulk on device (src/fea_solver.py:30-68): Ke n×36 row-major, L n. */
int mfea_element_stiffness(mfea_handle* h, int64_t n, const double* p1s, const double* p2s,
                           double E, double A, double I, double* Ke, double* L);
/* Export the assembled global K (active elements only) as scalar CSR over the
 * 3·n_nodes DOFs in original order, same pattern as the reference's
 * csr_matrix (explicit zeros kept, duplicates summed).  Call with indptr ==
 * NULL to query *nnz. */
int mfea_export_csr(mfea_handle* h, int64_t* nnz, int64_t* indptr, int32_t* indices,
                    double* data);
/* solve_system(K, known_dofs, known_vals) for an arbitrary caller-supplied
 * scalar CSR K (src/fea_solver.py:112-135), on device. U: n out. */
int mfea_solve_csr(mfea_handle* h, int64_t n, const int64_t* indptr, const int32_t* indices,
                   const double* data, int64_t n_known, const int64_t* known_dofs,
                   const double* known_vals, const mfea_solve_opts* opts, double* U,
                   mfea_stats* st);

/* ---- introspection / measurement ------------------------------------------- */
typedef struct {
  int64_t n_nodes, n_elems;
  int64_t n_free_nodes;     /* free rows (3 DOF each)                               */
  int64_t n_top, n_known;   /* grip rows                                            */
  int64_t n_slices;         /* SELL-64 slices                                       */
  int64_t n_slots;          /* slot rows × 64 = allocated slot entries              */
  int64_t free_incidences;  /* Σ row_len over free rows = valid slots the SpMV reads */
  int32_t planar;           /* all z == 0                                           */
  int32_t cg_lanes;         /* 1: CG iterations run on the wave-local lane operator */
  int64_t n_lanes;          /* lanes of that operator (owners + helpers + padding)   */
  int64_t n_halo;           /* lanes with an out-of-wave slot (one push per iteration) */
  int32_t n_parts;          /* partitions of the solve (ranks, or mfea_debug_set_parts)  */
  int32_t part;             /* this handle's (first) partition                         */
  int64_t n_pairs;          /* cut free-free elements of that partition (records/iter)  */
  int64_t n_ghost;          /* its ghost rows (other partitions' nodes)                */
  int32_t halo_compact;     /* lane operator: 1 compact halo records, 0 one per lane   */
  int32_t block_size;       /* lane CG kernels: threads per block                      */
  int64_t grid;             /* lane CG kernels: blocks per launch                      */
} mfea_info;
int mfea_get_info(mfea_handle* h, mfea_info* info);
/* Launches the dominant kernel — the fused SpMV + single-reduction CG iteration —
 * `reps` times on the handle's stream between two HIP events (on the current
 * vectors, identical work each launch) and returns the average launch duration.
 * Call after mfea_solve (it overwrites the solver state). */
int mfea_profile_iteration(mfea_handle* h, int precond, int reps, double* avg_ms);
/* MFEA_PC_GAMG: the SpMV kernel alone — w = A_0 u (f64 blocks) with the CG's
 * four partial sums — replayed `reps` times back to back as one captured
 * graph between two HIP events; average launch duration.  After a GAMG solve
 * (partitioned handles: the first partition's kernel over its own rows). */
int mfea_profile_spmv(mfea_handle* h, int reps, double* avg_ms);

/* ---- record writer (host only: needs no device, no handle) ------------------ */
/* Writes one of the driver's end-of-run CSV records, byte-identical to the
 * reference's writers: src/fea_solver.py:297-316 (pandas to_csv — shortest
 * round-trip floats as numpy/Python repr, NaN as an empty field, True/False,
 * node_displacements headed 0..n_cols-1) with style MFEA_CSV_PANDAS, or
 * src/fea_petsc.cpp:433-516 (setprecision(12), 1/0, node_i_x…node_i_z header)
 * with MFEA_CSV_PETSC.  values: n_rows×n_cols row-major f64 (STRESS, DISP,
 * FORCE); flags: n_rows×n_cols bytes (ACTIVE).  Rows get the 1-based step
 * column, except FORCE (n_cols = 2: total_displacement, total_force).
 * n_threads formats column chunks in parallel (output identical for any). */
#define MFEA_CSV_PANDAS 0
#define MFEA_CSV_PETSC 1
#define MFEA_REC_STRESS 0 /* stress_record.csv       */
#define MFEA_REC_ACTIVE 1 /* active_elements.csv     */
#define MFEA_REC_DISP 2   /* node_displacements.csv  */
#define MFEA_REC_FORCE 3  /* force_displacement.csv  */
int mfea_write_record_csv(const char* path, int style, int kind, int64_t n_rows, int64_t n_cols,
                          const double* values, const uint8_t* flags, int n_threads);
/* The same record as a NumPy .npy sidecar (the CSV's text is what
 * dominates at 1 M DOF; a binary copy reloads in milliseconds): the raw
 * n_rows × n_cols array without the step column, '<f8' (values) or '|b1'
 * (flags, ACTIVE), C order, readable by np.load(allow_pickle=False). */
int mfea_write_record_npy(const char* path, int kind, int64_t n_rows, int64_t n_cols, const double* values,
                          const uint8_t* flags);

/* ---- network producer (host only) ------------------------------------------- */
/* The hyphal growth model of src/mycelium_sim_2D.cpp (main :529-588, process
 * functions :236-414), native and multi-threaded, for networks of millions of
 * nodes.  With mfea_grow_default_params (the reference's
 * constants :17-33, 5×5 inoculum, 150 steps, seed 42) and snapshot_every = 1
 * it writes byte-identical nodes.csv / elements.csv (export_geometry :477-515),
 * mycelium_growth_stats.csv and snapshots/step_NNNN.csv to the reference
 * binary's.  Larger networks: more inoculation sites / a larger dish / more
 * steps (substrate_E and omega0 are totals: scale them with the area). */
typedef struct {
  uint64_t seed;                     /* mt19937_64 seed (:17, argv[1])              */
  double h0, dt, lambda_angle, P_branch, c_g, D, M_cap, omega0;
  int32_t t_steps, h0_per_point;     /* growth steps; hyphae per inoculation site   */
  double anastomosis_tol, wall_thickness, dish_size, substrate_width, substrate_E;
  int32_t inoc_nx, inoc_ny;          /* inoculum grid (:143-159), centred           */
  double inoc_dist;                  /* its spacing, mm                             */
  double voxel_size;                 /* spatial hash voxel (:553, 0.1 mm)           */
  int32_t snapshot_every;            /* 0: none; k: step_%04d.csv every k steps      */
  const char* snapshot_dir;          /* where the snapshots go (must exist)          */
  int32_t verbose;                   /* 1: the reference's stderr progress lines     */
  int32_t threads;                   /* 0: all hardware threads; results identical   */
} mfea_grow_params;
typedef struct mfea_grow_net mfea_grow_net;
void mfea_grow_default_params(mfea_grow_params* p);
int mfea_grow(const mfea_grow_params* p, mfea_grow_net** out);
int mfea_grow_info(const mfea_grow_net* g, int64_t* n_nodes, int64_t* n_elems, int64_t* n_hyphae);
/* xyz (3·n_nodes) as nodes.csv carries them (6 significant digits, read back);
 * e2n (2·n_elems) 0-based node rows as elements.csv.  Either may be NULL. */
int mfea_grow_mesh(const mfea_grow_net* g, double* xyz, int32_t* e2n);
/* nodes.csv, elements.csv and mycelium_growth_stats.csv into dir (must exist) */
int mfea_grow_write(const mfea_grow_net* g, const char* dir);
void mfea_grow_free(mfea_grow_net* g);

/* ---- multi-GPU (one process per GPU, RCCL over xGMI) ----------------------- */
/* Replaces the PETSC_COMM_WORLD row-block distribution of
 * src/fea_petsc_parallel.cpp:169-171, 234-268, 330-409 and its MPI reductions.
 * unique_id: the 128-byte ncclUniqueId made by rank 0 (mfea_dist_unique_id)
 * and broadcast by the caller.  Every rank then passes the WHOLE mesh and the
 * same grips to mfea_set_mesh / mfea_set_bc; the handle keeps the part of the
 * network it owns (partition.hpp: a px × py grid of strips with equal
 * free-node counts, boundaries at the fewest crossing elements), the elements
 * touching it and the far ends of cut elements as ghost rows.
 * Exchanges per CG iteration (one RCCL group of point-to-point transfers each):
 *   Jacobi / block Jacobi — one kernel per GPU, one group (the cut rows' CG
 *     records to the neighbours + the 4 partial sums to every rank);
 *   GAMG (distributed V-cycle) — per split level a halo of the smoother's x
 *     and of the residual on the way down and of the coarse correction and x
 *     on the way up, one all-gather into the first replicated level, the u
 *     halo of w = A u and the sums: 4·(split levels) + 2 groups.
 * All ranks derive bitwise identical α, β and stopping decisions.
 * Partitioned handles: mfea_get_displacement writes the owned nodes' entries,
 * mfea_get_stress / mfea_get_active the entries of elements whose first node
 * is owned (others untouched; mfea_gather_results collects all on rank 0);
 * mfea_post returns the global force and count. */
int mfea_dist_unique_id(uint8_t* unique_id /* 128 bytes */);
int mfea_dist_init(mfea_handle* h, int rank, int world, const uint8_t* unique_id);
/* Partition layout: 0 = strips along x, 1 = along y, -1 (default) = the
 * px × py grid (a factorisation of the world size) whose boundaries cross the
 * fewest elements (partition.hpp).  Takes effect at the next build. */
int mfea_set_partition_axis(mfea_handle* h, int axis);
/* Which nodes / elements this handle reports (1 = its own): every node
 * belongs to one partition, every element to the partition of its first
 * node.  Either array may be NULL.  One partition: all ones. */
int mfea_get_ownership(mfea_handle* h, uint8_t* node_owned /* n_nodes */, uint8_t* elem_owned /* n_elems */);
/* The step's records gathered on rank 0 — the displacement of every node and
 * the stress / activity of every element, as one partition would return them
 * (the reference gathers U to rank 0, src/fea_petsc_parallel.cpp:373-378,
 * while every rank writes the same record files, :491-574; here rank 0 alone
 * writes).  Collective over the RCCL world: every rank calls it; rank 0's
 * arrays are filled, the others' are not touched (may be NULL).  Handles
 * without an RCCL world fill the arrays directly.  Any array may be NULL. */
int mfea_gather_results(mfea_handle* h, double* U /* 3·n_nodes */, double* stress /* n_elems */,
                        uint8_t* active /* n_elems */);

#ifdef __cplusplus
}
#endif
#endif /* MFEA_H */
