/* mfea_debug.h — diagnostics of the mfea engine (not part of the reference's
 * interface; no reference counterpart).  Same ABI rules as mfea.h. */
#ifndef MFEA_DEBUG_H
#define MFEA_DEBUG_H
#include <stdint.h>

#include "mfea.h"

#ifdef __cplusplus
extern "C" {
#endif

/* One traced launch of the CG iteration kernel in the running state that
 * mfea_profile_iteration sets up.  For every wave w (block·4 + wave), out[4w+k]
 * holds s_memrealtime (100 MHz) at k = 0 entry, 1 partials reduced (α, β
 * known), 2 SpMV of its last row done, 3 its stores drained.  cap >= 4·waves. */
int mfea_debug_trace_iteration(mfea_handle* h, int precond, uint64_t* out, int64_t cap,
                               int64_t* n_waves);

/* Runs the partitioned solve of mfea_dist_init with `nparts` partitions held
 * by this one handle on its one device: the same partition plan, kernels and
 * exchange schedule, with device copies in place of RCCL (tests the
 * multi-GPU path on one GPU).  axis as mfea_set_partition_axis. */
int mfea_debug_set_parts(mfea_handle* h, int nparts, int axis);

/* The host's global element activity (E bytes, original order) as the
 * partitioned GAMG plan reads it (capi.hip global_active: kept current by
 * mfea_set_active and the failed-element ids each post exchanges; a rebuild
 * gathers it afresh).  One partition: the device activity. */
int mfea_debug_global_active(mfea_handle* h, uint8_t* out);

/* The free nodes with no path of active elements to a grip node, as the
 * kept GAMG hierarchy masks them (kernels.hip launch_floating: connected
 * components on the device, for the device's current activity): out[n] = 1
 * for such a node n (original order, n_nodes bytes).  One partition. */
int mfea_debug_floating(mfea_handle* h, uint8_t* out);

/* Tuning options of a handle (experiments and tests; the defaults are the
 * measured best; the library reads no environment variables).  Names:
 *   "graph" 0|1          single-partition CG chunks as hipGraph replays (1)
 *   "dist_graph" 0|1     partitioned chunks, exchanges included, likewise (1)
 *   "order" -1|0|k       free-row order: DFS (-1), natural (0), degree sort in windows of k
 *   "lane_dof" 0|3       planar meshes on 2 DOFs per node (0) or 3
 *   "cg_kernel" 0|1|2    Jacobi CG kernel: by density (0), lanes (1), SELL (2)
 *   "ell_block" 64..512  lane kernels: threads per block (256)
 *   "ell_maxg" n         lane kernels: grid cap (0 = 512)
 *   "ell_compact" 0|1    lane kernels: compact halo records (1)
 *   "amg_tail_rows" n    GAMG: deep levels of ≤ n rows in one workgroup (2048; 0 off)
 *   "amg_tail_lds" 0|1   GAMG: the tail's vectors in LDS (1) or global memory (0)
 *   "amg_restrict_lanes" 0|1|2|4|8  GAMG: lanes per coarse row of the restriction (0: by width)
 *   "amg_op_lanes" 0|1|2|4        GAMG: lanes per row of the operators below level 0 (0: by width)
 *   "dist_timeout_ms" n  RCCL waits: give up after n ms
 *   "part_slack_pct" n   partition boundaries move ≤ n % of a strip to the
 *                        fewest crossing elements (35; 0 = equal free-node counts)
 *   "amg_max_levels" 1..32  GAMG: hierarchy depth cap (32)
 *   "amg_dist" -1|0|1    partitioned GAMG: block Jacobi over per-partition hierarchies (0),
 *                        the distributed V-cycle of one global hierarchy (1), or per
 *                        active set whichever of the two solved faster (-1)
 *   "amg_rep_rows" n     distributed V-cycle (four-step form): levels of at most n rows replicated (32768)
 *   "amg_dist_cycle" 0|1 distributed V-cycle: the compact form, level 0 split and every level
 *                        below replicated (1), or the four-step form over the split levels (0)
 *   "dist_sums" 0|1      GAMG over RCCL: the CG's per-rank sums as one all-reduce of a
 *                        zero-padded [world][4] buffer (1) or send / receive pairs (0)
 *   "amg_reuse" 0|1      GAMG: keep the hierarchy over element failures, floating pieces
 *                        masked (1), or rebuild it for every new active set (0)
 *   "amg_rebuild_pct" n  GAMG: a kept hierarchy is rebuilt once a solve needs more than
 *                        n % of the iterations it took on its own set (800), or
 *   "amg_rebuild_rent" n once the time its solves spent on iterations above that count
 *                        reaches n % of the time its host build took (100; 0: off)
 *   "amg_coarse_rho_ppm" n  GAMG: ρ̂ of the levels below 0, ppm (1750000: ω = 0.76, level 0
 *                        then at its exact ρ̂ = 2); 0: the Gershgorin rule max(2, g / 1.45)
 *                        everywhere.  A solve failing with it falls back to 0 for the
 *                        handle's lifetime (read-only "amg_safe_omega" = 1)
 *   "amg_cycle" 0|1      GAMG: four-step V(1,1) levels (0) or the compact two-sweep form (1)
 *   "amg_collapse" -1|0|k  compact cycle: collapse the levels below k into one operator
 *                        (-1: the highest level whose operator fits the budget below; 0 off)
 *   "amg_collapse_mb" n, "amg_collapse_pairs" n  that budget: MB of blocks (32), product pairs (8e6)
 *   "amg_spatial" -1|0|1 GAMG labels in Z-order: by locality (-1), off, on
 *   "amg_up_lanes" 0|1|2|4  compact up sweep: lanes per P̃ row (0: by width)
 *   "amg_fuse_setup" 0|1 GAMG numeric setup: compact operators in the Galerkin launches (1)
 *   "amg_theta_ppm" n    GAMG strength threshold θ in ppm (PETSc -pc_gamg_threshold; 0)
 *   "sweep_piece" 1..64  SOR / ICC: rows per chain piece at most (64; sweep.hip)
 *   "cc_tile" 512|1024|2048|4096  floating rows on the device (kernels.hip launch_floating):
 *                        rows per LDS union-find tile (1024)
 *   "setup_entry" 0|1    GAMG / SOR / ICC (one partition, option graph 1): the solve's entry
 *                        launches — level-0 b, the first preconditioner application, w = A u,
 *                        update 0 — captured in the numeric setup's graph (1; off while
 *                        phase_times records the setup's end)
 *   "amg_a0_slot" 0|1    GAMG at a fixed level-0 ω without the fused P_0 / Ã_0 pass: level
 *                        0's blocks and D⁻¹ one thread per SELL position (1) instead of
 *                        one per row (0); the same bits
 *   "combo_graph" 0|1    with batch_graph: the batch, finish and post behind the numeric
 *                        setup in the setup's graph — one graph launch per step (1)
 *   "graph_start" 0|1    GAMG / SOR / ICC, graphs on, no phase events: the CG start
 *                        (k_cg_init_finalize) at the head of the setup graph (1)
 *   "step_graph" 0|1     mfea_step, one partition, GAMG / SOR / ICC, graphs on, no phase
 *                        events, asm_kernel 0: the assembly with the fused RHS and the CG
 *                        start at the head of the setup graph (0: measured slower — the
 *                        eager assembly overlaps the host's plan checks)
 *   "batch_graph" 0|1    mfea_step, one partition, GAMG / SOR / ICC, graphs on, no phase
 *                        events: the solve's planned batch, its finish and the post as ONE
 *                        captured graph of the batch's exact length (1)
 *   "spec_post" 0|1      mfea_step, one partition, GAMG / SOR / ICC: the post kernels enqueued
 *                        behind the solve's planned batch, one host wait for both (1); a
 *                        batch that was not the last has its post's failures undone
 *   "asm_kernel" 0|1|2   assembly: row gather, GAMG RHS fused (0); element colours, one
 *                        launch per colour (1); element pass + row pass (2) — DESIGN.md §0
 * Read-only: "sweep_colors", "sweep_pieces" (the last SOR / ICC plan), "asm_colours"
 * (the element colouring's colours once asm_kernel 1 or 2 has run; 0 before).
 * Options that change the symbolic layout rebuild it at the next call. */
int mfea_set_option(mfea_handle* h, const char* name, int64_t value);

/* The current value of an option of mfea_set_option (as it would be passed
 * back: part_slack_pct in percent, dist_timeout_ms in ms), or of the
 * read-only "amg_dist_chosen": the partitioned GAMG form in use — the one
 * option "amg_dist" names, or with "amg_dist" -1 the one picked for the
 * current active set (0 block Jacobi, 1 global hierarchy, -1 not yet). */
int mfea_get_option(mfea_handle* h, const char* name, int64_t* value);

/* The MFEA_PC_GAMG hierarchy for the current active set (built if needed;
 * partitioned handles: the global hierarchy of option "amg_dist" 1):
 * *n_levels levels; for level l < cap: rows[l] (nodes / aggregates),
 * blocks[l] (stored ND×ND blocks of A_l, diagonal included) and pblocks[l]
 * (blocks of the prolongator P_l; 0 on the coarsest level).  *pair_items =
 * index-list entries of the numeric setup; *nd = DOFs per node; *n_dist =
 * levels split over the partitions (0: one partition); ptblocks (may be
 * NULL): blocks of the compact cycle's P̃_l = (I − ω D⁻¹ A) P_l (= of R̃_l). */
int mfea_debug_amg_info(mfea_handle* h, int* n_levels, int64_t* rows, int64_t* blocks,
                        int64_t* pblocks, int cap, int64_t* pair_items, int* nd, int* n_dist,
                        int64_t* ptblocks);

/* One MFEA_PC_GAMG V-cycle u = M r on the assembled operator (call after
 * mfea_assemble; runs the numeric setup first).  r, u: n_nodes × ND in
 * original node order (ND = the hierarchy's DOFs per node, 2 on planar
 * meshes); entries of grip nodes are ignored / written 0.  Partitioned
 * handles run the distributed V-cycle (option "amg_dist" 1). */
int mfea_debug_amg_vcycle(mfea_handle* h, const double* r, double* u);

/* After mfea_debug_amg_vcycle: level l's V-cycle vector `which` (0 b, 1 x,
 * 2 t, 3 e; level 0: b = the CG's r, e = its u) in the level's natural
 * (aggregation) row order, n_l × ND; partitioned: each row from its owner.
 * Returns the row count in *n. */
int mfea_debug_amg_vector(mfea_handle* h, int l, int which, double* out, int64_t cap, int64_t* n);

#ifdef __cplusplus
}
#endif
#endif
