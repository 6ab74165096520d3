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

/* The MFEA_PC_GAMG hierarchy for the current active set (built if needed):
 * *n_levels levels; for level l < cap: rows[l] (nodes / aggregates),
 * blocks[l] (stored ND×ND blocks of A_l, diagonal included) and pblocks[l]
 * (blocks of the prolongator P_l; 0 on the coarsest level).  *pair_items =
 * index-list entries of the numeric setup; *nd = DOFs per node. */
int mfea_debug_amg_info(mfea_handle* h, int* n_levels, int64_t* rows, int64_t* blocks,
                        int64_t* pblocks, int cap, int64_t* pair_items, int* nd);

#ifdef __cplusplus
}
#endif
#endif
