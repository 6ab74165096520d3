// partition.hpp — multi-GPU partition of the filament network (host C++, once
// per mesh / BC set).  SURVEY.md §8(e); stands in for the PETSc row-block
// distribution of src/fea_petsc_parallel.cpp:169-171, 234-268.
//
// Nodes are cut into a px × py grid of strips (px along x, each cut into py
// along y; the factorisation of `world` with the fewest cut elements, or 1-D
// strips along a given axis) with equal FREE-node counts, each boundary then
// moved (by at most `slack` × the strip size) to the position crossed by the
// fewest elements; known (grip) nodes follow the strip they lie in.  Rank r owns its strip's nodes and every
// element with an owned endpoint (owner-computes: a cut element is assembled by
// both sides, identically), so assembly needs no communication.  Its local
// mesh = owned nodes + ghost nodes (the far endpoints of cut elements).
//
// Exchange plans (both sides enumerate them in the same order, so no
// negotiation is needed):
//   pairs — one per cut element joining two FREE nodes of different ranks,
//           ordered by (peer rank, global element id).  Pair k of rank A with
//           peer B and B's pair with peer A are the same element.  The lane
//           holding the cut element's slot on each side sends its row's CG
//           record and reads the other side's (the cross-rank form of the
//           halo record of symbolic.hpp).
//   xhalo — per peer, the owned free nodes the peer holds as ghosts (sorted
//           by global id): their displacement is sent once per solve so the
//           reaction and stress kernels see U at both ends of every element.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace mfea {

struct PartPlan {
  int world = 1, rank = 0, axis = 0;
  std::vector<int32_t> owner;     // rank of every global node (node_owner)
  // local mesh: nodes and elements in ascending global id
  std::vector<int64_t> node_g;    // local node → global node
  std::vector<uint8_t> ghost;     // local node owned by another rank
  std::vector<int64_t> elem_g;    // local element → global element
  std::vector<uint8_t> elem_own;  // reported by this rank (owner of its first node)
  std::vector<double> xyz;        // local nodes × 3
  std::vector<int64_t> e2n;       // local elements × 2, local node ids
  std::vector<int64_t> top, bot;  // local ids of grip nodes (owned and ghost), list order
  // CG record exchange
  std::vector<int32_t> elem_pair;  // per local element: pair index, -1
  std::vector<int32_t> peers;      // ranks with >= 1 pair, ascending
  std::vector<int64_t> peer_off, peer_cnt;
  int64_t n_pairs = 0;
  // displacement halo
  std::vector<int32_t> xpeers;  // ranks exchanging displacements with this one, ascending
  std::vector<int64_t> xsend_off, xsend_cnt, xrecv_off, xrecv_cnt;
  std::vector<int64_t> xsend_node, xrecv_node;  // local node ids, concatenated per peer
};

// Owner rank of every node.  axis: 0 = strips along x, 1 = along y, -1 = the
// px × py grid with the fewest cut elements (axis_used: 0, 1, or 2 = a 2-D
// grid).  Known nodes are those in top ∪ bot.  slack: 0 = equal
// free-node counts; s > 0 = boundaries at the fewest crossing elements within
// ±s × nfree / world free nodes of the equal cut (clamped to 0.45).
std::vector<int32_t> node_owner(int64_t N, const double* xyz, int64_t E, const int64_t* e2n,
                                const std::vector<int64_t>& top, const std::vector<int64_t>& bot,
                                int world, int axis, double slack, int* axis_used);

// Builds rank `rank`'s plan.  Elements with out-of-range endpoints are
// rejected (skip_invalid = false) or left out of every rank (true).
std::string build_partition(int64_t N, const double* xyz, int64_t E, const int64_t* e2n,
                            bool skip_invalid, const std::vector<int64_t>& top,
                            const std::vector<int64_t>& bot, int world, int rank, int axis,
                            double slack, PartPlan& plan);

}  // namespace mfea
