// symbolic.hpp — host-side symbolic phase of the mfea engine (once per mesh/BC set).
//
// The reference rebuilds its sparse pattern every load step: a Python COO list
// of 36 triplets per element handed to scipy's csr_matrix (src/fea_solver.py:88-105),
// or unpreallocated PETSc MatSetValue calls (src/fea_petsc.cpp:229-263).  Here
// the pattern is built once, on the host, as a node-block sliced ELL
// ("SELL-64"): one matrix row = one node (3 DOF), one slice = 64 consecutive
// rows = one wavefront, one slot = one incident element of the row.  Only the
// values change between steps (element deactivation zeroes a slot).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace mfea {

constexpr int kSlice = 64;  // rows per slice = wavefront width on CDNA4

// kGhost: a free node owned by another partition (multi-GPU); its row holds
// coordinates and, after a solve, the owner's displacement — never solved here.
enum NodeCode : uint8_t { kFree = 0, kTop = 1, kBot = 2, kGhost = 3 };

struct Pattern {
  int64_t n_nodes = 0, n_elems = 0;
  int64_t n_free = 0;   // free nodes occupy permuted rows [0, n_free)
  int64_t n_top = 0;    // top grip rows [n_free, n_free + n_top) in top-list order
  int64_t n_known = 0;  // known rows [n_free, n_nodes) (ghost rows included)
  int64_t n_ghost = 0;  // rows of other partitions' nodes, [n_nodes - n_ghost, n_nodes)
  std::vector<int32_t> perm;   // perm[new] = original node
  std::vector<int32_t> iperm;  // iperm[orig] = new
  std::vector<uint8_t> code;   // code[new] (kFree / kTop / kBot; bottom overrides top)
  // SELL-64: slice s covers rows [64 s, 64 s + 64); its slots are
  // slice_ptr[s] .. slice_ptr[s+1]-1; entry (slot t, lane l) lives at t*64 + l.
  std::vector<int32_t> slice_ptr;  // n_slices + 1
  std::vector<int32_t> row_len;    // per permuted row: incident (non-self-loop) elements
  std::vector<int32_t> s_col;      // permuted neighbour row, -1 = pad
  std::vector<int32_t> s_elem;     // element id (original order), -1 = pad
  std::vector<int32_t> e2n_perm;   // E×2 permuted endpoints (-1,-1 for skipped elements)
  std::vector<double> xyz_perm;    // N×3 coordinates in permuted order
  std::vector<uint8_t> elem_valid; // 0 for elements skipped (out of range)
  int64_t n_slices() const { return (int64_t)slice_ptr.size() - 1; }
  int64_t n_slots() const { return slice_ptr.empty() ? 0 : (int64_t)slice_ptr.back(); }
  bool planar = false;             // every z == 0
};

// Element colouring for the element-centric assembly (kernels.hip
// k_assemble_colour, option "asm_kernel" 1; BASELINE north_star's "one
// wavefront per element batch … colour-partitioned writes"): no two elements
// of one colour share a node, so a colour's element batches add their S_e
// into the two endpoint rows' diagonal blocks without atomics or conflicts.
// Greedy over the elements by their first row (the lowest colour free at both
// endpoints, ≤ 64 colours); within a colour the elements run by that row, so
// a batch's slot writes land in neighbouring rows.  entry: per colour a run of
// element ids padded to whole 64-element batches (−1), cstart[c] its start;
// pos[2e], pos[2e+1]: the element's SELL positions in its two rows (−1 for
// skipped / self-loop elements, which the assembly leaves out).
struct ElemColour {
  int colors = 0;
  std::vector<int32_t> cstart;  // colors + 1, in entries
  std::vector<int32_t> entry;   // element id or −1
  std::vector<int32_t> pos;     // E × 2
};
std::string build_elem_colour(const Pattern& P, ElemColour& out);

// sort_window: 0/1 = original node order, kOrderDFS = depth-first order of the
// free-node graph (default; chains contiguous), >1 = degree sort inside
// windows of that many rows.
constexpr int kOrderDFS = -1;

// Validates and builds.  Returns "" on success, else an error message.
// skip_invalid: drop elements with out-of-range node ids (src/fea_petsc.cpp:241)
// instead of failing (src/fea_solver.py:82-83 raises).
// ghost (multi-GPU, partition.hpp): nodes owned by another partition.  They
// take the last rows — a ghost grip node keeps its kTop / kBot code (its value
// is prescribed), a ghost free node gets kGhost — and never enter the free,
// top or bottom blocks.
std::string build_pattern(int64_t n_nodes, const double* xyz, int64_t n_elems, const int64_t* e2n,
                          bool skip_invalid, const std::vector<int64_t>& top,
                          const std::vector<int64_t>& bot, int sort_window, Pattern& P,
                          const std::vector<uint8_t>* ghost = nullptr);

// ---------------------------------------------------------------------------
// Wave-local CG operator ("ELL-3 lanes") over the free rows [0, n_free).
//
// One lane = one wavefront lane of the CG iteration kernel.  A free row gets
// an OWNER lane, plus HELPER lanes directly after it when it has more than
// three free-neighbour slots or more than one out-of-wave neighbour; a group
// never straddles a 64-lane wave (inert padding lanes).  Every lane holds up
// to three slots (k-major arrays [k][n_lanes]); slots to grip (known) rows
// are dropped (u = 0 there).  A slot's neighbour u_j comes from
//   - the lane of j's owner in the SAME wave: a cross-lane permute, or
//   - a halo record (slot 0 only, ≤ 1 per lane) that j's group pushed in the
//     previous launch: partner[lane] is the lane whose record this lane's
//     slot-0 partner reads, i.e. where this lane pushes its owner's (r, s, w).
// So an iteration needs no neighbour index loads: one memory round trip.
constexpr int kEllSlots = 3;
constexpr uint32_t kEllNone = 0xFF, kEllHalo = 0xFE;  // = kSrcNone / kSrcHalo (kernels.hpp)

struct Ell {
  int64_t n_lanes = 0;            // multiple of 64 (0 when n_free == 0)
  std::vector<int32_t> lane_row;  // owner lane → row; helper / inert → -1
  std::vector<int32_t> row_lane;  // free row → owner lane
  std::vector<int32_t> info;      // owner: #helpers; helper: -(distance to owner); inert: 0
  std::vector<uint32_t> code;     // byte k = source of slot k: lane 0..63, kEllHalo, kEllNone
  std::vector<int32_t> partner;   // push target lane of slot 0 (halo), -1
  std::vector<int32_t> src_pos;   // [k][n_lanes] SELL position of the slot, -1
  std::vector<int32_t> nbr_lane;  // [k][n_lanes] owner lane of the neighbour, -1
  // compact halo records: the in-partition halo lanes, numbered in lane order
  int64_t n_hrec = 0;
  std::vector<int32_t> hrec;      // per lane: its record index, -1
  std::vector<uint64_t> hmask;    // per wave: lanes owning a record
  std::vector<int32_t> hbase;     // per wave: index of its first record
};

// Builds the lanes for P's free rows.  Returns "" on success.
// elem_pair (multi-GPU): per element, its cross-partition pair index
// (partition.hpp).  A slot to a kGhost row is a REMOTE halo slot: always slot 0
// of its lane, and partner = -2 - pair (the lane sends its owner's record to
// that pair's send slot and reads the peer's record from the receive slot).
std::string build_ell(const Pattern& P, Ell& L, const std::vector<int32_t>* elem_pair = nullptr);

// Scalar CSR over the 3·N DOFs in original order, pattern = the reference's
// csr_matrix pattern for the active set (src/fea_solver.py:93-105):
// block (n,m) present iff an active element joins n and m (or n == m and n has
// an active incident element); all 9 entries of a present block are stored.
// diag/vals are the device arrays copied back (6 symmetric components each).
void export_csr(const Pattern& P, const std::vector<uint8_t>& active,
                const std::vector<double>& diag6 /* 6×N SoA */,
                const std::vector<double>& val6 /* 6×(slots·64) SoA */, std::vector<int64_t>& indptr,
                std::vector<int32_t>& indices, std::vector<double>& data);

}  // namespace mfea
