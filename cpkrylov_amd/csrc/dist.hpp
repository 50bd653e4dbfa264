// dist.hpp -- host plan of the row-block distributed solve (DESIGN.md
// section 7).  Host-only: ownership of the degrees of freedom, the per-rank slice of the
// exact LDL' factor, the separator solve and the halo plans of the distributed SpMVs.
//
// Ownership follows the top of the elimination tree.  The tree is cut below a small set T of
// separator pivots into disjoint subtrees, and the subtrees (in pivot order, so each rank's
// share is a few contiguous pieces of the ordering) are split into P balanced runs.  A
// subtree's forward and backward sweeps need nothing outside the subtree except, backward,
// the separator values; the separator rows need a few subtree values from every rank.  So one
// allgather per apply of those values makes every rank able to solve T redundantly in the
// exported factor's order -- the distributed apply is bit-identical to the 1-GPU one.
#pragma once
#include <cstdint>
#include <vector>

#include "dev.hpp"
#include "host.hpp"

namespace cpk {

struct TreeSplit {
    int P = 1;
    std::vector<int32_t> node_rank;  // factor row -> owning rank, -1 for separator rows
    std::vector<int32_t> T;          // separator rows, ascending
};
// tol: accepted load imbalance (max/avg - 1); T grows until it is met or T reaches tmax rows.
// Every rank must pass the same tol (each builds the same global plan independently).
constexpr double kSplitTol = 0.03;
// Akry (optional): the Krylov operator's (1,1) block A (n x n).  Isolated rows (no factor
// entries) then follow the rank of a dof A couples them with, which keeps the Krylov SpMV's
// halo small (S50's slack rows couple only through A).
TreeSplit split_tree(const Factor &f, int P, double tol = kSplitTol, int64_t tmax = -1, const HCsr *Akry = nullptr);

// Dof ownership.  Rank r's local vectors are [owned x-part dofs ascending; owned y-part dofs
// ascending], so the solvers' [x; y] index ranges keep their meaning locally.
struct DofMap {
    int P = 1;
    int64_t n = 0, m = 0, N = 0;
    std::vector<int32_t> owner;  // dof -> rank
    std::vector<int32_t> lidx;   // dof -> index in the owner's local vector
    std::vector<int64_t> n_loc, m_loc;
    std::vector<int32_t> dofs(int rank) const;  // local index -> dof
};
DofMap make_dofmap(const Factor &f, const TreeSplit &ts, int64_t n);

// A distributed CSR: rank-local rows (local vector order) with each row's entries in the
// global matrix's column order.  Column c < N_loc is local; c >= N_loc is a ghost read from
// the allgathered halo buffer at position c - N_loc = owner * kstride + slot.
struct DistCsr {
    HCsr a;                     // nrows = local rows, ncols = N_loc (+ ghost space)
    int64_t nloc = 0;           // local vector length (first ghost column)
    int64_t kmax = 0;           // halo payload per rank
    int64_t kstride = 0;        // slots per rank in the halo buffer: kmax + spare
    std::vector<int32_t> send;  // local indices this rank publishes, in slot order
};
// rows_x_only: only the x-part rows (the shift's [A B'] rows); spare: extra slots per rank
// after the halo values (a solver's partial sums ride there, solvers.hip)
DistCsr dist_csr(const HCsr &K, const DofMap &dm, int rank, bool rows_x_only, int64_t spare = 0);

// This rank's slice of the factor and the separator solve.
struct RankPlan {
    int P = 1, rank = 0;
    int64_t nsub = 0;                           // subtree rows of this rank
    Factor Fsub;                                // local subtree factor; perm = local vector index
    std::vector<int64_t> key;                   // exported-factor row of each local row (sum order)
    std::vector<std::vector<BwdExtra>> extra;   // backward entries into separator rows (col nsub + t)
    // separators (replicated on every rank)
    int64_t nT = 0, kt = 0;                     // T rows; allgather payload per rank
    std::vector<int64_t> tf_ptr;                // forward rows of T: col >= 0 payload position,
    std::vector<int32_t> tf_col;                //   col < 0 separator -(t + 1)
    std::vector<double> tf_val;
    std::vector<int32_t> tf_src;                // payload position of each T row's own input
    std::vector<int64_t> tb_ptr;                // backward rows of T (rows of L below t), descending
    std::vector<int32_t> tb_col;
    std::vector<double> tb_val;
    std::vector<double> DT;
    std::vector<int32_t> tlev_ptr, tlev_rows;   // T rows grouped by level
    std::vector<int32_t> tsend;                 // local rows whose w this rank publishes
    std::vector<int32_t> tdof;                  // rank 0: local vector index of each T dof (else empty)
};
RankPlan make_rank_plan(const Factor &f, const TreeSplit &ts, const DofMap &dm, int rank);

// blkdiag(A, C) and hstack(A, B') as global CSR (B' taken from Kp's upper-right block)
HCsr hstack_ab(const HCsr &A, const HCsr &Kp, int64_t n);

}  // namespace cpk
