// host.hpp -- host-side sparse structures, ordering and the static-pivot LDL' factorization
// that replaces MATLAB's ldl() inside opLDL2 (ops/opLDL2.m:81-86).
#pragma once
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace cpk {

// Error carrying a cpk_status code across C++ layers; converted at the C ABI.
struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

// Host CSR: 64-bit row pointers, 32-bit sorted column indices, no duplicates.
struct HCsr {
    int64_t nrows = 0, ncols = 0;
    std::vector<int64_t> ptr;
    std::vector<int32_t> ind;
    std::vector<double> val;
    int64_t nnz() const { return ptr.empty() ? 0 : ptr.back(); }
};

HCsr csr_from_csr(int64_t nr, int64_t nc, const int64_t *rp, const int32_t *ci, const double *v);
HCsr csr_from_csc(int64_t nr, int64_t nc, const size_t *jc, const size_t *ir, const double *pr);
HCsr transpose(const HCsr &a);
// Kp = [A B'; B C]  (opLDL2.m:81); throws CPK_ERR_DIM unless check_kp_dims passes
void check_kp_dims(const HCsr &A, const HCsr &B, const HCsr &C);  // opLDL2.m:61-75
HCsr assemble_kp(const HCsr &A, const HCsr &B, const HCsr &C);
// source of every Kp entry: (block << 40) | entry index, block 0 = A, 1 = B (B and B' entries),
// 2 = C, in assemble_kp's entry order (inputs that pass check_kp_dims)
std::vector<int64_t> kp_value_sources(const HCsr &A, const HCsr &B, const HCsr &C);
// blkdiag(A, C): the Krylov operator's diagonal blocks, used to fuse u = A*v and t = C*q.
HCsr blkdiag(const HCsr &A, const HCsr &C);
bool is_diagonal(const HCsr &a);

// ---- ordering --------------------------------------------------------------------------
enum OrderKind { ORD_NATURAL = 0, ORD_GFIRST_ND = 1, ORD_GFIRST_MD = 2, ORD_ND = 3, ORD_MD = 4 };
// Fill-reducing symmetric ordering of Kp (n = size of the (1,1) block). perm[k] = old index.
std::vector<int32_t> order_kp(const HCsr &Kp, int64_t n, int *kind_out);
// host threads for the analysis (CPK_THREADS, else OMP_NUM_THREADS, else the hardware's)
int host_threads();
// f(lo, hi) over contiguous chunks of [0, n) on up to host_threads() threads; for loops whose
// iterations write disjoint data (results do not depend on the thread count)
template <class F>
void parallel_for(int64_t n, F f, int64_t grain = 4096) {
    const int64_t T = std::min<int64_t>(host_threads(), (n + grain - 1) / grain);
    if (T <= 1) {
        if (n > 0) f(int64_t(0), n);
        return;
    }
    std::vector<std::thread> th;
    const int64_t chunk = (n + T - 1) / T;
    for (int64_t t = 1; t < T; t++) {
        const int64_t lo = t * chunk, hi = std::min(n, lo + chunk);
        if (lo < hi) th.emplace_back([=] { f(lo, hi); });
    }
    f(int64_t(0), std::min(n, chunk));
    for (auto &x : th) x.join();
}
// Rows of a column-compressed pattern (columns Lp / Li of an N x N matrix): rptr (N + 1), and
// for row i its columns rcol[rptr[i] ..) ascending with their column slots ridx (the serial
// column-by-column transpose, exactly), on host_threads() threads: each thread buckets the
// entries of an equal share of the columns by the thread owning their row, then places the
// rows it owns from those buckets in column order.  rcol / ridx must hold Lp[N] entries.
void transpose_pattern(int64_t N, const int64_t *Lp, const int32_t *Li, uint32_t *rptr, int32_t *rcol, int32_t *ridx);
// CPK_TIMING=1: wall times of the sub-phases of a host phase on stderr (diagnostic)
struct SubClock {
    bool on = getenv("CPK_TIMING") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void lap(const char *what) {
        if (!on) return;
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[cpk]   %-40s %8.3f s\n", what, std::chrono::duration<double>(now - t).count());
        t = now;
    }
};
// building blocks (exposed for tests)
std::vector<int32_t> min_degree(const HCsr &graph);
std::vector<int32_t> nested_dissection(const HCsr &graph, int leaf_size);

// ---- factorization -----------------------------------------------------------------------
// P'*Kp*P = L*D*L', L unit lower (strict part stored), D diagonal (1x1 static pivots).
struct Factor {
    int64_t N = 0;
    std::vector<int32_t> perm;   // perm[k] = original index of pivot k
    std::vector<int64_t> Lp;     // CSC of strict lower L
    std::vector<int32_t> Li;
    std::vector<double> Lx;
    std::vector<double> D;
    std::vector<int32_t> parent; // elimination tree
};
// Symbolic data of the up-looking factorization, for its numeric phase on the device
// (ldl.hip): row patterns of L (ascending), each row entry's CSC slot, the Kp entries that seed
// each row, and the rows grouped by elimination-tree height (rows of one height are independent).
struct LdlSymbolic {
    int64_t N = 0;
    std::vector<int32_t> Rp;      // row k of strict L: columns Rc[Rp[k] .. Rp[k+1]), ascending
    std::vector<int32_t> Rc;
    std::vector<int32_t> Rcsc;    // CSC slot (index into Factor::Li / Lx) of row entry t
    std::vector<int32_t> kp_ptr;  // seeds of row k: [kp_ptr[k], kp_ptr[k+1]) in Kp's entry order
    std::vector<int32_t> kp_tgt;  // row-entry slot t, or -1 for the pivot (diagonal) itself
    std::vector<uint32_t> kp_src; // Kp entry index of the seed
    std::vector<int32_t> lev_ptr; // rows of height h: lev_rows[lev_ptr[h] .. lev_ptr[h+1])
    std::vector<int32_t> lev_rows;
};
// Up-looking LDL'.  Row k's pattern (the reach of its Kp entries in the elimination tree) is
// processed in ascending column order, so the device numeric phase (ldl.hip), which walks the
// same pattern in the same order, reproduces L and D bit for bit.  numeric = false: structure
// only (Lx, D left empty); sym: also return the symbolic data of the device phase.
Factor ldl_factor(const HCsr &Kp, const std::vector<int32_t> &perm, int nthreads, LdlSymbolic *sym = nullptr,
                  bool numeric = true);

// ---- SpTRSV schedule ---------------------------------------------------------------------
// The elimination tree is cut into blocks: sets of whole subtrees of at most R rows and at
// most CAP forward / backward factor entries (so a block fits in LDS), solved by one
// workgroup each.  Blocks form rounds (block-level sets): a round's blocks only
// depend on earlier rounds, so one kernel launch per round and sweep suffices.  Inside a
// block, rows are grouped into intra-block levels separated by workgroup barriers.
struct Schedule {
    int64_t N = 0;
    std::vector<int32_t> order;        // new position -> old (factor) index: a topological relabel
    std::vector<int64_t> round_ptr;    // blocks of round r: [round_ptr[r], round_ptr[r+1])
    std::vector<int64_t> blk_row;      // block b rows: [blk_row[b], blk_row[b+1]) (new numbering)
    std::vector<int64_t> blk_lvl;      // block b levels: lvl_row[blk_lvl[b] .. blk_lvl[b+1]]
    std::vector<int64_t> lvl_row;      // level boundaries (row positions), one array for all blocks
    int64_t max_levels = 0;
    int64_t depth = 0;
};
// Round 0 (the wide bottom of the tree) uses blocks of (R0 rows, CAP0 entries); the upper
// rounds use (R1, CAP1), typically larger so that few launches cover the top of the tree.
// Round 0 peels subtrees of weight <= SUB0 (default CAP0) and packs them into blocks of CAP0:
// a block's level count is that of its tallest subtree, so packing several short subtrees
// per block cuts the barrier-separated level passes per row.
// extra_bwd[v] / extra_fwd[v]: backward / forward entries of row v outside the factor (the
// distributed separators' backward terms into T; T's own forward terms on the exchanged payload)
Schedule build_schedule(const Factor &f, int64_t R0, int64_t CAP0, int64_t R1, int64_t CAP1, int64_t SUB0 = 0,
                        const std::vector<int64_t> *extra_bwd = nullptr, const std::vector<int64_t> *extra_fwd = nullptr);
// Apply the schedule's relabel to the factor (values unchanged, exact data movement).
// src (optional): src[t] = index into f.Li / f.Lx of the relabelled factor's entry t.
Factor relabel(const Factor &f, const Schedule &s, std::vector<int32_t> *src = nullptr);

}  // namespace cpk
