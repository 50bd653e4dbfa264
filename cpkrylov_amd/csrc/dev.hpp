// dev.hpp -- device objects of libcpk (HBM-resident matrices, factor, workspaces) and the
// kernel launchers.  Included by host C++ (compiled with g++) and by the HIP units.
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <tuple>
#include <string>
#include <vector>

#include "cpk.h"
#include "host.hpp"

namespace cpk {

#define CPK_HIP(call)                                                                                   \
    do {                                                                                                \
        hipError_t e_ = (call);                                                                         \
        if (e_ != hipSuccess)                                                                           \
            throw ::cpk::Error(CPK_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_));        \
    } while (0)

template <class T>
struct DBuf {
    T *p = nullptr;
    size_t n = 0;
    DBuf() = default;
    DBuf(const DBuf &) = delete;
    DBuf &operator=(const DBuf &) = delete;
    DBuf(DBuf &&o) noexcept : p(o.p), n(o.n) { o.p = nullptr, o.n = 0; }
    DBuf &operator=(DBuf &&o) noexcept {
        if (this != &o) release(), p = o.p, n = o.n, o.p = nullptr, o.n = 0;
        return *this;
    }
    ~DBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr, n = 0;
    }
    void alloc(size_t count) {
        release();
        n = count;
        if (count) {
            hipError_t e = hipMalloc(&p, count * sizeof(T));
            if (e != hipSuccess) throw Error(CPK_ERR_NOMEM, "hipMalloc of " + std::to_string(count * sizeof(T)) + " bytes failed");
        }
    }
    void upload(const T *h, size_t count) {
        alloc(count);
        if (count) CPK_HIP(hipMemcpy(p, h, count * sizeof(T), hipMemcpyHostToDevice));
    }
    void upload(const std::vector<T> &h) { upload(h.data(), h.size()); }
    void zero(hipStream_t s) {
        if (n) CPK_HIP(hipMemsetAsync(p, 0, n * sizeof(T), s));
    }
    size_t bytes() const { return n * sizeof(T); }
};

// Collectives of a distributed context, enqueued on the context stream.  RCCL over xGMI in
// production; SimComm runs several ranks as threads sharing one GPU (tests on a 1-GPU box).
struct Comm {
    virtual ~Comm() = default;
    virtual void allreduce_sum(double *buf, size_t n, hipStream_t s) = 0;
    // integer sums (exact_dots: the superaccumulator digits of every rank, xacc.hpp)
    virtual void allreduce_sum_i64(int64_t *buf, size_t n, hipStream_t s) = 0;
    virtual void allgather(const double *send, double *recv, size_t n, hipStream_t s) = 0;
    // elementwise maximum over the ranks, in place on device memory: the status agreement of a
    // distributed solve (solvers.hip, agree_status) -- a rank-local failure reaches every rank
    virtual void allreduce_max_i64(int64_t *buf, size_t n, hipStream_t s) = 0;
    virtual bool capturable() const = 0;  // may be captured into a hipGraph
    virtual bool has_peers() const { return true; }  // false: the timing stand-in (no exchange)
    // rank `root`'s n host bytes at p to every rank's p (the distributed construction's analysis,
    // precond.cpp); n is the same on every rank.  Only where has_peers().  A receiver that passes
    // p = nullptr takes part and discards the bytes (a receiver that could not allocate keeps the
    // broadcast sequence, so the root never waits for it; the construction then fails everywhere).
    virtual void broadcast_host(void *p, size_t n, int root, hipStream_t s) = 0;
    virtual void release_staging() {}  // broadcast_host's device staging, kept across calls
    virtual int kind() const = 0;   // CPK_COMM_RCCL / _SIM / _NULL (cpk_ctx_get_info)
    virtual int count() const = 0;  // ranks of the communicator (RCCL: ncclCommCount)
};

// Sweep configuration: rows and entries staged per block, threads per block, round 0 / upper
// rounds (engine option "sweep": "rows,cap,threads" for both, or "R0,CAP0,T0,R1,CAP1,T1[,SUB0]").
// Default (r03 v40, profiles/r03_sub0_ab_v39.txt / r03_upper256_ab_v40.txt): round 0 peels subtrees
// of weight <= 480 (fewer levels per round-0 block: 9.75 -> 8.57 at S10) and the upper rounds use
// 256-thread blocks of <= 512 rows / 3072 entries, four per CU, so the doubled first upper round
// (1024 blocks at S10) stays co-resident: S10 875-879 -> 887-898 it/s.
struct SweepConfig {
    int rows[2] = {192, 512}, cap[2] = {576, 3072}, threads[2] = {64, 256};
    int sub0 = 480;  // round-0 subtree cap (0: cap[0])
};
// The distributed preconditioner's default for P > 1 (each rank schedules only its own
// subtrees): the single-GPU default's lower round-0 subtrees give a rank's 1.25 M rows at S10 /
// P = 8 a third sweep round, 0.337 against 0.311-0.321 ms per iteration
// (profiles/r03_dist_timing_v41.log), so such a rank keeps the round-0 blocks uncapped with
// 512-thread upper blocks.  A 1-rank communicator holds the whole system: the single-GPU default
// (profiles/r04_dist_v3.txt: 815 it/s with the distributed default against 892 on one GPU).
SweepConfig dist_sweep_default();

// Engine options of a context (opts.cpp; cpk_ctx_set_option).  None changes a result: they
// select equivalent execution paths (each is tested bit-exact against the default) or the
// sweep schedule and the distributed split, which every rank must build identically -- so a
// distributed preconditioner compares a hash of all of them across ranks before its first
// collective.  A context starts from the CPK_<NAME> environment variables, read once when it
// is created; objects built later see its current values.
struct EngineOpts {
    SweepConfig sweep;            // sweep:              LDS staging of the sweep schedule
    bool sweep_set = false;       //                     sweep given explicitly (else the per-path default)
    double split_tol = 0.03;      // split_tol:          distributed subtree weight tolerance
    bool host_factor = false;     // host_factor:        numeric LDL' on the host (reference path)
    bool no_pipe = false;         // no_pipe:            round 0 one workgroup per block
    bool no_upper = false;        // no_upper:           upper rounds through the generic kernels
    bool no_col16 = false;        // no_col16:           round-0 forward columns as int32
    bool no_dataflow = false;     // no_dataflow:        upper rounds always on the level loop
    bool all_dataflow = false;    // all_dataflow:       upper rounds always on the dataflow loop (tests)
    bool no_colsweep = false;     // no_colsweep:        upper rounds never on the column sweep
    bool all_colsweep = false;    // all_colsweep:       upper blocks of <= 256 rows always on the column sweep (tests)
    bool no_sched_resid = false;  // no_sched_resid:     refinement residual in original order
    bool no_fused_resid = false;  // no_fused_resid:     refinement residual as its own SpMV
    int r0_xcd_chunk = 16;        // r0_xcd_chunk:       K > 0: runs of K consecutive round-0 blocks share an XCD
    bool tsolve_global = false;   // tsolve_global:      separator records read from HBM
    bool tsolve_sweep = false;    // tsolve_sweep:       separator solved by the block sweeps (the path of a large T)
    bool no_piggy = false;        // no_piggy:           cpminres alpha by its own allreduce
    bool no_halo_merge = false;   // no_halo_merge:      cpminres beta by its own allreduce
    bool no_graph = false;        // no_graph:           no hipGraph capture of iterations
    bool no_fuse_last = false;    // no_fuse_last:       the last sweep round as two launches
    bool no_tkr = false;          // no_tkr:             distributed refinement residual through the Kp halo
    bool no_minres_fuse = false;  // no_minres_fuse:     cpminres update as its own pass (normalise + w, x)
    bool no_chain = false;        // no_chain:           upper rounds one launch per round (not the sweep chain)
    bool no_bcast_analysis = false;  // no_bcast_analysis: every rank of a distributed preconditioner runs the global analysis
    int chain_wide = 256;         // chain_wide:         rounds of at most this many blocks join the sweep chain
    bool dist_graph = true;       // dist_graph:         capture collectives in the graphs
    bool dist1 = false;           // dist1:              a 1-rank communicator runs the distributed path
                                  //                     (diagnostic; set before building operators)
    bool exact_dots = false;      // exact_dots:         every inner product the correctly rounded exact sum
                                  //                     of its TwoProd pairs (xacc.hpp): order-independent,
                                  //                     the oracle's orc_set_exact values bit for bit; the
                                  //                     one option that changes results (last bits)
    int batch = 0;                // batch:              fixed iterations per graph (0: adaptive)
    bool profile_fwd_sched = false;     // profile_fwd_sched: diagnostic, the profiled forward reads its input in schedule order
    bool profile_passes = false;  // profile_passes:     diagnostic, cpdqgmres runs eagerly with HIP events around its
                                  //                     passes (cpk_debug_pass_times: the bench's s50 block)
    // fail_inject: test hook, "R:site" -- rank R of a distributed solve fails locally at `site`:
    // "setup" (before the solve's first collective), "batch:K" (a host error after its K-th graph
    // batch) or "chain:K" (the sweep chain's device error word set after batch K).  Rank-local by
    // design, so it is NOT part of the plan agreement's hash (tests/test_gpu_dist.py)
    std::string fail_inject;
};
EngineOpts engine_opts_from_env();
// name as in the comments above; throws CPK_ERR_ARGS on an unknown name or a bad value
void set_engine_option(EngineOpts &o, const std::string &name, const std::string &value);
// dist: the value a distributed preconditioner uses (the sweep's per-path default)
std::string get_engine_option(const EngineOpts &o, const std::string &name, bool dist = false);
// the sweep configuration a preconditioner of this path is built with
SweepConfig effective_sweep(const EngineOpts &o, bool dist);
// every option as "name=value;name=value;..." (the effective sweep, and sweep_set as its own
// entry), and the inverse: a spec of that form applied on top of o
std::string engine_opts_string(const EngineOpts &o, bool dist);
void apply_engine_options(EngineOpts &o, const std::string &spec);
uint64_t engine_opts_hash(const EngineOpts &o);  // FNV-1a over every option

// Execution context: one GPU, one stream, reduction workspace (and a Comm when nranks > 1).
struct Ctx {
    EngineOpts opts;
    int device = 0, rank = 0, nranks = 1;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    DBuf<double> partials;   // per-workgroup partial sums of the grid reductions
    DBuf<unsigned> counter;  // arrival tickets
    DBuf<double> red;        // distributed mode: local sums awaiting the allreduce
    // exact_dots: sub-accumulators of the exact reductions (zero between launches) and, in
    // distributed mode, the digits awaiting the int64 allreduce (xacc.hpp)
    DBuf<int64_t> xsub, xred;
    Comm *comm = nullptr;    // owned by the C-ABI context object
    // the distributed path: a communicator of more than one rank.  A 1-rank communicator has
    // nothing to exchange and runs the single-GPU path (the same bits) unless engine option
    // dist1 asks for the distributed kernels (tests; DESIGN.md section 7's 1-rank comparison).
    // The timing stand-in (NullComm) declares nranks > 1.
    bool dist() const { return comm != nullptr && (nranks > 1 || opts.dist1); }
    // profile_passes: the last profiled solve's per-pass sums (cpk_debug_pass_times):
    // [iterations, Krylov SpMV ms, M*z ms, window dots ms, orthogonalisation ms, direction ms,
    //  sum of the dots' window sizes, sum of the direction's window sizes]
    double pass_ms[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    bool exact() const { return opts.exact_dots; }
    // reduction workspace for grids of up to `count` partial sums (and, in exact mode, the
    // sub-accumulators of at least 4 sums); ensure_xacc: room for `nsums` exact sums per launch
    void ensure_partials(size_t count);
    void ensure_xacc(size_t nsums);
};

// HBM-resident CSR with a row-block partition for the LDS-staged streaming SpMV.
constexpr int kSpmvCap = 2048;      // entries staged in LDS per workgroup
constexpr int kSpmvMaxRows = 1024;  // rows per workgroup
// 6 waves per SIMD (<= 80 VGPRs): the reducing epilogues otherwise take 82 and run 5
#ifndef CPK_SPMV_WAVES
#define CPK_SPMV_WAVES 6
#endif
struct DMat {
    int64_t nrows = 0, ncols = 0, nnz = 0, nblk = 0;
    DBuf<uint32_t> ptr;
    DBuf<int32_t> col;
    DBuf<double> val;
    DBuf<int32_t> blk;  // row-block boundaries [nblk + 1]
    bool is_diag = false;
    uint64_t gen = 0;   // unique per upload (keys cached solver graphs)
    // distributed rows (DistCsr): columns >= nloc read the allgathered halo buffer
    int64_t nloc = -1, kmax = 0, kstride = 0, nsend = 0;
    DBuf<int32_t> send;         // local indices published to the other ranks
    DBuf<double> sbuf, rbuf;    // halo payload [kstride], allgathered halo [nranks * kstride]
    bool halo() const { return nloc >= 0; }
    // ghost columns to read (a distributed matrix with a non-empty halo): the SpMV's HALO variant
    bool ghosts() const { return halo() && kmax > 0; }
    size_t bytes() const { return ptr.bytes() + col.bytes() + val.bytes() + blk.bytes(); }
};
void make_dmat(const HCsr &a, DMat &d);
struct DistCsr;
void make_dist_dmat(const DistCsr &a, int nranks, DMat &d);
// allgather the halo of x (local vector) into A.rbuf
void launch_halo(Ctx &c, const DMat &A, const double *x, bool packed = false);
// r = xin - A*y with A's columns >= A.nloc read from halo[c - nloc] (no exchange)
void launch_spmv_resid_loc(Ctx &c, const DMat &A, const double *xin, int64_t neg_from, const double *y, double *r,
                           const int *run, const double *halo);

// A sweep chain's tasks in topological order (task = kind << 28 | block; kind 0 forward, 1 last,
// 2 backward), each task's producer tasks (dptr / didx), a done flag per task and {epoch,
// ticket, error} (zero at build); tpb: the block kernel it runs (256 or 512 threads)
enum { kChainFull = 0, kChainFwd = 1, kChainBwd = 2 };
struct DChain {
    int64_t ntask = 0;
    int tpb = 0;
    DBuf<int32_t> task, dptr, didx;
    DBuf<uint32_t> flag, ctrl;
};

// HBM-resident factor + sweep schedule (rows in schedule order).
struct DFactor {
    int64_t N = 0, nnz = 0, nblk = 0, nlvl = 0;
    DBuf<uint32_t> fptr;  // forward rows of strict lower L, columns ascending
    DBuf<int32_t> fcol;
    // the upper rounds' rows [urow0, N): leading outside-term count of each row's forward and
    // backward entries, [2 (row - urow0) + bwd] (the kernels' fold_known; empty: fold_prefix)
    DBuf<int16_t> ufold;
    DBuf<int16_t> ustep;  // the row's step in its block's column sweep, same layout
    int32_t urow0 = 0;
    // the column sweep's staged column of every entry of the upper rounds' rows, per direction
    // (kernels.hip kCsOut / kCsStep): in-block, the column's step | the run of outside entries
    // behind it << 8; outside, kCsOut.  ucode[dir][e - ucode0[dir]] for entry e of fcol / bcol
    DBuf<int16_t> ucode[2];
    uint32_t ucode0[2] = {0, 0};
    DBuf<int16_t> fcol16;  // round 0 when every forward entry is local: column - block's first row (else empty)
    int64_t nnz16 = 0;     // forward entries stored in fcol16 (10 bytes each instead of 12)
    DBuf<double> fval;
    DBuf<uint32_t> bptr;  // backward rows (= columns of L), row indices descending
    DBuf<int32_t> bcol;
    DBuf<double> bval;
    DBuf<double> D;
    DBuf<int32_t> perm;     // perm[k] = original index of pivot k
    DBuf<int32_t> blk_lvl;  // [nblk + 1]
    DBuf<int32_t> lvl_row;  // [nlvl + 1]
    DBuf<int32_t> meta;     // [nblk][8]: r0, r1, l0, l1, fwd e0, e1, bwd e0, e1
    bool pipelined = true;  // round 0 through the persistent pipelined kernel (set before make_dfactor)
    bool no_upper = false;  // upper rounds through the generic kernels (set before make_dfactor)
    bool no_col16 = false;  // no int16 round-0 forward columns (set before make_dfactor)
    int dataflow = 0;       // upper-round level loops: 0 the host model per block, 1 never, 2 always
    int colsweep = 0;       // the column sweep (levels_colsweep): 0 the host model per block, 1 never, 2 always
    // engine options of the preconditioner's context when it was built (launch-time paths)
    bool no_fused_resid = false;
    bool fuse_last = false;  // single GPU, no entries outside the factor: the last round fwd + bwd in one launch
    bool skip0 = true;       // round 0's level-0 rows have no forward entries (false: a separator's T sweep)
    int64_t round0_rows = -1;  // round 0 is the rows [0, round0_rows) (-1: not a leading row range)
    // rows of round 0 whose backward value the pipelined kernel does not store back into w in a
    // sweep launched with wdead (launch_sptrsv_bwd): the byte models drop them
    int64_t bwd_dead_w_rows() const { return pipelined && round0_rows > 0 ? round0_rows : 0; }
    std::vector<int32_t> hmeta;  // host copy of meta
    std::vector<int64_t> hmodel; // the upper blocks' loop-cost model (mark_dataflow; diagnostic)
    // (first, last) block of a launch -> its blocks' largest rows / entries (the LDS image, kernels.hip)
    mutable std::map<std::pair<int64_t, int64_t>, std::pair<int, int>> img_cache;
    // round-0 blocks assigned to the persistent launch's workgroups by modelled cost (plan_round0),
    // per kernel variant v (0 forward, 1 forward with the fused refinement residual, 2 backward):
    // workgroup g runs the BlkMeta records ameta[v][aptr[v][g] .. aptr[v][g + 1]); agrid[v] = the
    // grid they were made for (0: none; the launch then strides over meta)
    DBuf<int32_t> aptr[3], ameta[3];
    int agrid[3] = {0, 0, 0};
    // the sweep chains (kernels.hip, sptrsv_chain_kernel): the narrow top rounds [chain_first, R)
    // in ONE launch whose blocks wait for their own producers (flags) instead of for whole
    // rounds.  kChainFull: those rounds forward, the last round (forward + backward) and those
    // rounds backward (single GPU, the last round fused); kChainFwd / kChainBwd: forward only /
    // backward only (a distributed solve, the separator exchange between them)
    DChain chain[3];
    int64_t chain_first = 1;  // the first chained round (the chains cover [chain_first, R))
    bool no_chain = false;  // engine option no_chain (set before make_dfactor)
    int chain_wide = 256;   // engine option chain_wide
    std::vector<int64_t> round_ptr;  // host copy: blocks per round
    std::vector<char> round_fits;    // host: every block of round r fits (sweep_rows[1], sweep_cap[1])
    int sweep_rows[2] = {192, 1024}, sweep_cap[2] = {576, 4096}, sweep_threads[2] = {64, 512};  // round 0 / rest
    size_t bytes() const {
        return fptr.bytes() + fcol.bytes() + fcol16.bytes() + ufold.bytes() + ustep.bytes() + ucode[0].bytes() + ucode[1].bytes() + fval.bytes() + bptr.bytes() + bcol.bytes() + bval.bytes() + D.bytes() +
               perm.bytes() + blk_lvl.bytes() + lvl_row.bytes() + meta.bytes();
    }
};
// a backward-sweep entry of row q referring to a row outside the factor (col >= N)
struct BwdExtra {
    int32_t col;
    int64_t key;
    double val;
};
// fsrc / bsrc (optional): the f.Li / f.Lx slot of every forward / backward device entry (the
// device numeric factorization fills fval / bval through them); f.Lx may be empty (zeros)
void make_dfactor(const Factor &f, const Schedule &s, DFactor &d, const std::vector<int64_t> *key = nullptr,
                  const std::vector<std::vector<BwdExtra>> *extra = nullptr, std::vector<int32_t> *fsrc = nullptr,
                  std::vector<int32_t> *bsrc = nullptr);
size_t sweep_lds_bytes(int R, int CAP);
// the round-0 block assignment of every kernel variant for the grids the launches will use;
// kps_ptr (optional): row pointers of Kp in schedule order (the fused-residual variant's cost)
void plan_round0(Ctx &c, DFactor &d, const int64_t *kps_ptr);

// ---- launchers (kernels.hip) -------------------------------------------------------------
// Flags: a kernel is a no-op when *run == 0 or *active == 0 (either pointer may be null).
// neg_from: input entries with index >= neg_from are negated on load (the reference's [u; -t]).
void launch_spmv(Ctx &c, const DMat &A, const double *x, double *y, const int *run);
// r = xin - A*y  (halo_packed: y's halo payload is already in A.sbuf, allgather only)
void launch_spmv_resid(Ctx &c, const DMat &A, const double *xin, int64_t neg_from, const double *y, double *r,
                       const int *run, const int *active, bool halo_packed = false);
// r = xin - A*y, and *active = (||r|| >= tol*||xin||) computed on device (opLDL2.m:176-177,183)
void launch_spmv_resid_norm(Ctx &c, const DMat &A, const double *xin, int64_t neg_from, const double *y, double *r,
                            double tol, int *active_out, const int *run, const int *active, bool halo_packed = false);
// y = A*x restricted to columns >= col_min (B'*v from the first n rows of Kp)
void launch_spmv_colmask(Ctx &c, const DMat &A, int64_t col_min, const double *x, double *y, const int *run);
// forward sweep w = L \ (P' * xin), backward sweep out (=|+=) P * (L' \ (D \ w))
// sched_in: xin is already in schedule order (no perm gather, no negation)
// xs (optional): also store the signed input in schedule order (the refinement residual's x)
// Distributed payloads packed by the sweeps' write-back (kernels.hip: PackArgs users)
struct PackArgs {
    const int32_t *slot = nullptr;
    double *buf = nullptr;
    const int32_t *tdof = nullptr;
    int ntdof = 0, nsend = 0, kt_data = 0;
    const double *x = nullptr;
    int64_t neg_from = 0;
    const double *piggy = nullptr;
};

// the forward input of a deferred last round (launch_sptrsv_fwd's defer, launch_sptrsv_bwd's last)
struct FwdIn {
    const double *xin = nullptr;
    int64_t neg_from = 0;
    int sched_in = 0;
    double *xs = nullptr;
    bool valid = false;
    int64_t from = 0;  // the deferred round (the last one; with chain, the first upper round)
    bool chain = false;  // every upper round deferred to the backward sweep's chain launch
};
// the sweep chain's error word (a producer wait timed out): CPK_ERR_HIP, cleared
void check_chain(const DFactor &F);
// the distributed solve's status word: host_code, raised to chain_code if a chain error word of
// any of the nf factors is set (kernels.hip, solve_status_kernel)
void launch_solve_status(Ctx &c, const DFactor *const *F, int nf, int64_t host_code, int64_t chain_code, int64_t *out);
bool debug_set_chain_error(Ctx &c, const DFactor &F);
bool fuse_last_ok(const DFactor &F);
// defer (optional): the last round is left to the backward sweep (sptrsv_last_kernel solves it
// forward and backward in one launch); *defer then says how, for launch_sptrsv_bwd's last
// pk (optional, distributed): the separator payload packed by the write-back; returns whether
// every round packed (else the caller packs with tpack_kernel)
bool launch_sptrsv_fwd(Ctx &c, const DFactor &F, const double *xin, int64_t neg_from, double *w, const int *run,
                       const int *active, bool sched_in = false, double *xs = nullptr, FwdIn *defer = nullptr,
                       const PackArgs *pk = nullptr);
// out == null: the solution stays in schedule order in w (and with add, ys += it in place);
// add with ys: out = P * (ys + solution), ys the previous solution in schedule order
// pk (optional, distributed): the output packed by the write-back, keyed by output index (out
// given) or by schedule row (out == null); returns whether every round packed
// wdead: nothing reads w after this sweep, so the pipelined round 0 (the sweep's last round)
// does not store its rows back into it (it still writes out / ys)
bool launch_sptrsv_bwd(Ctx &c, const DFactor &F, double *w, double *out, bool add, const int *run,
                       const int *active, double *ys = nullptr, const FwdIn *last = nullptr, const PackArgs *pk = nullptr,
                       bool wdead = false);
// r = xin(perm) - A*y with A = P'*Kp*P in schedule order (rows and columns), y in schedule
// order (perm null: xin is the signed input already in schedule order, see launch_sptrsv_fwd);
// order; each row sums its entries in Kp's column order, so r(k) equals row perm(k) of the
// original-order residual bit for bit
void launch_spmv_resid_sched(Ctx &c, const DMat &A, const int32_t *perm, const double *xin, int64_t neg_from,
                             const double *y, double *r, const int *run);
// fused refinement input: r = xs - Kps*y, then the forward sweep in place on r (schedule order);
// round 0 forms r inside the sweep, the rows above it by the round-0 kernel's workgroups after
// their blocks.  Bit-identical to launch_spmv_resid_sched + launch_sptrsv_fwd(sched_in).  False
// (nothing launched): no matching configuration.
// pk / packed (distributed): the separator payload packed by the sweep's write-back, and whether
// every round packed it (else the caller packs with tpack_kernel)
bool launch_sptrsv_fwd_resid(Ctx &c, const DFactor &F, const DMat &Kps, const double *xs, const double *y, double *r,
                             const int *run, FwdIn *defer = nullptr, const PackArgs *pk = nullptr,
                             bool *packed = nullptr);
// buf[slot[q]] = w[q] for q < n with slot[q] >= 0 (a payload the sweeps' write-back did not pack)
void launch_pack_slots(Ctx &c, const int32_t *slot, int64_t n, const double *w, double *buf, const int *run);
int debug_pipe_stamps(uint64_t *out, int npairs);  // diagnostic build only (CPK_PIPE_STAMPS)
int64_t debug_blk_cycles(uint64_t *out, int64_t n);  // likewise: [4][1 << 17] per-block cycles
// Kps row blocks of the rows [row0, nrows) (A.blk with a boundary at row0)
// out[i] = x[idx[i]]
void launch_gather(Ctx &c, const double *x, const int32_t *idx, int64_t n, double *out);
// small vector helpers
void launch_set_concat(Ctx &c, double *dst, const double *a, int64_t na, int64_t nb);  // dst = [a; 0]

// ---- distributed mode (comm.cpp, kernels.hip) --------------------------------------------
Comm *make_rccl_comm(int nranks, int rank, const unsigned char *uid);
void rccl_unique_id(unsigned char *uid);
struct SimGroup;
SimGroup *simgroup_create(int nranks);
void simgroup_destroy(SimGroup *g);
Comm *make_sim_comm(SimGroup *g, int rank);
Comm *make_null_comm(int rank, int nranks);  // diagnostic timing stand-in (cpk_ctx_create_null)
void launch_sum_slots(hipStream_t s, const double *slots, int P, size_t n, double *out);
void launch_sum_slots_i64(hipStream_t s, const int64_t *slots, int P, size_t n, int64_t *out);
struct DSep;
// pack this rank's separator payload (w rows read by T, rank 0: +-x at the T dofs), allgather
// t = x_eff - g with x_eff[i] = (i >= neg_from ? -x[i] : x[i])  (the GHN residual update)
void launch_sub_state(Ctx &c, const double *x, int64_t neg_from, const double *g, int64_t N, double *t,
                      const int *run);
// packed: the payload is already in S.sbuf (the forward sweep packed it): the allgather only
void launch_sep_exchange(Ctx &c, const DSep &S, const double *w, const double *x, int64_t neg_from,
                         const double *piggy_src = nullptr, bool packed = false);
// redundant separator solve into wT (= w + nsub); rank 0 writes (add: accumulates) y at the T dofs
// hslot / hbuf (optional): also pack y's Kp halo at the T dofs (PackArgs, backward)
// tkr_* (optional, Precond::tkr): first form the T rows' refinement residual (launch_tkr_resid's
// arithmetic, inside the prefix kernel when that path runs) from y's T values tkr_yT (default: wT,
// which this solve overwrites last)
void launch_sep_solve(Ctx &c, const DSep &S, double *wT, double *y, bool add, const int *run, const int *active,
                      const int32_t *hslot = nullptr, double *hbuf = nullptr, const int32_t *tkr_ptr = nullptr,
                      const int32_t *tkr_col = nullptr, const double *tkr_val = nullptr,
                      const double *tkr_yT = nullptr);
// the T rows' refinement residual after the refinement's separator exchange, on every rank:
// S.rbuf[tf_src[t]] (the T input +-x sent by rank 0) -= Kp row t * y, y from wT (T columns) and
// the exchange's extra slots (subtree columns); each row summed in Kp's column order from 0.0
void launch_tkr_resid(Ctx &c, const DSep &S, const int32_t *ptr, const int32_t *col, const double *val,
                      const double *wT, const int *run, const int *active);

// ---- device numeric LDL' (ldl.hip) --------------------------------------------------------
struct DLdl {
    int64_t N = 0, nnz = 0, nf = 0, nb = 0;
    std::vector<int32_t> lev_ptr;  // host: rows by elimination-tree height
    std::vector<int32_t> lev_long; // host: height l's long rows (one wave each) start at lev_long[l]
    int64_t max_long = 0;          // longest pattern among them
    DBuf<int32_t> lev_rows, Rp, Rc, Rcsc, Lp, Li, kp_ptr, kp_tgt, fsrc, bsrc, dsrc;
    DBuf<uint32_t> kp_src;
    DBuf<int64_t> kp_from;  // Kp entry -> (block << 40 | entry) of A11 / B / C22 (refactorization)
    DBuf<double> Lx, D, Y;  // L in CSC order, D in pivot order, per-row-entry scratch
    DBuf<int> bad;
    bool sym_ready = false;  // dldl_setup_sym done
    bool ready = false;
};
// the two halves of dldl_setup: the symbolic data (uploadable while the host still builds the
// schedule) and the value sources of the sweep layouts; ready after both
void dldl_setup_sym(DLdl &d, const LdlSymbolic &sym, const Factor &f);
void dldl_setup_src(DLdl &d, const std::vector<int32_t> &fsrc, const std::vector<int32_t> &bsrc,
                    const std::vector<int32_t> &order);
void dldl_setup(DLdl &d, const LdlSymbolic &sym, const Factor &f, const std::vector<int32_t> &fsrc,
                const std::vector<int32_t> &bsrc, const std::vector<int32_t> &order);
// numeric factorization from the device Kp values, then DFactor's sweep values and D;
// throws CPK_ERR_FACTOR on a zero or NaN pivot
void dldl_factor(Ctx &c, DLdl &d, const double *kpv, DFactor &dF);
// the numeric phase alone into caller-owned Lx (CSC order) / D (pivot order); throws on a bad
// pivot having written only Lx, D and d's scratch (a refactorization commits after it returns)
void dldl_numeric(Ctx &c, DLdl &d, const double *kpv, double *Lx, double *D);
// DFactor's sweep values and D from d.Lx / d.D
void dldl_fill(Ctx &c, const DLdl &d, DFactor &dF);
// Value maps (distributed preconditioner): a device array built from index-valued factor data
// (value = source index + 1, 0 = no source) is captured as map[q] = value - 1 and refilled as
// x[q] = map[q] >= 0 ? src[map[q]] : 0.0
void vmap_capture(Ctx &c, const double *x, size_t n, DBuf<int32_t> &map);
void vmap_fill(Ctx &c, const int32_t *map, size_t n, const double *src, double *x);
// Kp values from the device values of A11, B, C22 through d.kp_from
void dldl_assemble_kp(Ctx &c, const DLdl &d, const double *a, const double *b, const double *cc, double *kpv);

// ---- preconditioner (precond.cpp) --------------------------------------------------------
// Host analysis of opLDL2's constructor: Kp assembly, ordering, LDL', sweep schedule.
struct Analysis {
    int64_t n = 0, m = 0, N = 0;
    HCsr Kp;
    Factor F0;  // the factor as exported: P'*Kp*P = L*D*L' in pivot order (the reference's view)
    Factor F;   // F0 relabelled to the schedule order (S.order[q] = F0 index of row q)
    Schedule S;
    int ordering = 0;
    double seconds = 0;
    SweepConfig sweep;
    // device_numeric: the host computed structure only (F0.Lx, F0.D empty); sym and rsrc feed
    // the device numeric phase (ldl.hip)
    bool device_numeric = false;
    LdlSymbolic sym;
    std::vector<int32_t> rsrc;  // F's entry t came from F0's entry rsrc[t]
    uint64_t input_hash = 0;    // this rank's own A11, B, C22 (pattern and values): the plan agreement
};
// on_symbolic (optional) runs on a second host thread as soon as the symbolic factor exists,
// beside the schedule and the relabelling (which only read it), and is joined before analyze
// returns: precond_create uploads the device factorization's symbolic data there
using SymbolicHook = std::function<void(const HCsr &Kp, const Factor &, const LdlSymbolic &)>;
// global_schedule = false: no schedule / relabelled factor of the whole system (a distributed
// preconditioner schedules each rank's subtrees itself; an.S and an.F stay empty)
Analysis analyze(const HCsr &A11, const HCsr &B, const HCsr &C22, const EngineOpts &o, bool device_numeric = false,
                 const SymbolicHook &on_symbolic = {}, bool global_schedule = true);

// The separator solve of a distributed preconditioner, device copy.
constexpr int64_t kSepPiggy = 2;  // spare payload slots per rank in the separator exchange
// spare slots per rank in the Krylov operator's halo exchange: the Lanczos beta partials ride
// there with the next vector's halo (solvers.hip, cpminres)
// block record flags (DFactor::meta, the l1 field): the dataflow level loop per direction for
// an upper-round block (mark_dataflow, kernels.hip); every reader of l1 masks them off
constexpr int kBlockModelW = 8;  // fields per (upper block, direction) of DFactor::hmodel
constexpr int32_t kMetaDfFwd = 1 << 30, kMetaDfBwd = 1 << 29, kMetaCsFwd = 1 << 28, kMetaCsBwd = 1 << 27,
                  kMetaCoFwd = 1 << 26, kMetaCoBwd = 1 << 25, kMetaL1Mask = (1 << 25) - 1;
constexpr int64_t kKrylovSpare = 2;
struct DSep {
    int64_t nT = 0, kt = 0, nlev = 0, nsend = 0, ntdof = 0;
    int64_t kt_data = 0;  // payload values of the plan; [kt_data, kt) are the piggyback slots
    DBuf<int32_t> tf_src, send, tdof;  // each T row's input position in the payload; tpack's rows; rank 0's T dofs
    DBuf<double> DT, sbuf, rbuf;
    // stepped solve (tprefix_kernel + tsolve_steps_kernel): forward rows split into their
    // leading payload terms (tk_*) and the rest; the level solve is nsf forward and nsb backward
    // steps (steps[s] = waves | barrier flag) of records rec_v / rec_m (kernels.hip);
    // tprefix_kernel writes the row prefixes into pre (pre[nT] = 1.0) and the rest's payload
    // terms (tr_*, pre-multiplied) into their records' values (tr_slot)
    DBuf<int32_t> tk_ptr, tk_col, tr_ptr, tr_col, tr_slot, steps;
    DBuf<int32_t> tslot;  // local schedule row -> payload slot (-1: not sent): the forward sweep packs
    DBuf<double> tk_val, tr_val, pre, rec_v;
    DBuf<uint32_t> rec_m;
    int64_t nsf = 0, nsb = 0, nrec = 0;
    size_t lds = 0;    // LDS bytes of the stepped solve with its records staged, 0 = too large
    size_t lds_g = 0;  // LDS bytes with the records left in HBM; 0 (or no records): the T sweep
    bool tsolve_global = false;  // engine option at construction
    // T sweep (dsep_sweep_setup): T's rows as a factor of their own, solved by the block sweep
    // kernels over the combined vector rbuf = [payload (P * kt); T in T's schedule order] -- the
    // separator solve of a T too large for one workgroup (no row or step limit)
    bool tsweep = false;
    int64_t tsw_base = 0;  // P * kt: where T's rows start in rbuf
    DFactor tsw;
    DBuf<int32_t> tsw_q;   // T row t -> its schedule position (rbuf[tsw_base + tsw_q[t]])
};
struct RankPlan;
// Split the forward rows of T and build the steps of the separator level solve.
void dsep_stage(DSep &T, const RankPlan &rp);
// Build the T sweep: T's rows scheduled into blocks and rounds (build_schedule) and laid out as
// a DFactor over the combined vector [payload (P * kt); T]; forced by the engine option
// tsolve_sweep, else used when the stepped solve does not fit one workgroup.
void dsep_sweep_setup(Ctx &c, DSep &T, const RankPlan &rp, int P);
// the stepped separator solve can hold T on this device (kernels.hip; the same predicate at
// setup and at launch)
bool sep_steps_fit(const DSep &S);
struct DofMap;

struct Precond {
    Ctx *ctx = nullptr;
    int64_t n = 0, m = 0, N = 0;   // local sizes (= global ones on one GPU)
    int64_t gn = 0, gm = 0, gN = 0;  // global sizes
    bool dist = false;
    int64_t nsub = 0;              // distributed: subtree rows of this rank (w holds nsub + nT)
    DSep sep;
    std::shared_ptr<DofMap> dofmap;
    HCsr Kp;             // host copy (divide, export)
    Factor F;            // exported factor (pivot order, pre-relabel); the device copy sums in its order
    Schedule S;
    int ordering = 0;
    DMat dKp;
    DFactor dF;
    DBuf<double> w, r;   // permuted work vector, refinement residual
    DLdl dl;             // device numeric factorization (single GPU); dl.ready: F.Lx / F.D live on the device
    // single GPU, forced refinement: Kp permuted into schedule order (P'*Kp*P, each row's
    // entries in Kp's order) so the refinement residual, the forward sweep's input and the
    // accumulated solution all stay in schedule order (apply); kps_from: Kps entry -> Kp entry
    DMat dKps;
    DBuf<int32_t> kps_from;
    bool fused_resid = false;  // the refinement residual fused into the forward sweep (launch_sptrsv_fwd_resid)
    DBuf<double> xs;     // the apply's signed input in schedule order (captured by the first forward sweep)
    uint64_t pattern_hash = 0;  // sparsity of (A11, B, C22): a refactorization must keep it
    DBuf<int> active;    // refinement predicate
    // public properties of opLDL2 (opLDL2.m:45-50)
    double nitref = 3, itref_tol = 1.0e-8, force_itref = 0, residual_update = 0;
    // opt-in handle semantics of the residual-update state (opLDL2.m:164-172 as reg_cpkrylov.m:
    // 47-52 intends): ghn = [op.Aty; op.Cy] persists between applies.  Off by default: Spot
    // operators are value objects, so in the reference the state never survives a multiply.
    bool handle = false;
    DBuf<double> ghn, t;
    double ptime = 0;
    // distributed preconditioner with the device factorization: every rank factors the whole
    // system on its own GPU (dl, global Kp values kpg) and gathers its share of the values --
    // local sweeps, separator solve, Kp rows -- through value maps built at construction
    DBuf<double> kpg;
    struct VMap {
        double *dst = nullptr;
        size_t n = 0;
        int src = 0;  // 0: L (CSC order), 1: D (pivot order), 2: Kp entries
        DBuf<int32_t> map;
    };
    std::vector<VMap> vmaps;
    void fill_vmaps();  // every mapped array from dl.Lx, dl.D, kpg
    // cached solvers (workspace + captured iteration graphs), keyed; see solvers.hip
    std::vector<std::pair<std::string, std::shared_ptr<void>>> solvers;
    // distributed rows of the Krylov operator and the shift products, which follow this
    // preconditioner's dof map (capi.cpp): keyed by (kind, matrix generation(s)); they die with it
    std::map<std::tuple<char, uint64_t, uint64_t>, std::unique_ptr<DMat>> dist_ops;
    // y = M*x  (opLDL2.multiply); all pointers on the device, enqueued on ctx->stream
    // piggy_src (distributed only, piggyback_ok()): kSepPiggy device values appended to the first
    // separator exchange's payload, e.g. a solver's deferred inner-product partials; after the
    // apply every rank finds rank r's values at sep.rbuf[r * sep.kt + sep.kt_data + j]
    void apply(const double *x, int64_t neg_from, double *y, const int *run, const double *piggy_src = nullptr);
    bool piggyback_ok() const { return dist && sep.kt > 0; }
    // the schedule-order refinement path (single GPU; CPK_NO_SCHED_RESID=1 forces the plain one)
    bool sched_path() const { return !dist && dKps.nnz > 0 && !no_sched; }
    bool no_sched = false;
    void set_handle(bool on);  // enabling or disabling clears the state
    // returns whether the backward sweep packed y's Kp halo (distributed: the residual's gather)
    // stage (tkr): 1 the apply's first solve (the backward sweep packs hslot2 into the separator
    // payload), 2 the refinement solve (its forward packs the T inputs from xT, the T rows'
    // residual is formed after the exchange); 0 neither
    bool ldl_solve(const double *xin, int64_t neg_from, double *y, bool add, const int *run, const int *act,
                   const double *piggy_src = nullptr, int stage = 0, const double *xT = nullptr, int64_t xT_neg = 0);
    DBuf<int32_t> hslot;  // distributed: local output index -> Kp halo slot (-1: none); empty: no packing
    // distributed, one forced refinement step: the residual without the Kp halo exchange
    // (DESIGN.md section 7).  Kp couples a subtree row only with its own subtree and with T, and
    // every rank holds T's solution (wT), so the local rows need no halo (dKpl: T-dof columns
    // read wT at nloc + t; rank 0's T rows left empty); the T rows' residual is formed by every
    // rank after the refinement's separator exchange, whose payload also carries the y values of
    // the subtree rows those rows read (hslot2: local index -> extra payload slot; tkr_*: the T
    // dofs' Kp rows, col >= 0 payload position, < 0 -(t + 1)), into the exchange's T-input slots
    DMat dKpl;
    DBuf<int32_t> hslot2, tkr_ptr, tkr_col;
    DBuf<double> tkr_val;
    bool tkr = false;
    // distributed, one forced refinement step, in schedule order: the first
    // solve keeps its solution in schedule order (w, T values in w[nsub..]); the residual of the
    // rank's subtree rows runs on Kp's local rows permuted into schedule order (dKpsl: columns are
    // schedule positions, T columns nsub + t, so both read w), fused into the refinement solve's
    // forward sweep; hslot2s: hslot2 keyed by schedule position; xs (nsub) the signed input
    DMat dKpsl;
    DBuf<int32_t> hslot2s;
    bool dsched = false;
    void dist_sched_apply(const double *x, int64_t neg_from, double *y, const int *run, const double *piggy_src);
    PackArgs fwd_pack(const double *xt, int64_t xt_neg, const double *piggy_src) const;
    bool steps1_forced() const { return nitref == 1 && force_itref != 0 && !(residual_update != 0 && handle); }
    // algorithmic HBM bytes of one apply
    double apply_bytes() const;
};
Precond *precond_create(Ctx &c, const HCsr &A11, const HCsr &B, const HCsr &C22);
// new values of A11, B, C22 (device CSR copies) with the sparsity the preconditioner was built
// with: Kp and the numeric factorization on the device, symbolic analysis reused; returns seconds
double precond_refactor(Precond &p, const DMat &A11, const DMat &B, const DMat &C22);
uint64_t pattern_hash(const HCsr &A11, const HCsr &B, const HCsr &C22);
// device data uploaded ahead of precond_create (during the analysis, SymbolicHook)
struct PrecondPre {
    DLdl dl;   // dldl_setup_sym done when dl.sym_ready
    DMat dKp;  // Kp uploaded when kp
    bool kp = false;
};
Precond *precond_create(Ctx &c, Analysis &&an, PrecondPre *pre = nullptr);
// distributed preconditioner of rank c.rank out of c.nranks
// Akry (optional): the Krylov operator's A, a placement hint for isolated rows (split_tree)
Precond *precond_create_dist(Ctx &c, Analysis &&an, const HCsr *Akry = nullptr);
// the same from the blocks: analysis (structure only unless host_factor), device factorization
// of the whole system on every rank, refactorization support
Precond *precond_create_dist(Ctx &c, const HCsr &A11, const HCsr &B, const HCsr &C22, const HCsr *Akry);

}  // namespace cpk
