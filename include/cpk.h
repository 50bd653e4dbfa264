/*
 * cpk.h -- C ABI of libcpk, the MI355X-native constraint-preconditioned Krylov engine.
 *
 * Drop-in boundary for optimizers/cpkrylov (MATLAB).  Each entry point names the reference
 * interface it replaces; INTEGRATION.md shows the MEX gateway / opSpot subclass / ctypes
 * binding a maintainer adds on the reference side.
 *
 * Conventions
 *   - Every function returns an int status (cpk_status).  On failure cpk_last_error()
 *     returns a message (thread-local, valid until the next call on that thread).
 *     No C++ exception crosses this boundary.
 *   - Input arrays are borrowed read-only for the duration of the call; the library
 *     copies what it keeps (to host memory and HBM).  Output arrays are caller-allocated.
 *   - Handles are owned by the library and freed by the matching *_destroy.
 *   - One host thread per context; a handle is not re-entrant.
 *   - All arithmetic is IEEE fp64.  Vectors are laid out [x-part (n); y-part (m)], as the
 *     reference's [x1; x2] (reg_cpkrylov.m:166-173).
 */
#ifndef CPK_H
#define CPK_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CPK_ABI_VERSION 3

typedef enum {
    CPK_OK = 0,
    CPK_ERR_INDEFINITE = 1, /* beta < -100*eps, or a negative squared norm (cpminres.m:195-199 etc.) */
    CPK_ERR_DIM = 2,        /* dimension mismatch (opLDL2.m:61-75) */
    CPK_ERR_ARGS = 3,       /* bad argument (reg_cpkrylov.m:122-125 "not enough inputs") */
    CPK_ERR_HIP = 4,        /* HIP runtime failure */
    CPK_ERR_RCCL = 5,       /* RCCL failure */
    CPK_ERR_FACTOR = 6,     /* zero pivot in the static-pivot LDL' (ldl at opLDL2.m:82) */
    CPK_ERR_NOMEM = 7,
    CPK_ERR_UNSUPPORTED = 8
} cpk_status;

/* Method ids: the function handles @cpcg, @cpcglanczos, @cpminres, @cpsymmlq, @cpgmres,
 * @cpdqgmres passed to reg_cpkrylov (reg_cpkrylov.m:67-68, :163). */
typedef enum {
    CPK_CG = 0,
    CPK_CGLANCZOS = 1,
    CPK_MINRES = 2,
    CPK_SYMMLQ = 3,
    CPK_GMRES = 4,
    CPK_DQGMRES = 5
} cpk_method;

/* The MATLAB `opts` struct.  A field takes effect only when its has_* flag is set
 * (MATLAB isfield(), e.g. cpminres.m:98-111); otherwise each solver's own default applies.
 * nitref/itref_tol/force_itref/residual_update are the fields reg_cpkrylov copies into M
 * (reg_cpkrylov.m:135-148), with opLDL2's setter semantics (opLDL2.m:97-115). */
typedef struct {
    double atol, rtol, btol;
    double itmax, restart, mem;
    double print;
    double nitref, itref_tol, force_itref, residual_update;
    int has_atol, has_rtol, has_btol, has_itmax, has_restart, has_mem, has_print;
    int has_nitref, has_itref_tol, has_force_itref, has_residual_update;
} cpk_opts;

/* stats / flag outputs (cpminres.m:250-252, cpsymmlq.m:363-367, cpcglanczos.m:311-325,
 * reg_cpkrylov.m:177-178).  History buffers are caller-allocated with capacity hist_cap
 * (itmax + 2 suffices for every method); a NULL buffer is skipped. */
typedef struct {
    int64_t niters;
    int solved;          /* flag.solved */
    int status;          /* cpcglanczos stats.status: 0 max iters, 1 residual small, 2 backward error small */
    double *hist;        /* residHistory (cpsymmlq: cgresidHistory) */
    double *hist_lq;     /* cpsymmlq lqresidHistory */
    double *hist_qr;     /* cpsymmlq qrresidHistory */
    int64_t hist_cap;
    int64_t hist_len, lq_len, qr_len;
    double ptime;        /* s, preconditioner setup (reg_cpkrylov.m:128-132) */
    double stime;        /* s, shift + method + recovery (reg_cpkrylov.m:150-175) */
    double loop_ms;      /* device time of the method call (HIP events on the solver stream) */
    double bytes_moved;  /* algorithmic HBM bytes of the method call (DESIGN.md section 5 model) */
} cpk_stats;

/* Factor summary of a preconditioner. */
typedef struct {
    int64_t n, m, N;
    int64_t nnz_kp;      /* nnz(Kp) */
    int64_t nnz_l;       /* nnz of the strict lower factor */
    int64_t nblocks;     /* SpTRSV work blocks */
    int64_t nrounds;     /* kernel launches per triangular sweep */
    int64_t max_block_levels;
    int64_t depth;       /* elimination-tree height */
    int64_t ordering;    /* 0 natural, 1 G-first + nested dissection, 2 G-first + minimum degree,
                            3 nested dissection, 4 minimum degree */
} cpk_pc_info;

typedef struct cpk_ctx_s *cpk_ctx;
typedef struct cpk_mat_s *cpk_mat;
typedef struct cpk_pc_s *cpk_pc;

const char *cpk_last_error(void);
int cpk_abi_version(void);

/* ---- context: device, streams, RCCL communicator ------------------------------------- */
/* Fill `id` (128 bytes) with an RCCL unique id on rank 0; broadcast it to the other ranks. */
int cpk_get_unique_id(unsigned char id[128]);
/* device < 0: use the current device.  nranks == 1 and unique_id == NULL: no communicator.
 * nranks > 1 requires a unique_id and runs the distributed path over RCCL.  A 1-rank RCCL
 * communicator (a torchrun world of one) has nothing to exchange: it runs the single-GPU path
 * unless engine option dist1 is set before the operators are built. */
int cpk_ctx_create(int device, int rank, int nranks, const unsigned char *unique_id, cpk_ctx *out);
/* Diagnostic timing stand-in (no reference counterpart): rank `rank` of an nranks-way
 * distributed context WITHOUT peers.  Every collective is a no-op (an allgather copies the
 * rank's own slot), so results are meaningless, but each kernel is exactly that rank's share of
 * the P-way solve: tools/dist_timing.py times one rank's work on one GPU with it.  Never used by
 * cpk_ctx_create; nranks must be > 1. */
int cpk_ctx_create_null(int device, int rank, int nranks, cpk_ctx *out);
/* Communicator kinds reported by cpk_ctx_get_info. */
enum { CPK_COMM_NONE = 0, CPK_COMM_RCCL = 1, CPK_COMM_SIM = 2, CPK_COMM_NULL = 3 };
/* info[8] = {device, rank, nranks, communicator kind (CPK_COMM_*), ranks the communicator holds
 * (RCCL: ncclCommCount; SimComm: the group's ranks; the timing stand-in: 1; none: 0),
 * distributed path (0/1), 0, 0}. */
int cpk_ctx_get_info(cpk_ctx ctx, int64_t *info);
/* Single-GPU rehearsal of the distributed path: `nranks` ranks as host threads of one process,
 * all on one device, exchanging through a shared HBM buffer instead of RCCL (RCCL refuses two
 * ranks on one GPU).  Each thread creates its context with cpk_ctx_create_sim and then makes
 * the same collective calls as an RCCL rank.  For tests; no hipGraph capture. */
typedef struct cpk_simgroup_s *cpk_simgroup;
int cpk_simgroup_create(int nranks, cpk_simgroup *out);
int cpk_simgroup_destroy(cpk_simgroup g);
int cpk_ctx_create_sim(int device, cpk_simgroup group, int rank, int nranks, cpk_ctx *out);
/* Engine options of a context (no reference counterpart: they choose among execution paths
 * that give identical results, and the sweep schedule / distributed split that every rank
 * must build identically).  A context starts from the CPK_<NAME> environment variables, read
 * once at creation; a change applies to preconditioners and solves created afterwards.
 * Names: sweep ("rows,cap,threads[,rows,cap,threads[,sub0]]"; unset, each path has its own
 * default: a distributed context reports and uses the distributed one), split_tol, host_factor,
 * no_pipe, no_upper, no_col16, no_dataflow, all_dataflow, no_colsweep, all_colsweep, no_chain, chain_wide
 * (rounds of at most this many blocks join the sweep chain, default 256), exact_dots, no_bcast_analysis
 * (every rank of a distributed preconditioner runs the global analysis instead of receiving rank 0's),
 * no_sched_resid, no_fused_resid, r0_xcd_chunk, tsolve_global, tsolve_sweep,
 * no_piggy, no_halo_merge, no_graph, no_fuse_last, no_tkr, no_minres_fuse, dist_graph, batch,
 * dist1 (a 1-rank communicator runs the distributed kernels; set before building operators),
 * profile_fwd_sched (diagnostic), sweep_set ("0" returns sweep to the per-path default),
 * profile_passes (diagnostic: cpdqgmres runs eagerly with events between its passes, read by
 * cpk_debug_pass_times), fail_inject ("rank:site[:n]", site setup / batch / chain: a test hook
 * that makes one rank of a distributed solve fail at that point).
 * Booleans as "0"/"1".  A distributed preconditioner allgathers a hash of its plan and of every
 * option but fail_inject at creation and fails (CPK_ERR_ARGS) on every rank unless all ranks
 * agree. */
int cpk_ctx_set_option(cpk_ctx ctx, const char *name, const char *value);
int cpk_ctx_get_option(cpk_ctx ctx, const char *name, char *buf, size_t cap);
/* Every engine option of the context as "name=value;name=value;..." (the form cpk_analyze's
 * `options` takes), with the sweep this context's path uses. */
int cpk_ctx_get_options(cpk_ctx ctx, char *buf, size_t cap);
int cpk_ctx_destroy(cpk_ctx ctx);
int cpk_ctx_synchronize(cpk_ctx ctx);

/* ---- sparse matrices (MATLAB sparse arrays A, B, C, G; reg_cpkrylov.m:1) -------------- */
/* MATLAB-native CSC: jc[ncols+1], ir[nnz] (0-based, mwIndex = size_t), pr[nnz].
 * ctx may be NULL for a host-only matrix (cpk_analyze); such a matrix cannot be used on a device. */
int cpk_mat_create_csc(cpk_ctx ctx, int64_t nrows, int64_t ncols, const size_t *jc, const size_t *ir,
                       const double *pr, cpk_mat *out);
/* CSR with 64-bit row pointers and 32-bit column indices. */
int cpk_mat_create_csr(cpk_ctx ctx, int64_t nrows, int64_t ncols, const int64_t *rowptr,
                       const int32_t *colind, const double *val, cpk_mat *out);
int cpk_mat_destroy(cpk_mat A);
/* y = A*x on the device (host vectors in/out); replaces MATLAB sparse mtimes A*v. */
int cpk_mat_spmv(cpk_mat A, const double *x, double *y);

/* ---- preconditioner: M = opLDL2(A, B, C), Kp = [A B'; B C] (ops/opLDL2.m:60-92) ------
 * Distributed contexts (nranks > 1): every rank passes the same global matrices; the library
 * partitions rows by the elimination tree.  Host-vector entry points
 * then take and return GLOBAL vectors on every rank; device-vector entry points take the
 * rank's LOCAL slice in the order cpk_pc_local_dofs reports ([x-part; y-part]). */
int cpk_pc_create(cpk_ctx ctx, cpk_mat A11, cpk_mat B, cpk_mat C22, double *ptime, cpk_pc *out);
/* cpk_pc_create with the Krylov operator's A (n x n) as a placement hint for a distributed
 * context: rows the factor leaves isolated are owned with the dofs A couples them with, so the
 * Krylov SpMV's halo stays small.  reg_cpkrylov (cpk_reg_solve) passes its A itself.  On one
 * GPU identical to cpk_pc_create; Akry may be NULL. */
int cpk_pc_create_hint(cpk_ctx ctx, cpk_mat A11, cpk_mat B, cpk_mat C22, cpk_mat Akry, double *ptime,
                       cpk_pc *out);
int cpk_pc_destroy(cpk_pc M);
/* Refactorization with new values and the same sparsity: opLDL2(G, B, C) rebuilt in an
 * interior-point outer loop (the constructor, opLDL2.m:60-92, called per outer iteration
 * through reg_cpkrylov.m:131).  Kp and the numeric LDL' (opLDL2.m:81-82) are recomputed on
 * the device from the matrices' device copies; ordering, elimination tree and sweep schedule
 * are reused.  The factors equal those of a fresh cpk_pc_create on the same values, bit for
 * bit.  Single GPU; CPK_ERR_ARGS when the sparsity differs, CPK_ERR_FACTOR on a zero pivot.
 * ptime: seconds of the refactorization. */
int cpk_pc_refactor(cpk_pc M, cpk_mat A11, cpk_mat B, cpk_mat C22, double *ptime);
/* M.nitref = ...; M.itref_tol = ...; etc. (opLDL2.m:45-50, 97-115), has_* fields select. */
int cpk_pc_set(cpk_pc M, const cpk_opts *opts);
int cpk_pc_get(cpk_pc M, double *nitref, double *itref_tol, double *force_itref, double *residual_update);
/* Opt-in (not in the reference): handle semantics of the residual-update state.  In the
 * reference, opLDL2 is a Spot value object, so the op.Aty / op.Cy written inside multiply
 * (opLDL2.m:169-171) are lost and residual_update is a functional no-op; cpk_pc_apply matches
 * that by default.  on != 0 keeps [op.Aty; op.Cy] on the device between applies, as the
 * residual update of reg_cpkrylov.m:47-52 (Gould-Hribar-Nocedal) intends; it takes effect while
 * residual_update is set.  Enabling or disabling clears the state.  Single-GPU contexts only
 * (CPK_ERR_UNSUPPORTED on a distributed preconditioner). */
int cpk_pc_set_handle(cpk_pc M, int on);
/* y = M*x (opLDL2.multiply, opLDL2.m:161-188).  Host vectors of length N. */
int cpk_pc_apply(cpk_pc M, const double *x, double *y);
/* Same on device pointers, enqueued on the context stream. */
int cpk_pc_apply_device(cpk_pc M, const double *d_x, double *d_y);
/* x = Kp*b (opLDL2.divide, opLDL2.m:193-195). */
int cpk_pc_divide(cpk_pc M, const double *b, double *x);
int cpk_pc_get_info(cpk_pc M, cpk_pc_info *info);
/* Local slice of a (distributed) preconditioner: n_loc x-part and m_loc y-part dofs; dofs[i] =
 * global index of local entry i (n_loc + m_loc entries).  One GPU: the identity. */
/* Diagnostic (not in the reference): the separator solve of a distributed preconditioner,
 * info[12] = {distributed, separator rows, levels, step records, LDS bytes with the records
 * staged (0: they do not fit), LDS bytes with the records left in HBM, payload per rank,
 * refinement residual without the Kp halo exchange, refinement in schedule order, its residual
 * fused into the forward sweep, separator solved by the block sweeps (T sweep), the T sweep's
 * rounds}. */
int cpk_pc_sep_info(cpk_pc M, int64_t *info);
/* Diagnostic (not in the reference): the sweep schedule as launched, info[8] = {rounds, round-0
 * blocks, blocks above round 0, grid of the cost-balanced round-0 assignment of the forward /
 * fused-residual forward / backward kernel (0: the launch strides), round 0 persistent, tasks of
 * the sweep chain (every upper round of a solve in one launch; 0: one launch per round)}. */
int cpk_pc_sweep_info(cpk_pc M, int64_t *info);
int cpk_pc_local_dofs(cpk_pc M, int64_t *n_loc, int64_t *m_loc, int32_t *dofs);
/* Export the factors P'*Kp*P = L*D*L': strict-lower L in CSC (Lcolptr[N+1], Lrowind[nnz_l],
 * Lval[nnz_l]), D[N], perm[N] (perm[k] = original index of pivot k).  Any pointer may be NULL. */
int cpk_pc_export(cpk_pc M, int64_t *Lcolptr, int32_t *Lrowind, double *Lval, double *D, int32_t *perm);

/* ---- host-only analysis (no GPU needed) ------------------------------------------------- */
/* The host half of cpk_pc_create: Kp assembly, fill-reducing ordering, static-pivot LDL' and
 * the triangular-sweep schedule.  Matrices for this call may be created with ctx == NULL.
 * Engine options: the CPK_<NAME> environment (as a new context starts), then `options`
 * ("name=value;...", NULL: none) on top -- pass cpk_ctx_get_options of a context to analyse
 * and plan exactly as that context's preconditioner would (sweep, split_tol). */
typedef struct cpk_analysis_s *cpk_analysis;
int cpk_analyze(cpk_mat A11, cpk_mat B, cpk_mat C22, const char *options, cpk_analysis *out);
int cpk_analysis_destroy(cpk_analysis an);
int cpk_analysis_get_info(cpk_analysis an, cpk_pc_info *info);
int cpk_analysis_export(cpk_analysis an, int64_t *Lcolptr, int32_t *Lrowind, double *Lval, double *D,
                        int32_t *perm);
/* Sweep schedule: round_ptr[nrounds+1] (blocks per round), blk_lvl[nblocks+1] (levels per
 * block, indices into lvl_row), lvl_row[nlevels+1] (first position of each level; last = N),
 * order[N] (order[q] = exported-factor row solved at schedule position q).  Each row sums its
 * entries in the exported factor's order: forward by ascending column, backward by
 * descending row -- the order of the reference's column-oriented solves. */
int cpk_analysis_schedule(cpk_analysis an, int64_t *nlevels, int64_t *round_ptr, int64_t *blk_lvl,
                          int64_t *lvl_row, int32_t *order);

/* ---- distributed plan (host-only) --------------------------------- */
/* The row-block plan of rank `rank` out of `nranks` for the system the analysis was built on
 * (A: n x n, C: m x m the Krylov operator's blocks), with the analysis' engine options
 * (split_tol).  Every rank computes the same global plan deterministically; a distributed
 * cpk_pc_create on a context with the same options builds exactly this.  Exposed for tests and
 * inspection: cpk_plan_array(plan, name, &count, out) copies array `name` (values as double
 * for *_val, fsub_Lx, fsub_D, extra_val, tf_val, tb_val, DT; every other array as int64) into
 * out (NULL: count only).  Names: sizes [P, rank, n, m, N, n_loc, m_loc, N_loc, nsub, nT, kt,
 * kp_kmax, ac_kmax, ab_kmax], dofs, node_rank, T, fsub_{Lp,Li,Lx,D,perm,parent,key},
 * extra_{ptr,col,key,val}, tf_{ptr,col,val,src}, tb_{ptr,col,val}, DT, tlev_{ptr,rows},
 * tsend, tdof, and {kp,ac,ab}_{ptr,col,val,send} for Kp, blkdiag(A,C) and [A B']. */
typedef struct cpk_plan_s *cpk_plan;
int cpk_analysis_plan(cpk_analysis an, cpk_mat A, cpk_mat C, int nranks, int rank, cpk_plan *out);
int cpk_plan_array(cpk_plan plan, const char *name, int64_t *count, void *out);
int cpk_plan_destroy(cpk_plan plan);

/* ---- solvers --------------------------------------------------------------------------- */
/* [x, y, stats, flag] = method(b, A, C, M, opts)   (kernels/cp*.m, e.g. cpminres.m:1).
 * b: n, x: n, y: m (host). */
int cpk_method_solve(cpk_ctx ctx, int method, const double *b, cpk_mat A, cpk_mat C, cpk_pc M,
                     const cpk_opts *opts, double *x, double *y, cpk_stats *stats);
/* Same with device-resident b (n) and xy (N = [x; y]); nothing crosses PCIe except the
 * stop flag polled between iteration batches and the history copied back at the end. */
int cpk_method_solve_device(cpk_ctx ctx, int method, const double *d_b, cpk_mat A, cpk_mat C, cpk_pc M,
                            const cpk_opts *opts, double *d_xy, cpk_stats *stats);
/* [x, stats, flag] = reg_cpkrylov(method, b, A, B, C, G, opts)  (reg_cpkrylov.m:1-180).
 * b: N, x: N (host).  If M_out != NULL the preconditioner built here is returned. */
int cpk_reg_solve(cpk_ctx ctx, int method, const double *b, cpk_mat A, cpk_mat B, cpk_mat C, cpk_mat G,
                  const cpk_opts *opts, double *x, cpk_stats *stats, cpk_pc *M_out);
/* reg_cpkrylov's shift + method + recovery with an existing M, device-resident b and x (N). */
int cpk_reg_solve_device(cpk_ctx ctx, int method, const double *d_b, cpk_mat A, cpk_mat B, cpk_mat C,
                         cpk_pc M, const cpk_opts *opts, double *d_x, cpk_stats *stats);

/* The driver's shift step alone (reg_cpkrylov.m:152-160): if any(b(n+1:N)), xy0 = M*[0; b2]
 * and b1 = b(1:n) - A*xy0(1:n) - B'*xy0(n+1:N); else b1 = b(1:n), xy0 = 0.  Device pointers:
 * d_b (N), d_b1 (n), d_xy0 (N).  *shifted reports whether the shift was taken. */
int cpk_reg_shift_device(cpk_ctx ctx, const double *d_b, cpk_mat A, cpk_mat B, cpk_mat C, cpk_pc M,
                         double *d_b1, double *d_xy0, int *shifted);

/* ---- measurement ----------------------------------------------------------------------- */
/* Average device time (HIP events on the context stream, `reps` back-to-back launches) and
 * algorithmic HBM bytes per launch of each kernel class of an
 * iteration.  Times in ms. */
typedef struct {
    double spmv_ms, spmv_bytes;      /* Krylov operator blkdiag(A, C) SpMV (u = A*v, t = C*q) */
    double resid_ms, resid_bytes;    /* saddle-point SpMV r = x - Kp*y (refinement residual) */
    double fwd_ms, fwd_bytes;        /* forward sweep w = L \ P'x (all rounds) */
    double bwd_ms, bwd_bytes;        /* backward sweep y = P (L' \ (D \ w)) (all rounds) */
    double apply_ms, apply_bytes;    /* one M*z with the current properties */
    int64_t fwd_launches, bwd_launches;
    double fwd_resid_ms, fwd_resid_bytes;  /* refinement input fused into the forward sweep: r = x - Kp*y,
                                              then w = L \ P'r (0 when the apply does not fuse it) */
    double bwd_dead_store_bytes;     /* (ABI 3) bytes of the work-vector store the profiled backward
                                        sweep skips (round 0's w, dead after the sweep): not in
                                        bwd_bytes; the r03 byte model counted them */
} cpk_profile;
int cpk_profile_kernels(cpk_ctx ctx, cpk_mat A, cpk_mat C, cpk_pc M, int reps, cpk_profile *out);

/* Diagnostic (no reference counterpart): per-workgroup (start, end) s_memrealtime stamps of the
 * last round-0 sweep launch, 100 MHz ticks; *copied = 0 unless the library was built with
 * -DCPK_PIPE_STAMPS (tools/pipe_stamps.py). */
int cpk_debug_pipe_stamps(uint64_t *out, int npairs, int *copied);
/* Diagnostic: per-block s_memtime cycles of the last round-0 launch of each kernel variant,
 * out[v * 131072 + block] for v = forward, forward with the fused refinement residual, backward,
 * backward accumulating; *copied = 0 unless built with -DCPK_PIPE_STAMPS (tools/blk_cycles.py). */
int cpk_debug_blk_cycles(uint64_t *out, int64_t n, int64_t *copied);
/* Diagnostic: the upper-round loop-cost model of a preconditioner's sweeps, 8 int64 per (upper
 * block, direction): block, direction (0 forward), rows, level-loop trips, dataflow trips (-1:
 * not modelled), outside terms behind in-block ones, column sweep valid, loop chosen (0 level,
 * 1 dataflow, 2 column sweep).  out = NULL: *copied = the total count. */
int cpk_debug_block_model(cpk_pc M, int64_t *out, int64_t n, int64_t *copied);
/* Diagnostic: the last cpdqgmres solve of this context run with engine option profile_passes
 * (eager batches, HIP events between its passes): out[8] = {iterations, Krylov SpMV ms, M*z ms,
 * window dots ms, orthogonalisation ms, direction ms, sum over the iterations of the dots'
 * window size, the same for the direction pass} (bench.py's s50 block: per-pass GB/s). */
int cpk_debug_pass_times(cpk_ctx ctx, double *out);

/* [c, s, d] = SymGivens(a, b)  (util/SymGivens.m:1-29) */
int cpk_symgivens(double a, double b, double *c, double *s, double *d);

#ifdef __cplusplus
}
#endif
#endif
