// capi.cpp -- the extern "C" boundary of libcpk (include/cpk.h).  Every entry point converts
// C++ exceptions into a cpk_status code plus a thread-local message.
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <new>
#include <string>

#include "cpk.h"
#include "dev.hpp"
#include "dist.hpp"
#include "solvers.hpp"

using namespace cpk;

struct cpk_ctx_s {
    Ctx c;
    std::unique_ptr<Comm> comm;
};

struct cpk_simgroup_s {
    SimGroup *g = nullptr;
    ~cpk_simgroup_s() {
        if (g) simgroup_destroy(g);
    }
};

struct cpk_mat_s {
    cpk_ctx_s *ctx = nullptr;
    uint64_t gen = 0;
    HCsr h;
    std::unique_ptr<DMat> d;                          // lazily uploaded
    std::map<uint64_t, std::unique_ptr<DMat>> ac;     // blkdiag(this, C) keyed by C's generation
    const DMat &dev() {
        if (!ctx) throw Error(CPK_ERR_ARGS, "host-only matrix (created with ctx == NULL) used on the device");
        if (!d) {
            d = std::make_unique<DMat>();
            make_dmat(h, *d);
        }
        return *d;
    }
    // distributed rows follow the preconditioner's dof map, so they are
    // cached in the Precond itself (Precond::dist_ops), keyed by the matrices' generations: they
    // die with the preconditioner, and a new preconditioner never sees an old one's rows
    const DMat &krylov_op(cpk_mat_s *C, Precond &M) {
        if (M.dist != ctx->c.dist())
            throw Error(CPK_ERR_ARGS, "engine option dist1 changed after the preconditioner was built");
        if (!M.dist) return blkdiag_with(C);
        auto &slot = M.dist_ops[{'K', gen, C->gen}];
        if (!slot) {
            auto m = std::make_unique<DMat>();
            make_dist_dmat(dist_csr(blkdiag(h, C->h), *M.dofmap, ctx->c.rank, false, kKrylovSpare), ctx->c.nranks,
                           *m);
            slot = std::move(m);
        }
        return *slot;
    }
    // shift rows of a distributed preconditioner: A*xy0(1:n) and B'*xy0(n+1:N), x-part rows
    std::pair<const DMat *, const DMat *> shift_ops(Precond &M) {
        auto &sa = M.dist_ops[{'A', gen, 0}];
        auto &sb = M.dist_ops[{'B', gen, 0}];
        if (!sa || !sb) {
            const int64_t n = M.gn, N = M.gN;
            HCsr a = h, bt;
            a.ncols = N;
            bt.nrows = n, bt.ncols = N;
            bt.ptr.assign(n + 1, 0);
            for (int64_t i = 0; i < n; i++) {
                for (int64_t q = M.Kp.ptr[i]; q < M.Kp.ptr[i + 1]; q++)
                    if (M.Kp.ind[q] >= n) bt.ind.push_back(M.Kp.ind[q]), bt.val.push_back(M.Kp.val[q]);
                bt.ptr[i + 1] = (int64_t)bt.ind.size();
            }
            auto ma = std::make_unique<DMat>(), mb = std::make_unique<DMat>();
            make_dist_dmat(dist_csr(a, *M.dofmap, ctx->c.rank, true), ctx->c.nranks, *ma);
            make_dist_dmat(dist_csr(bt, *M.dofmap, ctx->c.rank, true), ctx->c.nranks, *mb);
            sa = std::move(ma), sb = std::move(mb);
        }
        return {sa.get(), sb.get()};
    }
    const DMat &blkdiag_with(cpk_mat_s *C) {
        if (!ctx) throw Error(CPK_ERR_ARGS, "host-only matrix (created with ctx == NULL) used on the device");
        auto it = ac.find(C->gen);
        if (it == ac.end()) {
            auto m = std::make_unique<DMat>();
            make_dmat(blkdiag(h, C->h), *m);
            it = ac.emplace(C->gen, std::move(m)).first;
        }
        return *it->second;
    }
};

struct cpk_analysis_s {
    Analysis an;
    EngineOpts opts;  // the options it was built with (cpk_analysis_plan's split_tol)
};

struct cpk_plan_s {
    TreeSplit ts;
    DofMap dm;
    RankPlan rp;
    DistCsr kp, ac, ab;
    int64_t n = 0, m = 0;
};

struct cpk_pc_s {
    cpk_ctx_s *ctx = nullptr;
    std::unique_ptr<Precond> p;
};

static thread_local std::string g_err;
static std::atomic<uint64_t> g_gen{1};

#define API_BEGIN try {
#define API_END                                                  \
    }                                                            \
    catch (const Error &e) {                                     \
        g_err = e.what();                                        \
        return e.code;                                           \
    }                                                            \
    catch (const std::bad_alloc &) {                             \
        g_err = "out of host memory";                            \
        return CPK_ERR_NOMEM;                                    \
    }                                                            \
    catch (const std::exception &e) {                            \
        g_err = e.what();                                        \
        return CPK_ERR_ARGS;                                     \
    }                                                            \
    return CPK_OK;

static void need(bool cond, const char *msg) {
    if (!cond) throw Error(CPK_ERR_ARGS, msg);
}

template <class T>
static void h2d(DBuf<T> &d, const T *h, size_t n) {
    d.alloc(n);
    if (n) CPK_HIP(hipMemcpy(d.p, h, n * sizeof(T), hipMemcpyHostToDevice));
}

// ---- distributed host vectors: global on every rank <-> local slices on the device ----------
static void scatter_global(const Precond &p, const double *h_glob, int64_t len_local, DBuf<double> &d) {
    const std::vector<int32_t> dofs = p.dofmap->dofs(p.ctx->rank);
    std::vector<double> loc((size_t)len_local);
    for (int64_t i = 0; i < len_local; i++) loc[i] = h_glob[dofs[i]];
    d.alloc((size_t)std::max<int64_t>(len_local, 1));
    if (len_local) CPK_HIP(hipMemcpy(d.p, loc.data(), len_local * sizeof(double), hipMemcpyHostToDevice));
}

static void gather_global(Ctx &c, const Precond &p, const double *d_loc, double *h_glob) {
    const DofMap &dm = *p.dofmap;
    int64_t mx = 1;
    for (int r = 0; r < dm.P; r++) mx = std::max<int64_t>(mx, dm.n_loc[r] + dm.m_loc[r]);
    DBuf<double> snd, rcv;
    snd.alloc((size_t)mx), rcv.alloc((size_t)(mx * dm.P));
    CPK_HIP(hipMemsetAsync(snd.p, 0, snd.bytes(), c.stream));
    if (p.N) CPK_HIP(hipMemcpyAsync(snd.p, d_loc, p.N * sizeof(double), hipMemcpyDeviceToDevice, c.stream));
    c.comm->allgather(snd.p, rcv.p, (size_t)mx, c.stream);
    std::vector<double> h((size_t)(mx * dm.P));
    CPK_HIP(hipMemcpyAsync(h.data(), rcv.p, rcv.bytes(), hipMemcpyDeviceToHost, c.stream));
    CPK_HIP(hipStreamSynchronize(c.stream));
    for (int64_t g = 0; g < dm.N; g++) h_glob[g] = h[(size_t)dm.owner[g] * mx + dm.lidx[g]];
}

extern "C" {

const char *cpk_last_error(void) { return g_err.c_str(); }
int cpk_abi_version(void) { return CPK_ABI_VERSION; }

int cpk_get_unique_id(unsigned char id[128]) {
    API_BEGIN
    need(id != nullptr, "id is NULL");
    rccl_unique_id(id);
    API_END
}

static std::unique_ptr<cpk_ctx_s> ctx_base(int device, int rank, int nranks) {
    need(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank/nranks");
    auto ctx = std::make_unique<cpk_ctx_s>();
    Ctx &c = ctx->c;
    if (device >= 0) CPK_HIP(hipSetDevice(device));
    CPK_HIP(hipGetDevice(&c.device));
    c.rank = rank, c.nranks = nranks;
    c.opts = engine_opts_from_env();
    CPK_HIP(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
    CPK_HIP(hipEventCreate(&c.ev0));
    CPK_HIP(hipEventCreate(&c.ev1));
    c.ensure_partials(4096);
    c.red.alloc(4096);  // distributed reductions (up to 2047 Arnoldi window pairs)
    return ctx;
}

int cpk_ctx_create(int device, int rank, int nranks, const unsigned char *unique_id, cpk_ctx *out) {
    API_BEGIN
    need(out != nullptr, "out is NULL");
    need(nranks == 1 || unique_id != nullptr, "unique_id required when nranks > 1");
    auto ctx = ctx_base(device, rank, nranks);
    if (unique_id) {  // a 1-rank communicator: the single-GPU path unless engine option dist1
        ctx->comm.reset(make_rccl_comm(nranks, rank, unique_id));
        ctx->c.comm = ctx->comm.get();
    }
    *out = ctx.release();
    API_END
}

int cpk_ctx_create_null(int device, int rank, int nranks, cpk_ctx *out) {
    API_BEGIN
    need(out != nullptr, "out is NULL");
    need(nranks > 1, "the timing stand-in needs nranks > 1");
    auto ctx = ctx_base(device, rank, nranks);
    ctx->comm.reset(make_null_comm(rank, nranks));  // diagnostic (comm.cpp): collectives are no-ops
    ctx->c.comm = ctx->comm.get();
    *out = ctx.release();
    API_END
}

int cpk_ctx_get_info(cpk_ctx ctx, int64_t *info) {
    API_BEGIN
    need(ctx && info, "NULL argument");
    const Ctx &c = ctx->c;
    const int64_t v[8] = {c.device, c.rank, c.nranks, c.comm ? c.comm->kind() : CPK_COMM_NONE,
                          c.comm ? c.comm->count() : 0, c.dist() ? 1 : 0, 0, 0};
    std::memcpy(info, v, sizeof v);
    API_END
}

int cpk_ctx_get_options(cpk_ctx ctx, char *buf, size_t cap) {
    API_BEGIN
    need(ctx && buf && cap > 0, "NULL argument");
    const std::string v = engine_opts_string(ctx->c.opts, ctx->c.dist() && ctx->c.nranks > 1);
    need(v.size() < cap, "buffer too small");
    std::memcpy(buf, v.c_str(), v.size() + 1);
    API_END
}

int cpk_simgroup_create(int nranks, cpk_simgroup *out) {
    API_BEGIN
    need(out && nranks >= 1, "bad argument");
    auto g = std::make_unique<cpk_simgroup_s>();
    g->g = simgroup_create(nranks);
    *out = g.release();
    API_END
}

int cpk_simgroup_destroy(cpk_simgroup g) {
    API_BEGIN
    delete g;
    API_END
}

int cpk_ctx_create_sim(int device, cpk_simgroup group, int rank, int nranks, cpk_ctx *out) {
    API_BEGIN
    need(out && group, "NULL argument");
    auto ctx = ctx_base(device, rank, nranks);
    ctx->comm.reset(make_sim_comm(group->g, rank));
    ctx->c.comm = ctx->comm.get();
    *out = ctx.release();
    API_END
}

int cpk_ctx_destroy(cpk_ctx ctx) {
    API_BEGIN
    if (!ctx) return CPK_OK;
    Ctx &c = ctx->c;
    (void)hipStreamSynchronize(c.stream);
    c.comm = nullptr;
    ctx->comm.reset();
    c.partials.release();
    c.counter.release();
    c.red.release();
    (void)hipEventDestroy(c.ev0);
    (void)hipEventDestroy(c.ev1);
    (void)hipStreamDestroy(c.stream);
    delete ctx;
    API_END
}

int cpk_ctx_set_option(cpk_ctx ctx, const char *name, const char *value) {
    API_BEGIN
    need(ctx && name && value, "NULL argument");
    set_engine_option(ctx->c.opts, name, value);
    API_END
}

int cpk_ctx_get_option(cpk_ctx ctx, const char *name, char *buf, size_t cap) {
    API_BEGIN
    need(ctx && name && buf && cap > 0, "NULL argument");
    const std::string v = get_engine_option(ctx->c.opts, name, ctx->c.dist() && ctx->c.nranks > 1);
    need(v.size() < cap, "buffer too small");
    std::memcpy(buf, v.c_str(), v.size() + 1);
    API_END
}

int cpk_ctx_synchronize(cpk_ctx ctx) {
    API_BEGIN
    need(ctx, "ctx is NULL");
    CPK_HIP(hipStreamSynchronize(ctx->c.stream));
    API_END
}

int cpk_mat_create_csc(cpk_ctx ctx, int64_t nrows, int64_t ncols, const size_t *jc, const size_t *ir,
                       const double *pr, cpk_mat *out) {
    API_BEGIN
    need(out != nullptr, "NULL argument");
    auto m = std::make_unique<cpk_mat_s>();
    m->ctx = ctx;
    m->gen = g_gen++;
    m->h = csr_from_csc(nrows, ncols, jc, ir, pr);
    *out = m.release();
    API_END
}

int cpk_mat_create_csr(cpk_ctx ctx, int64_t nrows, int64_t ncols, const int64_t *rowptr, const int32_t *colind,
                       const double *val, cpk_mat *out) {
    API_BEGIN
    need(out != nullptr, "NULL argument");
    auto m = std::make_unique<cpk_mat_s>();
    m->ctx = ctx;
    m->gen = g_gen++;
    m->h = csr_from_csr(nrows, ncols, rowptr, colind, val);
    *out = m.release();
    API_END
}

int cpk_mat_destroy(cpk_mat A) {
    API_BEGIN
    delete A;
    API_END
}

int cpk_mat_spmv(cpk_mat A, const double *x, double *y) {
    API_BEGIN
    need(A && (x || !A->h.ncols) && (y || !A->h.nrows), "NULL argument");
    Ctx &c = A->ctx->c;
    const DMat &d = A->dev();
    DBuf<double> dx, dy;
    h2d(dx, x, (size_t)A->h.ncols);
    dy.alloc((size_t)A->h.nrows);
    launch_spmv(c, d, dx.p, dy.p, nullptr);
    if (A->h.nrows) CPK_HIP(hipMemcpyAsync(y, dy.p, A->h.nrows * sizeof(double), hipMemcpyDeviceToHost, c.stream));
    CPK_HIP(hipStreamSynchronize(c.stream));
    API_END
}

int cpk_pc_create(cpk_ctx ctx, cpk_mat A11, cpk_mat B, cpk_mat C22, double *ptime, cpk_pc *out) {
    API_BEGIN
    need(ctx && A11 && B && C22 && out, "opLDL2: Invalid number of arguments.");
    auto pc = std::make_unique<cpk_pc_s>();
    pc->ctx = ctx;
    if (ctx->c.dist()) pc->p.reset(precond_create_dist(ctx->c, A11->h, B->h, C22->h, nullptr));
    else pc->p.reset(precond_create(ctx->c, A11->h, B->h, C22->h));
    if (ptime) *ptime = pc->p->ptime;
    *out = pc.release();
    API_END
}

int cpk_pc_create_hint(cpk_ctx ctx, cpk_mat A11, cpk_mat B, cpk_mat C22, cpk_mat Akry, double *ptime,
                       cpk_pc *out) {
    API_BEGIN
    need(ctx && A11 && B && C22 && out, "opLDL2: Invalid number of arguments.");
    auto pc = std::make_unique<cpk_pc_s>();
    pc->ctx = ctx;
    if (ctx->c.dist())
        pc->p.reset(precond_create_dist(ctx->c, A11->h, B->h, C22->h, Akry ? &Akry->h : nullptr));
    else pc->p.reset(precond_create(ctx->c, A11->h, B->h, C22->h));
    if (ptime) *ptime = pc->p->ptime;
    *out = pc.release();
    API_END
}

int cpk_pc_refactor(cpk_pc M, cpk_mat A11, cpk_mat B, cpk_mat C22, double *ptime) {
    API_BEGIN
    need(M && A11 && B && C22, "opLDL2: Invalid number of arguments.");
    Precond &p = *M->p;
    if (A11->h.nrows != p.gn || C22->h.nrows != p.gm || B->h.nrows != p.gm || B->h.ncols != p.gn)
        throw Error(CPK_ERR_DIM, "Incompatible dimensions.");
    if (!p.dl.ready)
        throw Error(CPK_ERR_UNSUPPORTED, "refactorization needs the device factorization (engine option host_factor off)");
    if (pattern_hash(A11->h, B->h, C22->h) != p.pattern_hash)
        throw Error(CPK_ERR_ARGS, "refactor: the sparsity of A11, B or C22 differs from the factored one");
    const double s = precond_refactor(p, A11->dev(), B->dev(), C22->dev());
    if (ptime) *ptime = s;
    API_END
}

int cpk_pc_destroy(cpk_pc M) {
    API_BEGIN
    delete M;
    API_END
}

static double matlab_round(double v) { return v < 0 ? -std::floor(-v + 0.5) : std::floor(v + 0.5); }

// opLDL2 setters (ops/opLDL2.m:97-115)
static void apply_props(Precond &p, const cpk_opts *o) {
    if (!o) return;
    if (o->has_nitref) p.nitref = std::max(0.0, matlab_round(o->nitref));
    if (o->has_itref_tol) p.itref_tol = o->itref_tol;  // `sef.itref_tol` typo: no clamp in effect
    if (o->has_residual_update) p.residual_update = o->residual_update;
    if (o->has_force_itref) p.force_itref = (o->force_itref != 0 && o->force_itref != 1) ? 0.0 : o->force_itref;
}

int cpk_pc_set(cpk_pc M, const cpk_opts *opts) {
    API_BEGIN
    need(M && opts, "NULL argument");
    apply_props(*M->p, opts);
    API_END
}

int cpk_pc_get(cpk_pc M, double *nitref, double *itref_tol, double *force_itref, double *residual_update) {
    API_BEGIN
    need(M, "NULL argument");
    if (nitref) *nitref = M->p->nitref;
    if (itref_tol) *itref_tol = M->p->itref_tol;
    if (force_itref) *force_itref = M->p->force_itref;
    if (residual_update) *residual_update = M->p->residual_update;
    API_END
}

int cpk_pc_set_handle(cpk_pc M, int on) {
    API_BEGIN
    need(M, "NULL argument");
    M->p->set_handle(on != 0);
    API_END
}

int cpk_pc_apply(cpk_pc M, const double *x, double *y) {
    API_BEGIN
    need(M && x && y, "NULL argument");
    Precond &p = *M->p;
    Ctx &c = M->ctx->c;
    DBuf<double> dx, dy;
    if (p.dist) scatter_global(p, x, p.N, dx);
    else h2d(dx, x, (size_t)p.N);
    dy.alloc((size_t)std::max<int64_t>(p.N, 1));
    p.apply(dx.p, p.N, dy.p, nullptr);
    if (p.dist) {
        gather_global(c, p, dy.p, y);
    } else {
        CPK_HIP(hipMemcpyAsync(y, dy.p, p.N * sizeof(double), hipMemcpyDeviceToHost, c.stream));
        CPK_HIP(hipStreamSynchronize(c.stream));
    }
    check_chain(p.dF);
    check_chain(p.sep.tsw);
    API_END
}

int cpk_pc_apply_device(cpk_pc M, const double *d_x, double *d_y) {
    API_BEGIN
    need(M && d_x && d_y, "NULL argument");
    M->p->apply(d_x, M->p->N, d_y, nullptr);
    API_END
}

int cpk_pc_divide(cpk_pc M, const double *b, double *x) {
    API_BEGIN
    need(M && b && x, "NULL argument");
    Precond &p = *M->p;
    Ctx &c = M->ctx->c;
    DBuf<double> db, dx;
    if (p.dist) scatter_global(p, b, p.N, db);
    else h2d(db, b, (size_t)p.N);
    dx.alloc((size_t)std::max<int64_t>(p.N, 1));
    launch_spmv(c, p.dKp, db.p, dx.p, nullptr);
    if (p.dist) {
        gather_global(c, p, dx.p, x);
    } else {
        CPK_HIP(hipMemcpyAsync(x, dx.p, p.N * sizeof(double), hipMemcpyDeviceToHost, c.stream));
        CPK_HIP(hipStreamSynchronize(c.stream));
    }
    API_END
}

int cpk_pc_get_info(cpk_pc M, cpk_pc_info *info) {
    API_BEGIN
    need(M && info, "NULL argument");
    const Precond &p = *M->p;
    info->n = p.gn, info->m = p.gm, info->N = p.gN;
    info->nnz_kp = p.Kp.nnz();
    info->nnz_l = (int64_t)p.F.Li.size();
    info->nblocks = (int64_t)p.S.blk_row.size() - 1;
    info->nrounds = (int64_t)p.S.round_ptr.size() - 1;
    info->max_block_levels = p.S.max_levels;
    info->depth = p.S.depth;
    info->ordering = p.ordering;
    API_END
}

int cpk_pc_export(cpk_pc M, int64_t *Lcolptr, int32_t *Lrowind, double *Lval, double *D, int32_t *perm) {
    API_BEGIN
    need(M, "NULL argument");
    const Precond &p = *M->p;
    const Factor &f = p.F;
    if (Lcolptr) std::memcpy(Lcolptr, f.Lp.data(), f.Lp.size() * sizeof(int64_t));
    if (Lrowind) std::memcpy(Lrowind, f.Li.data(), f.Li.size() * sizeof(int32_t));
    if (p.dl.ready) {  // values computed on the device (ldl.hip): CSC order, pivot order
        if (Lval && !f.Li.empty()) CPK_HIP(hipMemcpy(Lval, p.dl.Lx.p, f.Li.size() * sizeof(double), hipMemcpyDeviceToHost));
        if (D && f.N) CPK_HIP(hipMemcpy(D, p.dl.D.p, (size_t)f.N * sizeof(double), hipMemcpyDeviceToHost));
    } else {
        if (Lval) std::memcpy(Lval, f.Lx.data(), f.Lx.size() * sizeof(double));
        if (D) std::memcpy(D, f.D.data(), f.D.size() * sizeof(double));
    }
    if (perm) std::memcpy(perm, f.perm.data(), f.perm.size() * sizeof(int32_t));
    API_END
}

static void check_method_dims(cpk_mat A, cpk_mat C, const cpk_pc_s *M) {
    need(A && C && M, "NULL argument");
    if (A->h.nrows != A->h.ncols || C->h.nrows != C->h.ncols) throw Error(CPK_ERR_DIM, "A and C must be square");
    if (A->h.nrows != M->p->gn || C->h.nrows != M->p->gm) throw Error(CPK_ERR_DIM, "A, C and M dimensions disagree");
}

static void check_dist_method(const Ctx &, int) {}

int cpk_method_solve_device(cpk_ctx ctx, int method, const double *d_b, cpk_mat A, cpk_mat C, cpk_pc M,
                            const cpk_opts *opts, double *d_xy, cpk_stats *stats) {
    API_BEGIN
    need(ctx && A && M && (d_xy || !M->p->N) && (d_b || !M->p->n), "NULL argument");
    check_method_dims(A, C, M);
    check_dist_method(ctx->c, method);
    const DMat &AC = A->krylov_op(C, *M->p);
    method_solve_device(ctx->c, method, d_b, AC, *M->p, opts, d_xy, stats);
    API_END
}

int cpk_method_solve(cpk_ctx ctx, int method, const double *b, cpk_mat A, cpk_mat C, cpk_pc M, const cpk_opts *opts,
                     double *x, double *y, cpk_stats *stats) {
    API_BEGIN
    need(ctx && b && x && A && C && M && (y || !C->h.nrows), "NULL argument");
    check_method_dims(A, C, M);
    check_dist_method(ctx->c, method);
    Ctx &c = ctx->c;
    Precond &p = *M->p;
    const int64_t n = p.n, m = p.m, N = n + m;
    const DMat &AC = A->krylov_op(C, p);
    DBuf<double> db, dxy;
    if (p.dist) scatter_global(p, b, n, db);
    else h2d(db, b, (size_t)n);
    dxy.alloc((size_t)std::max<int64_t>(N, 1));
    auto t0 = std::chrono::steady_clock::now();
    method_solve_device(c, method, db.p, AC, p, opts, dxy.p, stats);
    if (p.dist) {
        std::vector<double> g((size_t)p.gN);
        gather_global(c, p, dxy.p, g.data());
        std::memcpy(x, g.data(), p.gn * sizeof(double));
        if (p.gm) std::memcpy(y, g.data() + p.gn, p.gm * sizeof(double));
    } else {
        CPK_HIP(hipMemcpy(x, dxy.p, n * sizeof(double), hipMemcpyDeviceToHost));
        if (m) CPK_HIP(hipMemcpy(y, dxy.p + n, m * sizeof(double), hipMemcpyDeviceToHost));
    }
    if (stats) stats->stime = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    API_END
}

// the shift's two products: 1 GPU reads rows < n of blkdiag(A, C) and of Kp (columns >= n);
// distributed mode has dedicated x-part row slices of [A 0] and [0 B']
struct ShiftOps {
    const DMat *A, *Bt;
    int64_t bt_colmin;
};
static ShiftOps shift_ops(cpk_mat A, cpk_mat C, Precond &p) {
    if (p.dist) {
        auto pr = A->shift_ops(p);
        return {pr.first, pr.second, 0};
    }
    return {&A->blkdiag_with(C), &p.dKp, p.n};
}

int cpk_reg_solve_device(cpk_ctx ctx, int method, const double *d_b, cpk_mat A, cpk_mat B, cpk_mat C, cpk_pc M,
                         const cpk_opts *opts, double *d_x, cpk_stats *stats) {
    API_BEGIN
    need(ctx && A && M && B && ((d_b && d_x) || !M->p->N), "NULL argument");
    check_method_dims(A, C, M);
    check_dist_method(ctx->c, method);
    const DMat &AC = A->krylov_op(C, *M->p);
    const ShiftOps so = shift_ops(A, C, *M->p);
    reg_solve_device(ctx->c, method, d_b, AC, *so.A, *so.Bt, so.bt_colmin, *M->p, opts, d_x, stats);
    if (stats) stats->ptime = M->p->ptime;
    API_END
}

int cpk_reg_shift_device(cpk_ctx ctx, const double *d_b, cpk_mat A, cpk_mat B, cpk_mat C, cpk_pc M, double *d_b1,
                         double *d_xy0, int *shifted) {
    API_BEGIN
    need(ctx && A && M && B && ((d_b && d_b1 && d_xy0) || !M->p->N), "NULL argument");
    check_method_dims(A, C, M);
    const ShiftOps so = shift_ops(A, C, *M->p);
    int s = reg_shift_device(ctx->c, d_b, *so.A, *so.Bt, so.bt_colmin, *M->p, d_b1, d_xy0);
    if (shifted) *shifted = s;
    API_END
}

int cpk_profile_kernels(cpk_ctx ctx, cpk_mat A, cpk_mat C, cpk_pc M, int reps, cpk_profile *out) {
    API_BEGIN
    need(ctx && out, "NULL argument");
    check_method_dims(A, C, M);
    profile_kernels(ctx->c, A->krylov_op(C, *M->p), *M->p, reps, out);
    API_END
}

int cpk_debug_pipe_stamps(uint64_t *out, int npairs, int *copied) {
    API_BEGIN
    need(out && copied, "NULL argument");
    *copied = debug_pipe_stamps(out, npairs);
    API_END
}

int cpk_debug_blk_cycles(uint64_t *out, int64_t n, int64_t *copied) {
    API_BEGIN
    need(out && copied, "NULL argument");
    *copied = debug_blk_cycles(out, n);
    API_END
}

int cpk_debug_pass_times(cpk_ctx ctx, double *out) {
    API_BEGIN
    need(ctx && out, "NULL argument");
    std::memcpy(out, ctx->c.pass_ms, sizeof ctx->c.pass_ms);
    API_END
}

int cpk_debug_block_model(cpk_pc M, int64_t *out, int64_t n, int64_t *copied) {
    API_BEGIN
    need(M && copied, "NULL argument");
    const std::vector<int64_t> &h = M->p->dF.hmodel;
    *copied = std::min<int64_t>(n, (int64_t)h.size());
    if (out && *copied) std::memcpy(out, h.data(), (size_t)*copied * sizeof(int64_t));
    API_END
}

int cpk_pc_sep_info(cpk_pc M, int64_t *info) {
    API_BEGIN
    need(M && info, "NULL argument");
    const Precond &p = *M->p;
    const DSep &T = p.sep;
    const int64_t v[12] = {p.dist ? 1 : 0, T.nT, T.nlev, T.nrec, (int64_t)T.lds, (int64_t)T.lds_g, T.kt, p.tkr ? 1 : 0,
                           p.dsched ? 1 : 0, (p.dsched && p.fused_resid && !p.dF.no_fused_resid) ? 1 : 0,
                           T.tsweep ? 1 : 0, T.tsweep ? (int64_t)T.tsw.round_ptr.size() - 1 : 0};
    std::memcpy(info, v, sizeof v);
    API_END
}

int cpk_pc_sweep_info(cpk_pc M, int64_t *info) {
    API_BEGIN
    need(M && info, "NULL argument");
    const DFactor &F = M->p->dF;
    const int64_t nr = (int64_t)F.round_ptr.size() - 1;
    const int64_t r0 = nr >= 1 ? F.round_ptr[1] - F.round_ptr[0] : 0;
    // the chain the sweeps launch: the full one (last round fused), else the forward one
    const int64_t chain = F.no_chain ? 0
                          : (F.chain[kChainFull].ntask > 0 && fuse_last_ok(F)) ? F.chain[kChainFull].ntask
                                                                               : F.chain[kChainFwd].ntask;
    const int64_t v[8] = {nr, r0, F.nblk - r0, F.agrid[0], F.agrid[1], F.agrid[2], F.pipelined ? 1 : 0, chain};
    std::memcpy(info, v, sizeof v);
    API_END
}

int cpk_pc_local_dofs(cpk_pc M, int64_t *n_loc, int64_t *m_loc, int32_t *dofs) {
    API_BEGIN
    need(M, "NULL argument");
    const Precond &p = *M->p;
    if (n_loc) *n_loc = p.n;
    if (m_loc) *m_loc = p.m;
    if (dofs) {
        if (p.dist) {
            const std::vector<int32_t> d = p.dofmap->dofs(M->ctx->c.rank);
            std::memcpy(dofs, d.data(), d.size() * sizeof(int32_t));
        } else {
            for (int64_t i = 0; i < p.N; i++) dofs[i] = (int32_t)i;
        }
    }
    API_END
}

int cpk_reg_solve(cpk_ctx ctx, int method, const double *b, cpk_mat A, cpk_mat B, cpk_mat C, cpk_mat G,
                  const cpk_opts *opts, double *x, cpk_stats *stats, cpk_pc *M_out) {
    API_BEGIN
    // reg_cpkrylov.m:122-125
    if (!ctx || !b || !A || !B || !C || !G || !x) throw Error(CPK_ERR_ARGS, "reg_cpkrylov: not enough inputs");
    Ctx &c = ctx->c;
    // M = opLDL2(G, B, -C)   (reg_cpkrylov.m:128-132)
    HCsr negC = C->h;
    for (auto &v : negC.val) v = -v;
    check_dist_method(c, method);
    auto pc = std::make_unique<cpk_pc_s>();
    pc->ctx = ctx;
    if (c.dist()) pc->p.reset(precond_create_dist(c, G->h, B->h, negC, &A->h));
    else pc->p.reset(precond_create(c, G->h, B->h, negC));
    Precond &p = *pc->p;
    apply_props(p, opts);  // reg_cpkrylov.m:135-148
    check_method_dims(A, C, pc.get());
    const int64_t N = p.N;
    const DMat &AC = A->krylov_op(C, p);
    const ShiftOps so = shift_ops(A, C, p);
    DBuf<double> db, dx;
    if (p.dist) scatter_global(p, b, N, db);
    else h2d(db, b, (size_t)N);
    dx.alloc((size_t)std::max<int64_t>(N, 1));
    reg_solve_device(c, method, db.p, AC, *so.A, *so.Bt, so.bt_colmin, p, opts, dx.p, stats);
    if (p.dist) gather_global(c, p, dx.p, x);
    else CPK_HIP(hipMemcpy(x, dx.p, N * sizeof(double), hipMemcpyDeviceToHost));
    if (stats) stats->ptime = pc->p->ptime;
    if (M_out) *M_out = pc.release();
    API_END
}

int cpk_analyze(cpk_mat A11, cpk_mat B, cpk_mat C22, const char *options, cpk_analysis *out) {
    API_BEGIN
    need(A11 && B && C22 && out, "NULL argument");
    auto a = std::make_unique<cpk_analysis_s>();
    a->opts = engine_opts_from_env();
    if (options) apply_engine_options(a->opts, options);
    a->an = analyze(A11->h, B->h, C22->h, a->opts);
    *out = a.release();
    API_END
}

int cpk_analysis_destroy(cpk_analysis an) {
    API_BEGIN
    delete an;
    API_END
}

int cpk_analysis_get_info(cpk_analysis a, cpk_pc_info *info) {
    API_BEGIN
    need(a && info, "NULL argument");
    const Analysis &an = a->an;
    info->n = an.n, info->m = an.m, info->N = an.N;
    info->nnz_kp = an.Kp.nnz();
    info->nnz_l = (int64_t)an.F0.Li.size();
    info->nblocks = (int64_t)an.S.blk_row.size() - 1;
    info->nrounds = (int64_t)an.S.round_ptr.size() - 1;
    info->max_block_levels = an.S.max_levels;
    info->depth = an.S.depth;
    info->ordering = an.ordering;
    API_END
}

int cpk_analysis_export(cpk_analysis a, int64_t *Lcolptr, int32_t *Lrowind, double *Lval, double *D, int32_t *perm) {
    API_BEGIN
    need(a, "NULL argument");
    const Factor &f = a->an.F0;
    if (Lcolptr) std::memcpy(Lcolptr, f.Lp.data(), f.Lp.size() * sizeof(int64_t));
    if (Lrowind) std::memcpy(Lrowind, f.Li.data(), f.Li.size() * sizeof(int32_t));
    if (Lval) std::memcpy(Lval, f.Lx.data(), f.Lx.size() * sizeof(double));
    if (D) std::memcpy(D, f.D.data(), f.D.size() * sizeof(double));
    if (perm) std::memcpy(perm, f.perm.data(), f.perm.size() * sizeof(int32_t));
    API_END
}

int cpk_analysis_schedule(cpk_analysis a, int64_t *nlevels, int64_t *round_ptr, int64_t *blk_lvl, int64_t *lvl_row,
                          int32_t *order) {
    API_BEGIN
    need(a, "NULL argument");
    const Schedule &s = a->an.S;
    if (order) std::memcpy(order, s.order.data(), s.order.size() * sizeof(int32_t));
    if (nlevels) *nlevels = (int64_t)s.lvl_row.size() - 1;
    if (round_ptr) std::memcpy(round_ptr, s.round_ptr.data(), s.round_ptr.size() * sizeof(int64_t));
    if (blk_lvl) std::memcpy(blk_lvl, s.blk_lvl.data(), s.blk_lvl.size() * sizeof(int64_t));
    if (lvl_row) std::memcpy(lvl_row, s.lvl_row.data(), s.lvl_row.size() * sizeof(int64_t));
    API_END
}

int cpk_analysis_plan(cpk_analysis a, cpk_mat A, cpk_mat C, int nranks, int rank, cpk_plan *out) {
    API_BEGIN
    need(a && A && C && out, "NULL argument");
    need(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank / nranks");
    const Analysis &an = a->an;
    need(A->h.nrows == an.n && A->h.ncols == an.n && C->h.nrows == an.m && C->h.ncols == an.m,
         "A and C must match the analysis' n and m");
    auto p = std::make_unique<cpk_plan_s>();
    p->n = an.n, p->m = an.m;
    p->ts = split_tree(an.F0, nranks, a->opts.split_tol, -1, &A->h);
    p->dm = make_dofmap(an.F0, p->ts, an.n);
    p->rp = make_rank_plan(an.F0, p->ts, p->dm, rank);
    p->kp = dist_csr(an.Kp, p->dm, rank, false);
    p->ac = dist_csr(blkdiag(A->h, C->h), p->dm, rank, false);
    p->ab = dist_csr(hstack_ab(A->h, an.Kp, an.n), p->dm, rank, true);
    *out = p.release();
    API_END
}

int cpk_plan_destroy(cpk_plan p) {
    API_BEGIN
    delete p;
    API_END
}

int cpk_plan_array(cpk_plan p, const char *name, int64_t *count, void *out) {
    API_BEGIN
    need(p && name && count, "NULL argument");
    const RankPlan &r = p->rp;
    const std::string nm(name);
    std::vector<int64_t> iv;
    std::vector<double> dv;
    bool isd = false;
    auto I = [&](const auto &v) { iv.assign(v.begin(), v.end()); };
    auto Dv = [&](const std::vector<double> &v) { dv = v, isd = true; };
    const DistCsr *dc = nm.rfind("kp_", 0) == 0 ? &p->kp : nm.rfind("ac_", 0) == 0 ? &p->ac : nm.rfind("ab_", 0) == 0 ? &p->ab : nullptr;
    const std::string sub = dc ? nm.substr(3) : nm;
    if (dc) {
        if (sub == "ptr") I(dc->a.ptr);
        else if (sub == "col") I(dc->a.ind);
        else if (sub == "val") Dv(dc->a.val);
        else if (sub == "send") I(dc->send);
        else throw Error(CPK_ERR_ARGS, "unknown plan array " + nm);
    } else if (nm == "sizes") {
        const int64_t nl = p->dm.n_loc[r.rank], ml = p->dm.m_loc[r.rank];
        iv = {r.P, r.rank, p->n, p->m, p->n + p->m, nl, ml, nl + ml, r.nsub, r.nT, r.kt, p->kp.kmax, p->ac.kmax, p->ab.kmax};
    } else if (nm == "dofs") I(p->dm.dofs(r.rank));
    else if (nm == "node_rank") I(p->ts.node_rank);
    else if (nm == "T") I(p->ts.T);
    else if (nm == "fsub_Lp") I(r.Fsub.Lp);
    else if (nm == "fsub_Li") I(r.Fsub.Li);
    else if (nm == "fsub_Lx") Dv(r.Fsub.Lx);
    else if (nm == "fsub_D") Dv(r.Fsub.D);
    else if (nm == "fsub_perm") I(r.Fsub.perm);
    else if (nm == "fsub_parent") I(r.Fsub.parent);
    else if (nm == "fsub_key") I(r.key);
    else if (nm == "extra_ptr" || nm == "extra_col" || nm == "extra_key" || nm == "extra_val") {
        std::vector<int64_t> ptr{0}, col, key;
        std::vector<double> val;
        for (const auto &e : r.extra) {
            for (const BwdExtra &x : e) col.push_back(x.col), key.push_back(x.key), val.push_back(x.val);
            ptr.push_back((int64_t)col.size());
        }
        if (nm == "extra_ptr") iv = ptr;
        else if (nm == "extra_col") iv = col;
        else if (nm == "extra_key") iv = key;
        else dv = val, isd = true;
    } else if (nm == "tf_ptr") I(r.tf_ptr);
    else if (nm == "tf_col") I(r.tf_col);
    else if (nm == "tf_val") Dv(r.tf_val);
    else if (nm == "tf_src") I(r.tf_src);
    else if (nm == "tb_ptr") I(r.tb_ptr);
    else if (nm == "tb_col") I(r.tb_col);
    else if (nm == "tb_val") Dv(r.tb_val);
    else if (nm == "DT") Dv(r.DT);
    else if (nm == "tlev_ptr") I(r.tlev_ptr);
    else if (nm == "tlev_rows") I(r.tlev_rows);
    else if (nm == "tsend") I(r.tsend);
    else if (nm == "tdof") I(r.tdof);
    else throw Error(CPK_ERR_ARGS, "unknown plan array " + nm);
    *count = isd ? (int64_t)dv.size() : (int64_t)iv.size();
    if (out) {
        if (isd) std::memcpy(out, dv.data(), dv.size() * sizeof(double));
        else std::memcpy(out, iv.data(), iv.size() * sizeof(int64_t));
    }
    API_END
}

int cpk_symgivens(double a, double b, double *c, double *s, double *d) {
    API_BEGIN
    need(c && s && d, "NULL argument");
    auto sign = [](double v) { return (double)((v > 0) - (v < 0)); };
    if (b == 0) {
        *c = (a == 0) ? 1.0 : sign(a), *s = 0.0, *d = std::fabs(a);
    } else if (a == 0) {
        *c = 0.0, *s = sign(b), *d = std::fabs(b);
    } else if (std::fabs(b) > std::fabs(a)) {
        double t = a / b;
        *s = sign(b) / std::sqrt(1 + t * t), *c = *s * t, *d = b / *s;
    } else {
        double t = b / a;
        *c = sign(a) / std::sqrt(1 + t * t), *s = *c * t, *d = a / *c;
    }
    API_END
}

}  // extern "C"
