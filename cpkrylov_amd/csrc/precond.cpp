// precond.cpp -- the constraint preconditioner M = opLDL2(G, B, -C) on the device.
//
// Construction replaces opLDL2's constructor (ops/opLDL2.m:60-92): assemble Kp = [A B'; B C],
// choose a fill-reducing ordering, factor P'*Kp*P = L*D*L' on the host, cut the elimination
// tree into the sweep schedule, and upload Kp, L, L', D and P to HBM.
// apply() replaces opLDL2.multiply (ops/opLDL2.m:161-188) with the effective semantics of the
// reference: Spot operators are value objects, so the residual-update state (Aty, Cy) written
// inside multiply never survives the call and the branch subtracts zeros -- it is skipped here
// (a functional no-op).  With force_itref the residual norms do not influence the loop and
// the residual after the last refinement step is never read, so neither is computed.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <atomic>
#include <cmath>
#include <exception>
#include <memory>
#include <thread>

#include "dev.hpp"
#include "dist.hpp"

namespace cpk {

// CPK_TIMING=1: per-phase wall times of the host analysis on stderr (diagnostic)
struct PhaseClock {
    const char *what;
    bool on;
    std::chrono::steady_clock::time_point t;
    explicit PhaseClock(const char *w) : what(w), on(getenv("CPK_TIMING") != nullptr), t(std::chrono::steady_clock::now()) {}
    void lap(const char *phase) {
        if (!on) return;
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[cpk] %s: %-32s %8.3f s\n", what, phase, std::chrono::duration<double>(now - t).count());
        t = now;
    }
};

Analysis analyze(const HCsr &A11, const HCsr &B, const HCsr &C22, const EngineOpts &o, bool device_numeric,
                 const SymbolicHook &on_symbolic, bool global_schedule) {
    auto t0 = std::chrono::steady_clock::now();
    PhaseClock pc("analyze");
    Analysis an;
    an.Kp = assemble_kp(A11, B, C22);  // dimension checks of opLDL2.m:61-75
    an.n = A11.nrows, an.m = C22.nrows, an.N = an.n + an.m;
    pc.lap("assemble");
    std::vector<int32_t> perm = order_kp(an.Kp, an.n, &an.ordering);
    pc.lap("order");
    an.device_numeric = device_numeric;
    Factor f0 = ldl_factor(an.Kp, perm, 1, device_numeric ? &an.sym : nullptr, !device_numeric);
    pc.lap(device_numeric ? "factor (symbolic)" : "factor");
    // the hook reads Kp, f0 and an.sym on its own thread while this one only reads f0 too
    std::exception_ptr hook_err;
    std::thread hook;
    if (on_symbolic)
        hook = std::thread([&] {
            try {
                on_symbolic(an.Kp, f0, an.sym);
            } catch (...) {
                hook_err = std::current_exception();
            }
        });
    try {
        an.sweep = o.sweep;
        if (global_schedule) {
            an.S = build_schedule(f0, an.sweep.rows[0], an.sweep.cap[0], an.sweep.rows[1], an.sweep.cap[1],
                                  an.sweep.sub0, nullptr);
            pc.lap("schedule");
            an.F = relabel(f0, an.S, device_numeric ? &an.rsrc : nullptr);
            pc.lap("relabel");
        }
    } catch (...) {
        if (hook.joinable()) hook.join();
        throw;
    }
    if (hook.joinable()) hook.join();
    if (hook_err) std::rethrow_exception(hook_err);
    an.F0 = std::move(f0);
    if (on_symbolic) pc.lap("symbolic hook (overlapped)");
    an.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return an;
}

Precond *precond_create(Ctx &c, Analysis &&an, PrecondPre *pre) {
    auto t0 = std::chrono::steady_clock::now();
    PhaseClock clk("precond_create");
    auto pc = std::make_unique<Precond>();
    pc->ctx = &c;
    pc->n = an.n, pc->m = an.m, pc->N = an.N;
    pc->gn = an.n, pc->gm = an.m, pc->gN = an.N;
    pc->ordering = an.ordering;
    pc->Kp = std::move(an.Kp);
    pc->S = std::move(an.S);
    for (int i = 0; i < 2; i++)  // before make_dfactor: the device layout follows the configuration
        pc->dF.sweep_rows[i] = an.sweep.rows[i], pc->dF.sweep_cap[i] = an.sweep.cap[i],
        pc->dF.sweep_threads[i] = an.sweep.threads[i];
    pc->dF.pipelined = !c.opts.no_pipe, pc->dF.no_upper = c.opts.no_upper, pc->dF.no_col16 = c.opts.no_col16;
    pc->dF.no_chain = c.opts.no_chain;
    pc->dF.chain_wide = c.opts.chain_wide;
    pc->dF.dataflow = c.opts.no_dataflow ? 1 : (c.opts.all_dataflow ? 2 : 0);
    pc->dF.colsweep = c.opts.no_colsweep ? 1 : (c.opts.all_colsweep ? 2 : 0);
    pc->dF.no_fused_resid = c.opts.no_fused_resid;
    pc->dF.fuse_last = !c.opts.no_fuse_last;  // single GPU: no entries outside the factor
    pc->no_sched = c.opts.no_sched_resid;
    // Kp and Kp in schedule order depend only on Kp and the pivot order: they are built and
    // uploaded on a second host thread while this one lays out and uploads the factor
    std::vector<int64_t> kps_ptr;
    std::exception_ptr kp_err;
    std::thread kp_thread([&] {
        try {
            CPK_HIP(hipSetDevice(c.device));
            if (pre && pre->kp) pc->dKp = std::move(pre->dKp);  // uploaded during the analysis
            else make_dmat(pc->Kp, pc->dKp);
            if (pc->Kp.nnz() > (int64_t)INT32_MAX) return;
            // Kp in schedule order: row q = Kp row perm_s[q] with its entries in Kp's order, columns
            // renumbered to schedule positions (perm_s = the relabelled factor's pivot order)
            const std::vector<int32_t> &ps = an.F.perm;
            const int64_t N = pc->N;
            std::vector<int32_t> pos(N);
            for (int64_t q = 0; q < N; q++) pos[ps[q]] = (int32_t)q;
            HCsr ks;
            ks.nrows = ks.ncols = N;
            ks.ptr.assign(N + 1, 0);
            for (int64_t q = 0; q < N; q++) ks.ptr[q + 1] = ks.ptr[q] + (pc->Kp.ptr[ps[q] + 1] - pc->Kp.ptr[ps[q]]);
            ks.ind.resize(pc->Kp.nnz());
            ks.val.resize(pc->Kp.nnz());
            std::vector<int32_t> from(pc->Kp.nnz());
            parallel_for(N, [&](int64_t lo, int64_t hi) {
                for (int64_t q = lo; q < hi; q++) {
                    int64_t t = ks.ptr[q];
                    for (int64_t p = pc->Kp.ptr[ps[q]]; p < pc->Kp.ptr[ps[q] + 1]; p++, t++)
                        ks.ind[t] = pos[pc->Kp.ind[p]], ks.val[t] = pc->Kp.val[p], from[t] = (int32_t)p;
                }
            });
            make_dmat(ks, pc->dKps);
            pc->kps_from.upload(from);
            kps_ptr = std::move(ks.ptr);
        } catch (...) {
            kp_err = std::current_exception();
        }
    });
    try {
        const std::vector<int64_t> key(pc->S.order.begin(), pc->S.order.end());
        if (an.device_numeric) {
            std::vector<int32_t> fsrc, bsrc;
            make_dfactor(an.F, pc->S, pc->dF, &key, nullptr, &fsrc, &bsrc);
            parallel_for((int64_t)fsrc.size(), [&](int64_t lo, int64_t hi) {  // relabelled slot -> exported (CSC) slot
                for (int64_t q = lo; q < hi; q++) fsrc[q] = an.rsrc[fsrc[q]];
            });
            parallel_for((int64_t)bsrc.size(), [&](int64_t lo, int64_t hi) {
                for (int64_t q = lo; q < hi; q++) bsrc[q] = an.rsrc[bsrc[q]];
            });
            if (pre && pre->dl.sym_ready) pc->dl = std::move(pre->dl);  // uploaded during the analysis
            else dldl_setup_sym(pc->dl, an.sym, an.F0);
            dldl_setup_src(pc->dl, fsrc, bsrc, pc->S.order);
        } else {
            make_dfactor(an.F, pc->S, pc->dF, &key);
        }
    } catch (...) {
        kp_thread.join();
        throw;
    }
    clk.lap("device factor layout + upload");
    kp_thread.join();
    if (kp_err) std::rethrow_exception(kp_err);
    clk.lap("Kp, Kp in schedule order (overlapped)");
    if (an.device_numeric) {
        dldl_factor(c, pc->dl, pc->dKp.val.p, pc->dF);
        CPK_HIP(hipStreamSynchronize(c.stream));
        clk.lap("numeric factorization (device)");
    }
    plan_round0(c, pc->dF, kps_ptr.empty() ? nullptr : kps_ptr.data());
    if (pc->dKps.nnz) pc->xs.alloc(pc->N);
    if (pc->dKps.nnz && pc->dF.round0_rows >= 0 && pc->dF.fcol16.n > 0)
        pc->fused_resid = true;
    clk.lap("round-0 assignment");
    an.F = Factor();
    pc->F = std::move(an.F0);
    pc->w.alloc(pc->N);
    pc->r.alloc(pc->N);
    pc->active.alloc(1);
    c.ensure_partials(std::max<size_t>(pc->dKp.nblk * 2, 4096));
    CPK_HIP(hipDeviceSynchronize());
    pc->ptime = an.seconds + std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return pc.release();
}

// Every rank builds the global analysis and its share of the plan on its own (DESIGN.md
// section 7), so all of them must agree on the inputs, the split and every engine option (the
// schedule, the separator exchange and the solvers' collective sequence follow from them).
// Before the first collective of any apply, the ranks allgather a hash of all of it; on a
// mismatch every rank throws the same error instead of exchanging mismatched payloads.
uint64_t plan_hash(const Ctx &c, const Analysis &an, const TreeSplit &ts) {
    uint64_t h = engine_opts_hash(c.opts);
    auto mix = [&](uint64_t v) { h = (h ^ v) * 1099511628211ull; };
    mix((uint64_t)c.nranks), mix((uint64_t)an.n), mix((uint64_t)an.m), mix((uint64_t)an.Kp.nnz());
    mix(an.input_hash);
    for (int32_t v : an.F0.perm) mix((uint32_t)v);
    for (int64_t v : an.F0.Lp) mix((uint64_t)v);
    for (int32_t v : ts.node_rank) mix((uint32_t)v);
    for (int32_t v : ts.T) mix((uint32_t)v);
    return h;
}

void check_plan_agreement(Ctx &c, uint64_t h) {
    if (!c.comm->has_peers()) return;
    const double mine[2] = {(double)(h >> 32), (double)(h & 0xffffffffull)};  // exact in fp64
    DBuf<double> snd, rcv;
    snd.alloc(2), rcv.alloc((size_t)2 * c.nranks);
    CPK_HIP(hipMemcpy(snd.p, mine, sizeof mine, hipMemcpyHostToDevice));
    c.comm->allgather(snd.p, rcv.p, 2, c.stream);
    std::vector<double> all((size_t)2 * c.nranks);
    CPK_HIP(hipMemcpyAsync(all.data(), rcv.p, rcv.bytes(), hipMemcpyDeviceToHost, c.stream));
    CPK_HIP(hipStreamSynchronize(c.stream));
    std::string bad;
    for (int r = 0; r < c.nranks; r++)
        if (all[2 * r] != all[0] || all[2 * r + 1] != all[1]) bad += (bad.empty() ? "" : ", ") + std::to_string(r);
    if (!bad.empty())
        throw Error(CPK_ERR_ARGS, "distributed preconditioner: the plan of rank(s) " + bad +
                                      " differs from rank 0's (inputs or engine options differ between ranks)");
}

Precond *precond_create_dist(Ctx &c, Analysis &&an, const HCsr *Akry) {
    auto t0 = std::chrono::steady_clock::now();
    PhaseClock clk("precond_create_dist");
    // device factorization (an.device_numeric): the host analysis holds the structure only; the
    // plan is built from an INDEX-valued factor (L entry p -> p + 1, D row v -> v + 1, Kp entry
    // q -> q + 1), so every value array of this rank's plan holds where its values come from.
    // Those become value maps (vmap_capture), and the device factorization of the whole system
    // fills them (fill_vmaps): the values a host-factored plan would copy, bit for bit.
    const bool devnum = an.device_numeric;
    SubClock sub;
    if (devnum) {
        an.F0.Lx.resize(an.F0.Li.size());
        an.F0.D.resize((size_t)an.F0.N);
        parallel_for((int64_t)an.F0.Lx.size(), [&](int64_t lo, int64_t hi) {
            for (int64_t p = lo; p < hi; p++) an.F0.Lx[p] = (double)(p + 1);
        }, 1 << 16);
        parallel_for(an.F0.N, [&](int64_t lo, int64_t hi) {
            for (int64_t v = lo; v < hi; v++) an.F0.D[v] = (double)(v + 1);
        }, 1 << 16);
    }
    sub.lap("dist: index-valued factor");
    auto pc = std::make_unique<Precond>();
    pc->ctx = &c;
    pc->dist = true;
    pc->gn = an.n, pc->gm = an.m, pc->gN = an.N;
    pc->ordering = an.ordering;
    const TreeSplit ts = split_tree(an.F0, c.nranks, c.opts.split_tol, -1, Akry);
    sub.lap("dist: split");
    check_plan_agreement(c, plan_hash(c, an, ts));
    sub.lap("dist: plan hash + agreement");
    auto dm = std::make_shared<DofMap>(make_dofmap(an.F0, ts, an.n));
    RankPlan rp = make_rank_plan(an.F0, ts, *dm, c.rank);
    sub.lap("dist: dof map + rank plan");
    pc->n = dm->n_loc[c.rank], pc->m = dm->m_loc[c.rank], pc->N = pc->n + pc->m;
    pc->nsub = rp.nsub;
    // local sweeps: schedule + relabel of this rank's subtrees, rows summed in exported order
    std::vector<int64_t> nextra(rp.nsub);
    for (int64_t j = 0; j < rp.nsub; j++) nextra[j] = (int64_t)rp.extra[j].size();
    // the rank's subtrees of a P > 1 split take the distributed default (dist_sweep_default); one
    // rank holds the whole system and takes the single-GPU one
    const SweepConfig sw = effective_sweep(c.opts, c.nranks > 1);
    Schedule S = build_schedule(rp.Fsub, sw.rows[0], sw.cap[0], sw.rows[1], sw.cap[1], sw.sub0, &nextra);
    for (int i = 0; i < 2; i++)
        pc->dF.sweep_rows[i] = sw.rows[i], pc->dF.sweep_cap[i] = sw.cap[i], pc->dF.sweep_threads[i] = sw.threads[i];
    pc->dF.pipelined = !c.opts.no_pipe, pc->dF.no_upper = c.opts.no_upper, pc->dF.no_col16 = c.opts.no_col16;
    pc->dF.no_chain = c.opts.no_chain;
    pc->dF.chain_wide = c.opts.chain_wide;
    pc->dF.dataflow = c.opts.no_dataflow ? 1 : (c.opts.all_dataflow ? 2 : 0);
    pc->dF.colsweep = c.opts.no_colsweep ? 1 : (c.opts.all_colsweep ? 2 : 0);
    pc->dF.no_fused_resid = c.opts.no_fused_resid;
    {
        Factor Fl = relabel(rp.Fsub, S);
        std::vector<int64_t> key(rp.nsub);
        std::vector<std::vector<BwdExtra>> extra(rp.nsub);
        std::vector<int32_t> pos(rp.nsub);
        for (int64_t q = 0; q < rp.nsub; q++) {
            key[q] = rp.key[S.order[q]];
            extra[q] = std::move(rp.extra[S.order[q]]);
            pos[S.order[q]] = (int32_t)q;
        }
        make_dfactor(Fl, S, pc->dF, &key, &extra);
        plan_round0(c, pc->dF, nullptr);
        std::vector<int32_t> send(rp.tsend.size());
        for (size_t i = 0; i < send.size(); i++) send[i] = pos[rp.tsend[i]];
        pc->sep.send.upload(send);
        pc->sep.nsend = (int64_t)send.size();
        // the forward sweep's write-back packs the payload: schedule row -> payload slot
        std::vector<int32_t> tsl((size_t)std::max<int64_t>(rp.nsub, 1), -1);
        for (size_t i = 0; i < send.size(); i++) tsl[send[i]] = (int32_t)i;
        pc->sep.tslot.upload(tsl);
    }
    sub.lap("dist: local schedule + layout");
    // separator solve
    DSep &T = pc->sep;
    // payload per rank: the plan's kt values, then kSepPiggy slots that can carry a solver's
    // deferred inner-product partials through the same allgather (Precond::apply, piggy_src):
    // positions r * kt + j of the plan become r * (kt + kSepPiggy) + j
    if (rp.kt > 0) {
        const int64_t kt0 = rp.kt, kt1 = kt0 + kSepPiggy;
        auto remap = [&](int32_t q) { return (int32_t)((q / kt0) * kt1 + q % kt0); };
        for (auto &q : rp.tf_col)
            if (q >= 0) q = remap(q);
        for (auto &q : rp.tf_src) q = remap(q);
        rp.kt = kt1;
    }
    // the refinement residual without the Kp halo exchange (Precond::tkr): the subtree rows the
    // T dofs' Kp rows read, per owner (ascending dof), ride in extra payload slots after the
    // plan's payload and the piggyback: positions r * kt1 + j become r * kt2 + j.  Every rank
    // decides from global data only, so all take the same path.
    std::vector<int32_t> tkr_ptr{0}, tkr_col, hslot2;
    std::vector<double> tkr_val;
    const int64_t kt1 = rp.kt;
    {
        const HCsr &K = an.Kp;
        std::vector<int32_t> tof((size_t)an.N, -1);  // dof -> T index
        for (int64_t t = 0; t < rp.nT; t++) tof[an.F0.perm[ts.T[t]]] = (int32_t)t;
        const bool want_tkr = !c.opts.no_tkr && rp.kt > 0 && rp.nT > 0;
        const bool want_sched = !c.opts.no_sched_resid && (rp.nT == 0 || want_tkr);
        // Kp(i, j) != 0 joins an ancestor and a descendant, so outside T a row couples only with
        // its own rank's rows: checked over the whole matrix (the same verdict on every rank)
        std::atomic<bool> coupled{want_tkr || want_sched};
        if (coupled && c.nranks > 1)
            parallel_for(K.nrows, [&](int64_t lo, int64_t hi) {
                for (int64_t d = lo; d < hi && coupled.load(std::memory_order_relaxed); d++)
                    if (tof[d] < 0)
                        for (int64_t p = K.ptr[d]; p < K.ptr[d + 1]; p++) {
                            const int32_t g = K.ind[p];
                            if (tof[g] < 0 && dm->owner[g] != dm->owner[d]) coupled = false;
                        }
            }, 1 << 16);
        const bool ok = want_tkr && coupled;
        std::vector<std::vector<int32_t>> need((size_t)c.nranks);
        for (int64_t t = 0; t < rp.nT && ok; t++) {
            const int32_t d = an.F0.perm[ts.T[t]];
            for (int64_t p = K.ptr[d]; p < K.ptr[d + 1]; p++) {
                const int32_t g = K.ind[p];
                if (tof[g] < 0) need[(size_t)dm->owner[g]].push_back(g);
            }
        }
        size_t kext = 0;
        std::vector<int32_t> epos((size_t)an.N, -1);
        for (auto &v : need) {
            std::sort(v.begin(), v.end());
            v.erase(std::unique(v.begin(), v.end()), v.end());
            for (size_t e = 0; e < v.size(); e++) epos[(size_t)v[e]] = (int32_t)e;
            kext = std::max(kext, v.size());
        }
        if (ok && kext > 0) {
            const int64_t kt2 = kt1 + (int64_t)kext;
            auto remap = [&](int32_t q) { return (int32_t)((q / kt1) * kt2 + q % kt1); };
            for (auto &q : rp.tf_col)
                if (q >= 0) q = remap(q);
            for (auto &q : rp.tf_src) q = remap(q);
            rp.kt = kt2;
            for (int64_t t = 0; t < rp.nT; t++) {
                const int32_t d = an.F0.perm[ts.T[t]];
                for (int64_t p = K.ptr[d]; p < K.ptr[d + 1]; p++) {
                    const int32_t g = K.ind[p];
                    tkr_col.push_back(tof[g] >= 0 ? -(tof[g] + 1)
                                                  : (int32_t)((int64_t)dm->owner[g] * kt2 + kt1 + epos[(size_t)g]));
                    tkr_val.push_back(devnum ? (double)(p + 1) : K.val[p]);
                }
                tkr_ptr.push_back((int32_t)tkr_col.size());
            }
            hslot2.assign((size_t)std::max<int64_t>(pc->N, 1), -1);
            for (size_t e = 0; e < need[(size_t)c.rank].size(); e++)
                hslot2[(size_t)dm->lidx[need[(size_t)c.rank][e]]] = (int32_t)(kt1 + (int64_t)e);
            // this rank's Kp rows: T-dof columns read wT (column nloc + t); rank 0's T rows empty
            const std::vector<int32_t> mine = dm->dofs(c.rank);
            const int64_t nloc = (int64_t)mine.size();
            HCsr kl;
            kl.nrows = nloc, kl.ncols = nloc + rp.nT;
            kl.ptr.assign(1, 0);
            for (int64_t i = 0; i < nloc; i++) {
                const int32_t d = mine[(size_t)i];
                if (tof[d] < 0)
                    for (int64_t p = K.ptr[d]; p < K.ptr[d + 1]; p++) {
                        const int32_t g = K.ind[p];
                        kl.ind.push_back(tof[g] >= 0 ? (int32_t)(nloc + tof[g]) : dm->lidx[g]);
                        kl.val.push_back(devnum ? (double)(p + 1) : K.val[p]);
                    }
                kl.ptr.push_back((int64_t)kl.ind.size());
            }
            make_dmat(kl, pc->dKpl);
            pc->dKpl.nloc = nloc;  // columns >= nloc: wT
            pc->tkr = true;
        }
        if (want_sched && coupled && (rp.nT == 0 || pc->tkr)) {
            // the subtree rows' Kp rows in schedule order, entries in Kp's order (so each row sum
            // is the residual SpMV's); columns: schedule positions, T dofs nsub + t
            const int64_t nsub = rp.nsub;
            const std::vector<int32_t> mine = dm->dofs(c.rank);
            std::vector<int32_t> spos(mine.size(), -1), lrow((size_t)nsub);
            for (int64_t q = 0; q < nsub; q++) {
                lrow[q] = rp.Fsub.perm[S.order[q]];
                spos[(size_t)lrow[q]] = (int32_t)q;
            }
            HCsr ks;
            ks.nrows = nsub, ks.ncols = nsub + rp.nT;
            ks.ptr.assign((size_t)nsub + 1, 0);
            for (int64_t q = 0; q < nsub; q++) {
                const int32_t d = mine[(size_t)lrow[q]];
                ks.ptr[q + 1] = ks.ptr[q] + (K.ptr[d + 1] - K.ptr[d]);
            }
            ks.ind.resize((size_t)ks.ptr[nsub]);
            ks.val.resize((size_t)ks.ptr[nsub]);
            std::atomic<bool> bad{false};
            parallel_for(nsub, [&](int64_t lo, int64_t hi) {
                for (int64_t q = lo; q < hi; q++) {
                    const int32_t d = mine[(size_t)lrow[q]];
                    int64_t t = ks.ptr[q];
                    for (int64_t p = K.ptr[d]; p < K.ptr[d + 1]; p++, t++) {
                        const int32_t g = K.ind[p];
                        const int32_t col = tof[g] >= 0 ? (int32_t)(nsub + tof[g]) : spos[(size_t)dm->lidx[g]];
                        if (col < 0) bad = true;
                        ks.ind[t] = col;
                        ks.val[t] = devnum ? (double)(p + 1) : K.val[p];
                    }
                }
            }, 1 << 14);
            if (bad) throw Error(CPK_ERR_FACTOR, "internal: a subtree row's Kp row leaves its rank");
            make_dmat(ks, pc->dKpsl);
            if (pc->tkr) {
                std::vector<int32_t> h2((size_t)std::max<int64_t>(nsub, 1), -1);
                for (int64_t q = 0; q < nsub; q++) h2[q] = hslot2[(size_t)lrow[q]];
                pc->hslot2s.upload(h2);
            }
            pc->xs.alloc((size_t)std::max<int64_t>(nsub, 1));
            pc->dsched = true;
            // the refinement residual fused into the round-0 forward sweep (launch_sptrsv_fwd_resid)
            pc->fused_resid = pc->dF.round0_rows >= 0 && pc->dF.fcol16.n > 0;
            // no separator: the last round's forward and backward meet in one launch, as on one GPU
            pc->dF.fuse_last = !c.opts.no_fuse_last && rp.nT == 0;
        }
    }
    sub.lap("dist: refinement without the Kp halo");
    T.nT = rp.nT, T.kt = rp.kt, T.nlev = (int64_t)rp.tlev_ptr.size() - 1, T.ntdof = (int64_t)rp.tdof.size();
    T.tsolve_global = c.opts.tsolve_global;
    T.kt_data = kt1 > 0 ? kt1 - kSepPiggy : 0;
    if (pc->tkr) pc->hslot2.upload(hslot2), pc->tkr_ptr.upload(tkr_ptr), pc->tkr_col.upload(tkr_col), pc->tkr_val.upload(tkr_val);
    T.tf_src.upload(rp.tf_src), T.DT.upload(rp.DT), T.tdof.upload(rp.tdof);
    dsep_stage(T, rp);
    // a T the stepped solve cannot hold (LDS, step table) goes through the block sweeps
    if (T.nT > 0 && (c.opts.tsolve_sweep || !sep_steps_fit(T))) dsep_sweep_setup(c, T, rp, c.nranks);
    T.sbuf.alloc((size_t)std::max<int64_t>(T.kt, 1));
    T.sbuf.zero(c.stream);
    T.rbuf.alloc((size_t)std::max<int64_t>(T.kt * c.nranks + (T.tsweep ? T.nT : 0), 1));
    sub.lap("dist: separator solve data");
    // refinement residual rows of Kp with their halo
    std::vector<int32_t> kp_send;
    if (devnum) {
        // index-valued Kp (entry q -> q + 1) in place of the values for the slice, then back
        std::vector<double> idx(an.Kp.val.size());
        parallel_for((int64_t)idx.size(), [&](int64_t lo, int64_t hi) {
            for (int64_t q = lo; q < hi; q++) idx[q] = (double)(q + 1);
        }, 1 << 16);
        std::swap(an.Kp.val, idx);
        DistCsr dk;
        try {
            dk = dist_csr(an.Kp, *dm, c.rank, false);
        } catch (...) {
            std::swap(an.Kp.val, idx);
            throw;
        }
        std::swap(an.Kp.val, idx);
        kp_send = dk.send;
        make_dist_dmat(dk, c.nranks, pc->dKp);
    } else {
        DistCsr dk = dist_csr(an.Kp, *dm, c.rank, false);
        kp_send = dk.send;
        make_dist_dmat(dk, c.nranks, pc->dKp);
    }
    {   // the backward sweep's write-back (and, at the T dofs of rank 0, the separator solve's)
        // packs the residual's Kp halo: output index -> slot
        std::vector<int32_t> hs((size_t)std::max<int64_t>(pc->N, 1), -1);
        for (size_t i = 0; i < kp_send.size(); i++) hs[kp_send[i]] = (int32_t)i;
        if (!kp_send.empty()) pc->hslot.upload(hs);
    }
    sub.lap("dist: Kp slice");
    clk.lap("rank plan + upload");
    if (devnum) {
        auto add = [&](DBuf<double> &x, int src) {
            if (!x.n) return;
            Precond::VMap m;
            m.dst = x.p, m.n = x.n, m.src = src;
            vmap_capture(c, x.p, x.n, m.map);
            pc->vmaps.push_back(std::move(m));
        };
        add(pc->dF.fval, 0), add(pc->dF.bval, 0), add(pc->dF.D, 1);
        add(T.DT, 1), add(T.tk_val, 0), add(T.tr_val, 0), add(T.rec_v, 0);
        add(T.tsw.fval, 0), add(T.tsw.bval, 0), add(T.tsw.D, 1);
        add(pc->dKp.val, 2);
        add(pc->dKpl.val, 2), add(pc->tkr_val, 2), add(pc->dKpsl.val, 2);
        dldl_setup(pc->dl, an.sym, an.F0, {}, {}, {});
        pc->kpg.upload(an.Kp.val);
        dldl_numeric(c, pc->dl, pc->kpg.p, pc->dl.Lx.p, pc->dl.D.p);
        pc->fill_vmaps();
        CPK_HIP(hipStreamSynchronize(c.stream));
        an.F0.Lx.clear(), an.F0.D.clear();  // the exported values come from the device (dl)
        clk.lap("numeric factorization (device, whole system) + value maps");
    }
    pc->Kp = std::move(an.Kp);
    pc->S = std::move(S);
    pc->F = std::move(an.F0);
    pc->dofmap = dm;
    an.F = Factor();
    pc->w.alloc((size_t)std::max<int64_t>(pc->nsub + T.nT, 1));
    pc->r.alloc((size_t)std::max<int64_t>(std::max<int64_t>(pc->N, pc->nsub + T.nT), 1));  // dsched: a work vector
    pc->active.alloc(1);
    c.ensure_partials(std::max<size_t>(pc->dKp.nblk * 2, 4096));
    CPK_HIP(hipDeviceSynchronize());
    pc->ptime = an.seconds + std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return pc.release();
}

// FNV-1a over the dimensions, the pattern and the value bits of the three blocks
static uint64_t input_hash(const HCsr &A11, const HCsr &B, const HCsr &C22) {
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](uint64_t v) { h = (h ^ v) * 1099511628211ull; };
    for (const HCsr *a : {&A11, &B, &C22}) {
        mix((uint64_t)a->nrows), mix((uint64_t)a->ncols);
        for (int64_t v : a->ptr) mix((uint64_t)v);
        for (int32_t v : a->ind) mix((uint32_t)v);
        for (double v : a->val) {
            uint64_t u;
            std::memcpy(&u, &v, sizeof u);
            mix(u);
        }
    }
    return h;
}

// The global analysis of a distributed preconditioner, once: rank 0 runs it and broadcasts the
// parts every rank's plan and device factorization read (Kp, the exported factor's structure,
// the device phase's symbolic data), field by field straight from and into the vectors; the
// other ranks skip the ordering and the symbolic factorization (S50 at P = 8: ~3.9 s of host
// work and its memory peak, 8 times over on one node's cores).  Each rank still hashes its own
// inputs into the plan agreement, so ranks given different matrices fail as before.  A failure
// on rank 0 travels with the broadcast: every rank throws its message.
namespace {
struct AnalysisBcast {
    Comm &cm;
    hipStream_t s;
    // a receiver that cannot hold a field (allocation failure) keeps taking part in every later
    // broadcast, discarding the bytes, so rank 0 never waits for it; the ranks then agree
    // (analyze_dist) and every one of them fails with the same error
    bool failed = false;
    std::string why;
    template <class T>
    void pod(T &v) { cm.broadcast_host(&v, sizeof v, 0, s); }
    template <class T>
    void vec(std::vector<T> &v) {
        uint64_t n = v.size();
        pod(n);
        if (!failed) {
            try {
                v.resize((size_t)n);
            } catch (const std::exception &e) {
                failed = true, why = e.what();
                std::vector<T>().swap(v);
            }
        }
        if (n) cm.broadcast_host(failed ? nullptr : v.data(), (size_t)n * sizeof(T), 0, s);
    }
    void run(Analysis &an) {
        pod(an.n), pod(an.m), pod(an.N), pod(an.ordering), pod(an.seconds), pod(an.sweep);
        uint8_t dn = an.device_numeric ? 1 : 0;
        pod(dn);
        an.device_numeric = dn != 0;
        pod(an.Kp.nrows), pod(an.Kp.ncols), vec(an.Kp.ptr), vec(an.Kp.ind), vec(an.Kp.val);
        pod(an.F0.N), vec(an.F0.perm), vec(an.F0.Lp), vec(an.F0.Li), vec(an.F0.Lx), vec(an.F0.D), vec(an.F0.parent);
        LdlSymbolic &y = an.sym;
        pod(y.N), vec(y.Rp), vec(y.Rc), vec(y.Rcsc), vec(y.kp_ptr), vec(y.kp_tgt), vec(y.kp_src), vec(y.lev_ptr),
            vec(y.lev_rows);
        vec(an.rsrc);
    }
};
}  // namespace

// every rank's vote (all must agree to broadcast: a rank that analyzes on its own while the
// others wait in a broadcast would never meet them)
static bool all_ranks(Ctx &c, bool mine) {
    DBuf<double> snd, rcv;
    snd.alloc(1), rcv.alloc((size_t)c.nranks);
    const double v = mine ? 1.0 : 0.0;
    CPK_HIP(hipMemcpy(snd.p, &v, sizeof v, hipMemcpyHostToDevice));
    c.comm->allgather(snd.p, rcv.p, 1, c.stream);
    std::vector<double> all((size_t)c.nranks);
    CPK_HIP(hipMemcpyAsync(all.data(), rcv.p, rcv.bytes(), hipMemcpyDeviceToHost, c.stream));
    CPK_HIP(hipStreamSynchronize(c.stream));
    for (double a : all)
        if (a != 1.0) return false;
    return true;
}

static Analysis analyze_dist(Ctx &c, const HCsr &A11, const HCsr &B, const HCsr &C22, bool dev) {
    Analysis an;
    if (c.nranks <= 1 || !c.comm->has_peers() || !all_ranks(c, !c.opts.no_bcast_analysis)) {
        an = analyze(A11, B, C22, c.opts, dev, {}, false);
    } else {
        const auto t0 = std::chrono::steady_clock::now();
        PhaseClock pcl("precond_create_dist");
        std::string err;
        if (c.rank == 0) {
            try {
                an = analyze(A11, B, C22, c.opts, dev, {}, false);
            } catch (const std::exception &e) {
                err = e.what();
                if (err.empty()) err = "analysis failed";
            }
        }
        AnalysisBcast bc{*c.comm, c.stream};
        std::vector<char> msg(err.begin(), err.end());
        bc.vec(msg);
        err.assign(msg.begin(), msg.end());
        if (!err.empty()) throw Error(CPK_ERR_ARGS, "distributed preconditioner (analysis on rank 0): " + err);
        pcl.lap(c.rank == 0 ? "global analysis (rank 0)" : "rank 0's global analysis (waiting)");
        try {
            bc.run(an);
        } catch (...) {
            c.comm->release_staging();
            throw;
        }
        c.comm->release_staging();
        if (!all_ranks(c, !bc.failed))
            throw Error(CPK_ERR_NOMEM, "distributed preconditioner: a rank could not hold rank 0's analysis" +
                                           (bc.failed ? " (this rank: " + bc.why + ")" : std::string()));
        if (c.rank != 0) an.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        pcl.lap("analysis broadcast from rank 0");
    }
    an.input_hash = input_hash(A11, B, C22);
    return an;
}

Precond *precond_create_dist(Ctx &c, const HCsr &A11, const HCsr &B, const HCsr &C22, const HCsr *Akry) {
    const bool dev = !c.opts.host_factor;
    // each rank schedules its own subtrees: no schedule of the whole system
    Precond *pc = precond_create_dist(c, analyze_dist(c, A11, B, C22, dev), Akry);
    pc->pattern_hash = pattern_hash(A11, B, C22);
    if (dev) pc->dl.kp_from.upload(kp_value_sources(A11, B, C22));
    return pc;
}

void Precond::fill_vmaps() {
    for (const VMap &m : vmaps)
        vmap_fill(*ctx, m.map.p, m.n, m.src == 0 ? dl.Lx.p : (m.src == 1 ? dl.D.p : kpg.p), m.dst);
}

uint64_t pattern_hash(const HCsr &A11, const HCsr &B, const HCsr &C22) {
    uint64_t h = 1469598103934665603ull;  // FNV-1a over the dimensions, row pointers and columns
    auto mix = [&](uint64_t v) { h = (h ^ v) * 1099511628211ull; };
    for (const HCsr *a : {&A11, &B, &C22}) {
        mix((uint64_t)a->nrows), mix((uint64_t)a->ncols);
        for (int64_t v : a->ptr) mix((uint64_t)v);
        for (int32_t v : a->ind) mix((uint32_t)v);
    }
    return h;
}

// Single GPU: the host does the symbolic analysis, the device the numeric factorization
// (engine option host_factor: host numeric, the reference path of the device one's parity tests).
Precond *precond_create(Ctx &c, const HCsr &A11, const HCsr &B, const HCsr &C22) {
    const bool dev = !c.opts.host_factor;
    // the refactorization's inputs (Kp's value sources, the sparsity hash) depend only on the
    // matrices: computed on a second host thread during the analysis, once the dimensions are
    // known to be consistent (kp_value_sources indexes by them)
    check_kp_dims(A11, B, C22);
    std::vector<int64_t> src;
    uint64_t hash = 0;
    std::exception_ptr side_err;
    std::thread side([&] {
        try {
            if (dev) src = kp_value_sources(A11, B, C22);
            hash = pattern_hash(A11, B, C22);
        } catch (...) {
            side_err = std::current_exception();
        }
    });
    // Kp and the device factorization's symbolic data are uploaded while the host builds the
    // schedule
    PrecondPre pre;
    SymbolicHook hook;
    if (dev)
        hook = [&](const HCsr &Kp, const Factor &f, const LdlSymbolic &sym) {
            CPK_HIP(hipSetDevice(c.device));
            dldl_setup_sym(pre.dl, sym, f);
            make_dmat(Kp, pre.dKp);
            pre.kp = true;
        };
    Analysis an;
    try {
        an = analyze(A11, B, C22, c.opts, dev, hook);
    } catch (...) {
        side.join();
        throw;
    }
    side.join();
    if (side_err) std::rethrow_exception(side_err);
    Precond *pc = precond_create(c, std::move(an), dev ? &pre : nullptr);
    pc->pattern_hash = hash;
    if (dev) pc->dl.kp_from.upload(src);
    return pc;
}

double precond_refactor(Precond &p, const DMat &A11, const DMat &B, const DMat &C22) {
    if (!p.dl.ready)
        throw Error(CPK_ERR_UNSUPPORTED, "refactorization needs the device factorization (engine option host_factor off)");
    auto t0 = std::chrono::steady_clock::now();
    Ctx &c = *p.ctx;
    if (p.dist) {
        // every rank refactors the whole system (as at construction) into scratch, then commits
        // its maps' values; collective-free, so each rank's result is the single-GPU one
        DBuf<double> kpv, Lx, D;
        kpv.alloc(std::max<size_t>(p.kpg.n, 1));
        Lx.alloc(p.dl.Lx.n);
        D.alloc(p.dl.D.n);
        dldl_assemble_kp(c, p.dl, A11.val.p, B.val.p, C22.val.p, kpv.p);
        dldl_numeric(c, p.dl, kpv.p, Lx.p, D.p);
        if (p.kpg.n) CPK_HIP(hipMemcpyAsync(p.kpg.p, kpv.p, p.kpg.bytes(), hipMemcpyDeviceToDevice, c.stream));
        CPK_HIP(hipMemcpyAsync(p.dl.Lx.p, Lx.p, Lx.bytes(), hipMemcpyDeviceToDevice, c.stream));
        CPK_HIP(hipMemcpyAsync(p.dl.D.p, D.p, D.bytes(), hipMemcpyDeviceToDevice, c.stream));
        p.fill_vmaps();
        if (!p.Kp.val.empty())
            CPK_HIP(hipMemcpyAsync(p.Kp.val.data(), p.kpg.p, p.Kp.val.size() * sizeof(double), hipMemcpyDeviceToHost,
                                   c.stream));
        CPK_HIP(hipStreamSynchronize(c.stream));
        // the shift's B' rows were built from the host Kp: rebuilt on next use (with the solvers
        // whose captured graphs may reference them)
        for (auto it = p.dist_ops.begin(); it != p.dist_ops.end();)
            it = std::get<0>(it->first) == 'B' ? p.dist_ops.erase(it) : std::next(it);
        p.solvers.clear();
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        p.ptime = s;
        return s;
    }
    // all or nothing: the new Kp and factor are formed in scratch buffers; a bad pivot throws
    // before anything the preconditioner holds (Kp, Kps, L, D, the sweep values) is touched
    DBuf<double> kpv, Lx, D;
    kpv.alloc((size_t)std::max<int64_t>(p.dKp.nnz, 1));
    Lx.alloc(p.dl.Lx.n);
    D.alloc(p.dl.D.n);
    dldl_assemble_kp(c, p.dl, A11.val.p, B.val.p, C22.val.p, kpv.p);
    dldl_numeric(c, p.dl, kpv.p, Lx.p, D.p);
    // commit (copies, not buffer swaps: captured solver graphs hold these addresses)
    if (p.dKp.nnz) CPK_HIP(hipMemcpyAsync(p.dKp.val.p, kpv.p, p.dKp.val.bytes(), hipMemcpyDeviceToDevice, c.stream));
    CPK_HIP(hipMemcpyAsync(p.dl.Lx.p, Lx.p, Lx.bytes(), hipMemcpyDeviceToDevice, c.stream));
    CPK_HIP(hipMemcpyAsync(p.dl.D.p, D.p, D.bytes(), hipMemcpyDeviceToDevice, c.stream));
    if (p.dKps.nnz) launch_gather(c, p.dKp.val.p, p.kps_from.p, p.dKps.nnz, p.dKps.val.p);
    dldl_fill(c, p.dl, p.dF);
    // a rebuilt opLDL2 starts with op.Aty = op.Cy = 0 (opLDL2.m:90-91): so does the handle state
    if (p.handle && p.ghn.n) p.ghn.zero(c.stream);
    // the host copy of Kp follows (divide / export read the device copies; the distributed
    // shift rows, built from the host copy, do not exist on one GPU)
    if (!p.Kp.val.empty())
        CPK_HIP(hipMemcpyAsync(p.Kp.val.data(), p.dKp.val.p, p.Kp.val.size() * sizeof(double), hipMemcpyDeviceToHost,
                               c.stream));
    CPK_HIP(hipStreamSynchronize(c.stream));
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    p.ptime = s;
    return s;
}

// y (=|+=) LDL * xin: forward sweep, [distributed: separator exchange + solve], backward sweep
bool Precond::ldl_solve(const double *xin, int64_t neg_from, double *y, bool add, const int *run,
                        const int *act, const double *piggy_src, int stage, const double *xT, int64_t xT_neg) {
    Ctx &c = *ctx;
    FwdIn last;  // single GPU: the last round forward + backward in one launch (sptrsv_last_kernel)
    if (!dist) {
        launch_sptrsv_fwd(c, dF, xin, neg_from, w.p, run, act, false, nullptr, &last);
        launch_sptrsv_bwd(c, dF, w.p, y, add, run, act, nullptr, &last);
        return false;
    }
    // distributed: the sweeps' write-back packs the separator payload (forward) and the Kp halo
    // of y (backward), so neither needs a gather launch
    // stage 2 (tkr): rank 0 sends the apply's own T inputs +-x (the T rows' residual is formed
    // from them after the exchange), not the refinement input's
    const double *xt = stage == 2 ? xT : xin;
    const int64_t xt_neg = stage == 2 ? xT_neg : neg_from;
    const PackArgs fp = fwd_pack(xt, xt_neg, piggy_src);
    const bool fpacked = launch_sptrsv_fwd(c, dF, xin, neg_from, w.p, run, act, false, nullptr, nullptr,
                                           sep.tslot.n ? &fp : nullptr);
    launch_sep_exchange(c, sep, w.p, xt, xt_neg, piggy_src, fpacked);
    const bool hpack = stage == 0 && hslot.n;
    launch_sep_solve(c, sep, w.p + nsub, y, add, run, act, hpack ? hslot.p : nullptr, dKp.sbuf.p,
                     stage == 2 ? tkr_ptr.p : nullptr, tkr_col.p, tkr_val.p);
    PackArgs bp;
    if (hpack) bp.slot = hslot.p, bp.buf = dKp.sbuf.p;
    if (stage == 1) bp.slot = hslot2.p, bp.buf = sep.sbuf.p;  // y of the rows T's Kp rows read
    return launch_sptrsv_bwd(c, dF, w.p, y, add, run, act, nullptr, nullptr, (hpack || stage == 1) ? &bp : nullptr);
}

// the forward sweep's separator payload: its rows' values by tslot, rank 0's T inputs +-xt[tdof]
// and the piggyback values (tpack_kernel's work, in the write-back)
PackArgs Precond::fwd_pack(const double *xt, int64_t xt_neg, const double *piggy_src) const {
    PackArgs fp;
    if (sep.tslot.n) {
        fp.slot = sep.tslot.p, fp.buf = sep.sbuf.p, fp.tdof = sep.tdof.p, fp.ntdof = (int)sep.ntdof;
        fp.nsend = (int)sep.nsend, fp.kt_data = (int)sep.kt_data, fp.x = xt, fp.neg_from = xt_neg;
        fp.piggy = piggy_src;
    }
    return fp;
}

// y = M*x with one forced refinement step, distributed, in schedule order:
// the single-GPU apply's kernels plus a separator exchange and solve inside each LDL solve.
//   solve 1: forward sweep (captures the signed input xs, packs the payload), exchange, separator
//            solve (rank 0: y at the T dofs), backward sweep kept in schedule order in w (packs the
//            subtree values T's Kp rows read into the payload's extra slots, hslot2s);
//   solve 2: r = xs - Kpsl*w fused into the forward sweep (w holds the subtree rows and T), the
//            exchange, the separator solve forming the T rows' residual x_T - Kp_T*y itself and
//            accumulating rank 0's T dofs, and the backward sweep writing y = P*(w + dy).
// Every row sums in the order of the single-GPU path: bit-identical to it and to the oracle.
void Precond::dist_sched_apply(const double *x, int64_t neg_from, double *y, const int *run,
                               const double *piggy_src) {
    Ctx &c = *ctx;
    const bool pk = sep.tslot.n > 0;
    FwdIn last;  // no separator (sep.nT == 0): the last round fused as on one GPU
    const PackArgs fp1 = fwd_pack(x, neg_from, piggy_src);
    const bool f1 = launch_sptrsv_fwd(c, dF, x, neg_from, w.p, run, nullptr, false, xs.p, &last, pk ? &fp1 : nullptr);
    launch_sep_exchange(c, sep, w.p, x, neg_from, piggy_src, f1);
    launch_sep_solve(c, sep, w.p + nsub, y, false, run, nullptr);
    PackArgs bp;
    if (hslot2s.n) bp.slot = hslot2s.p, bp.buf = sep.sbuf.p;
    const bool b1 = launch_sptrsv_bwd(c, dF, w.p, nullptr, false, run, nullptr, nullptr, &last, hslot2s.n ? &bp : nullptr);
    if (hslot2s.n && !b1) launch_pack_slots(c, hslot2s.p, nsub, w.p, sep.sbuf.p, run);
    // solve 2: rank 0 sends the apply's own T inputs (the T rows' residual is formed from them)
    const PackArgs fp2 = fwd_pack(x, neg_from, nullptr);
    bool f2 = false;
    FwdIn last2;
    if (!(fused_resid && launch_sptrsv_fwd_resid(c, dF, dKpsl, xs.p, w.p, r.p, run, &last2, pk ? &fp2 : nullptr, &f2))) {
        launch_spmv_resid_sched(c, dKpsl, nullptr, xs.p, 0, w.p, r.p, run);  // r = x - op.A*y (subtree rows)
        f2 = launch_sptrsv_fwd(c, dF, r.p, N, r.p, run, nullptr, true, nullptr, &last2, pk ? &fp2 : nullptr);
    }
    launch_sep_exchange(c, sep, r.p, x, neg_from, nullptr, f2);
    launch_sep_solve(c, sep, r.p + nsub, y, true, run, nullptr, nullptr, nullptr, tkr ? tkr_ptr.p : nullptr, tkr_col.p,
                     tkr_val.p, w.p + nsub);
    launch_sptrsv_bwd(c, dF, r.p, y, true, run, nullptr, w.p, &last2, nullptr, true);  // y = P*(ys + dy); r dead
}

void Precond::set_handle(bool on) {
    if (on && dist) throw Error(CPK_ERR_UNSUPPORTED, "handle semantics of the residual update: single-GPU only");
    handle = on;
    if (on) {
        if (ghn.n < (size_t)N) ghn.alloc(N), t.alloc(N);
        ghn.zero(ctx->stream);
        CPK_HIP(hipStreamSynchronize(ctx->stream));
    }
}

void Precond::apply(const double *x, int64_t neg_from, double *y, const int *run, const double *piggy_src) {
    Ctx &c = *ctx;
    bool have_xs = false;  // the first forward sweep left the signed x in schedule order (xs)
    bool hpacked = false;  // distributed: y's Kp halo packed by the last backward sweep
    if (residual_update != 0 && handle) {
        // y = op.LDL * [x(1:n) - op.Aty; x(n+1:N) - op.Cy]; then op.Aty = op.A(1:n, n+1:N) * y2,
        // op.Cy = op.A(n+1:N, n+1:N) * y2 = the columns n+1:N of Kp times y2  (opLDL2.m:164-172)
        launch_sub_state(c, x, neg_from, ghn.p, N, t.p, run);
        ldl_solve(t.p, N, y, false, run, nullptr, piggy_src);
        launch_spmv_colmask(c, dKp, n, y, ghn.p, run);
    } else if (nitref >= 1 && force_itref != 0 && sched_path()) {
        // y = op.LDL * x kept in schedule order (w) for the refinement below: no scatter; the
        // forward sweep also leaves the signed input in schedule order (xs) for the residual
        FwdIn last;
        launch_sptrsv_fwd(c, dF, x, neg_from, w.p, run, nullptr, false, xs.n ? xs.p : nullptr, &last);
        have_xs = xs.n > 0;
        launch_sptrsv_bwd(c, dF, w.p, nullptr, false, run, nullptr, nullptr, &last);
    } else if (dist && dsched && steps1_forced()) {
        dist_sched_apply(x, neg_from, y, run, piggy_src);
        return;
    } else if (dist && tkr && steps1_forced()) {
        // distributed, one forced refinement step, no Kp halo exchange (Precond::tkr): y = LDL*x
        // packs the y values the T rows' residual needs into the separator payload; the local
        // rows' residual reads T's values from wT; the refinement solve forms the T rows' own
        ldl_solve(x, neg_from, y, false, run, nullptr, piggy_src, 1);
        launch_spmv_resid_loc(c, dKpl, x, neg_from, y, r.p, run, w.p + nsub);  // r = x - op.A*y
        ldl_solve(r.p, N, y, true, run, nullptr, nullptr, 2, x, neg_from);    // y = y + op.LDL*r
        return;
    } else {
        // y = op.LDL * x   (opLDL2.m:165-167); the residual-update branch subtracts the zero
        // state of a value object and its SpMVs are dead: skipped
        hpacked = ldl_solve(x, neg_from, y, false, run, nullptr, piggy_src);
    }
    if (nitref <= 0) return;
    const int64_t steps = (int64_t)nitref;
    if (force_itref != 0 && sched_path()) {
        // every step runs and the norms are dead; everything stays in schedule order until the
        // last backward sweep scatters y = P * (ys + dy)
        for (int64_t s = 0; s < steps; s++) {
            // r = x - op.A*y; the refinement solve runs in place on r (each row reads its own
            // input before it writes); y += op.LDL*r
            FwdIn last;
            if (!(have_xs && (fused_resid && launch_sptrsv_fwd_resid(c, dF, dKps, xs.p, w.p, r.p, run, &last)))) {
                if (have_xs) launch_spmv_resid_sched(c, dKps, nullptr, xs.p, 0, w.p, r.p, run);
                else launch_spmv_resid_sched(c, dKps, dF.perm.p, x, neg_from, w.p, r.p, run);
                launch_sptrsv_fwd(c, dF, r.p, N, r.p, run, nullptr, true, nullptr, &last);
            }
            // r is formed again by the next step's residual: its round-0 rows are not stored back
            launch_sptrsv_bwd(c, dF, r.p, s + 1 == steps ? y : nullptr, true, run, nullptr, w.p, &last, nullptr, true);
        }
        return;
    }
    if (force_itref != 0) {
        // every step runs; rNorm/xNorm and the final residual are dead
        for (int64_t s = 0; s < steps; s++) {
            launch_spmv_resid(c, dKp, x, neg_from, y, r.p, run, nullptr, hpacked);  // r = x - op.A*y
            hpacked = ldl_solve(r.p, N, y, true, run, nullptr);                    // y = y + op.LDL*r
        }
        return;
    }
    // data-dependent refinement: the predicate lives on the device, kernels test it
    launch_spmv_resid_norm(c, dKp, x, neg_from, y, r.p, itref_tol, active.p, run, nullptr, hpacked);
    for (int64_t s = 0; s < steps; s++) {
        // a skipped step (active == 0) leaves y and its packed halo as they were
        hpacked = ldl_solve(r.p, N, y, true, run, active.p);
        if (s + 1 < steps)
            launch_spmv_resid_norm(c, dKp, x, neg_from, y, r.p, itref_tol, active.p, run, active.p, hpacked);
    }
}

double Precond::apply_bytes() const {
    const double ghn_bytes = (residual_update != 0 && handle)
                                 ? 32.0 * N + 12.0 * (double)dKp.nnz + 4.0 * (N + 1) + 16.0 * N : 0.0;
    // SpTRSV sweep over the strict factor (l entries): 12*l + 4*(N+1) + 16*N (vector in/out)
    // + 4*N (perm) ; backward adds D (8*N) and the scatter (8*N, +8*N when accumulating).
    const double l = (double)dF.nnz, Nn = (double)N;
    const double fwd = 12 * l - 2 * (double)dF.nnz16 + 4 * (Nn + 1) + 16 * Nn + 4 * Nn;  // fcol16: 10 B per entry
    const double bwd = 12 * l + 4 * (Nn + 1) + 16 * Nn + 4 * Nn + 8 * Nn + 8 * Nn;
    const double kp = 12 * (double)dKp.nnz + 4 * (Nn + 1) + 8 * Nn /*y*/ + 8 * Nn /*x*/ + 8 * Nn /*r*/;
    const int64_t steps = nitref > 0 ? (int64_t)nitref : 0;
    const DMat &Ks = dist ? dKpsl : dKps;  // distributed: the rank's subtree rows (dist_sched_apply)
    if (steps && force_itref != 0 && (sched_path() || (dsched && steps1_forced())) && !(residual_update != 0 && handle)) {
        // schedule-order path: the first backward sweep keeps its solution (no perm, no
        // scatter); the residual gathers x through perm; the refinement forward sweeps read it
        // contiguously (no perm); each refinement backward sweep reads ys contiguously and only
        // the last scatters
        const double bwd_keep = 12 * l + 4 * (Nn + 1) + 16 * Nn + 8 * Nn;
        const double kps = 12 * (double)Ks.nnz + 4 * (Nn + 1) + 8 * Nn /*y*/ +
                           (xs.n ? 8 * Nn /*xs*/ : 12 * Nn /*x(perm)*/) + 8 * Nn /*r*/;
        const double fwd_s = 12 * l - 2 * (double)dF.nnz16 + 4 * (Nn + 1) + 16 * Nn;
        const double dead = 8.0 * (double)dF.bwd_dead_w_rows();  // round 0's w, not stored back
        const double bwd_acc = 12 * l + 4 * (Nn + 1) + 16 * Nn + 8 * Nn + 8 * Nn /*ys*/ - dead;
        double b = fwd + (xs.n ? 8 * Nn : 0.0) /*xs written*/ + bwd_keep + steps * (kps + fwd_s + bwd_acc) + (4 + 8) * Nn /*last: perm + scatter*/ +
                   (steps - 1) * 8.0 * Nn /*ys written back in place*/;
        // fused refinement input (launch_sptrsv_fwd_resid): r is neither written nor read back
        if (xs.n && fused_resid && dF.pipelined && !dF.no_fused_resid)
            b -= steps * 16.0 * Nn;
        return b;
    }
    double b = fwd + bwd;
    b += steps * (kp + fwd + bwd + 8 * Nn);
    return b + ghn_bytes;
}

}  // namespace cpk
