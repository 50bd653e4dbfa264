// factor.cpp -- static-pivot sparse LDL' of the constraint preconditioner (replaces MATLAB's
// [L,D,P] = ldl(op.A), ops/opLDL2.m:82) and the block/round schedule for the device
// triangular sweeps that replace op.LDL = P*inv(L')*inv(D)*inv(L)*P' (ops/opLDL2.m:86).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <atomic>
#include <cstdlib>
#include <memory>
#include <numeric>
#include <thread>

#include "cpk.h"
#include "host.hpp"

namespace cpk {

// Up-looking (row-by-row) LDL': row k of L is the solution of a sparse triangular system
// whose pattern is the reach of row k's entries in the elimination tree (the up-looking
// algorithm of T. A. Davis, "Direct Methods for Sparse Linear Systems", SIAM 2006, sec. 4.7 /
// LDL: ldl_symbolic, ldl_numeric).  Here the reach of each row is visited in ascending column
// order (a topological order of the row's triangular solve) instead of the stack order, so a
// device thread walking the sorted row pattern performs the same operations in the same order.
// Symbolic phase only (the device runs the numeric one), threaded.  The same outputs as the
// serial loop below with numeric == false: the elimination tree by Liu's algorithm with path
// compression (cs_etree), then every row's pattern -- the union of the tree paths from its Kp
// entries up to the row, sorted ascending -- rows in parallel (each thread stamps its own
// marker array), then the columns of L by a parallel transpose that keeps each column's rows
// ascending (the serial loop's order).
static Factor ldl_symbolic_threaded(const HCsr &Kp, const std::vector<int32_t> &perm, LdlSymbolic &sym) {
    const int64_t N = Kp.nrows;
    Factor f;
    f.N = N;
    f.perm = perm;
    std::vector<int32_t> pinv(N);
    for (int64_t k = 0; k < N; k++) pinv[perm[k]] = (int32_t)k;
    f.parent.assign(N, -1);
    {
        std::vector<int32_t> anc(N, -1);
        for (int64_t k = 0; k < N; k++) {
            const int32_t r = perm[k];
            for (int64_t p = Kp.ptr[r]; p < Kp.ptr[r + 1]; p++) {
                int32_t i = pinv[Kp.ind[p]];
                while (i != -1 && i < k) {
                    const int32_t nx = anc[i];
                    anc[i] = (int32_t)k;
                    if (nx == -1) f.parent[i] = (int32_t)k;
                    i = nx;
                }
            }
        }
    }
    // row patterns and seeds, rows in parallel chunks
    const int T = std::max(1, std::min<int>(host_threads(), (int)((N + 65535) / 65536)));
    struct Chunk {
        std::vector<int32_t> rc, tgt;
        std::vector<uint32_t> src;
        std::vector<int32_t> rcnt, scnt;  // per row: pattern length, seed count
    };
    std::vector<Chunk> ch(T);
    const int64_t cs = (N + T - 1) / T;
    std::vector<std::thread> th;
    auto work = [&](int t) {
        const int64_t lo = t * cs, hi = std::min<int64_t>(N, lo + cs);
        Chunk &c = ch[t];
        c.rcnt.resize(std::max<int64_t>(hi - lo, 0)), c.scnt.resize(std::max<int64_t>(hi - lo, 0));
        std::vector<int32_t> flag(N, -1), pat;  // one marker array per thread (N int32)
        for (int64_t k = lo; k < hi; k++) {
            flag[k] = (int32_t)k;
            pat.clear();
            const int32_t r = perm[k];
            for (int64_t p = Kp.ptr[r]; p < Kp.ptr[r + 1]; p++)
                for (int32_t i = pinv[Kp.ind[p]]; i < k && flag[i] != k; i = f.parent[i]) {
                    pat.push_back(i);
                    flag[i] = (int32_t)k;
                }
            std::sort(pat.begin(), pat.end());
            c.rc.insert(c.rc.end(), pat.begin(), pat.end());
            c.rcnt[k - lo] = (int32_t)pat.size();
            int32_t ns = 0;
            for (int64_t p = Kp.ptr[r]; p < Kp.ptr[r + 1]; p++) {
                const int32_t i = pinv[Kp.ind[p]];
                if (i > k) continue;
                // row-local slot of i in the sorted pattern (rebased later)
                c.tgt.push_back(i == k ? -1 : (int32_t)(std::lower_bound(pat.begin(), pat.end(), i) - pat.begin()));
                c.src.push_back((uint32_t)p);
                ns++;
            }
            c.scnt[k - lo] = ns;
        }
    };
    for (int t = 1; t < T; t++) th.emplace_back(work, t);
    work(0);
    for (auto &x : th) x.join();
    sym.N = N;
    sym.Rp.assign(N + 1, 0);
    sym.kp_ptr.assign(N + 1, 0);
    for (int t = 0; t < T; t++)
        for (size_t q = 0; q < ch[t].rcnt.size(); q++) {
            const int64_t k = t * cs + (int64_t)q;
            sym.Rp[k + 1] = sym.Rp[k] + ch[t].rcnt[q];
            sym.kp_ptr[k + 1] = sym.kp_ptr[k] + ch[t].scnt[q];
        }
    if ((int64_t)sym.Rp[N] > INT32_MAX || sym.kp_ptr[N] < 0)
        throw Error(CPK_ERR_NOMEM, "factor too large for 32-bit entry offsets");
    const int64_t nnz = sym.Rp[N];
    {
        // the large outputs are zero-filled on threads of their own: the first touch of fresh
        // pages (kernel faults) is the cost of a resize, and it runs in parallel this way
        std::vector<std::thread> al;
        al.emplace_back([&] { sym.Rc.resize(nnz); });
        al.emplace_back([&] { sym.kp_tgt.resize(sym.kp_ptr[N]); });
        al.emplace_back([&] { sym.kp_src.resize(sym.kp_ptr[N]); });
        al.emplace_back([&] { f.Li.resize(nnz); });
        al.emplace_back([&] { f.Lp.assign(N + 1, 0); });
        sym.Rcsc.resize(nnz);
        for (auto &x : al) x.join();
    }
    {
        std::vector<std::thread> cp;
        auto copy = [&](int t) {
            const int64_t k0 = t * cs;
            if (ch[t].rcnt.empty()) return;
            std::copy(ch[t].rc.begin(), ch[t].rc.end(), sym.Rc.begin() + sym.Rp[k0]);
            // seeds: row-local slots -> row-entry slots
            int64_t o = sym.kp_ptr[k0];
            for (size_t q = 0; q < ch[t].rcnt.size(); q++) {
                const int32_t base = sym.Rp[k0 + (int64_t)q];
                for (int32_t s = 0; s < ch[t].scnt[q]; s++, o++) {
                    const int32_t tg = ch[t].tgt[o - sym.kp_ptr[k0]];
                    sym.kp_tgt[o] = tg < 0 ? -1 : base + tg;
                    sym.kp_src[o] = ch[t].src[o - sym.kp_ptr[k0]];
                }
            }
            std::vector<int32_t>().swap(ch[t].rc);
        };
        for (int t = 1; t < T; t++) cp.emplace_back(copy, t);
        copy(0);
        for (auto &x : cp) x.join();
    }
    // columns of L: rows in ascending order within each column (the serial loop's lnz[i]++ order)
    parallel_for(nnz, [&](int64_t lo, int64_t hi) {  // column counts: a histogram, order-free
        for (int64_t q = lo; q < hi; q++) __atomic_fetch_add(&f.Lp[sym.Rc[q] + 1], (int64_t)1, __ATOMIC_RELAXED);
    }, 1 << 18);
    for (int64_t i = 0; i < N; i++) f.Lp[i + 1] += f.Lp[i];
    {
        // a parallel transpose: thread t owns the row range rcut[t] .. rcut[t+1) and the column
        // range ccut[t] .. ccut[t+1) (equal entry counts each).  Every thread sorts its rows'
        // entries into one bucket per column owner (row entries in ascending row order); each
        // owner then places its buckets in thread order, so a column's rows stay ascending: the
        // placement of the serial lnz[i]++ loop, with each entry visited three times in all
        // rather than once per thread
        std::vector<int64_t> ccut(T + 1, N), rcut(T + 1, N);
        ccut[0] = rcut[0] = 0;
        for (int t = 1; t < T; t++) {
            ccut[t] = std::upper_bound(f.Lp.begin(), f.Lp.end(), nnz * t / T) - f.Lp.begin() - 1;
            rcut[t] = std::upper_bound(sym.Rp.begin(), sym.Rp.end(), (int32_t)(nnz * t / T)) - sym.Rp.begin() - 1;
        }
        std::vector<uint8_t> owner(N);
        for (int t = 0; t < T; t++) std::fill(owner.begin() + ccut[t], owner.begin() + ccut[t + 1], (uint8_t)t);
        // bucket (t, u): row entries q of thread t's rows whose column thread u owns
        std::vector<std::vector<int64_t>> boff(T, std::vector<int64_t>(T + 1, 0));
        std::vector<std::vector<int32_t>> bq(T);  // thread t's entries, grouped by owner
        std::vector<std::thread> cth;
        auto bucket = [&](int t) {
            const int32_t q0 = sym.Rp[rcut[t]], q1 = sym.Rp[rcut[t + 1]];
            std::vector<int64_t> &o = boff[t];
            for (int32_t q = q0; q < q1; q++) o[owner[sym.Rc[q]] + 1]++;
            for (int u = 0; u < T; u++) o[u + 1] += o[u];
            std::vector<int64_t> nx(o.begin(), o.end() - 1);
            bq[t].resize((size_t)(q1 - q0));
            for (int32_t q = q0; q < q1; q++) bq[t][nx[owner[sym.Rc[q]]]++] = q;
        };
        auto place = [&](int u) {
            const int64_t c0 = ccut[u];
            std::vector<int64_t> nx(f.Lp.begin() + c0, f.Lp.begin() + ccut[u + 1]);
            for (int t = 0; t < T; t++) {  // row ranges ascending, rows ascending within each
                int64_t k = rcut[t];
                for (int64_t s = boff[t][u]; s < boff[t][u + 1]; s++) {
                    const int32_t q = bq[t][s];
                    while (sym.Rp[k + 1] <= q) k++;
                    const int64_t p2 = nx[sym.Rc[q] - c0]++;
                    f.Li[p2] = (int32_t)k;
                    sym.Rcsc[q] = (int32_t)p2;
                }
            }
        };
        for (int t = 1; t < T; t++) cth.emplace_back(bucket, t);
        bucket(0);
        for (auto &x : cth) x.join();
        cth.clear();
        for (int u = 1; u < T; u++) cth.emplace_back(place, u);
        place(0);
        for (auto &x : cth) x.join();
    }
    return f;
}

static void height_levels(const Factor &f, LdlSymbolic *sym);

Factor ldl_factor(const HCsr &Kp, const std::vector<int32_t> &perm, int /*nthreads*/, LdlSymbolic *sym,
                  bool numeric) {
    if (!numeric && sym && Kp.nrows > 0) {
        Factor f = ldl_symbolic_threaded(Kp, perm, *sym);
        height_levels(f, sym);
        return f;
    }
    const int64_t N = Kp.nrows;
    Factor f;
    f.N = N;
    f.perm = perm;
    std::vector<int32_t> pinv(N);
    for (int64_t k = 0; k < N; k++) pinv[perm[k]] = (int32_t)k;
    f.parent.assign(N, -1);
    std::vector<int32_t> flag(N);
    std::vector<int64_t> lnz(N, 0);
    // symbolic: etree + column counts
    for (int64_t k = 0; k < N; k++) {
        flag[k] = (int32_t)k;
        const int32_t r = perm[k];
        for (int64_t p = Kp.ptr[r]; p < Kp.ptr[r + 1]; p++) {
            int32_t i = pinv[Kp.ind[p]];
            if (i >= k) continue;
            for (; flag[i] != k; i = f.parent[i]) {
                if (f.parent[i] == -1) f.parent[i] = (int32_t)k;
                lnz[i]++;
                flag[i] = (int32_t)k;
            }
        }
    }
    f.Lp.assign(N + 1, 0);
    for (int64_t k = 0; k < N; k++) f.Lp[k + 1] = f.Lp[k] + lnz[k];
    if (f.Lp[N] > INT32_MAX) throw Error(CPK_ERR_NOMEM, "factor too large for 32-bit entry offsets");
    const int64_t nnz = f.Lp[N];
    f.Li.resize(nnz);
    if (numeric) f.Lx.resize(nnz), f.D.resize(N);
    if (sym) {
        sym->N = N;
        sym->Rp.assign(N + 1, 0);
        sym->Rc.resize(nnz);
        sym->Rcsc.resize(nnz);
        sym->kp_ptr.assign(N + 1, 0);
        sym->kp_tgt.clear();
        sym->kp_src.clear();
        sym->kp_tgt.reserve((size_t)(Kp.nnz() / 2 + N));
        sym->kp_src.reserve((size_t)(Kp.nnz() / 2 + N));
    }
    std::vector<double> y(numeric ? N : 0, 0.0);
    std::vector<int32_t> pattern(N), slot(sym ? N : 0);
    std::fill(lnz.begin(), lnz.end(), 0);
    int64_t rpos = 0;
    for (int64_t k = 0; k < N; k++) {
        int64_t top = N;
        flag[k] = (int32_t)k;
        const int32_t r = perm[k];
        for (int64_t p = Kp.ptr[r]; p < Kp.ptr[r + 1]; p++) {
            int32_t i = pinv[Kp.ind[p]];
            if (i > k) continue;
            if (numeric) y[i] += Kp.val[p];
            int64_t len = 0;
            for (; flag[i] != k; i = f.parent[i]) {
                pattern[len++] = i;
                flag[i] = (int32_t)k;
            }
            while (len > 0) pattern[--top] = pattern[--len];
        }
        std::sort(pattern.begin() + top, pattern.end());
        if (sym) {
            for (int64_t q = top; q < N; q++) slot[pattern[q]] = (int32_t)(rpos + (q - top));
            for (int64_t p = Kp.ptr[r]; p < Kp.ptr[r + 1]; p++) {
                const int32_t i = pinv[Kp.ind[p]];
                if (i > k) continue;
                sym->kp_tgt.push_back(i == k ? -1 : slot[i]);
                sym->kp_src.push_back((uint32_t)p);
            }
            sym->kp_ptr[k + 1] = (int32_t)sym->kp_tgt.size();
        }
        double d = numeric ? y[k] : 0.0;
        if (numeric) y[k] = 0.0;
        for (; top < N; top++) {
            const int32_t i = pattern[top];
            const int64_t p2 = f.Lp[i] + lnz[i];
            if (numeric) {
                const double yi = y[i];
                y[i] = 0.0;
                for (int64_t p = f.Lp[i]; p < p2; p++) y[f.Li[p]] -= f.Lx[p] * yi;
                const double lki = yi / f.D[i];
                d -= lki * yi;
                f.Lx[p2] = lki;
            }
            f.Li[p2] = (int32_t)k;
            if (sym) sym->Rc[rpos] = i, sym->Rcsc[rpos] = (int32_t)p2, rpos++;
            lnz[i]++;
        }
        if (sym) sym->Rp[k + 1] = (int32_t)rpos;
        if (!numeric) continue;
        if (d == 0.0 || !(d == d))
            throw Error(CPK_ERR_FACTOR, "ldl: zero or NaN pivot at position " + std::to_string(k) +
                                            " (static 1x1 pivoting needs G > 0 on the nullspace and C > 0)");
        f.D[k] = d;
    }
    if (sym) height_levels(f, sym);
    return f;
}

// rows by elimination-tree height: a row depends only on its descendants
static void height_levels(const Factor &f, LdlSymbolic *sym) {
    const int64_t N = f.N;
    {
        if (sym->kp_tgt.size() > (size_t)INT32_MAX) throw Error(CPK_ERR_NOMEM, "too many Kp entries for the device factorization");
        std::vector<int32_t> h(N, 0);
        int32_t hmax = 0;
        for (int64_t v = 0; v < N; v++) {
            if (f.parent[v] >= 0) h[f.parent[v]] = std::max(h[f.parent[v]], h[v] + 1);
            hmax = std::max(hmax, h[v]);
        }
        sym->lev_ptr.assign((size_t)hmax + 2, 0);
        for (int64_t v = 0; v < N; v++) sym->lev_ptr[h[v] + 1]++;
        for (int32_t l = 0; l <= hmax; l++) sym->lev_ptr[l + 1] += sym->lev_ptr[l];
        sym->lev_rows.resize(N);
        std::vector<int32_t> nx(sym->lev_ptr.begin(), sym->lev_ptr.end() - 1);
        for (int64_t v = 0; v < N; v++) sym->lev_rows[nx[h[v]]++] = (int32_t)v;
    }
}

Schedule build_schedule(const Factor &f, int64_t R0, int64_t CAP0, int64_t R1, int64_t CAP1, int64_t SUB0,
                        const std::vector<int64_t> *extra_bwd, const std::vector<int64_t> *extra_fwd) {
    if (SUB0 <= 0 || SUB0 > CAP0) SUB0 = CAP0;
    const int64_t N = f.N;
    SubClock clk;
    Schedule s;
    s.N = N;
    // Node weights: a block is staged in LDS when it holds at most R rows, at most CAP forward
    // entries (rows of L) and at most CAP backward entries (columns of L).  With
    // wt(v) = max(CAP/R, fwd(v), bwd(v)), a cluster of total weight <= CAP meets all three.
    std::vector<int32_t> ent(N), nfwd(N, 0);  // nfwd: forward entries (row counts of L)
    parallel_for((int64_t)f.Li.size(), [&](int64_t lo, int64_t hi) {  // a histogram: order-free
        for (int64_t p = lo; p < hi; p++) __atomic_fetch_add(&nfwd[f.Li[p]], 1, __ATOMIC_RELAXED);
    }, 1 << 18);
    parallel_for(N, [&](int64_t lo, int64_t hi) {
        for (int64_t v = lo; v < hi; v++)
            ent[v] = (int32_t)std::max<int64_t>(nfwd[v] + (extra_fwd ? (*extra_fwd)[v] : 0),
                                                f.Lp[v + 1] - f.Lp[v] + (extra_bwd ? (*extra_bwd)[v] : 0));
    });
    const int64_t u0 = std::max<int64_t>(1, CAP0 / std::max<int64_t>(R0, 1));
    const int64_t u1 = std::max<int64_t>(1, CAP1 / std::max<int64_t>(R1, 1));
    auto wt0 = [&](int64_t v) { return std::max<int64_t>(u0, ent[v]); };
    auto wt1 = [&](int64_t v) { return std::max<int64_t>(u1, ent[v]); };
    auto capof = [&](int32_t r) { return r == 0 ? CAP0 : CAP1; };
    // children lists and the tree height (for reporting), one ascending pass each
    std::vector<int32_t> cptr(N + 2, 0), height(N, 0);
    for (int64_t v = 0; v < N; v++) {
        const int32_t p = f.parent[v];
        if (p >= 0) cptr[p + 1]++, height[p] = std::max(height[p], height[v] + 1);
        s.depth = std::max<int64_t>(s.depth, height[v] + 1);
    }
    for (int64_t v = 0; v < N; v++) cptr[v + 1] += cptr[v];
    std::vector<int32_t> kids(cptr[N]);
    {
        std::vector<int32_t> nx(cptr.begin(), cptr.begin() + N);
        for (int64_t v = 0; v < N; v++)
            if (f.parent[v] >= 0) kids[nx[f.parent[v]]++] = (int32_t)v;
    }
    std::vector<int32_t>().swap(height);
    clk.lap("schedule: weights, children, heights");
    std::vector<int32_t> closed_round(N, -1);  // >= 0 iff v roots a cluster
    // (1) Layer peeling: round r takes the maximal subtrees of at most R rows of the tree that
    //     remains after rounds 0..r-1.  On bushy (nested-dissection) trees the remainder
    //     shrinks geometrically and a few rounds suffice.
    std::vector<int32_t> alive(N);
    for (int64_t v = 0; v < N; v++) alive[v] = (int32_t)v;
    std::vector<char> is_alive(N, 1);
    // per round, written for every alive row before any read (the parent of an alive row is alive)
    std::unique_ptr<int64_t[]> sz(new int64_t[N]);
    std::unique_ptr<int32_t[]> root_of(new int32_t[N]);
    int32_t round = 0;
    while (!alive.empty()) {
        for (int32_t v : alive) sz[v] = 0;
        const int64_t u = round == 0 ? u0 : u1;
        // round 0 peels subtrees of weight <= SUB0 and packs several of them per block
        const int64_t CAP = round == 0 ? SUB0 : capof(round);
        for (int32_t v : alive) {  // ascending: children before parents
            sz[v] += std::max<int64_t>(u, ent[v]);
            if (f.parent[v] >= 0 && is_alive[f.parent[v]]) sz[f.parent[v]] += sz[v];
        }
        const size_t before = alive.size();
        for (size_t q = alive.size(); q-- > 0;) {  // descending: parents before children
            const int32_t v = alive[q], p = f.parent[v];
            if (sz[v] > CAP) root_of[v] = -1;
            else if (p < 0 || sz[p] > CAP) root_of[v] = v, closed_round[v] = round;
            else root_of[v] = root_of[p];
        }
        std::vector<int32_t> rest;
        rest.reserve(alive.size());
        for (int32_t v : alive) {
            if (root_of[v] >= 0) is_alive[v] = 0;
            else rest.push_back(v);
        }
        alive.swap(rest);
        round++;
        if (!alive.empty() && round >= 8 && alive.size() * 2 > before) break;  // chain-like tree
    }
    clk.lap("schedule: layer peeling");
    // (2) Greedy bottom-up clustering of what peeling left (chain-like upper trees): a node's
    //     open cluster absorbs its children's open clusters, closing the largest ones until it
    //     fits in R rows.  Peeled children are already-closed clusters.
    // read only for alive nodes (a peeled row's parent is peeled too), each written before its
    // parent reads it: no initialisation
    std::unique_ptr<int64_t[]> open_size(new int64_t[N]);
    std::unique_ptr<int32_t[]> open_dep(new int32_t[N]);
    std::vector<int32_t> tmp;
    const int64_t CAP = CAP1;
    for (int32_t v : alive) {
        int64_t total = wt1(v);
        tmp.clear();
        for (int64_t q = cptr[v]; q < cptr[v + 1]; q++)
            if (closed_round[kids[q]] < 0) tmp.push_back(kids[q]), total += open_size[kids[q]];
        if (total > CAP) {
            std::sort(tmp.begin(), tmp.end(), [&](int32_t a, int32_t b) {
                return open_size[a] != open_size[b] ? open_size[a] > open_size[b] : a < b;
            });
            for (int32_t c : tmp) {
                if (total <= CAP) break;
                closed_round[c] = open_dep[c] + 1;
                total -= open_size[c];
            }
        }
        int32_t dep = -1;
        for (int64_t q = cptr[v]; q < cptr[v + 1]; q++) {
            const int32_t c = kids[q];
            dep = std::max(dep, closed_round[c] >= 0 ? closed_round[c] : open_dep[c]);
        }
        open_size[v] = total;
        open_dep[v] = dep;
        if (f.parent[v] < 0) closed_round[v] = dep + 1;
    }
    // cluster membership (top-down): a non-root joins its parent's cluster
    // and the cluster sizes (a root comes before its members, so it starts its sum)
    std::vector<int32_t> cl(N, -1);
    std::unique_ptr<int64_t[]> csize(new int64_t[N]);
    int32_t nrounds = 0;
    for (int64_t v = N - 1; v >= 0; v--) {
        if (closed_round[v] >= 0) nrounds = std::max(nrounds, closed_round[v] + 1);
        const bool root = closed_round[v] >= 0;
        const int32_t c = root ? (int32_t)v : cl[f.parent[v]];
        cl[v] = c;
        const int64_t w = closed_round[c] == 0 ? wt0(v) : wt1(v);
        csize[c] = root ? w : csize[c] + w;
    }
    clk.lap("schedule: clustering");
    // pack the clusters of one round into blocks of <= R rows (clusters taken in root order)
    std::vector<std::vector<int32_t>> roots_by_round(nrounds);
    for (int64_t v = 0; v < N; v++)
        if (closed_round[v] >= 0) roots_by_round[closed_round[v]].push_back((int32_t)v);
    int32_t *cluster_block = root_of.get();  // free after the peeling; read for cluster roots only
    int32_t nb = 0;
    s.round_ptr.assign(1, 0);
    for (int32_t r = 0; r < nrounds; r++) {
        const int64_t cap = capof(r);
        int64_t fill = cap + 1;
        for (int32_t c : roots_by_round[r]) {
            if (fill + csize[c] > cap) {
                nb++;
                fill = 0;
            }
            cluster_block[c] = nb - 1;
            fill += csize[c];
        }
        s.round_ptr.push_back(nb);
    }
    // new order: blocks ascending (= rounds ascending), then level, then old index
    std::vector<int32_t> block(N);
    std::vector<int64_t> bcount(nb + 1, 0);
    for (int64_t v = 0; v < N; v++) {
        block[v] = cluster_block[cl[v]];
        bcount[block[v] + 1]++;
    }
    for (int32_t b = 0; b < nb; b++) bcount[b + 1] += bcount[b];
    s.blk_row.assign(bcount.begin(), bcount.end());
    s.order.resize(N);
    {
        std::vector<int64_t> nx(bcount.begin(), bcount.end() - 1);
        for (int64_t v = 0; v < N; v++) s.order[nx[block[v]]++] = (int32_t)v;
    }
    clk.lap("schedule: blocks and order");
    // intra-block levels, blocks in parallel: a block's rows are disjoint from every other
    // block's, and in ascending old index (a topological order: L's columns point to rows of
    // larger index), so level[j] is final when column j is visited
    std::vector<int32_t> level(N, 0);
    parallel_for(nb, [&](int64_t lo, int64_t hi) {
        for (int64_t b = lo; b < hi; b++)
            for (int64_t q = s.blk_row[b]; q < s.blk_row[b + 1]; q++) {
                const int32_t j = s.order[q];
                for (int64_t p = f.Lp[j]; p < f.Lp[j + 1]; p++) {
                    const int32_t i = f.Li[p];
                    if (block[i] == block[j]) level[i] = std::max(level[i], level[j] + 1);
                }
            }
    }, 64);
    s.blk_lvl.assign(1, 0);
    s.lvl_row.clear();
    parallel_for(nb, [&](int64_t lo, int64_t hi) {  // blocks sort independently
        for (int64_t b = lo; b < hi; b++)
            std::stable_sort(s.order.begin() + s.blk_row[b], s.order.begin() + s.blk_row[b + 1],
                             [&](int32_t a, int32_t c) { return level[a] < level[c]; });
    }, 256);
    for (int32_t b = 0; b < nb; b++) {
        int32_t prev = -1;
        for (int64_t q = s.blk_row[b]; q < s.blk_row[b + 1]; q++) {
            const int32_t l = level[s.order[q]];
            if (l != prev) s.lvl_row.push_back(q), prev = l;
        }
        s.blk_lvl.push_back((int64_t)s.lvl_row.size());
        s.max_levels = std::max<int64_t>(s.max_levels, s.blk_lvl[b + 1] - s.blk_lvl[b]);
    }
    s.lvl_row.push_back(N);
    clk.lap("schedule: intra-block levels");
    return s;
}

Factor relabel(const Factor &f, const Schedule &s, std::vector<int32_t> *src) {
    const int64_t N = f.N;
    std::vector<int32_t> pos(N);
    parallel_for(N, [&](int64_t lo, int64_t hi) {  // order is a permutation: disjoint writes
        for (int64_t q = lo; q < hi; q++) pos[s.order[q]] = (int32_t)q;
    }, 1 << 16);
    Factor g;
    g.N = N;
    g.perm.resize(N);
    if (!f.D.empty()) g.D.resize(N);
    g.parent.resize(N);
    parallel_for(N, [&](int64_t lo, int64_t hi) {
        for (int64_t q = lo; q < hi; q++) {
            int32_t old = s.order[q];
            g.perm[q] = f.perm[old];
            if (!f.D.empty()) g.D[q] = f.D[old];
            g.parent[q] = f.parent[old] >= 0 ? pos[f.parent[old]] : -1;
        }
    }, 1 << 16);
    g.Lp.assign(N + 1, 0);
    for (int64_t q = 0; q < N; q++) {
        int32_t old = s.order[q];
        g.Lp[q + 1] = g.Lp[q] + (f.Lp[old + 1] - f.Lp[old]);
    }
    const bool vals = (int64_t)f.D.size() == N;  // numeric factor (Lx may be empty: no entries)
    {
        std::vector<std::thread> al;  // zero-fills (first touch of fresh pages) side by side
        if (vals) al.emplace_back([&] { g.Lx.resize(f.Lx.size()); });
        if (src) al.emplace_back([&] { src->resize(f.Li.size()); });
        g.Li.resize(f.Li.size());
        for (auto &x : al) x.join();
    }
    std::atomic<bool> bad{false};
    parallel_for(N, [&](int64_t lo, int64_t hi) {  // columns relabel independently
        std::vector<std::pair<int32_t, int64_t>> col;
        for (int64_t q = lo; q < hi; q++) {
            int32_t old = s.order[q];
            const int64_t len = f.Lp[old + 1] - f.Lp[old];
            if (len <= 32) {  // short columns: insertion sort in place (new indices are distinct)
                const int64_t b = g.Lp[q];
                int64_t sp[32];
                for (int64_t t = 0; t < len; t++) {
                    const int64_t p = f.Lp[old] + t;
                    const int32_t r = pos[f.Li[p]];
                    int64_t u = t;
                    for (; u > 0 && g.Li[b + u - 1] > r; u--) g.Li[b + u] = g.Li[b + u - 1], sp[u] = sp[u - 1];
                    g.Li[b + u] = r, sp[u] = p;
                }
                for (int64_t t = 0; t < len; t++) {
                    if (g.Li[b + t] <= q) bad = true;
                    if (vals) g.Lx[b + t] = f.Lx[sp[t]];
                    if (src) (*src)[b + t] = (int32_t)sp[t];
                }
                continue;
            }
            col.clear();
            for (int64_t p = f.Lp[old]; p < f.Lp[old + 1]; p++) col.emplace_back(pos[f.Li[p]], p);
            std::sort(col.begin(), col.end(), [](auto &a, auto &b) { return a.first < b.first; });
            for (size_t t = 0; t < col.size(); t++) {
                if (col[t].first <= q) bad = true;
                g.Li[g.Lp[q] + t] = col[t].first;
                if (vals) g.Lx[g.Lp[q] + t] = f.Lx[col[t].second];
                if (src) (*src)[g.Lp[q] + t] = (int32_t)col[t].second;
            }
        }
    });
    if (bad) throw Error(CPK_ERR_FACTOR, "internal: relabel is not topological");
    return g;
}

}  // namespace cpk
