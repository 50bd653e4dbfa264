// ordering.cpp -- fill-reducing symmetric orderings for the constraint preconditioner Kp.
//
// MATLAB's ldl() (ops/opLDL2.m:82) picks its own (MA57) ordering and 2x2 pivots; neither can
// be reproduced, and only the exact solve with Kp matters for the Krylov iterates.  Kp is
// symmetric quasi-definite for G > 0, C_user > 0, so an LDL' with 1x1 pivots exists for every
// symmetric ordering.  The ordering is chosen for fill AND for triangular-solve parallelism:
//   - G diagonal (every example and synthetic case): eliminate the G block first (its nodes
//     are independent leaves), then order the Schur-complement graph S = pattern(C + B G^-1 B')
//     by nested dissection (large) or minimum degree (small);
//   - otherwise nested dissection / minimum degree on the whole graph of Kp.
#include <algorithm>
#include <cstdio>
#include <atomic>
#include <cstdlib>
#include <memory>
#include <thread>
#include <cstring>
#include <numeric>
#include <queue>
#include <set>

#include "cpk.h"
#include "host.hpp"

namespace cpk {

static constexpr int64_t kMdLimit = 60000;  // exact minimum degree up to this many nodes
static constexpr int kNdLeaf = 4;

// symmetric adjacency graph (no self loops, sorted unique neighbours) from undirected edges:
// bucketed by endpoint, then each row sorted and deduplicated on its own
static HCsr graph_from_edges(int64_t nv, std::vector<std::pair<int32_t, int32_t>> &edges) {
    std::vector<int64_t> cnt(nv + 1, 0);
    for (auto &e : edges)
        if (e.first != e.second) cnt[e.first + 1]++, cnt[e.second + 1]++;
    for (int64_t i = 0; i < nv; i++) cnt[i + 1] += cnt[i];
    std::vector<int32_t> adj(cnt[nv]);
    {
        std::vector<int64_t> nx(cnt.begin(), cnt.end() - 1);
        for (auto &e : edges)
            if (e.first != e.second) adj[nx[e.first]++] = e.second, adj[nx[e.second]++] = e.first;
    }
    edges.clear();
    edges.shrink_to_fit();
    std::vector<int64_t> deg(nv, 0);
    parallel_for(nv, [&](int64_t lo, int64_t hi) {
        for (int64_t i = lo; i < hi; i++) {
            auto b0 = adj.begin() + cnt[i], b1 = adj.begin() + cnt[i + 1];
            std::sort(b0, b1);
            deg[i] = std::unique(b0, b1) - b0;
        }
    });
    HCsr g;
    g.nrows = g.ncols = nv;
    g.ptr.assign(nv + 1, 0);
    for (int64_t i = 0; i < nv; i++) g.ptr[i + 1] = g.ptr[i] + deg[i];
    g.ind.resize(g.ptr[nv]);
    parallel_for(nv, [&](int64_t lo, int64_t hi) {
        for (int64_t i = lo; i < hi; i++) std::copy(adj.begin() + cnt[i], adj.begin() + cnt[i] + deg[i], g.ind.begin() + g.ptr[i]);
    });
    return g;
}

// The Schur-complement graph on the m constraint rows of Kp (G diagonal): the clique of each G
// column's B entries plus C's pattern, the graph graph_from_edges builds from those edges.  Its
// neighbour lists end sorted and unique, so the order in which entries land does not matter:
// threads count and place theirs concurrently (relaxed atomic slots), with no edge list.
static HCsr schur_graph(const HCsr &Kp, int64_t n, int64_t m) {
    std::vector<int64_t> cnt(m + 1, 0);
    auto cliques = [&](auto &&add) {
        parallel_for(n, [&](int64_t lo, int64_t hi) {
            int32_t nb[64];
            std::vector<int32_t> big;
            for (int64_t j = lo; j < hi; j++) {
                int k = 0;
                big.clear();
                for (int64_t p = Kp.ptr[j]; p < Kp.ptr[j + 1]; p++)
                    if (Kp.ind[p] >= n) {
                        if (k < 64) nb[k] = Kp.ind[p] - (int32_t)n;
                        else big.push_back(Kp.ind[p] - (int32_t)n);
                        k++;
                    }
                auto at = [&](int t) { return t < 64 ? nb[t] : big[t - 64]; };
                for (int a = 0; a < k; a++)
                    for (int b = a + 1; b < k; b++)
                        if (at(a) != at(b)) add(at(a), at(b)), add(at(b), at(a));
            }
        }, 1 << 16);
        parallel_for(m, [&](int64_t lo, int64_t hi) {
            for (int64_t i = lo; i < hi; i++)
                for (int64_t p = Kp.ptr[n + i]; p < Kp.ptr[n + i + 1]; p++) {
                    const int32_t c = Kp.ind[p];
                    if (c >= n && c - n != i) add((int32_t)i, c - (int32_t)n), add(c - (int32_t)n, (int32_t)i);
                }
        }, 1 << 16);
    };
    cliques([&](int32_t u, int32_t) { __atomic_fetch_add(&cnt[u + 1], (int64_t)1, __ATOMIC_RELAXED); });
    for (int64_t i = 0; i < m; i++) cnt[i + 1] += cnt[i];
    std::vector<int32_t> adj(cnt[m]);
    {
        std::vector<int64_t> nx(cnt.begin(), cnt.end() - 1);
        cliques([&](int32_t u, int32_t v) { adj[__atomic_fetch_add(&nx[u], (int64_t)1, __ATOMIC_RELAXED)] = v; });
    }
    std::vector<int64_t> deg(m, 0);
    parallel_for(m, [&](int64_t lo, int64_t hi) {
        for (int64_t i = lo; i < hi; i++) {
            auto b0 = adj.begin() + cnt[i], b1 = adj.begin() + cnt[i + 1];
            std::sort(b0, b1);
            deg[i] = std::unique(b0, b1) - b0;
        }
    });
    HCsr g;
    g.nrows = g.ncols = m;
    g.ptr.assign(m + 1, 0);
    for (int64_t i = 0; i < m; i++) g.ptr[i + 1] = g.ptr[i] + deg[i];
    g.ind.resize(g.ptr[m]);
    parallel_for(m, [&](int64_t lo, int64_t hi) {
        for (int64_t i = lo; i < hi; i++) std::copy(adj.begin() + cnt[i], adj.begin() + cnt[i] + deg[i], g.ind.begin() + g.ptr[i]);
    });
    return g;
}

// Exact minimum degree on the explicit elimination graph; ties broken by lowest index.
std::vector<int32_t> min_degree(const HCsr &g) {
    const int64_t nv = g.nrows;
    std::vector<std::vector<int32_t>> adj(nv);
    for (int64_t i = 0; i < nv; i++)
        for (int64_t p = g.ptr[i]; p < g.ptr[i + 1]; p++)
            if (g.ind[p] != i) adj[i].push_back(g.ind[p]);
    std::set<std::pair<int64_t, int32_t>> pq;
    for (int64_t i = 0; i < nv; i++) pq.insert({(int64_t)adj[i].size(), (int32_t)i});
    std::vector<char> dead(nv, 0);
    std::vector<int32_t> order;
    order.reserve(nv);
    std::vector<int32_t> mark(nv, -1), merged;
    while (!pq.empty()) {
        int32_t v = pq.begin()->second;
        pq.erase(pq.begin());
        dead[v] = 1;
        order.push_back(v);
        std::vector<int32_t> nb;
        for (int32_t u : adj[v])
            if (!dead[u]) nb.push_back(u);
        for (int32_t u : nb) {
            pq.erase({(int64_t)adj[u].size(), u});
            // adj[u] <- (adj[u] U nb) \ {u, v, dead}
            merged.clear();
            for (int32_t w : adj[u])
                if (!dead[w] && mark[w] != u) mark[w] = u, merged.push_back(w);
            for (int32_t w : nb)
                if (w != u && mark[w] != u) mark[w] = u, merged.push_back(w);
            adj[u].swap(merged);
            pq.insert({(int64_t)adj[u].size(), u});
        }
        adj[v].clear();
        adj[v].shrink_to_fit();
    }
    return order;
}

// ---- nested dissection by BFS level structures (George-Liu) ------------------------------
// The two halves of a dissection are independent, so large halves are ordered on their own
// threads.  Every subset writes its nodes to its own precomputed range of the output (half A,
// then half B, then the separator), and every decision depends only on the subset itself, so
// the ordering is the same for any number of threads.
namespace {
struct Nd {
    const HCsr &g;
    std::unique_ptr<std::atomic<int32_t>[]> label;  // subset id of each node
    // BFS distance and visit stamp of each node, twice: the pseudo-peripheral search keeps the
    // best start's BFS in one copy while it tries a candidate in the other
    std::vector<int32_t> dist_[2], stamp_[2];
    std::vector<int32_t> &dist = dist_[0], &stamp = stamp_[0];
    std::vector<int32_t> out;
    // Subset labels only need to be unique: each thread draws them from a block of its own (one
    // shared atomic per kLabelBlock labels).  Visit stamps only need to grow along a node's
    // chain of subsets (a subset's BFS stamps exceed every stamp its ancestors left on its
    // nodes; disjoint subsets never see each other's), so each subset counts them on from the
    // value its parent reached: no shared counter, the same decisions
    static constexpr int32_t kLabelBlock = 1 << 12;
    std::atomic<int32_t> next_block{1};
    const uint64_t gen = [] {
        static std::atomic<uint64_t> g{1};
        return g.fetch_add(1);
    }();  // which dissection a thread's block belongs to
    int32_t new_label() {
        thread_local uint64_t owner = 0;
        thread_local int32_t next = 0, end = 0;
        if (owner != gen || next == end) {
            owner = gen;
            next = next_block.fetch_add(kLabelBlock, std::memory_order_relaxed);
            end = next + kLabelBlock;
        }
        return next++;
    }
    std::atomic<int> spare_threads;
    int leaf;
    Nd(const HCsr &gg, int lf, int threads)
        : g(gg), label(new std::atomic<int32_t>[gg.nrows]), dist_{std::vector<int32_t>(gg.nrows, 0), std::vector<int32_t>(gg.nrows, 0)},
          stamp_{std::vector<int32_t>(gg.nrows, -1), std::vector<int32_t>(gg.nrows, -1)}, out(gg.nrows),
          spare_threads(threads - 1), leaf(lf) {
        for (int64_t i = 0; i < gg.nrows; i++) label[i].store(0, std::memory_order_relaxed);
    }
    int32_t lab_of(int32_t v) const { return label[v].load(std::memory_order_relaxed); }
    void set_lab(int32_t v, int32_t l) { label[v].store(l, std::memory_order_relaxed); }

    // BFS within nodes of `lab` from `src`; fills `bfs` in visit order, returns eccentricity.
    // Nodes of other subsets (possibly relabelled concurrently by another thread) never carry
    // `lab`, so reading their labels is harmless.
    int32_t bfs(int32_t src, int32_t lab, std::vector<int32_t> &bfs_order, int32_t &st, int32_t &ctr, int buf = 0) {
        std::vector<int32_t> &dst = dist_[buf], &stm = stamp_[buf];
        st = ++ctr;
        bfs_order.clear();
        bfs_order.push_back(src);
        stm[src] = st;
        dst[src] = 0;
        for (size_t h = 0; h < bfs_order.size(); h++) {
            int32_t v = bfs_order[h];
            for (int64_t p = g.ptr[v]; p < g.ptr[v + 1]; p++) {
                int32_t w = g.ind[p];
                if (lab_of(w) != lab || stm[w] == st) continue;
                stm[w] = st;
                dst[w] = dst[v] + 1;
                bfs_order.push_back(w);
            }
        }
        return dst[bfs_order.back()];
    }

    void emit(std::vector<int32_t> &nodes, int64_t pos) {
        std::sort(nodes.begin(), nodes.end());
        for (int32_t v : nodes) out[pos++] = v;
    }

    // a and b in parallel when both are large and a thread is spare
    template <class FA, class FB>
    void both(size_t na, FA fa, FB fb) {
        if (na > 20000 && spare_threads.fetch_sub(1) > 0) {
            std::thread t(fa);
            fb();
            t.join();
            spare_threads.fetch_add(1);
            return;
        }
        if (na > 20000) spare_threads.fetch_add(1);
        fa();
        fb();
    }

    // order the nodes of subset `nodes` (all carry label `lab`) into out[pos, pos + |nodes|).
    // bfs_ordered: the subset is connected and `nodes` is already its BFS order from nodes[0]
    // (the near half of a dissection: the parent's BFS restricted to it), so the component
    // search is skipped -- it would visit the same nodes in the same order
    void run(std::vector<int32_t> nodes, int32_t lab, int64_t pos, int32_t ctr, bool bfs_ordered = false) {
        // CPK_TIMING: the phases of the top subsets (at least 1/16 of the graph), on stderr
        const size_t n0 = nodes.size();
        SubClock clk;
        clk.on = clk.on && (int64_t)n0 * 16 >= g.nrows && n0 > 100000;
        int nbfs = 0;
        auto phase = [&](const char *w) {
            if (!clk.on) return;
            char buf[96];
            snprintf(buf, sizeof buf, "  nd %zu: %s (%d BFS)", n0, w, nbfs);
            clk.lap(buf);
        };
        std::vector<int32_t> order;
        order.reserve(n0);  // capacity only: no pages are touched until used, no regrowth copies
        int32_t st = 0;
        if ((int64_t)nodes.size() <= leaf) {
            emit(nodes, pos);
            return;
        }
        // split into connected components first (one linear pass over the subset)
        if (bfs_ordered) order = nodes;
        else bfs(nodes[0], lab, order, st, ctr), nbfs++;
        if (order.size() < nodes.size()) {
            std::vector<std::pair<int32_t, std::vector<int32_t>>> comps;
            const int32_t stamp0 = st;  // this subset's later BFS get newer stamps
            for (int32_t v : nodes) {
                if (lab_of(v) != lab || (stamp[v] != stamp0 && stamp[v] > stamp0)) continue;  // relabelled or seen
                int32_t c_st;
                if (stamp[v] == stamp0) {  // the component found by the first BFS
                    comps.emplace_back(new_label(), order);
                } else {
                    std::vector<int32_t> c;
                    bfs(v, lab, c, c_st, ctr);
                    comps.emplace_back(new_label(), std::move(c));
                }
                for (int32_t w : comps.back().second) set_lab(w, comps.back().first);
            }
            run_comps(comps, 0, pos, ctr);
            return;
        }
        // pseudo-peripheral node; the best start's BFS stays in buffer `cur`, so it is not redone
        int32_t start = order.back();
        int cur = 0;
        phase("components");
        int32_t ecc = bfs(start, lab, order, st, ctr, cur);
        nbfs = 1;
        for (int it = 0; it < 4; it++) {
            int32_t cand = order.back();
            std::vector<int32_t> o2;
            o2.reserve(n0);
            int32_t st2;
            int32_t e2 = bfs(cand, lab, o2, st2, ctr, 1 - cur);
            nbfs++;
            if (e2 <= ecc) break;
            ecc = e2, start = cand, order.swap(o2), st = st2, cur = 1 - cur;
        }
        const std::vector<int32_t> &dist = dist_[cur], &stamp = stamp_[cur];
        if (ecc < 2) {  // too shallow to dissect
            emit(nodes, pos);
            return;
        }
        // level sizes; split at the level reaching half of the nodes
        std::vector<int64_t> lsz(ecc + 1, 0);
        for (int32_t v : order) lsz[dist[v]]++;
        int64_t acc = 0, half = (int64_t)nodes.size() / 2;
        int32_t s = 1;
        for (int32_t l = 0; l <= ecc; l++) {
            acc += lsz[l];
            if (acc >= half) {
                s = l;
                break;
            }
        }
        s = std::max<int32_t>(1, std::min<int32_t>(s, ecc - 1));
        // separator: level-s nodes adjacent to level s+1 (the rest join part A)
        const int32_t la = new_label(), lb = new_label(), ls = new_label();
        std::vector<int32_t> a, b, sep;
        a.reserve(order.size()), b.reserve(order.size()), sep.reserve(order.size());
        for (int32_t v : order) {
            int32_t d = dist[v];
            if (d < s) a.push_back(v);
            else if (d > s) b.push_back(v);
            else {
                bool touches = false;
                for (int64_t p = g.ptr[v]; p < g.ptr[v + 1] && !touches; p++) {
                    int32_t w = g.ind[p];
                    touches = lab_of(w) == lab && stamp[w] == st && dist[w] == s + 1;
                }
                (touches ? sep : a).push_back(v);
            }
        }
        for (int32_t v : a) set_lab(v, la);
        for (int32_t v : b) set_lab(v, lb);
        for (int32_t v : sep) set_lab(v, ls);
        nodes.clear();
        nodes.shrink_to_fit();
        const int64_t pa = pos, pb = pos + (int64_t)a.size(), ps = pb + (int64_t)b.size();
        emit(sep, ps);
        phase("peripheral search");
        const size_t na = std::min(a.size(), b.size());
        // part A (levels < s, and level-s nodes without a neighbour at s + 1) is connected through
        // the BFS tree and listed in BFS order from `start`; part B may fall apart
        both(na, [&] { run(std::move(a), la, pa, ctr, true); }, [&] { run(std::move(b), lb, pb, ctr); });
    }

    // components [i, end) into consecutive output ranges starting at pos
    void run_comps(std::vector<std::pair<int32_t, std::vector<int32_t>>> &comps, size_t i, int64_t pos, int32_t ctr) {
        for (; i < comps.size(); i++) {
            const size_t sz = comps[i].second.size();
            if (i + 1 < comps.size() && sz > 20000) {
                auto &c = comps[i];
                both(sz, [&] { run(std::move(c.second), c.first, pos, ctr); },
                     [&, i] { run_comps(comps, i + 1, pos + (int64_t)sz, ctr); });
                return;
            }
            run(std::move(comps[i].second), comps[i].first, pos, ctr);
            pos += (int64_t)sz;
        }
    }
};
}  // namespace

int host_threads() {
    const char *e = getenv("CPK_THREADS");
    if (!e) e = getenv("OMP_NUM_THREADS");
    int t = e ? atoi(e) : 0;
    if (t <= 0) t = (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(t, 64));
}

std::vector<int32_t> nested_dissection(const HCsr &g, int leaf_size) {
    Nd nd(g, leaf_size, host_threads());
    std::vector<int32_t> all(g.nrows);
    std::iota(all.begin(), all.end(), 0);
    if (g.nrows) nd.run(std::move(all), 0, 0, 0);
    return std::move(nd.out);
}

std::vector<int32_t> order_kp(const HCsr &Kp, int64_t n, int *kind_out) {
    SubClock clk;
    auto sub_lap = [&](const char *what) { clk.lap(what); };
    const int64_t N = Kp.nrows, m = N - n;
    bool g_diag = true;
    for (int64_t i = 0; i < n && g_diag; i++)
        for (int64_t p = Kp.ptr[i]; p < Kp.ptr[i + 1]; p++)
            if (Kp.ind[p] < n && Kp.ind[p] != i) {
                g_diag = false;
                break;
            }
    std::vector<int32_t> perm(N);
    if (g_diag && m > 0) {
        // Schur-complement graph on the m block: cliques of each G column's B entries + C pattern
        HCsr S = schur_graph(Kp, n, m);
        sub_lap("order: Schur graph");
        std::vector<int32_t> os;
        if (m <= kMdLimit) {
            os = min_degree(S);
            *kind_out = ORD_GFIRST_MD;
        } else {
            os = nested_dissection(S, kNdLeaf);
            *kind_out = ORD_GFIRST_ND;
        }
        sub_lap("order: dissection");
        for (int64_t i = 0; i < n; i++) perm[i] = (int32_t)i;
        for (int64_t i = 0; i < m; i++) perm[n + i] = (int32_t)(n + os[i]);
    } else {
        std::vector<std::pair<int32_t, int32_t>> edges;
        for (int64_t i = 0; i < N; i++)
            for (int64_t p = Kp.ptr[i]; p < Kp.ptr[i + 1]; p++)
                if (Kp.ind[p] != i) edges.emplace_back((int32_t)i, Kp.ind[p]);
        HCsr g = graph_from_edges(N, edges);
        if (N <= kMdLimit) {
            perm = min_degree(g);
            *kind_out = ORD_MD;
        } else {
            perm = nested_dissection(g, kNdLeaf);
            *kind_out = ORD_ND;
        }
    }
    return perm;
}

}  // namespace cpk
