// dist.cpp -- host plan of the distributed solve (see dist.hpp).  Every rank runs the same
// deterministic analysis and builds the same global plan, so no setup communication is
// needed beyond the RCCL communicator itself.
#include <cstdlib>
#include "dist.hpp"

#include <algorithm>
#include <cmath>
#include <numeric>
#include <queue>
#include <string>

#include "cpk.h"

namespace cpk {

TreeSplit split_tree(const Factor &f, int P, double tol, int64_t tmax, const HCsr *Akry) {
    const int64_t N = f.N;
    TreeSplit ts;
    ts.P = std::max(P, 1);
    ts.node_rank.assign(N, 0);
    if (ts.P == 1 || N == 0) return ts;
    if (tmax < 0) tmax = std::max<int64_t>(256, N / 100);
    if (!(tol > 0 && tol < 1)) throw Error(CPK_ERR_ARGS, "split_tree: load tolerance must lie in (0, 1)");
    // work weight of a row: its forward and backward entries plus the row itself
    // (row counts of L by a relaxed-atomic histogram; every weight is an exact integer)
    std::vector<int32_t> nrow(N, 0);
    parallel_for((int64_t)f.Li.size(), [&](int64_t lo, int64_t hi) {
        for (int64_t p = lo; p < hi; p++) __atomic_fetch_add(&nrow[f.Li[p]], 1, __ATOMIC_RELAXED);
    }, 1 << 18);
    std::vector<double> W(N);
    parallel_for(N, [&](int64_t lo, int64_t hi) {
        for (int64_t v = lo; v < hi; v++) W[v] = 1.0 + (double)nrow[v] + (double)(f.Lp[v + 1] - f.Lp[v]);
    }, 1 << 16);
    for (int64_t v = 0; v < N; v++)  // subtree weights (children precede parents)
        if (f.parent[v] >= 0) W[f.parent[v]] += W[v];
    std::vector<int64_t> cptr(N + 1, 0);
    for (int64_t v = 0; v < N; v++)
        if (f.parent[v] >= 0) cptr[f.parent[v] + 1]++;
    for (int64_t v = 0; v < N; v++) cptr[v + 1] += cptr[v];
    std::vector<int32_t> kids(cptr[N]);
    {
        std::vector<int64_t> nx(cptr.begin(), cptr.end() - 1);
        for (int64_t v = 0; v < N; v++)
            if (f.parent[v] >= 0) kids[nx[f.parent[v]]++] = (int32_t)v;
    }
    double total = 0;
    std::priority_queue<std::pair<double, int32_t>> heap;  // candidate subtree roots by weight
    std::vector<char> is_cand(N, 0), inT(N, 0), iso(N, 0);
    // isolated rows (no factor entries at all: e.g. G pivots no constraint touches) are solved
    // by a division; they are placed by dof locality at the end instead of by the tree
    parallel_for(N, [&](int64_t lo, int64_t hi) {
        for (int64_t v = lo; v < hi; v++)
            iso[v] = f.parent[v] < 0 && nrow[v] == 0 && f.Lp[v + 1] == f.Lp[v] && cptr[v + 1] == cptr[v];
    }, 1 << 16);
    for (int64_t v = 0; v < N; v++)
        if (f.parent[v] < 0 && !iso[v]) heap.push({W[v], (int32_t)v}), is_cand[v] = 1, total += W[v];
    // cut below the heaviest subtree until every candidate is light: a contiguous split of the
    // candidates into P runs is then within (1 + tol) of the average load
    auto avg = [&]() { return total / ts.P; };
    while (!heap.empty() && (int64_t)ts.T.size() < tmax) {
        const auto [w, v] = heap.top();
        if (w <= tol * avg() && (int64_t)heap.size() >= 4 * (int64_t)ts.P) break;
        heap.pop();
        is_cand[v] = 0, inT[v] = 1;
        ts.T.push_back(v);
        double sk = 0;  // the candidates lose v's subtree and gain its children's
        for (int64_t q = cptr[v]; q < cptr[v + 1]; q++) sk += W[kids[q]];
        total += sk - W[v];
        for (int64_t q = cptr[v]; q < cptr[v + 1]; q++) heap.push({W[kids[q]], kids[q]}), is_cand[kids[q]] = 1;
    }
    std::sort(ts.T.begin(), ts.T.end());
    // candidates ordered by their separator parent (then pivot index), split into P contiguous
    // runs at the average-load boundaries.  Keying by the parent keeps the small subtrees that
    // hang off a separator (e.g. the G-first leaves) next to the separator's other children in
    // the ordering, so a rank's share stays spatially compact and the halos small.
    std::vector<int32_t> cand;
    for (int64_t v = 0; v < N; v++)
        if (is_cand[v]) cand.push_back((int32_t)v);
    auto ckey = [&](int32_t v) { return f.parent[v] >= 0 ? f.parent[v] : v; };
    std::stable_sort(cand.begin(), cand.end(), [&](int32_t a, int32_t b) { return ckey(a) < ckey(b); });
    std::vector<int32_t> cand_rank(cand.size(), 0);
    {
        double tot = 0;
        for (int32_t v : cand) tot += W[v];
        double acc = 0;
        int r = 0;
        for (size_t i = 0; i < cand.size(); i++) {
            const double w = W[cand[i]];
            // move to the next run when this subtree's midpoint passes the run boundary
            while (r + 1 < ts.P && acc + 0.5 * w > tot * (r + 1) / ts.P) r++;
            cand_rank[i] = r;
            acc += w;
        }
    }
    // ranks of the subtree rows: top-down from the candidates (parents follow children, so
    // walk descending and inherit the parent's rank below a candidate)
    std::vector<int32_t> rank_of(N, -1);
    for (size_t i = 0; i < cand.size(); i++) rank_of[cand[i]] = cand_rank[i];
    for (int64_t v = N - 1; v >= 0; v--) {
        if (inT[v] || iso[v]) continue;
        if (rank_of[v] < 0) {
            const int32_t p = f.parent[v];
            if (p < 0 || inT[p]) throw Error(CPK_ERR_FACTOR, "internal: split_tree lost a subtree root");
            rank_of[v] = rank_of[p];
        }
    }
    std::vector<int32_t> node_of(N);  // dof -> tree node
    parallel_for(N, [&](int64_t lo, int64_t hi) {
        for (int64_t v = lo; v < hi; v++) node_of[f.perm[v]] = (int32_t)v;
    }, 1 << 16);
    // isolated rows take the rank of the nearest preceding (else following) dof
    {
        int32_t last = -1;
        for (int64_t g = 0; g < N; g++) {
            const int32_t v = node_of[g];
            if (!iso[v]) last = inT[v] ? 0 : rank_of[v];
            else if (last >= 0) rank_of[v] = last;
        }
        last = 0;
        for (int64_t g = N - 1; g >= 0; g--) {
            const int32_t v = node_of[g];
            if (!iso[v]) last = inT[v] ? 0 : rank_of[v];
            else if (rank_of[v] < 0) rank_of[v] = last;
        }
    }
    // Rows drive the Krylov side (vectors, SpMV rows), so long stretches of consecutive isolated
    // dofs (S50: the slack blocks no constraint touches, nZ/2 rows each) are split into P equal
    // contiguous parts, part r to rank r, instead of all following one neighbour.  A slack row
    // couples (in A) with the bounded variable at the same relative position of its block, so
    // equal parts in dof order land next to each rank's share of those variables.
    {
        const int64_t min_run = 64 * (int64_t)ts.P;
        for (int64_t g = 0; g < N;) {
            if (!iso[node_of[g]]) {
                g++;
                continue;
            }
            int64_t e = g;
            while (e < N && iso[node_of[e]]) e++;
            if (e - g >= min_run)
                for (int64_t q = g; q < e; q++) rank_of[node_of[q]] = (int32_t)(((q - g) * ts.P) / (e - g));
            g = e;
        }
    }
    // with the Krylov operator known, an isolated row takes the rank of the first dof its A row
    // couples it with that the tree placed (the slack rows of S50 couple with one bounded
    // variable each): the halo of A then holds only the coupling across rank boundaries
    if (Akry) {
        for (int64_t v = 0; v < N; v++) {
            if (!iso[v] || inT[v]) continue;
            const int64_t g = f.perm[v];
            if (g >= Akry->nrows) continue;
            for (int64_t p = Akry->ptr[g]; p < Akry->ptr[g + 1]; p++) {
                const int32_t c = Akry->ind[p];
                if (c == g || c >= N) continue;
                const int32_t u = node_of[c];
                if (!iso[u] && !inT[u]) {
                    rank_of[v] = rank_of[u];
                    break;
                }
            }
        }
    }
    for (int64_t v = 0; v < N; v++) ts.node_rank[v] = inT[v] ? -1 : rank_of[v];
    return ts;
}

std::vector<int32_t> DofMap::dofs(int rank) const {
    std::vector<int32_t> d((size_t)(n_loc[rank] + m_loc[rank]));
    for (int64_t g = 0; g < N; g++)
        if (owner[g] == rank) d[lidx[g]] = (int32_t)g;
    return d;
}

DofMap make_dofmap(const Factor &f, const TreeSplit &ts, int64_t n) {
    DofMap dm;
    dm.P = ts.P, dm.N = f.N, dm.n = n, dm.m = f.N - n;
    dm.owner.assign(f.N, 0);
    dm.lidx.assign(f.N, 0);
    for (int64_t v = 0; v < f.N; v++) dm.owner[f.perm[v]] = std::max(ts.node_rank[v], 0);  // T dofs: rank 0
    dm.n_loc.assign(ts.P, 0), dm.m_loc.assign(ts.P, 0);
    for (int64_t g = 0; g < n; g++) dm.lidx[g] = (int32_t)dm.n_loc[dm.owner[g]]++;
    for (int64_t g = n; g < f.N; g++) dm.lidx[g] = (int32_t)(dm.n_loc[dm.owner[g]] + dm.m_loc[dm.owner[g]]++);
    return dm;
}

DistCsr dist_csr(const HCsr &K, const DofMap &dm, int rank, bool rows_x_only, int64_t spare) {
    const int64_t rows_end = rows_x_only ? dm.n : dm.N;
    if (K.nrows != rows_end || K.ncols != dm.N) throw Error(CPK_ERR_DIM, "dist_csr: matrix shape does not match the dof map");
    // slot of every dof some other rank reads (per owner, ascending dof)
    std::vector<char> need(dm.N, 0);
    for (int64_t g = 0; g < rows_end; g++) {
        const int32_t q = dm.owner[g];
        for (int64_t p = K.ptr[g]; p < K.ptr[g + 1]; p++)
            if (dm.owner[K.ind[p]] != q) need[K.ind[p]] = 1;
    }
    std::vector<int64_t> cnt(dm.P, 0);
    std::vector<int32_t> slot(dm.N, -1);
    for (int64_t c = 0; c < dm.N; c++)
        if (need[c]) slot[c] = (int32_t)cnt[dm.owner[c]]++;
    DistCsr d;
    d.kmax = *std::max_element(cnt.begin(), cnt.end());
    d.kstride = d.kmax + spare;
    const int64_t nl = dm.n_loc[rank], ml = dm.m_loc[rank];
    d.nloc = nl + ml;
    for (int64_t c = 0; c < dm.N; c++)
        if (need[c] && dm.owner[c] == rank) d.send.push_back(dm.lidx[c]);
    // local rows in local order
    const std::vector<int32_t> dofs = dm.dofs(rank);
    const int64_t nrows = rows_x_only ? nl : nl + ml;
    d.a.nrows = nrows;
    d.a.ncols = d.nloc + (int64_t)dm.P * d.kstride;
    d.a.ptr.assign(nrows + 1, 0);
    for (int64_t i = 0; i < nrows; i++) d.a.ptr[i + 1] = d.a.ptr[i] + (K.ptr[dofs[i] + 1] - K.ptr[dofs[i]]);
    d.a.ind.resize(d.a.ptr[nrows]);
    d.a.val.resize(d.a.ptr[nrows]);
    for (int64_t i = 0; i < nrows; i++) {
        const int32_t g = dofs[i];
        int64_t o = d.a.ptr[i];
        for (int64_t p = K.ptr[g]; p < K.ptr[g + 1]; p++, o++) {  // global column order kept
            const int32_t c = K.ind[p];
            d.a.ind[o] = dm.owner[c] == rank ? dm.lidx[c] : (int32_t)(d.nloc + (int64_t)dm.owner[c] * d.kstride + slot[c]);
            d.a.val[o] = K.val[p];
        }
    }
    return d;
}

RankPlan make_rank_plan(const Factor &f, const TreeSplit &ts, const DofMap &dm, int rank) {
    const int64_t N = f.N;
    RankPlan rp;
    rp.P = ts.P, rp.rank = rank;
    std::vector<int32_t> loc(N, -1), tpos(N, -1);
    for (int64_t v = 0; v < N; v++)
        if (ts.node_rank[v] == rank) loc[v] = (int32_t)rp.nsub++;
    rp.nT = (int64_t)ts.T.size();
    for (int64_t t = 0; t < rp.nT; t++) tpos[ts.T[t]] = (int32_t)t;
    // ---- local subtree factor: columns of this rank's rows, restricted to its rows; entries
    //      in separator rows become backward extras
    Factor &F = rp.Fsub;
    F.N = rp.nsub;
    F.Lp.assign(rp.nsub + 1, 0);
    F.D.resize(rp.nsub), F.perm.resize(rp.nsub), F.parent.assign(rp.nsub, -1);
    rp.key.resize(rp.nsub);
    rp.extra.assign(rp.nsub, {});
    for (int64_t v = 0; v < N; v++) {
        const int32_t j = loc[v];
        if (j < 0) continue;
        F.D[j] = f.D[v];
        F.perm[j] = dm.lidx[f.perm[v]];
        rp.key[j] = v;
        if (f.parent[v] >= 0 && loc[f.parent[v]] >= 0) F.parent[j] = loc[f.parent[v]];
        for (int64_t p = f.Lp[v]; p < f.Lp[v + 1]; p++) {
            const int32_t i = f.Li[p];
            if (loc[i] >= 0) {
                F.Li.push_back(loc[i]);
                F.Lx.push_back(f.Lx[p]);
            } else if (tpos[i] >= 0) {
                rp.extra[j].push_back(BwdExtra{(int32_t)(rp.nsub + tpos[i]), (int64_t)i, f.Lx[p]});
            } else {
                throw Error(CPK_ERR_FACTOR, "internal: factor entry couples two ranks' subtrees");
            }
        }
        F.Lp[j + 1] = (int64_t)F.Li.size();
    }
    // ---- separator inputs: subtree rows read by T rows, grouped by owner, ascending
    std::vector<int32_t> jpos(N, -1);
    std::vector<int64_t> jcnt(ts.P, 0);
    std::vector<std::vector<std::pair<int32_t, double>>> trow(rp.nT);  // forward rows of T
    for (int64_t j = 0; j < N; j++)
        for (int64_t p = f.Lp[j]; p < f.Lp[j + 1]; p++) {
            const int32_t i = f.Li[p];
            if (tpos[i] < 0) continue;
            trow[tpos[i]].push_back({(int32_t)j, f.Lx[p]});  // j ascending: the sum order
            if (tpos[j] < 0 && jpos[j] < 0) jpos[j] = (int32_t)jcnt[ts.node_rank[j]]++;
        }
    // jpos was assigned in ascending j within each owner
    rp.kt = 0;
    for (int q = 0; q < ts.P; q++) rp.kt = std::max<int64_t>(rp.kt, jcnt[q] + (q == 0 ? rp.nT : 0));
    for (int64_t j = 0; j < N; j++)
        if (jpos[j] >= 0 && ts.node_rank[j] == rank) rp.tsend.push_back(loc[j]);
    // ---- separator rows
    rp.tf_ptr.assign(rp.nT + 1, 0);
    rp.tb_ptr.assign(rp.nT + 1, 0);
    rp.DT.resize(rp.nT);
    rp.tf_src.resize(rp.nT);
    std::vector<int32_t> lvl(rp.nT, 0);
    int32_t nlev = 0;
    for (int64_t t = 0; t < rp.nT; t++) {
        const int32_t v = ts.T[t];
        rp.DT[t] = f.D[v];
        rp.tf_src[t] = (int32_t)(jcnt[0] + t);  // rank 0 publishes the T inputs after its own rows
        for (const auto &[j, x] : trow[t]) {
            if (tpos[j] >= 0) {
                rp.tf_col.push_back(-(tpos[j] + 1));
                lvl[t] = std::max(lvl[t], lvl[tpos[j]] + 1);
            } else {
                rp.tf_col.push_back((int32_t)((int64_t)ts.node_rank[j] * rp.kt + jpos[j]));
            }
            rp.tf_val.push_back(x);
        }
        rp.tf_ptr[t + 1] = (int64_t)rp.tf_col.size();
        nlev = std::max(nlev, lvl[t] + 1);
        for (int64_t p = f.Lp[v + 1] - 1; p >= f.Lp[v]; p--) {  // rows below t, descending
            const int32_t i = f.Li[p];
            if (tpos[i] < 0) throw Error(CPK_ERR_FACTOR, "internal: separator row above a subtree row");
            rp.tb_col.push_back(tpos[i]);
            rp.tb_val.push_back(f.Lx[p]);
        }
        rp.tb_ptr[t + 1] = (int64_t)rp.tb_col.size();
    }
    rp.tlev_ptr.assign(nlev + 1, 0);
    for (int64_t t = 0; t < rp.nT; t++) rp.tlev_ptr[lvl[t] + 1]++;
    for (int32_t l = 0; l < nlev; l++) rp.tlev_ptr[l + 1] += rp.tlev_ptr[l];
    rp.tlev_rows.resize(rp.nT);
    {
        std::vector<int32_t> nx(rp.tlev_ptr.begin(), rp.tlev_ptr.end() - 1);
        for (int64_t t = 0; t < rp.nT; t++) rp.tlev_rows[nx[lvl[t]]++] = (int32_t)t;
    }
    if (rank == 0)
        for (int64_t t = 0; t < rp.nT; t++) rp.tdof.push_back(dm.lidx[f.perm[ts.T[t]]]);
    return rp;
}

HCsr hstack_ab(const HCsr &A, const HCsr &Kp, int64_t n) {
    // rows 0..n-1 of [A, Kp(0:n, n:N)] with columns in global order (A's columns < n first)
    HCsr o;
    o.nrows = n, o.ncols = Kp.ncols;
    o.ptr.assign(n + 1, 0);
    for (int64_t i = 0; i < n; i++) {
        int64_t c = A.ptr[i + 1] - A.ptr[i];
        for (int64_t p = Kp.ptr[i]; p < Kp.ptr[i + 1]; p++) c += Kp.ind[p] >= n;
        o.ptr[i + 1] = o.ptr[i] + c;
    }
    o.ind.reserve(o.ptr[n]);
    o.val.reserve(o.ptr[n]);
    for (int64_t i = 0; i < n; i++) {
        for (int64_t p = A.ptr[i]; p < A.ptr[i + 1]; p++) o.ind.push_back(A.ind[p]), o.val.push_back(A.val[p]);
        for (int64_t p = Kp.ptr[i]; p < Kp.ptr[i + 1]; p++)
            if (Kp.ind[p] >= n) o.ind.push_back(Kp.ind[p]), o.val.push_back(Kp.val[p]);
    }
    return o;
}

}  // namespace cpk
