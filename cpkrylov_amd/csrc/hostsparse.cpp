// hostsparse.cpp -- host CSR conversions and the Kp = [A B'; B C] assembly (ops/opLDL2.m:81).
#include <algorithm>
#include <numeric>
#include <thread>

#include "cpk.h"
#include "host.hpp"

namespace cpk {

void transpose_pattern(int64_t N, const int64_t *Lp, const int32_t *Li, uint32_t *rptr, int32_t *rcol, int32_t *ridx) {
    const int64_t nnz = Lp[N];
    const int T = (int)std::max<int64_t>(1, std::min<int64_t>(host_threads(), (nnz + 262143) / 262144));
    // thread t: columns ccut[t] .. ccut[t+1) (equal entry counts) for the bucketing, rows
    // t * rs .. (t + 1) * rs for the placement
    std::vector<int64_t> ccut(T + 1, N);
    ccut[0] = 0;
    for (int t = 1; t < T; t++) ccut[t] = std::upper_bound(Lp, Lp + N + 1, nnz * t / T) - Lp - 1;
    const int64_t rs = (N + T - 1) / T;
    std::vector<std::vector<int64_t>> boff(T, std::vector<int64_t>(T + 1, 0));
    std::vector<std::vector<int32_t>> bp(T);  // thread t's column slots, grouped by row owner
    std::vector<std::thread> th;
    auto bucket = [&](int t) {
        const int64_t p0 = Lp[ccut[t]], p1 = Lp[ccut[t + 1]];
        std::vector<int64_t> &o = boff[t];
        for (int64_t p = p0; p < p1; p++) o[Li[p] / rs + 1]++;
        for (int u = 0; u < T; u++) o[u + 1] += o[u];
        std::vector<int64_t> nx(o.begin(), o.end() - 1);
        bp[t].resize((size_t)(p1 - p0));
        for (int64_t p = p0; p < p1; p++) bp[t][nx[Li[p] / rs]++] = (int32_t)p;
    };
    std::vector<int64_t> base(T + 1, 0);  // entries of the rows before each row range
    auto place = [&](int u) {
        const int64_t r0 = std::min<int64_t>(N, u * rs), r1 = std::min<int64_t>(N, r0 + rs);
        std::vector<uint32_t> cnt(r1 - r0 + 1, 0);
        for (int t = 0; t < T; t++)
            for (int64_t s = boff[t][u]; s < boff[t][u + 1]; s++) cnt[Li[bp[t][s]] - r0 + 1]++;
        uint32_t acc = (uint32_t)base[u];
        for (int64_t i = r0; i < r1; i++) acc += cnt[i - r0 + 1], cnt[i - r0 + 1] = acc;
        cnt[0] = (uint32_t)base[u];
        for (int64_t i = r0; i < r1; i++) rptr[i + 1] = cnt[i - r0 + 1];
        for (int t = 0; t < T; t++) {  // column ranges ascending, columns ascending within each
            int64_t j = ccut[t];
            for (int64_t s = boff[t][u]; s < boff[t][u + 1]; s++) {
                const int32_t p = bp[t][s];
                while (Lp[j + 1] <= p) j++;
                const uint32_t q = cnt[Li[p] - r0]++;
                rcol[q] = (int32_t)j;
                ridx[q] = p;
            }
        }
    };
    for (int t = 1; t < T; t++) th.emplace_back(bucket, t);
    bucket(0);
    for (auto &x : th) x.join();
    th.clear();
    for (int u = 0; u < T; u++) {
        int64_t tot = 0;
        for (int t = 0; t < T; t++) tot += boff[t][u + 1] - boff[t][u];
        base[u + 1] = base[u] + tot;
    }
    rptr[0] = 0;
    for (int u = 1; u < T; u++) th.emplace_back(place, u);
    place(0);
    for (auto &x : th) x.join();
}

// Canonicalise: sort each row by column, sum duplicates (MATLAB sparse arrays never hold any).
static void canonicalise(HCsr &a) {
    std::vector<int64_t> ptr(a.nrows + 1, 0);
    std::vector<int32_t> ind;
    std::vector<double> val;
    ind.reserve(a.ind.size());
    val.reserve(a.val.size());
    std::vector<std::pair<int32_t, double>> row;
    for (int64_t i = 0; i < a.nrows; i++) {
        row.clear();
        for (int64_t p = a.ptr[i]; p < a.ptr[i + 1]; p++) row.emplace_back(a.ind[p], a.val[p]);
        bool sorted = std::is_sorted(row.begin(), row.end(),
                                     [](auto &x, auto &y) { return x.first < y.first; });
        if (!sorted) std::stable_sort(row.begin(), row.end(), [](auto &x, auto &y) { return x.first < y.first; });
        for (size_t q = 0; q < row.size(); q++) {
            if (!ind.empty() && (int64_t)ind.size() > ptr[i] && ind.back() == row[q].first)
                val.back() += row[q].second;
            else
                ind.push_back(row[q].first), val.push_back(row[q].second);
        }
        ptr[i + 1] = (int64_t)ind.size();
    }
    a.ptr.swap(ptr);
    a.ind.swap(ind);
    a.val.swap(val);
}

HCsr csr_from_csr(int64_t nr, int64_t nc, const int64_t *rp, const int32_t *ci, const double *v) {
    if (nr < 0 || nc < 0 || nr > INT32_MAX || nc > INT32_MAX) throw Error(CPK_ERR_DIM, "matrix dimensions out of range");
    if (nr > 0 && (!rp || (rp[nr] > 0 && (!ci || !v)))) throw Error(CPK_ERR_ARGS, "NULL CSR array");
    HCsr a;
    a.nrows = nr, a.ncols = nc;
    a.ptr.assign(rp, rp + nr + 1);
    if (a.ptr.empty()) a.ptr.push_back(0);
    int64_t nnz = a.ptr.back() - a.ptr.front();
    if (a.ptr.front() != 0) for (auto &p : a.ptr) p -= rp[0];
    a.ind.assign(ci + rp[0], ci + rp[0] + nnz);
    a.val.assign(v + rp[0], v + rp[0] + nnz);
    for (int64_t i = 0; i < nr; i++)
        if (a.ptr[i + 1] < a.ptr[i]) throw Error(CPK_ERR_ARGS, "CSR row pointers not monotone");
    for (auto c : a.ind)
        if (c < 0 || c >= nc) throw Error(CPK_ERR_ARGS, "CSR column index out of range");
    canonicalise(a);
    return a;
}

HCsr csr_from_csc(int64_t nr, int64_t nc, const size_t *jc, const size_t *ir, const double *pr) {
    if (nr < 0 || nc < 0 || nr > INT32_MAX || nc > INT32_MAX) throw Error(CPK_ERR_DIM, "matrix dimensions out of range");
    if (nc > 0 && !jc) throw Error(CPK_ERR_ARGS, "NULL CSC array");
    size_t nnz = nc > 0 ? jc[nc] - jc[0] : 0;
    if (nnz && (!ir || !pr)) throw Error(CPK_ERR_ARGS, "NULL CSC array");
    HCsr a;
    a.nrows = nr, a.ncols = nc;
    a.ptr.assign(nr + 1, 0);
    for (int64_t j = 0; j < nc; j++)
        for (size_t p = jc[j]; p < jc[j + 1]; p++) {
            if (ir[p] >= (size_t)nr) throw Error(CPK_ERR_ARGS, "CSC row index out of range");
            a.ptr[ir[p] + 1]++;
        }
    for (int64_t i = 0; i < nr; i++) a.ptr[i + 1] += a.ptr[i];
    a.ind.resize(nnz);
    a.val.resize(nnz);
    std::vector<int64_t> next(a.ptr.begin(), a.ptr.end() - 1);
    for (int64_t j = 0; j < nc; j++)  // columns ascend, so every row comes out sorted
        for (size_t p = jc[j]; p < jc[j + 1]; p++) {
            int64_t q = next[ir[p]]++;
            a.ind[q] = (int32_t)j;
            a.val[q] = pr[p];
        }
    canonicalise(a);
    return a;
}

HCsr transpose(const HCsr &a) {
    HCsr t;
    t.nrows = a.ncols, t.ncols = a.nrows;
    t.ptr.assign(t.nrows + 1, 0);
    for (auto c : a.ind) t.ptr[c + 1]++;
    for (int64_t i = 0; i < t.nrows; i++) t.ptr[i + 1] += t.ptr[i];
    t.ind.resize(a.nnz());
    t.val.resize(a.nnz());
    std::vector<int64_t> next(t.ptr.begin(), t.ptr.end() - 1);
    for (int64_t i = 0; i < a.nrows; i++)
        for (int64_t p = a.ptr[i]; p < a.ptr[i + 1]; p++) {
            int64_t q = next[a.ind[p]]++;
            t.ind[q] = (int32_t)i;
            t.val[q] = a.val[p];
        }
    return t;
}

void check_kp_dims(const HCsr &A, const HCsr &B, const HCsr &C) {
    // dimension checks of opLDL2.m:61-75 (same messages)
    if (A.nrows != A.ncols || C.nrows != C.ncols) throw Error(CPK_ERR_DIM, "First and last arguments must be square.");
    if (B.ncols != A.nrows || B.nrows != C.nrows) throw Error(CPK_ERR_DIM, "Incompatible dimensions.");
    if (A.nrows + C.nrows > INT32_MAX) throw Error(CPK_ERR_DIM, "N exceeds the 32-bit index range");
}

HCsr assemble_kp(const HCsr &A, const HCsr &B, const HCsr &C) {
    check_kp_dims(A, B, C);
    const int64_t n = A.nrows, m = C.nrows, N = n + m;
    HCsr K;
    K.nrows = K.ncols = N;
    // the entry arrays are zero-filled (first touch of fresh pages) on their own threads while
    // this one transposes B
    const int64_t nnz = A.nnz() + 2 * B.nnz() + C.nnz();
    std::thread zi([&] { K.ind.resize(nnz); }), zv([&] { K.val.resize(nnz); });
    HCsr Bt;
    try {
        Bt = transpose(B);
    } catch (...) {
        zi.join(), zv.join();
        throw;
    }
    K.ptr.assign(N + 1, 0);
    for (int64_t i = 0; i < n; i++) K.ptr[i + 1] = K.ptr[i] + (A.ptr[i + 1] - A.ptr[i]) + (Bt.ptr[i + 1] - Bt.ptr[i]);
    for (int64_t i = 0; i < m; i++)
        K.ptr[n + i + 1] = K.ptr[n + i] + (B.ptr[i + 1] - B.ptr[i]) + (C.ptr[i + 1] - C.ptr[i]);
    zi.join(), zv.join();
    // row i: [A row; B' row shifted by n] (i < n), [B row; C row shifted by n] (i >= n)
    auto put = [&](int64_t row, const HCsr &L, int64_t li, int32_t lshift, const HCsr &R, int64_t ri, int32_t rshift) {
        int64_t q = K.ptr[row];
        for (int64_t p = L.ptr[li]; p < L.ptr[li + 1]; p++, q++) K.ind[q] = L.ind[p] + lshift, K.val[q] = L.val[p];
        for (int64_t p = R.ptr[ri]; p < R.ptr[ri + 1]; p++, q++) K.ind[q] = R.ind[p] + rshift, K.val[q] = R.val[p];
    };
    parallel_for(N, [&](int64_t lo, int64_t hi) {
        for (int64_t i = lo; i < hi; i++) {
            if (i < n) put(i, A, i, 0, Bt, i, (int32_t)n);
            else put(i, B, i - n, 0, C, i - n, (int32_t)n);
        }
    });
    return K;
}

std::vector<int64_t> kp_value_sources(const HCsr &A, const HCsr &B, const HCsr &C) {
    const int64_t n = A.nrows, m = C.nrows;
    // B' rows with B's entry index of each entry (the order transpose() produces: rows of B ascending)
    std::vector<int64_t> tp(n + 1, 0);
    for (int64_t p = 0; p < B.nnz(); p++) tp[B.ind[p] + 1]++;
    for (int64_t j = 0; j < n; j++) tp[j + 1] += tp[j];
    std::vector<int64_t> ti(B.nnz()), nx(tp.begin(), tp.end() - 1);
    for (int64_t i = 0; i < m; i++)
        for (int64_t p = B.ptr[i]; p < B.ptr[i + 1]; p++) ti[nx[B.ind[p]]++] = p;
    const int64_t kB = int64_t(1) << 40, kC = int64_t(2) << 40;
    std::vector<int64_t> src;
    src.reserve(A.nnz() + 2 * B.nnz() + C.nnz());
    for (int64_t i = 0; i < n; i++) {
        for (int64_t p = A.ptr[i]; p < A.ptr[i + 1]; p++) src.push_back(p);
        for (int64_t q = tp[i]; q < tp[i + 1]; q++) src.push_back(kB | ti[q]);
    }
    for (int64_t i = 0; i < m; i++) {
        for (int64_t p = B.ptr[i]; p < B.ptr[i + 1]; p++) src.push_back(kB | p);
        for (int64_t p = C.ptr[i]; p < C.ptr[i + 1]; p++) src.push_back(kC | p);
    }
    return src;
}

HCsr blkdiag(const HCsr &A, const HCsr &C) {
    const int64_t n = A.nrows, m = C.nrows;
    HCsr K;
    K.nrows = n + m;
    K.ncols = A.ncols + C.ncols;
    K.ptr.assign(n + m + 1, 0);
    K.ind.reserve(A.nnz() + C.nnz());
    K.val.reserve(A.nnz() + C.nnz());
    for (int64_t i = 0; i < n; i++) {
        for (int64_t p = A.ptr[i]; p < A.ptr[i + 1]; p++) K.ind.push_back(A.ind[p]), K.val.push_back(A.val[p]);
        K.ptr[i + 1] = (int64_t)K.ind.size();
    }
    for (int64_t i = 0; i < m; i++) {
        for (int64_t p = C.ptr[i]; p < C.ptr[i + 1]; p++)
            K.ind.push_back((int32_t)(A.ncols + C.ind[p])), K.val.push_back(C.val[p]);
        K.ptr[n + i + 1] = (int64_t)K.ind.size();
    }
    return K;
}

bool is_diagonal(const HCsr &a) {
    for (int64_t i = 0; i < a.nrows; i++)
        for (int64_t p = a.ptr[i]; p < a.ptr[i + 1]; p++)
            if (a.ind[p] != i) return false;
    return true;
}

}  // namespace cpk
