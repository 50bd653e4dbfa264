// ldl.hip -- numeric phase of the LDL' factorization on the device.
//
// Replaces the numeric half of [L,D,P] = ldl(op.A) (ops/opLDL2.m:82) and its refactorization
// when G, B or C change with the same sparsity (the IPM outer loop that rebuilds opLDL2 per
// iteration).  The host keeps the symbolic analysis (ordering, elimination tree, the pattern of
// every row of L, the sweep schedule; factor.cpp: ldl_factor(..., sym, numeric = false)).
//
// Up-looking by rows: row k of L solves L(0:k,0:k) y = Kp(perm, perm)(0:k, k) over its pattern
// (the reach of its Kp entries in the elimination tree) and D(k) = Kp(k,k) - sum l_ki y_i.  A
// row depends only on its descendants in the tree, so rows of one tree height run
// concurrently, one thread per row, one launch per height.  Each thread walks its row pattern in
// ascending column order and, for each column i, column i's entries above row k in ascending
// row order -- exactly the operations and order of the host's ldl_factor -- so L and D equal
// the host factorization bit for bit (-ffp-contract=off: no FMA is formed).
//
// The values land in CSC order (the exported factor's layout); ldl_fill_kernel then gathers
// them into the forward / backward sweep layouts of DFactor (schedule order, summation order of
// the exported factor) and D into schedule order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>

#include "dev.hpp"

namespace cpk {

__global__ __launch_bounds__(256) void ldl_rows_kernel(
    const int32_t *__restrict__ rows, int nrows, const int32_t *__restrict__ Rp, const int32_t *__restrict__ Rc,
    const int32_t *__restrict__ Rcsc, const int32_t *__restrict__ Lp, const int32_t *__restrict__ Li,
    double *__restrict__ Lx, double *__restrict__ D, double *__restrict__ Y, const int32_t *__restrict__ kp_ptr,
    const int32_t *__restrict__ kp_tgt, const uint32_t *__restrict__ kp_src, const double *__restrict__ kpv,
    int *__restrict__ bad) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= nrows) return;
    const int32_t k = rows[idx];
    const int32_t t0 = Rp[k], t1 = Rp[k + 1];
    for (int32_t t = t0; t < t1; t++) Y[t] = 0.0;
    // seeds: y(i) += Kp(perm(k), perm(i)) for the row's entries left of and on the diagonal
    double d = 0.0;
    for (int32_t q = kp_ptr[k]; q < kp_ptr[k + 1]; q++) {
        const int32_t tg = kp_tgt[q];
        const double v = kpv[kp_src[q]];
        if (tg < 0) d += v;
        else Y[tg] += v;
    }
    for (int32_t t = t0; t < t1; t++) {
        const int32_t i = Rc[t];
        const double yi = Y[t];
        // y(j) -= L(j,i) * y(i) for column i's rows j < k; every such j is in row k's pattern
        // (right of i), found by merging the two ascending lists
        int32_t s = t + 1;
        const int32_t p1 = Lp[i + 1];
        for (int32_t p = Lp[i]; p < p1; p++) {
            const int32_t j = Li[p];
            if (j >= k) break;
            while (s < t1 && Rc[s] < j) s++;
            if (s >= t1 || Rc[s] != j) {  // impossible for a consistent symbolic analysis
                atomicOr(bad, 2);
                return;
            }
            Y[s] -= Lx[p] * yi;
        }
        const double lki = yi / D[i];
        d -= lki * yi;
        Lx[Rcsc[t]] = lki;
    }
    D[k] = d;
    if (d == 0.0 || !(d == d)) {
        atomicOr(bad, 1);
        atomicMin(bad + 1, k);
    }
}

// Long rows (a pattern of kLdlWaveMin or more columns): one wave per row.  The dense top of a
// factor (cvxqp1_m: the last ~470 rows form one chain of tree levels, each row's pattern the
// whole separator) made the one-thread-per-row kernel walk ~10 M dependent steps on one lane
// per level (seconds).  Here the row's y lives in LDS, and for each column i of the pattern (in
// the same ascending order) the lanes take column i's entries j < k together: each finds j's
// slot in the row's sorted pattern by binary search and subtracts L(j,i) y(i) -- distinct slots,
// so the updates of one column are independent, and every slot still receives its updates in
// ascending column order.  The seeds and the pivot run on lane 0 in the thread kernel's order.
// Same operations in the same order per value: bit-identical to the host factorization.
constexpr int kLdlWaveMin = 48;
__global__ __launch_bounds__(64) void ldl_rows_wave_kernel(
    const int32_t *__restrict__ rows, const int32_t *__restrict__ Rp, const int32_t *__restrict__ Rc,
    const int32_t *__restrict__ Rcsc, const int32_t *__restrict__ Lp, const int32_t *__restrict__ Li,
    double *__restrict__ Lx, double *__restrict__ D, const int32_t *__restrict__ kp_ptr,
    const int32_t *__restrict__ kp_tgt, const uint32_t *__restrict__ kp_src, const double *__restrict__ kpv,
    int *__restrict__ bad) {
    extern __shared__ __attribute__((aligned(16))) double ly[];  // y[n] | pattern columns[n]
    const int lane = threadIdx.x;
    const int32_t k = rows[blockIdx.x];
    const int32_t t0 = Rp[k], n = Rp[k + 1] - t0;
    int32_t *rc = reinterpret_cast<int32_t *>(ly + n);
    for (int32_t t = lane; t < n; t += 64) ly[t] = 0.0, rc[t] = Rc[t0 + t];
    __syncthreads();
    double d = 0.0;
    if (lane == 0)  // seeds in Kp's entry order (a slot may receive several)
        for (int32_t q = kp_ptr[k]; q < kp_ptr[k + 1]; q++) {
            const int32_t tg = kp_tgt[q];
            const double v = kpv[kp_src[q]];
            if (tg < 0) d += v;
            else ly[tg - t0] += v;
        }
    __syncthreads();
    for (int32_t t = 0; t < n; t++) {
        const int32_t i = rc[t];
        const double yi = ly[t];
        const int32_t p0 = Lp[i], p1 = Lp[i + 1];
        for (int32_t p = p0 + lane; p < p1; p += 64) {
            const int32_t j = Li[p];
            if (j < k) {  // column i's rows are ascending: those below k follow, and are skipped
                int32_t lo = t + 1, hi = n;  // first slot with rc >= j
                while (lo < hi) {
                    const int32_t mid = (lo + hi) >> 1;
                    if (rc[mid] < j) lo = mid + 1;
                    else hi = mid;
                }
                if (lo >= n || rc[lo] != j) atomicOr(bad, 2);  // impossible for a consistent analysis
                else ly[lo] -= Lx[p] * yi;
            }
        }
        if (lane == 0) {
            const double lki = yi / D[i];
            d -= lki * yi;
            Lx[Rcsc[t0 + t]] = lki;
        }
        __syncthreads();
    }
    if (lane == 0) {
        D[k] = d;
        if (d == 0.0 || !(d == d)) {
            atomicOr(bad, 1);
            atomicMin(bad + 1, k);
        }
    }
}

// sweep layouts of DFactor from the CSC values, D into schedule order
__global__ void ldl_fill_kernel(int64_t nf, int64_t nb, int64_t N, const int32_t *__restrict__ fsrc,
                                const int32_t *__restrict__ bsrc, const int32_t *__restrict__ dsrc,
                                const double *__restrict__ Lx, const double *__restrict__ Dp, double *__restrict__ fval,
                                double *__restrict__ bval, double *__restrict__ Ds) {
    const int64_t n = nf > nb ? (nf > N ? nf : N) : (nb > N ? nb : N);
    for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x) {
        if (q < nf) fval[q] = Lx[fsrc[q]];
        if (q < nb) bval[q] = Lx[bsrc[q]];
        if (q < N) Ds[q] = Dp[dsrc[q]];
    }
}

// Kp's values from the user's blocks: src = (block << 40) | entry, block 0 = A11 (G),
// 1 = B (B or B' entries), 2 = C22
__global__ void kp_assemble_kernel(int64_t nnz, const int64_t *__restrict__ src, const double *__restrict__ a,
                                   const double *__restrict__ b, const double *__restrict__ c, double *__restrict__ kpv) {
    for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < nnz; q += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = src[q];
        const int64_t blk = s >> 40, e = s & ((int64_t(1) << 40) - 1);
        kpv[q] = blk == 0 ? a[e] : (blk == 1 ? b[e] : c[e]);
    }
}

void dldl_setup_sym(DLdl &d, const LdlSymbolic &sym, const Factor &f) {
    d.N = f.N;
    d.nnz = (int64_t)f.Li.size();
    d.lev_ptr = sym.lev_ptr;
    // within each height: the short rows first, then the long ones (ldl_rows_wave_kernel)
    std::vector<int32_t> rows = sym.lev_rows;
    const int64_t nlev = (int64_t)d.lev_ptr.size() - 1;
    d.lev_long.assign((size_t)std::max<int64_t>(nlev, 0), 0);
    d.max_long = 0;
    for (int64_t l = 0; l < nlev; l++) {
        auto b = rows.begin() + d.lev_ptr[l], e = rows.begin() + d.lev_ptr[l + 1];
        auto mid = std::stable_partition(b, e, [&](int32_t k) { return sym.Rp[k + 1] - sym.Rp[k] < kLdlWaveMin; });
        d.lev_long[l] = (int32_t)(mid - rows.begin());
        for (auto it = mid; it != e; ++it) d.max_long = std::max<int64_t>(d.max_long, sym.Rp[*it + 1] - sym.Rp[*it]);
    }
    SubClock clk;
    d.lev_rows.upload(rows);
    d.Rp.upload(sym.Rp);
    d.Rc.upload(sym.Rc);
    d.Rcsc.upload(sym.Rcsc);
    std::vector<int32_t> lp(f.Lp.begin(), f.Lp.end());
    d.Lp.upload(lp);
    d.Li.upload(f.Li);
    d.kp_ptr.upload(sym.kp_ptr);
    d.kp_tgt.upload(sym.kp_tgt);
    d.kp_src.upload(sym.kp_src);
    d.Lx.alloc((size_t)std::max<int64_t>(d.nnz, 1));
    d.D.alloc((size_t)std::max<int64_t>(d.N, 1));
    d.Y.alloc((size_t)std::max<int64_t>(d.nnz, 1));
    d.bad.alloc(2);
    d.sym_ready = true;
    clk.lap("ldl setup: symbolic uploads");
}

void dldl_setup_src(DLdl &d, const std::vector<int32_t> &fsrc, const std::vector<int32_t> &bsrc,
                    const std::vector<int32_t> &order) {
    if (!d.sym_ready) throw Error(CPK_ERR_ARGS, "internal: value sources before the symbolic data");
    d.nf = (int64_t)fsrc.size(), d.nb = (int64_t)bsrc.size();
    d.fsrc.upload(fsrc);
    d.bsrc.upload(bsrc);
    d.dsrc.upload(order);
    d.ready = true;
}

void dldl_setup(DLdl &d, const LdlSymbolic &sym, const Factor &f, const std::vector<int32_t> &fsrc,
                const std::vector<int32_t> &bsrc, const std::vector<int32_t> &order) {
    dldl_setup_sym(d, sym, f);
    dldl_setup_src(d, fsrc, bsrc, order);
}

void dldl_assemble_kp(Ctx &c, const DLdl &d, const double *a, const double *b, const double *cc, double *kpv) {
    const int64_t nnz = (int64_t)d.kp_from.n;
    if (!nnz) return;
    const int grid = (int)std::min<int64_t>((nnz + 255) / 256, 4096);
    hipLaunchKernelGGL(kp_assemble_kernel, dim3(grid), dim3(256), 0, c.stream, nnz, d.kp_from.p, a, b, cc, kpv);
    CPK_HIP(hipGetLastError());
}

void dldl_numeric(Ctx &c, DLdl &d, const double *kpv, double *Lx, double *D) {
    if (!d.ready) throw Error(CPK_ERR_ARGS, "internal: device factorization without its symbolic data");
    const int init[2] = {0, 0x7fffffff};
    CPK_HIP(hipMemcpyAsync(d.bad.p, init, sizeof init, hipMemcpyHostToDevice, c.stream));
    const int64_t nlev = (int64_t)d.lev_ptr.size() - 1;
    // long rows whose y does not fit in LDS stay on the thread kernel (global scratch)
    const size_t lds = 12 * (size_t)d.max_long;
    static const bool big_lds = hipFuncSetAttribute((const void *)ldl_rows_wave_kernel,
                                                    hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    const bool wave = d.max_long > 0 && (lds <= 64 * 1024 || (big_lds && lds <= 160 * 1024));
    for (int64_t l = 0; l < nlev; l++) {
        const int32_t a = d.lev_ptr[l], z = d.lev_ptr[l + 1], w = wave ? d.lev_long[l] : z;
        if (w > a)
            hipLaunchKernelGGL(ldl_rows_kernel, dim3((unsigned)((w - a + 255) / 256)), dim3(256), 0, c.stream,
                               d.lev_rows.p + a, w - a, d.Rp.p, d.Rc.p, d.Rcsc.p, d.Lp.p, d.Li.p, Lx, D, d.Y.p,
                               d.kp_ptr.p, d.kp_tgt.p, d.kp_src.p, kpv, d.bad.p);
        if (z > w)
            hipLaunchKernelGGL(ldl_rows_wave_kernel, dim3((unsigned)(z - w)), dim3(64), lds, c.stream, d.lev_rows.p + w,
                               d.Rp.p, d.Rc.p, d.Rcsc.p, d.Lp.p, d.Li.p, Lx, D, d.kp_ptr.p, d.kp_tgt.p, d.kp_src.p,
                               kpv, d.bad.p);
    }
    CPK_HIP(hipGetLastError());
    int bad[2];
    CPK_HIP(hipMemcpyAsync(bad, d.bad.p, sizeof bad, hipMemcpyDeviceToHost, c.stream));
    CPK_HIP(hipStreamSynchronize(c.stream));
    if (bad[0] & 2) throw Error(CPK_ERR_FACTOR, "ldl (device): inconsistent symbolic structure");
    if (bad[0] & 1)
        throw Error(CPK_ERR_FACTOR, "ldl: zero or NaN pivot at position " + std::to_string(bad[1]) +
                                        " (static 1x1 pivoting needs G > 0 on the nullspace and C > 0)");
}

void dldl_fill(Ctx &c, const DLdl &d, DFactor &dF) {
    const int64_t n = std::max(std::max(d.nf, d.nb), d.N);
    if (!n) return;
    const int grid = (int)std::min<int64_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(ldl_fill_kernel, dim3(grid), dim3(256), 0, c.stream, d.nf, d.nb, d.N, d.fsrc.p, d.bsrc.p,
                       d.dsrc.p, d.Lx.p, d.D.p, dF.fval.p, dF.bval.p, dF.D.p);
    CPK_HIP(hipGetLastError());
}

__global__ void vmap_capture_kernel(const double *__restrict__ x, int64_t n, int32_t *__restrict__ map) {
    for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x)
        map[q] = (int32_t)x[q] - 1;  // exact: indices < 2^31
}

__global__ void vmap_fill_kernel(const int32_t *__restrict__ map, int64_t n, const double *__restrict__ src,
                                 double *__restrict__ x) {
    for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x) {
        const int32_t s = map[q];
        x[q] = s >= 0 ? src[s] : 0.0;
    }
}

void vmap_capture(Ctx &c, const double *x, size_t n, DBuf<int32_t> &map) {
    map.alloc(n);
    if (!n) return;
    const int grid = (int)std::min<size_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(vmap_capture_kernel, dim3(grid), dim3(256), 0, c.stream, x, (int64_t)n, map.p);
    CPK_HIP(hipGetLastError());
}

void vmap_fill(Ctx &c, const int32_t *map, size_t n, const double *src, double *x) {
    if (!n) return;
    const int grid = (int)std::min<size_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(vmap_fill_kernel, dim3(grid), dim3(256), 0, c.stream, map, (int64_t)n, src, x);
    CPK_HIP(hipGetLastError());
}

void dldl_factor(Ctx &c, DLdl &d, const double *kpv, DFactor &dF) {
    dldl_numeric(c, d, kpv, d.Lx.p, d.D.p);
    dldl_fill(c, d, dF);
}

}  // namespace cpk
