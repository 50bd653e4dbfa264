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

void dldl_setup(DLdl &d, const LdlSymbolic &sym, const Factor &f, const std::vector<int32_t> &fsrc,
                const std::vector<int32_t> &bsrc, const std::vector<int32_t> &order) {
    d.N = f.N;
    d.nnz = (int64_t)f.Li.size();
    d.nf = (int64_t)fsrc.size(), d.nb = (int64_t)bsrc.size();
    d.lev_ptr = sym.lev_ptr;
    d.lev_rows.upload(sym.lev_rows);
    d.Rp.upload(sym.Rp);
    d.Rc.upload(sym.Rc);
    d.Rcsc.upload(sym.Rcsc);
    std::vector<int32_t> lp(f.Lp.begin(), f.Lp.end());
    d.Lp.upload(lp);
    d.Li.upload(f.Li);
    d.kp_ptr.upload(sym.kp_ptr);
    d.kp_tgt.upload(sym.kp_tgt);
    d.kp_src.upload(sym.kp_src);
    d.fsrc.upload(fsrc);
    d.bsrc.upload(bsrc);
    d.dsrc.upload(order);
    d.Lx.alloc((size_t)std::max<int64_t>(d.nnz, 1));
    d.D.alloc((size_t)std::max<int64_t>(d.N, 1));
    d.Y.alloc((size_t)std::max<int64_t>(d.nnz, 1));
    d.bad.alloc(2);
    d.ready = true;
}

void dldl_assemble_kp(Ctx &c, const DLdl &d, const double *a, const double *b, const double *cc, double *kpv) {
    const int64_t nnz = (int64_t)d.kp_from.n;
    if (!nnz) return;
    const int grid = (int)std::min<int64_t>((nnz + 255) / 256, 4096);
    hipLaunchKernelGGL(kp_assemble_kernel, dim3(grid), dim3(256), 0, c.stream, nnz, d.kp_from.p, a, b, cc, kpv);
    CPK_HIP(hipGetLastError());
}

void dldl_factor(Ctx &c, DLdl &d, const double *kpv, DFactor &dF) {
    if (!d.ready) throw Error(CPK_ERR_ARGS, "internal: device factorization without its symbolic data");
    const int init[2] = {0, 0x7fffffff};
    CPK_HIP(hipMemcpyAsync(d.bad.p, init, sizeof init, hipMemcpyHostToDevice, c.stream));
    const int64_t nlev = (int64_t)d.lev_ptr.size() - 1;
    for (int64_t l = 0; l < nlev; l++) {
        const int32_t a = d.lev_ptr[l], z = d.lev_ptr[l + 1];
        if (z <= a) continue;
        const int nr = z - a;
        hipLaunchKernelGGL(ldl_rows_kernel, dim3((unsigned)((nr + 255) / 256)), dim3(256), 0, c.stream,
                           d.lev_rows.p + a, nr, d.Rp.p, d.Rc.p, d.Rcsc.p, d.Lp.p, d.Li.p, d.Lx.p, d.D.p, d.Y.p,
                           d.kp_ptr.p, d.kp_tgt.p, d.kp_src.p, kpv, d.bad.p);
    }
    CPK_HIP(hipGetLastError());
    int bad[2];
    CPK_HIP(hipMemcpyAsync(bad, d.bad.p, sizeof bad, hipMemcpyDeviceToHost, c.stream));
    CPK_HIP(hipStreamSynchronize(c.stream));
    if (bad[0] & 2) throw Error(CPK_ERR_FACTOR, "ldl (device): inconsistent symbolic structure");
    if (bad[0] & 1)
        throw Error(CPK_ERR_FACTOR, "ldl: zero or NaN pivot at position " + std::to_string(bad[1]) +
                                        " (static 1x1 pivoting needs G > 0 on the nullspace and C > 0)");
    const int64_t n = std::max(std::max(d.nf, d.nb), d.N);
    if (!n) return;
    const int grid = (int)std::min<int64_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(ldl_fill_kernel, dim3(grid), dim3(256), 0, c.stream, d.nf, d.nb, d.N, d.fsrc.p, d.bsrc.p,
                       d.dsrc.p, d.Lx.p, d.D.p, dF.fval.p, dF.bval.p, dF.D.p);
    CPK_HIP(hipGetLastError());
}

}  // namespace cpk
