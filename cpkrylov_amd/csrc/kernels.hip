// kernels.hip -- sparse kernels of the preconditioner apply and the Krylov operator
// (gfx950 / CDNA4, wave64).  All arithmetic is fp64 with FMA contraction disabled
// (-ffp-contract=off), and every row sum runs in increasing column order from 0, the
// accumulation order of MATLAB's sparse mtimes and column-oriented sparse mldivide, so the
// per-row results equal the CPU oracle bit for bit given equal inputs.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "dev.hpp"
#include "devutil.hpp"
#include "spmv.hpp"

namespace cpk {

void Ctx::ensure_partials(size_t count) {
    if (partials.n < count) partials.alloc(count);
    if (!counter.n) {
        counter.alloc(64);
        CPK_HIP(hipMemset(counter.p, 0, counter.bytes()));
    }
}

// ---- device matrix layout -------------------------------------------------------------------
void make_dmat(const HCsr &a, DMat &d) {
    if (a.nnz() > (int64_t)UINT32_MAX) throw Error(CPK_ERR_UNSUPPORTED, "more than 2^32 nonzeros in one matrix");
    d.nrows = a.nrows, d.ncols = a.ncols, d.nnz = a.nnz();
    std::vector<uint32_t> ptr(a.ptr.begin(), a.ptr.end());
    std::vector<int32_t> blk{0};
    int64_t r0 = 0;
    for (int64_t r = 0; r < a.nrows; r++) {
        int64_t rows = r - r0, ents = a.ptr[r + 1] - a.ptr[r0];
        if (rows > 0 && (rows >= kSpmvMaxRows || ents > kSpmvCap)) {
            blk.push_back((int32_t)r);
            r0 = r;
        }
    }
    if (a.nrows > 0) blk.push_back((int32_t)a.nrows);
    d.nblk = (int64_t)blk.size() - 1;
    d.ptr.upload(ptr);
    d.col.upload(a.ind);
    d.val.upload(a.val);
    d.blk.upload(blk);
    d.is_diag = is_diagonal(a);
}

// ---- factor layout ---------------------------------------------------------------------------
void make_dfactor(const Factor &f, const Schedule &s, DFactor &d) {
    const int64_t N = f.N;
    d.N = N;
    d.nnz = (int64_t)f.Li.size();
    // forward rows: transpose of the CSC (columns ascend, so rows come out with ascending columns)
    std::vector<uint32_t> fptr(N + 1, 0);
    for (int32_t i : f.Li) fptr[i + 1]++;
    for (int64_t i = 0; i < N; i++) fptr[i + 1] += fptr[i];
    std::vector<int32_t> fcol(d.nnz);
    std::vector<double> fval(d.nnz);
    {
        std::vector<uint32_t> nx(fptr.begin(), fptr.end() - 1);
        for (int64_t j = 0; j < N; j++)
            for (int64_t p = f.Lp[j]; p < f.Lp[j + 1]; p++) {
                uint32_t q = nx[f.Li[p]]++;
                fcol[q] = (int32_t)j;
                fval[q] = f.Lx[p];
            }
    }
    // backward rows: the CSC columns with row indices in descending order
    std::vector<uint32_t> bptr(N + 1);
    std::vector<int32_t> bcol(d.nnz);
    std::vector<double> bval(d.nnz);
    for (int64_t j = 0; j <= N; j++) bptr[j] = (uint32_t)f.Lp[j];
    for (int64_t j = 0; j < N; j++) {
        int64_t a = f.Lp[j], b = f.Lp[j + 1];
        for (int64_t p = a; p < b; p++) bcol[a + (b - 1 - p)] = f.Li[p], bval[a + (b - 1 - p)] = f.Lx[p];
    }
    d.fptr.upload(fptr);
    d.fcol.upload(fcol);
    d.fval.upload(fval);
    d.bptr.upload(bptr);
    d.bcol.upload(bcol);
    d.bval.upload(bval);
    d.D.upload(f.D);
    d.perm.upload(f.perm);
    d.nblk = (int64_t)s.blk_row.size() - 1;
    d.nlvl = (int64_t)s.lvl_row.size() - 1;
    std::vector<int32_t> bl(s.blk_lvl.begin(), s.blk_lvl.end()), lr(s.lvl_row.begin(), s.lvl_row.end());
    d.blk_lvl.upload(bl);
    d.lvl_row.upload(lr);
    d.round_ptr = s.round_ptr;
}

// ---- SpMV launchers --------------------------------------------------------------------------
namespace {
struct EpiStore {
    double *y;
    const int *run;
    __device__ bool skip() const { return run && *run == 0; }
    __device__ const double *xvec(const double *x) const { return x; }
    __device__ void row(int64_t r, double acc) { y[r] = acc; }
    __device__ void finish() {}
};
struct EpiResid {
    const double *xin;
    int64_t neg_from;
    double *r;
    const int *run, *active;
    __device__ bool skip() const { return cpk::skip(run, active); }
    __device__ const double *xvec(const double *x) const { return x; }
    __device__ void row(int64_t i, double acc) {
        double xi = xin[i];
        if (i >= neg_from) xi = -xi;
        r[i] = xi - acc;
    }
    __device__ void finish() {}
};
struct EpiResidNorm {
    const double *xin;
    int64_t neg_from;
    double *r;
    double tol;
    int *active_out;
    RedBuf rb;
    const int *run, *active;
    double rr = 0.0, xx = 0.0;
    __device__ bool skip() const { return cpk::skip(run, active); }
    __device__ const double *xvec(const double *x) const { return x; }
    __device__ void row(int64_t i, double acc) {
        double xi = xin[i];
        if (i >= neg_from) xi = -xi;
        double ri = xi - acc;
        r[i] = ri;
        rr += ri * ri;
        xx += xi * xi;
    }
    __device__ void finish() {
        double v[2] = {rr, xx}, tot[2];
        if (grid_sum<2>(v, rb, tot) && threadIdx.x == 0) {
            // while nit < nitref & (rNorm >= itref_tol * xNorm | force_itref)   (opLDL2.m:183)
            double rNorm = sqrt(tot[0]), xNorm = sqrt(tot[1]);
            *active_out = (rNorm >= tol * xNorm) ? 1 : 0;
        }
    }
};
}  // namespace

static inline int grid_of(const DMat &A) { return (int)A.nblk; }

void launch_spmv(Ctx &c, const DMat &A, const double *x, double *y, const int *run) {
    if (!A.nblk) return;
    EpiStore e{y, run};
    hipLaunchKernelGGL(spmv_stream<EpiStore>, dim3(grid_of(A)), dim3(kBlock), 0, c.stream, A.ptr.p, A.col.p,
                       A.val.p, A.blk.p, x, (int64_t)0, e);
    CPK_HIP(hipGetLastError());
}

void launch_spmv_colmask(Ctx &c, const DMat &A, int64_t col_min, const double *x, double *y, const int *run) {
    if (!A.nblk) return;
    EpiStore e{y, run};
    hipLaunchKernelGGL(spmv_stream<EpiStore>, dim3(grid_of(A)), dim3(kBlock), 0, c.stream, A.ptr.p, A.col.p,
                       A.val.p, A.blk.p, x, col_min, e);
    CPK_HIP(hipGetLastError());
}

void launch_spmv_resid(Ctx &c, const DMat &A, const double *xin, int64_t neg_from, const double *y, double *r,
                       const int *run, const int *active) {
    if (!A.nblk) return;
    EpiResid e{xin, neg_from, r, run, active};
    hipLaunchKernelGGL(spmv_stream<EpiResid>, dim3(grid_of(A)), dim3(kBlock), 0, c.stream, A.ptr.p, A.col.p,
                       A.val.p, A.blk.p, y, (int64_t)0, e);
    CPK_HIP(hipGetLastError());
}

void launch_spmv_resid_norm(Ctx &c, const DMat &A, const double *xin, int64_t neg_from, const double *y, double *r,
                            double tol, int *active_out, const int *run, const int *active) {
    if (!A.nblk) return;
    c.ensure_partials((size_t)A.nblk * 2);
    EpiResidNorm e{xin, neg_from, r, tol, active_out, RedBuf{c.partials.p, c.counter.p}, run, active};
    hipLaunchKernelGGL(spmv_stream<EpiResidNorm>, dim3(grid_of(A)), dim3(kBlock), 0, c.stream, A.ptr.p, A.col.p,
                       A.val.p, A.blk.p, y, (int64_t)0, e);
    CPK_HIP(hipGetLastError());
}

// ---- level-scheduled triangular sweeps -------------------------------------------------------
// One workgroup per schedule block.  A block holds whole elimination subtrees; its rows are
// contiguous and grouped by intra-block level, so a level is a contiguous row range and the
// only synchronisation inside a block is a workgroup barrier between levels.  Rows of other
// blocks that a block reads were written by an earlier launch (earlier round).
__global__ __launch_bounds__(kBlock) void sptrsv_fwd_kernel(
    int64_t blk0, const int32_t *__restrict__ blk_lvl, const int32_t *__restrict__ lvl_row,
    const uint32_t *__restrict__ ptr, const int32_t *__restrict__ col, const double *__restrict__ val,
    const int32_t *__restrict__ perm, const double *__restrict__ xin, int64_t neg_from, double *w,
    const int *run, const int *active) {
    if (skip(run, active)) return;
    const int64_t b = blk0 + blockIdx.x;
    const int l0 = blk_lvl[b], l1 = blk_lvl[b + 1];
    for (int l = l0; l < l1; l++) {
        const int r0 = lvl_row[l], r1 = lvl_row[l + 1];
        for (int k = r0 + (int)threadIdx.x; k < r1; k += kBlock) {
            const int32_t src = perm[k];
            double acc = xin[src];
            if (src >= neg_from) acc = -acc;
            const uint32_t e1 = ptr[k + 1];
            for (uint32_t e = ptr[k]; e < e1; e++) acc -= val[e] * w[col[e]];
            w[k] = acc;
        }
        __syncthreads();
    }
}

template <bool ADD>
__global__ __launch_bounds__(kBlock) void sptrsv_bwd_kernel(
    int64_t blk0, const int32_t *__restrict__ blk_lvl, const int32_t *__restrict__ lvl_row,
    const uint32_t *__restrict__ ptr, const int32_t *__restrict__ col, const double *__restrict__ val,
    const double *__restrict__ D, const int32_t *__restrict__ perm, double *w, double *out, const int *run,
    const int *active) {
    if (skip(run, active)) return;
    const int64_t b = blk0 + blockIdx.x;
    const int l0 = blk_lvl[b], l1 = blk_lvl[b + 1];
    for (int l = l1 - 1; l >= l0; l--) {
        const int r0 = lvl_row[l], r1 = lvl_row[l + 1];
        for (int k = r0 + (int)threadIdx.x; k < r1; k += kBlock) {
            double acc = w[k] / D[k];
            const uint32_t e1 = ptr[k + 1];
            for (uint32_t e = ptr[k]; e < e1; e++) acc -= val[e] * w[col[e]];
            w[k] = acc;
            const int32_t dst = perm[k];
            if (ADD) out[dst] = out[dst] + acc;
            else out[dst] = acc;
        }
        __syncthreads();
    }
}

void launch_sptrsv_fwd(Ctx &c, const DFactor &F, const double *xin, int64_t neg_from, double *w, const int *run,
                       const int *active) {
    const int64_t R = (int64_t)F.round_ptr.size() - 1;
    for (int64_t r = 0; r < R; r++) {
        const int64_t b0 = F.round_ptr[r], nb = F.round_ptr[r + 1] - b0;
        if (!nb) continue;
        hipLaunchKernelGGL(sptrsv_fwd_kernel, dim3((unsigned)nb), dim3(kBlock), 0, c.stream, b0, F.blk_lvl.p,
                           F.lvl_row.p, F.fptr.p, F.fcol.p, F.fval.p, F.perm.p, xin, neg_from, w, run, active);
    }
    CPK_HIP(hipGetLastError());
}

void launch_sptrsv_bwd(Ctx &c, const DFactor &F, double *w, double *out, bool add, const int *run,
                       const int *active) {
    const int64_t R = (int64_t)F.round_ptr.size() - 1;
    for (int64_t r = R - 1; r >= 0; r--) {
        const int64_t b0 = F.round_ptr[r], nb = F.round_ptr[r + 1] - b0;
        if (!nb) continue;
        if (add)
            hipLaunchKernelGGL(sptrsv_bwd_kernel<true>, dim3((unsigned)nb), dim3(kBlock), 0, c.stream, b0,
                               F.blk_lvl.p, F.lvl_row.p, F.bptr.p, F.bcol.p, F.bval.p, F.D.p, F.perm.p, w, out, run,
                               active);
        else
            hipLaunchKernelGGL(sptrsv_bwd_kernel<false>, dim3((unsigned)nb), dim3(kBlock), 0, c.stream, b0,
                               F.blk_lvl.p, F.lvl_row.p, F.bptr.p, F.bcol.p, F.bval.p, F.D.p, F.perm.p, w, out, run,
                               active);
    }
    CPK_HIP(hipGetLastError());
}

// ---- small helpers ---------------------------------------------------------------------------
__global__ void set_concat_kernel(double *dst, const double *a, int64_t na, int64_t nb) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < na + nb; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = i < na ? a[i] : 0.0;
}

void launch_set_concat(Ctx &c, double *dst, const double *a, int64_t na, int64_t nb) {
    int64_t tot = na + nb;
    if (!tot) return;
    int grid = (int)std::min<int64_t>((tot + kBlock - 1) / kBlock, 2048);
    hipLaunchKernelGGL(set_concat_kernel, dim3(grid), dim3(kBlock), 0, c.stream, dst, a, na, nb);
    CPK_HIP(hipGetLastError());
}

}  // namespace cpk
