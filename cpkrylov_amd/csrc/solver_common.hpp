// solver_common.hpp -- device state + generic streaming kernels shared by the six solvers.
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <type_traits>

#include "dev.hpp"
#include "devutil.hpp"
#include "xacc.hpp"

namespace cpk {

constexpr double kEps = 2.220446049250313e-16;  // MATLAB eps

// Scalar state of a solve, resident in HBM.  Every recurrence scalar of the reference
// solvers lives here and is updated by the single-thread epilogue of a reduction kernel, so
// the host never sits on the iteration's critical path.
struct DState {
    int64_t k;        // completed iterations (MATLAB k / itn)
    int64_t itmax;
    int64_t nh, nh2, nh3;  // history lengths
    int64_t hcap;
    int stop;         // loop condition is false (or an error occurred)
    int running;      // the current iteration is live
    int err;          // 1: indefinite (beta < -100 eps or negative squared norm)
    int flag;         // solver-specific flag (symmlq: moved to CG point)
    int64_t err_iter;
    int exact;        // engine option exact_dots: norm([a b]) by xnorm2 (the oracle's formula)
    double err_val;
    double atol, rtol, btol, stopTol, bstopTol, residNorm;
    // Lanczos family
    double alpha, beta, beta1, oldeps, delta, gamma, gammabar, deltabar, epsln, cs, sn, tau, taubar;
    // cpcg
    double rn2, pAp, qCq;
    // cpcglanczos
    double dg, low, eta, zeta, rhobar, xxNorm2, xNorm, taul, deltal, opNorm2, oldbeta, bkerr, opNorm;
    // cpsymmlq
    double epsdelzeta, epsilonzeta, bstep, snprod, matnorm2, cgresid, lqresid, qrresid, den, betaold, epsilon, zcs,
        zsn, zetabar;
    // cpgmres / cpdqgmres
    int64_t restart, mem, kin, hrow;
    double hk1;
    double *H, *c, *s, *g, *z;
    double *hist, *hist2, *hist3, *aux;
};

__device__ __forceinline__ void push(double *h, int64_t &len, int64_t cap, double v) {
    if (len < cap) h[len] = v;
    len++;
}

// MATLAB norm([a b]) of a 2-vector (cpminres.m:218, cpsymmlq.m:239,291,324)
__device__ __forceinline__ double norm2(const DState *st, double a, double b) {
    return st->exact ? xnorm2(a, b) : hypot(a, b);
}

__device__ __forceinline__ double msign(double a) { return (double)((a > 0) - (a < 0)); }

// util/SymGivens.m:1-29
__device__ __forceinline__ void sym_givens(double a, double b, double &c, double &s, double &d) {
    if (b == 0) {
        c = (a == 0) ? 1.0 : msign(a);
        s = 0.0;
        d = fabs(a);
    } else if (a == 0) {
        c = 0.0;
        s = msign(b);
        d = fabs(b);
    } else if (fabs(b) > fabs(a)) {
        double t = a / b;
        s = msign(b) / sqrt(1 + t * t);
        c = s * t;
        d = b / s;
    } else {
        double t = b / a;
        c = msign(a) / sqrt(1 + t * t);
        s = c * t;
        d = a / c;
    }
}

#ifndef CPK_EW_GRID
#define CPK_EW_GRID 1024
#endif
constexpr int kEwGrid = CPK_EW_GRID;  // fixed grid of the streaming vector kernels (deterministic partials)

// Elementwise kernel over [0, N): F::setup() loads scalars (false => no-op), F::operator()(i).
template <class F>
__global__ __launch_bounds__(kBlock) void ew_kernel(int64_t N, F f) {
    if (!f.setup()) return;
    for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < N; i += (int64_t)gridDim.x * kBlock) f(i);
}

// Elementwise + grid reduction of NV sums: F::operator()(i, acc), F::fin(tot) in the last workgroup.
// A: the accumulator (double: the default fixed-tree sums; XAcc: exact_dots, xacc.hpp).
template <int NV, class F, class A = double>
__global__ __launch_bounds__(kBlock) void ewred_kernel(int64_t N, F f, RedBuf rb) {
    if (!f.setup()) return;
    A acc[NV];
#pragma unroll
    for (int j = 0; j < NV; j++) acc_init(acc[j], rb.xsub, j, NV);
    for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < N; i += (int64_t)gridDim.x * kBlock) f(i, acc);
    double tot[NV];
    if (grid_sum<NV>(acc, rb, tot) && threadIdx.x == 0) f.fin(tot);
}

// Tiled forms for the Arnoldi window passes: each thread takes kTile elements per step,
// kBlock apart (every load coalesced), and F::tile() runs the window loop once for all of them:
// a window coefficient and basis pointer read from LDS serve kTile elements, and kTile
// independent chains keep more loads in flight.  Each element's arithmetic is unchanged.
constexpr int kTile = 4;
template <class F>
__global__ __launch_bounds__(kBlock) void ewt_kernel(int64_t N, F f) {
    if (!f.setup()) return;
    for (int64_t i0 = blockIdx.x * (int64_t)kBlock * kTile + threadIdx.x; i0 < N;
         i0 += (int64_t)gridDim.x * kBlock * kTile)
        f.tile(i0, N);
}
template <int NV, class F, class A = double>
__global__ __launch_bounds__(kBlock) void ewtred_kernel(int64_t N, F f, RedBuf rb) {
    if (!f.setup()) return;
    A acc[NV];
#pragma unroll
    for (int j = 0; j < NV; j++) acc_init(acc[j], rb.xsub, j, NV);
    for (int64_t i0 = blockIdx.x * (int64_t)kBlock * kTile + threadIdx.x; i0 < N;
         i0 += (int64_t)gridDim.x * kBlock * kTile)
        f.tile(i0, N, acc);
    double tot[NV];
    if (grid_sum<NV>(acc, rb, tot) && threadIdx.x == 0) f.fin(tot);
}

// Single-thread scalar step.
template <class F>
__global__ void scalar_kernel(F f) {
    if (threadIdx.x == 0 && blockIdx.x == 0) f();
}

inline int ew_grid(int64_t N) { return (int)std::max<int64_t>(1, std::min<int64_t>((N + kBlock - 1) / kBlock, kEwGrid)); }

template <class F>
inline void launch_ew(Ctx &c, int64_t N, const F &f) {
    hipLaunchKernelGGL(ew_kernel<F>, dim3(ew_grid(N)), dim3(kBlock), 0, c.stream, N, f);
}
// Distributed mode: the reduction kernel leaves its local sums in c.red, RCCL allreduces them
// and this single-thread kernel runs the epilogue on the global sums (identical on every rank).
// Every reduction grid has at least one workgroup, so a rank with no rows still writes its zero
// sums; when the step is not live the kernel writes nothing, and the epilogue, which tests the
// same device predicate, ignores the buffer.
template <class F>
__global__ void ewred_fin_kernel(F f, const double *tot) {
    if (threadIdx.x || blockIdx.x) return;
    if (f.setup()) f.fin(tot);
}
template <int NV, class F>
inline void launch_ewred(Ctx &c, int64_t N, const F &f) {
    c.ensure_partials((size_t)ew_grid(N) * NV);
    const bool dist = c.dist();
    if (c.exact())
        hipLaunchKernelGGL((ewred_kernel<NV, F, XAcc>), dim3(ew_grid(N)), dim3(kBlock), 0, c.stream, N, f, red_buf(c));
    else
        hipLaunchKernelGGL((ewred_kernel<NV, F>), dim3(ew_grid(N)), dim3(kBlock), 0, c.stream, N, f, red_buf(c));
    if (dist) {
        allreduce_red(c, NV);
        hipLaunchKernelGGL(ewred_fin_kernel<F>, dim3(1), dim3(64), 0, c.stream, f, (const double *)c.red.p);
    }
}
#ifndef CPK_EWT_GRID
#define CPK_EWT_GRID kEwGrid
#endif
inline int ewt_grid(int64_t N) {
    return (int)std::max<int64_t>(1, std::min<int64_t>((N + kBlock - 1) / kBlock, CPK_EWT_GRID));
}
template <class F>
inline void launch_ewt(Ctx &c, int64_t N, const F &f) {
    hipLaunchKernelGGL(ewt_kernel<F>, dim3(ewt_grid(N)), dim3(kBlock), 0, c.stream, N, f);
}
template <int NV, class F>
inline void launch_ewtred(Ctx &c, int64_t N, const F &f) {
    c.ensure_partials((size_t)ewt_grid(N) * NV);
    const bool dist = c.dist();
    if (c.exact())
        hipLaunchKernelGGL((ewtred_kernel<NV, F, XAcc>), dim3(ewt_grid(N)), dim3(kBlock), 0, c.stream, N, f,
                           red_buf(c));
    else
        hipLaunchKernelGGL((ewtred_kernel<NV, F>), dim3(ewt_grid(N)), dim3(kBlock), 0, c.stream, N, f, red_buf(c));
    if (dist) {
        allreduce_red(c, NV);
        hipLaunchKernelGGL(ewred_fin_kernel<F>, dim3(1), dim3(64), 0, c.stream, f, (const double *)c.red.p);
    }
}
template <class F>
inline void launch_scalar(Ctx &c, const F &f) {
    hipLaunchKernelGGL(scalar_kernel<F>, dim3(1), dim3(64), 0, c.stream, f);
}

// SpMV epilogue of the Krylov operator blkdiag(A, C) applied to a Lanczos/direction vector,
// with the two inner products <y(1:n), x(1:n)> and <y(n+1:N), x(n+1:N)> of the result against
// the input (alpha = dot(u,vk) + dot(t,qk), pAp and qCq).  F::select(st) picks the input
// vector and the finalize runs F::fin(st, tot).
// F::kNorm (cpminres, fused update): the input is the previous step's unnormalised vector;
// every value read is divided by F::norm(st) (when > 0: the division MinresUpdate would have
// stored, so the same bits), and each row's normalised value is stored to F::out(st) -- the
// normalisation pass folded into the product that reads the vector next.
#ifndef CPK_SPMV_NORM_WAVES
#define CPK_SPMV_NORM_WAVES 5
#endif
template <class F, class A = double>
struct EpiKrylov {
    DState *st;
    const double *xsel;  // resolved input vector
    double *y;
    int64_t n;
    RedBuf rb;
    F f;
    A dn{}, dm{};
    // exact mode: fewer waves (the two expansions take 12 VGPRs where the sums took 4)
    static constexpr int kWaves = std::is_same<A, XAcc>::value ? 4 : (F::kNorm ? CPK_SPMV_NORM_WAVES : CPK_SPMV_WAVES);
    double nb = 0.0;          // F::kNorm: the divisor (0: none)
    double *xo = nullptr;     // F::kNorm: where the normalised input goes
    __device__ bool skip() { return f.skip(st); }
    __device__ const double *xvec(const double *base) {
        xsel = f.select(st, base);
        if constexpr (F::kNorm) nb = f.norm(st), xo = f.out(st);
        acc_init(dn, rb.xsub, 0, 2), acc_init(dm, rb.xsub, 1, 2);
        return xsel;
    }
    __device__ double xl(double v) const {
        if constexpr (F::kNorm) return nb > 0 ? v / nb : v;
        return v;
    }
    __device__ double pre(int64_t r) const { return xl(xsel[r]); }
    __device__ void row(int64_t r, double acc, double xr) {
        y[r] = acc;
        if constexpr (F::kNorm)
            if (xo) xo[r] = xr;
        if (r < n) dadd(dn, acc, xr);
        else dadd(dm, acc, xr);
    }
    __device__ void finish() {
        A v[2] = {dn, dm};
        double tot[2];
        if (grid_sum<2>(v, rb, tot) && threadIdx.x == 0) f.fin(st, tot);
    }
};

}  // namespace cpk
