// solvers.hip -- the six constraint-preconditioned Krylov solvers on the device.
//
// Each solver restates its MATLAB kernel (kernels/cp*.m) as a short sequence of fused HIP
// kernels per iteration.  Vectors are N-vectors [x-part; y-part], so the reference's pairs
// (vk, qk), (u, t), (wv, wq), (x, y) each live in one HBM array and one streaming pass
// updates both halves.  All recurrence scalars stay on the device (DState); a solver
// iteration is captured once into a hipGraph and replayed in batches, and the host only
// polls the stop flag between batches.  Elementwise updates keep MATLAB's left-to-right
// evaluation order with FMA contraction disabled.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <exception>
#include <functional>
#include <memory>
#include <string>

#include "solver_common.hpp"
#include "solvers.hpp"
#include "spmv.hpp"

namespace cpk {

namespace {

constexpr double kEps100 = 100 * kEps;

// ----------------------------------------------------------------------------------------------
// Krylov SpMV policies (first kernel of an iteration): pick the input vector from the
// iteration index and run the scalar step that consumes the two inner products.
// ----------------------------------------------------------------------------------------------
struct PolStart {  // starts an iteration: decides `running` from `stop`
    __device__ static bool start(DState *st) {
        const bool s = st->stop != 0;
        if (blockIdx.x == 0 && threadIdx.x == 0) st->running = s ? 0 : 1;
        return s;
    }
};

// cpminres.m:187-189 / cpcglanczos.m:232-234 / cpsymmlq.m:231-268 : u = A*vk; t = C*qk; alpha
// cpminres with the fused update (raw set): the input is the previous Lanczos step's
// unnormalised vector; the product divides what it reads by beta and stores vk normalised
// into its ring slot (EpiKrylov::kNorm), the pass MinresUpdate made on its own before
template <int KIND, bool NORM = false>
struct PolLanczosSpmv {
    static_assert(!NORM || KIND == 0, "the fused update is cpminres's");
    static constexpr bool kNorm = NORM;
    const double *VQ;
    int64_t N;
    int slot_shift;  // vk = VQ[(kk + slot_shift) % 3]
    const double *raw = nullptr;  // NORM: the unnormalised input
    __device__ bool skip(DState *st) { return PolStart::start(st); }
    __device__ bool ran(DState *st) const { return st->running != 0; }
    __device__ const double *select(DState *st, const double *) {
        if (NORM) return raw;
        const int64_t kk = st->k + 1;
        return VQ + ((kk + slot_shift) % 3) * N;
    }
    __device__ double norm(DState *st) const { return st->beta; }
    __device__ double *out(DState *st) const {
        const int64_t kk = st->k + 1;
        return const_cast<double *>(VQ) + ((kk + slot_shift) % 3) * N;
    }
    __device__ void fin(DState *st, const double *tot) {
        const int64_t kk = st->k + 1;
        if (KIND == 1) {  // cpcglanczos
            st->alpha = tot[0] + tot[1];
            st->dg = st->alpha - st->low * st->low * st->dg;
            st->zeta = st->eta / st->dg;
        } else if (KIND == 2) {  // cpsymmlq: the loop-head norm estimates (cpsymmlq.m:233-252)
            const double matnorm = sqrt(st->matnorm2);
            const double epsmat = matnorm * kEps;
            double den = st->gammabar;
            if (den == 0) den = epsmat;
            st->den = den;
            st->lqresid = norm2(st, st->epsdelzeta, st->epsilonzeta);
            st->qrresid = st->snprod * st->beta1;
            st->cgresid = st->qrresid * st->beta / fabs(den);
            push(st->hist2, st->nh2, st->hcap, st->lqresid);
            push(st->hist3, st->nh3, st->hcap, st->qrresid);
            push(st->hist, st->nh, st->hcap, st->cgresid);
            st->betaold = st->beta;
            st->alpha = tot[0] + tot[1];
        } else {  // cpminres
            st->alpha = tot[0] + tot[1];
        }
        st->k = kk;
    }
};

// cpcg.m:151-154 : Ap = A*p; pAp; Cq = C*q; qCq; alpha = residNorm2/(pAp+qCq)
struct PolCgSpmv {
    static constexpr bool kNorm = false;
    const double *PQ;
    __device__ bool skip(DState *st) { return PolStart::start(st); }
    __device__ bool ran(DState *st) const { return st->running != 0; }
    __device__ const double *select(DState *, const double *) { return PQ; }
    __device__ void fin(DState *st, const double *tot) {
        const int64_t kk = st->k + 1;
        st->pAp = tot[0];
        st->qCq = tot[1];
        st->alpha = st->rn2 / (st->pAp + st->qCq);
        if (st->aux) {
            st->aux[3 * (kk - 1) + 0] = st->pAp;
            st->aux[3 * (kk - 1) + 1] = st->qCq;
            st->aux[3 * (kk - 1) + 2] = st->alpha;
        }
        st->k = kk;
    }
};

// GMRES family: u = A*V_k; t = C*Q_k (no inner products needed)
struct PolArnoldiSpmv {
    static constexpr bool kNorm = false;
    const double *V;
    int64_t N;
    int64_t ring;  // 0: GMRES (column k-1), >0: DQGMRES ring size mem+1
    __device__ bool skip(DState *st) { return PolStart::start(st); }
    __device__ bool ran(DState *st) const { return st->running != 0; }
    __device__ const double *select(DState *st, const double *) {
        const int64_t kk = st->k + 1;
        const int64_t pos = ring ? (kk - 1) % ring : (kk - 1);
        return V + pos * N;
    }
    __device__ void fin(DState *st, const double *) { st->k = st->k + 1; }
};

// Pre-step spmv (cpsymmlq.m:198-200): no running/stop logic.
struct PolPlainSpmv {
    static constexpr bool kNorm = false;
    const double *X;
    __device__ bool skip(DState *) { return false; }
    __device__ bool ran(DState *) const { return true; }
    __device__ const double *select(DState *, const double *) { return X; }
    __device__ void fin(DState *st, const double *tot) { st->alpha = tot[0] + tot[1]; }
};

// distributed mode: publish the halo of the vector the policy selects, then run the epilogue
// on the allreduced inner products
template <class P>
__global__ void krylov_pack_kernel(P pol, DState *st, const int32_t *__restrict__ idx, int64_t n, double *out) {
    const double *x = pol.select(st, nullptr);
    double nb = 0.0;
    if constexpr (P::kNorm) nb = pol.norm(st);
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const double v = x[idx[i]];
        out[i] = nb > 0 ? v / nb : v;
    }
}
template <class P>
__global__ void krylov_fin_kernel(P pol, DState *st, const double *tot) {
    if (threadIdx.x || blockIdx.x) return;
    if (pol.ran(st)) pol.fin(st, tot);
}

// distributed mode with the partials carried by the separator exchange (Precond::apply with
// piggy_src = c.red): the epilogue on the rank-ordered sum of every rank's two partials
template <class P>
__global__ void krylov_fin_sep_kernel(P pol, DState *st, const double *rbuf, int nranks, int64_t kt,
                                      int64_t kt_data) {
    if (threadIdx.x || blockIdx.x) return;
    if (!pol.ran(st)) return;
    double tot[2] = {0.0, 0.0};
    for (int r = 0; r < nranks; r++)
        for (int j = 0; j < 2; j++) tot[j] += rbuf[(int64_t)r * kt + kt_data + j];
    pol.fin(st, tot);
}
template <class P>
void launch_krylov_fin_sep(Ctx &c, const DSep &S, DState *st, const P &pol) {
    hipLaunchKernelGGL(krylov_fin_sep_kernel<P>, dim3(1), dim3(64), 0, c.stream, pol, st, (const double *)S.rbuf.p,
                       c.nranks, S.kt, S.kt_data);
    CPK_HIP(hipGetLastError());
}

// distributed mode: publish the halo of the vector the policy selects
template <class P>
void launch_krylov_halo(Ctx &c, const DMat &AC, DState *st, const P &pol) {
    if (AC.nsend > 0)
        hipLaunchKernelGGL(krylov_pack_kernel<P>, dim3((unsigned)std::min<int64_t>((AC.nsend + 255) / 256, 1024)),
                           dim3(256), 0, c.stream, pol, st, AC.send.p, AC.nsend, AC.sbuf.p);
    c.comm->allgather(AC.sbuf.p, AC.rbuf.p, (size_t)AC.kstride, c.stream);
}

// distributed, the Lanczos step's beta partials carried by the next vector's halo exchange: the
// step's reduction leaves the two local sums in the payload's spare slots, and its last
// workgroup recomputes the new vector's halo entries with the step's own formula (the other
// workgroups' stores are not yet visible across XCDs) into the payload.  After the allgather
// one block sums the partials in rank order, runs the step's epilogue and normalises the
// received halo exactly as the owners normalise their rows (MinresUpdate: v = v / beta when
// beta > 0).
template <class F>
__global__ __launch_bounds__(kBlock) void lanczos_step_halo_kernel(int64_t N, F f, RedBuf rb,
                                                                   const int32_t *__restrict__ idx, int64_t nsend,
                                                                   double *sbuf) {
    if (!f.setup()) return;
    double acc[2] = {0.0, 0.0};
    for (int64_t i0 = blockIdx.x * (int64_t)kBlock * kTile + threadIdx.x; i0 < N; i0 += (int64_t)gridDim.x * kBlock * kTile)
        f.tile(i0, N, acc);  // the tiled order of ewtred_kernel (the 1-GPU step): the same partials
    double tot[2];
    bool last = false;
    grid_sum<2>(acc, rb, tot, &last);  // rb.defer: the payload's spare slots
    if (!last) return;
    for (int64_t j = threadIdx.x; j < nsend; j += kBlock) sbuf[j] = f.value(idx[j]);
}
template <class F>
__global__ void lanczos_fin_halo_kernel(F f, DState *st, double *rbuf, int nranks, int64_t kstride, int64_t kmax) {
    __shared__ int live;
    if (threadIdx.x == 0) {
        double tot[2] = {0.0, 0.0};
        for (int r = 0; r < nranks; r++)
            for (int j = 0; j < 2; j++) tot[j] += rbuf[(int64_t)r * kstride + kmax + j];
        live = f.setup();
        if (live) f.fin(tot);
    }
    __syncthreads();
    if (!live || !(st->running) || !(st->beta > 0)) return;
    const double beta = st->beta;
    for (int64_t i = threadIdx.x; i < (int64_t)nranks * kstride; i += blockDim.x)
        if (i % kstride < kmax) rbuf[i] = rbuf[i] / beta;
}
template <class F>
void launch_lanczos_step_halo(Ctx &c, const DMat &AC, DState *st, int64_t N, const F &f) {
    c.ensure_partials((size_t)ew_grid(N) * 2);
    hipLaunchKernelGGL((lanczos_step_halo_kernel<F>), dim3(ew_grid(N)), dim3(kBlock), 0, c.stream, N, f,
                       RedBuf{c.partials.p, c.counter.p, AC.sbuf.p + AC.kmax}, (const int32_t *)AC.send.p, AC.nsend,
                       AC.sbuf.p);
    c.comm->allgather(AC.sbuf.p, AC.rbuf.p, (size_t)AC.kstride, c.stream);
    hipLaunchKernelGGL(lanczos_fin_halo_kernel<F>, dim3(1), dim3(256), 0, c.stream, f, st, AC.rbuf.p, c.nranks,
                       AC.kstride, AC.kmax);
    CPK_HIP(hipGetLastError());
}

// defer (distributed): leave the local partials in c.red for the caller to carry
// halo_ready: the input's halo is already in AC.rbuf (launch_lanczos_step_halo)
template <class P, class A>
void launch_krylov_spmv_as(Ctx &c, const DMat &AC, DState *st, double *y, int64_t n, const P &pol) {
    using E = EpiKrylov<P, A>;
    E e{st, nullptr, y, n, red_buf(c), pol};
    const unsigned grid = AC.ghosts() ? spmv_grid<E, true>(AC.nblk) : spmv_grid<E, false>(AC.nblk);
    if (AC.ghosts())
        hipLaunchKernelGGL((spmv_stream<E, true>), dim3(grid), dim3(kBlock), 0, c.stream, AC.ptr.p, AC.col.p, AC.val.p,
                           AC.blk.p, AC.nblk, (const double *)nullptr, (int64_t)0, e, (const double *)AC.rbuf.p,
                           AC.nloc);
    else
        hipLaunchKernelGGL((spmv_stream<E, false>), dim3(grid), dim3(kBlock), 0, c.stream, AC.ptr.p, AC.col.p,
                           AC.val.p, AC.blk.p, AC.nblk, (const double *)nullptr, (int64_t)0, e,
                           (const double *)nullptr, (int64_t)0);
}
template <class P>
void launch_krylov_spmv(Ctx &c, const DMat &AC, DState *st, double *y, int64_t n, const P &pol, bool defer = false,
                        bool halo_ready = false) {
    const bool dist = c.dist();
    if (defer && c.exact()) throw Error(CPK_ERR_ARGS, "internal: deferred Krylov partials in exact mode");
    if (AC.halo() && AC.kmax > 0 && !halo_ready) launch_krylov_halo(c, AC, st, pol);
    if (c.exact()) launch_krylov_spmv_as<P, XAcc>(c, AC, st, y, n, pol);
    else launch_krylov_spmv_as<P, double>(c, AC, st, y, n, pol);
    if (dist && !defer) {
        allreduce_red(c, 2);
        hipLaunchKernelGGL(krylov_fin_kernel<P>, dim3(1), dim3(64), 0, c.stream, pol, st, (const double *)c.red.p);
    }
}

// ----------------------------------------------------------------------------------------------
// shared Lanczos pieces
// ----------------------------------------------------------------------------------------------
// vkp1 = vprec(1:n) - alpha*vk - beta*vkm1 ; qkp1 = qk - vprec(n+1:N); qkp1 = qkp1 - alpha*qk - beta*qkm1
// + beta_new = dot(u, vkp1) + dot(t, qkp1)      (cpminres.m:191-194, identical in the others)
// the fused Lanczos + MINRES pass streams its vectors: nontemporal loads and stores (A/B: CPK_LANCZOS_NT)
#ifndef CPK_LANCZOS_NT
#define CPK_LANCZOS_NT 1
#endif
#if CPK_LANCZOS_NT
#define NTL(p) __builtin_nontemporal_load(p)
#define NTS(p, v) __builtin_nontemporal_store((v), (p))
#else
#define NTL(p) (*(p))
#define NTS(p, v) (*(p) = (v))
#endif
template <int KIND>
struct LanczosStep {
    DState *st;
    double *VQ;
    const double *vprec, *ut;
    double *xy, *W;
    int64_t n, N;
    int sk, skm1, skp1;  // slot offsets relative to kk
    double alpha, beta, zeta;
    const double *vk, *vkm1;
    double *vkp1;
    // distributed cpminres: alpha's partials ride in the separator exchange (sep: its allgathered
    // payload) and every workgroup sums them itself, in rank order (the α epilogue of
    // krylov_fin_sep_kernel, without its dispatch); fin commits alpha and the iteration count
    const double *sep = nullptr;
    int sep_ranks = 0;
    int64_t sep_kt = 0, sep_data = 0, kk = 0;
    // cpminres, fused update (raw set): the new vector goes to raw unnormalised (the next
    // Krylov product normalises it), and from the second iteration on this pass also makes the
    // previous iteration's MinresUpdate w/x update (cpminres.m:221-232): its vk is this step's
    // vkm1, and its scalars are still in the state (this step's epilogue replaces them)
    double *raw = nullptr;
    bool upd = false;
    double u_oldeps = 0, u_delta = 0, u_gamma = 1, u_tau = 0;
    const double *u_w1 = nullptr, *u_w2 = nullptr;
    double *u_wn = nullptr;
    __device__ bool setup() {
        if (!st->running) return false;
        kk = st->k;
        alpha = st->alpha;
        if (sep) {
            double tot[2] = {0.0, 0.0};
            for (int r = 0; r < sep_ranks; r++)
                for (int j = 0; j < 2; j++) tot[j] += sep[(int64_t)r * sep_kt + sep_data + j];
            alpha = tot[0] + tot[1];
            kk += 1;
        }
        beta = st->beta;
        zeta = st->zeta;
        vk = VQ + ((kk + sk) % 3) * N;
        vkm1 = VQ + ((kk + skm1) % 3) * N;
        vkp1 = VQ + ((kk + skp1) % 3) * N;
        if (KIND == 0 && raw) {
            vkp1 = raw;
            upd = kk >= 2;
            if (upd) {  // MinresUpdate's slots at its iteration kp = kk - 1
                const int64_t kp = kk - 1;
                u_oldeps = st->oldeps, u_delta = st->delta, u_gamma = st->gamma, u_tau = st->tau;
                u_wn = W + (kp % 3) * N;
                u_w2 = W + ((kp + 2) % 3) * N;
                u_w1 = W + ((kp + 1) % 3) * N;
            }
        }
        return true;
    }
    // the previous iteration's w/x update of entry i; vprev = its vk (this step's vkm1)
    __device__ void minres_wx(int64_t i, double vprev, double w1, double w2, double x) {
        const double w = (vprev - u_oldeps * w1 - u_delta * w2) / u_gamma;
        u_wn[i] = w;
        xy[i] = (i < n) ? x + u_tau * w : x - u_tau * w;
    }
    // the new (not yet normalised) Lanczos vector's entry i
    __device__ double value(int64_t i) const {
        if (i < n) return vprec[i] - alpha * vk[i] - beta * vkm1[i];
        const double v = vk[i] - vprec[i];
        return v - alpha * vk[i] - beta * vkm1[i];
    }
    template <class A>
    __device__ void operator()(int64_t i, A *acc) {
        const double v = value(i);
        if (i < n) {
            dadd(acc[0], ut[i], v);
            if (KIND == 1) xy[i] = xy[i] + zeta * W[i];  // cpcglanczos.m:238 x = x + zeta*wv
        } else {
            dadd(acc[1], ut[i], v);
            if (KIND == 1) xy[i] = xy[i] - zeta * W[i];  // y = y - zeta*wq
        }
        vkp1[i] = v;
        if (KIND == 0 && upd) minres_wx(i, vkm1[i], u_w1[i], u_w2[i], xy[i]);
    }
    // kTile elements kBlock apart (ewtred_kernel): every load of the tile in flight at once; the
    // per-element arithmetic and the thread's accumulation order over its elements are unchanged
    template <class A>
    __device__ void tile(int64_t i0, int64_t Nn, A *acc) {
        if (i0 + (kTile - 1) * kBlock >= Nn) {
            for (int e = 0; e < kTile; e++)
                if (i0 + e * kBlock < Nn) (*this)(i0 + e * kBlock, acc);
            return;
        }
        if (KIND == 0 && upd) {
            tile_upd(i0, acc);
            return;
        }
        double p[kTile], a[kTile], b[kTile], u[kTile];
#pragma unroll
        for (int e = 0; e < kTile; e++) {
            const int64_t i = i0 + e * kBlock;
            p[e] = vprec[i], a[e] = vk[i], b[e] = vkm1[i], u[e] = ut[i];
        }
#pragma unroll
        for (int e = 0; e < kTile; e++) {
            const int64_t i = i0 + e * kBlock;
            double v;
            if (i < n) {
                v = p[e] - alpha * a[e] - beta * b[e];
                dadd(acc[0], u[e], v);
                if (KIND == 1) xy[i] = xy[i] + zeta * W[i];
            } else {
                const double t = a[e] - p[e];
                v = t - alpha * a[e] - beta * b[e];
                dadd(acc[1], u[e], v);
                if (KIND == 1) xy[i] = xy[i] - zeta * W[i];
            }
            vkp1[i] = v;
        }
    }
    // tile() with the fused MINRES update: all seven loads of the tile in flight at once; the
    // step's arithmetic and accumulation order as in tile(), the update's as in MinresUpdate
    template <class A>
    __device__ void tile_upd(int64_t i0, A *acc) {
        double p[kTile], a[kTile], b[kTile], u[kTile], w1[kTile], w2[kTile], x[kTile];
#pragma unroll
        for (int e = 0; e < kTile; e++) {
            const int64_t i = i0 + e * kBlock;
            p[e] = NTL(vprec + i), a[e] = vk[i], b[e] = NTL(vkm1 + i), u[e] = NTL(ut + i);
            w1[e] = NTL(u_w1 + i), w2[e] = NTL(u_w2 + i), x[e] = NTL(xy + i);
        }
#pragma unroll
        for (int e = 0; e < kTile; e++) {
            const int64_t i = i0 + e * kBlock;
            double v;
            if (i < n) {
                v = p[e] - alpha * a[e] - beta * b[e];
                dadd(acc[0], u[e], v);
            } else {
                const double t = a[e] - p[e];
                v = t - alpha * a[e] - beta * b[e];
                dadd(acc[1], u[e], v);
            }
            NTS(vkp1 + i, v);
            const double w = (b[e] - u_oldeps * w1[e] - u_delta * w2[e]) / u_gamma;  // minres_wx
            NTS(u_wn + i, w);
            NTS(xy + i, (i < n) ? x[e] + u_tau * w : x[e] - u_tau * w);
        }
    }
    __device__ void fin(const double *tot);
};

__device__ inline bool check_beta(DState *st, double raw, int64_t kk) {
    if (raw < -kEps100) {
        st->err = 1;
        st->err_val = raw;
        st->err_iter = kk;
        st->stop = 1;
        return false;
    }
    return true;
}

// cpminres.m:195-235
template <>
__device__ void LanczosStep<0>::fin(const double *tot) {
    if (sep) st->alpha = alpha, st->k = kk;  // PolLanczosSpmv<0>::fin's part
    const double raw = tot[0] + tot[1];
    const int64_t kk = st->k;
    if (!check_beta(st, raw, kk)) return;
    const double b = sqrt(fabs(raw));
    const double oldeps = st->epsln;
    const double delta = st->cs * st->deltabar + st->sn * st->alpha;
    const double gammabar = st->sn * st->deltabar - st->cs * st->alpha;
    st->epsln = st->sn * b;
    st->deltabar = -st->cs * b;
    const double gamma = norm2(st, gammabar, b);
    const double cs = gammabar / gamma, sn = b / gamma;
    st->tau = cs * st->taubar;
    st->taubar = sn * st->taubar;
    st->cs = cs, st->sn = sn;
    st->oldeps = oldeps, st->delta = delta, st->gamma = gamma, st->gammabar = gammabar;
    st->beta = b;
    st->residNorm = st->taubar;
    push(st->hist, st->nh, st->hcap, st->residNorm);
    st->stop = !(st->residNorm > st->stopTol && kk < st->itmax);
}

// cpcglanczos.m:247-295
template <>
__device__ void LanczosStep<1>::fin(const double *tot) {
    const double raw = tot[0] + tot[1];
    const int64_t kk = st->k;
    if (!check_beta(st, raw, kk)) return;
    const double b = sqrt(fabs(raw));
    st->beta = b;
    st->low = b / st->dg;
    st->eta = -st->low * st->eta;
    if (st->btol > 0) {
        const double rho = sqrt(st->rhobar * st->rhobar + st->low * st->low);
        const double cs = st->rhobar / rho;
        const double sn = st->low / rho;
        const double num = st->zeta - st->deltal * st->taul;
        const double taubar = num / st->rhobar;
        st->taul = num / rho;
        st->xNorm = sqrt(st->xxNorm2 + taubar * taubar);
        st->xxNorm2 = st->xxNorm2 + st->taul * st->taul;
        st->deltal = sn;
        st->rhobar = -cs;
        st->opNorm2 = st->opNorm2 + st->alpha * st->alpha + b * b + st->oldbeta * st->oldbeta;
        st->opNorm = sqrt(st->opNorm2);
        st->bkerr = st->opNorm * st->xNorm + st->beta1;
        st->bstopTol = st->btol * st->bkerr;
        if (st->aux) {
            st->aux[3 * (kk - 1) + 0] = st->bkerr;
            st->aux[3 * (kk - 1) + 1] = st->opNorm;
            st->aux[3 * (kk - 1) + 2] = st->xNorm;
        }
    }
    st->residNorm = b * fabs(st->zeta);
    push(st->hist, st->nh, st->hcap, st->residNorm);
    st->oldbeta = b;
    st->stop = !(st->residNorm > st->stopTol && st->residNorm > st->bstopTol && kk < st->itmax);
}

// cpsymmlq.m:273-313
template <>
__device__ void LanczosStep<2>::fin(const double *tot) {
    const double raw = tot[0] + tot[1];
    const int64_t kk = st->k;
    if (!check_beta(st, raw, kk)) return;
    const double b = sqrt(fabs(raw));
    st->beta = b;
    st->matnorm2 = st->matnorm2 + st->alpha * st->alpha + b * b + st->betaold * st->betaold;
    const double gamma = norm2(st, st->gammabar, st->betaold);
    const double cs = st->gammabar / gamma, sn = st->betaold / gamma;
    const double delta = cs * st->deltabar + sn * st->alpha;
    st->gammabar = sn * st->deltabar - cs * st->alpha;
    const double epsilon = sn * b;
    st->deltabar = -cs * b;
    const double zeta = st->epsdelzeta / gamma;
    st->zcs = zeta * cs;
    st->zsn = zeta * sn;
    st->cs = cs, st->sn = sn;
    st->bstep = st->bstep + st->snprod * cs * zeta;
    st->snprod = st->snprod * sn;
    st->epsdelzeta = st->epsilonzeta - delta * zeta;
    st->epsilonzeta = -epsilon * zeta;
    st->stop = !(st->cgresid > st->stopTol && kk < st->itmax);
}

// ----------------------------------------------------------------------------------------------
// device kernels as functors
// ----------------------------------------------------------------------------------------------
// Common solver init: vkp1 = vprec(1:n), qkp1 = -vprec(n+1:N), beta = dot(u, vkp1), plus zeroing.
template <int KIND>
struct InitLanczos {
    DState *st;
    const double *vprec, *b;
    double *v1, *v0, *z2, *xy;
    int64_t n;
    __device__ bool setup() { return true; }
    template <class A>
    __device__ void operator()(int64_t i, A *acc) {
        double v;
        if (i < n) {
            v = vprec[i];
            dadd(acc[0], b[i], v);
        } else {
            v = -vprec[i];
        }
        v1[i] = v;
        if (v0) v0[i] = 0.0;
        if (z2) z2[i] = 0.0;
        xy[i] = 0.0;
    }
    __device__ void fin(const double *tot) {
        const double raw = tot[0];
        st->k = 0;
        st->running = 0;
        if (!check_beta(st, raw, 0)) return;
        const double b1 = sqrt(fabs(raw));
        if (KIND == 0) {  // cpminres.m:141-164
            st->beta = b1;
            st->residNorm = b1;
            st->taubar = b1;
            st->cs = -1, st->sn = 0, st->deltabar = 0, st->epsln = 0;
            st->stopTol = st->atol + st->rtol * st->residNorm;
            push(st->hist, st->nh, st->hcap, st->residNorm);
            st->stop = !(st->residNorm > st->stopTol && 0 < st->itmax);
        } else if (KIND == 1) {  // cpcglanczos.m:154-198
            st->beta = b1;
            st->beta1 = b1;
            st->residNorm = b1;
            push(st->hist, st->nh, st->hcap, st->residNorm);
            st->dg = 0, st->low = 1, st->eta = b1;
            st->rhobar = 1, st->xxNorm2 = 0, st->xNorm = 0, st->taul = 0, st->deltal = 0;
            st->oldbeta = 0, st->opNorm2 = 0;
            st->stopTol = st->atol + st->rtol * st->residNorm;
            st->bstopTol = st->btol * st->beta1;
            st->stop = !(st->residNorm > st->stopTol && st->residNorm > st->bstopTol && 0 < st->itmax);
        } else {  // cpsymmlq.m:148-189
            st->beta1 = b1;
            st->beta = b1;
            st->cgresid = b1;
            st->stopTol = st->atol + st->rtol * st->cgresid;
            if (st->cgresid <= st->stopTol) {
                st->lqresid = b1, st->qrresid = b1;
                push(st->hist, st->nh, st->hcap, st->cgresid);
                push(st->hist2, st->nh2, st->hcap, st->lqresid);
                push(st->hist3, st->nh3, st->hcap, st->qrresid);
                st->flag = 2;  // done before the loop
                st->stop = 1;
            } else {
                st->stop = 0;
            }
        }
    }
};

// if beta > 0: v1 = v1/beta ; optional copy w = v1   (cpminres.m:143-149)
struct NormalizeCopy {
    DState *st;
    double *v, *w;
    int which;  // 0: beta, 1: residNorm, 2: hk1
    double s;
    __device__ bool setup() {
        s = which == 0 ? st->beta : which == 1 ? st->residNorm : st->hk1;
        return true;
    }
    __device__ void operator()(int64_t i) {
        if (which == 0 ? s > 0 : s != 0) v[i] = v[i] / s;
        if (w) w[i] = v[i];
    }
};

// cpminres.m:202-232 (normalisation of vkp1 and the w/x/y updates).  tail (fused update):
// after the loop, the last iteration's w/x update, which no next Lanczos step made
struct MinresUpdate {
    DState *st;
    double *VQ, *W, *xy;
    int64_t n, N;
    bool tail = false;
    double beta, oldeps, delta, gamma, tau;
    const double *vk, *w1, *w2;
    double *vkp1, *wn;
    __device__ bool setup() {
        if (tail ? st->k < 1 : !st->running) return false;
        const int64_t kk = st->k;
        beta = tail ? 0.0 : st->beta;  // tail: vkp1 is not normalised (beta > 0 fails)
        oldeps = st->oldeps, delta = st->delta, gamma = st->gamma, tau = st->tau;
        vk = VQ + (kk % 3) * N;
        vkp1 = VQ + ((kk + 1) % 3) * N;
        wn = W + (kk % 3) * N;
        w2 = W + ((kk + 2) % 3) * N;
        w1 = W + ((kk + 1) % 3) * N;
        return true;
    }
    __device__ void operator()(int64_t i) {
        if (beta > 0) vkp1[i] = vkp1[i] / beta;
        const double w = (vk[i] - oldeps * w1[i] - delta * w2[i]) / gamma;
        wn[i] = w;
        xy[i] = (i < n) ? xy[i] + tau * w : xy[i] - tau * w;
    }
    __device__ void tile(int64_t i0, int64_t Nn) {  // ewt_kernel: the tile's loads all in flight
        if (i0 + (kTile - 1) * kBlock >= Nn) {
            for (int e = 0; e < kTile; e++)
                if (i0 + e * kBlock < Nn) (*this)(i0 + e * kBlock);
            return;
        }
        double q[kTile], a[kTile], b1[kTile], b2[kTile], x[kTile];
#pragma unroll
        for (int e = 0; e < kTile; e++) {
            const int64_t i = i0 + e * kBlock;
            q[e] = vkp1[i], a[e] = vk[i], b1[e] = w1[i], b2[e] = w2[i], x[e] = xy[i];
        }
#pragma unroll
        for (int e = 0; e < kTile; e++) {
            const int64_t i = i0 + e * kBlock;
            if (beta > 0) vkp1[i] = q[e] / beta;
            const double w = (a[e] - oldeps * b1[e] - delta * b2[e]) / gamma;
            wn[i] = w;
            xy[i] = (i < n) ? x[e] + tau * w : x[e] - tau * w;
        }
    }
};

// cpcglanczos.m:256-268 : normalise vkp1; wv = vkp1 - low*wv
struct CglUpdate {
    DState *st;
    double *VQ, *W;
    int64_t N;
    double beta, low;
    double *vkp1;
    __device__ bool setup() {
        if (!st->running) return false;
        beta = st->beta, low = st->low;
        vkp1 = VQ + ((st->k + 1) % 3) * N;
        return true;
    }
    __device__ void operator()(int64_t i) {
        if (beta > 0) vkp1[i] = vkp1[i] / beta;
        W[i] = vkp1[i] - low * W[i];
    }
};

// cpsymmlq.m:280-306 : normalise vkp1; x/y LQ update; w update
struct SymmlqUpdate {
    DState *st;
    double *VQ, *W, *xy;
    int64_t n, N;
    double beta, zcs, zsn, cs, sn;
    const double *vk;
    double *vkp1;
    __device__ bool setup() {
        if (!st->running) return false;
        const int64_t kk = st->k;
        beta = st->beta, zcs = st->zcs, zsn = st->zsn, cs = st->cs, sn = st->sn;
        vk = VQ + ((kk + 1) % 3) * N;
        vkp1 = VQ + ((kk + 2) % 3) * N;
        return true;
    }
    __device__ void operator()(int64_t i) {
        if (beta > 0) vkp1[i] = vkp1[i] / beta;
        const double w = W[i], v = vk[i];
        if (i < n) xy[i] = xy[i] + zcs * w + zsn * v;
        else xy[i] = xy[i] - zcs * w - zsn * v;
        W[i] = sn * w - cs * v;
    }
};

// cpsymmlq.m:198-225 pre-step Lanczos vector (no vkm1 term)
struct SymmlqPre {
    DState *st;
    const double *vk, *vprec, *ut;
    double *vkp1;
    int64_t n;
    double alpha;
    __device__ bool setup() {
        alpha = st->alpha;
        return true;
    }
    template <class A>
    __device__ void operator()(int64_t i, A *acc) {
        double v;
        if (i < n) {
            v = vprec[i] - alpha * vk[i];
            dadd(acc[0], ut[i], v);
        } else {
            v = vk[i] - vprec[i];
            v = v - alpha * vk[i];
            dadd(acc[1], ut[i], v);
        }
        vkp1[i] = v;
    }
    __device__ void fin(const double *tot) {
        const double raw = tot[0] + tot[1];
        if (raw < -kEps100) {
            st->err = 3;  // "Iter 0, 2nd Lanczos vec"
            st->err_val = raw;
            st->err_iter = 0;
            st->stop = 1;
            return;
        }
        const double b = sqrt(fabs(raw));
        st->beta = b;
        st->gammabar = st->alpha;
        st->deltabar = b;
        st->epsdelzeta = st->beta1;
        st->epsilonzeta = 0;
        st->bstep = 0;
        st->snprod = 1;
        st->matnorm2 = st->alpha * st->alpha + b * b;
        st->k = 0;
        st->stop = !(st->cgresid > st->stopTol && 0 < st->itmax);
    }
};

// cpsymmlq.m:317-339 post-loop scalars (single thread)
struct SymmlqPostScalar {
    DState *st;
    __device__ void operator()() {
        const double matnorm = sqrt(st->matnorm2);
        const double epsmat = matnorm * kEps;
        double den = st->gammabar;
        if (den == 0) den = epsmat;
        st->den = den;
        st->lqresid = norm2(st, st->epsdelzeta, st->epsilonzeta);
        st->qrresid = st->snprod * st->beta1;
        push(st->hist2, st->nh2, st->hcap, st->lqresid);
        push(st->hist3, st->nh3, st->hcap, st->qrresid);
        st->flag = 0;
        if (st->cgresid < st->lqresid) {
            st->zetabar = st->epsdelzeta / den;
            st->bstep = st->bstep + st->snprod * st->zetabar;
            st->flag = 1;
        }
    }
};
struct SymmlqMoveCg {
    DState *st;
    double *xy;
    const double *W;
    int64_t n;
    double z;
    __device__ bool setup() {
        if (st->flag != 1) return false;
        z = st->zetabar;
        return true;
    }
    __device__ void operator()(int64_t i) { xy[i] = (i < n) ? xy[i] + z * W[i] : xy[i] - z * W[i]; }
};
// cpsymmlq.m:342-347 : x = x + (bstep/beta1)*vk ; y = y - (bstep/beta1)*qk, qk = -vprec2
struct SymmlqFirstStep {
    DState *st;
    double *xy;
    const double *vprec;
    int64_t n;
    double bs;
    __device__ bool setup() {
        bs = st->bstep / st->beta1;
        return true;
    }
    __device__ void operator()(int64_t i) {
        if (i < n) xy[i] = xy[i] + bs * vprec[i];
        else xy[i] = xy[i] - bs * (-vprec[i]);
    }
};

// ---- cpcg ----------------------------------------------------------------------------------
struct CgInit0 {  // g = -b ; w = 0 ; x = 0 ; a = 0
    const double *b;
    double *GW, *XA;
    int64_t n;
    __device__ bool setup() { return true; }
    __device__ void operator()(int64_t i) {
        GW[i] = i < n ? -b[i] : 0.0;
        XA[i] = 0.0;
    }
};
struct CgInit1 {  // p = -r; q = -u; residNorm2 = g'*r   (cpcg.m:126-133)
    DState *st;
    const double *RU, *GW;
    double *PQ;
    int64_t n;
    __device__ bool setup() { return true; }
    template <class A>
    __device__ void operator()(int64_t i, A *acc) {
        PQ[i] = -RU[i];
        if (i < n) dadd(acc[0], GW[i], RU[i]);
    }
    __device__ void fin(const double *tot) {
        st->k = 0;
        st->running = 0;
        st->rn2 = tot[0];
        if (st->rn2 < 0) {
            st->err = 2, st->err_val = st->rn2, st->err_iter = 0, st->stop = 1;
            return;
        }
        st->residNorm = sqrt(st->rn2);
        st->stopTol = st->atol + st->rtol * st->residNorm;
        push(st->hist, st->nh, st->hcap, st->residNorm);
        st->stop = !(st->residNorm > st->stopTol && 0 < st->itmax);
    }
};
struct CgStep {  // x += alpha p; a += alpha q; g += alpha Ap; w += alpha Cq   (cpcg.m:161-164)
    DState *st;
    double *XA, *GW;
    const double *PQ, *APCQ;
    double alpha;
    __device__ bool setup() {
        if (!st->running) return false;
        alpha = st->alpha;
        return true;
    }
    __device__ void operator()(int64_t i) {
        XA[i] = XA[i] + alpha * PQ[i];
        GW[i] = GW[i] + alpha * APCQ[i];
    }
};
struct CgResid {  // t = a + u; residNorm2_new = g'*r + t'*w   (cpcg.m:166-176)
    DState *st;
    const double *XA, *RU, *GW;
    double *TT;
    int64_t n;
    __device__ bool setup() { return st->running != 0; }
    template <class A>
    __device__ void operator()(int64_t i, A *acc) {
        if (i < n) {
            dadd(acc[0], GW[i], RU[i]);
        } else {
            const double t = XA[i] + RU[i];
            TT[i] = t;
            dadd(acc[1], t, GW[i]);
        }
    }
    __device__ void fin(const double *tot) {
        const int64_t kk = st->k;
        const double nw = tot[0] + tot[1];
        st->beta = nw / st->rn2;
        st->rn2 = nw;
        if (st->rn2 < 0) {
            st->err = 2, st->err_val = st->rn2, st->err_iter = kk, st->stop = 1;
            return;
        }
        st->residNorm = sqrt(st->rn2);
        push(st->hist, st->nh, st->hcap, st->residNorm);
        st->stop = !(st->residNorm > st->stopTol && kk < st->itmax);
    }
};
struct CgDir {  // p = -r + beta*p; q = -t + beta*q
    DState *st;
    const double *RU, *TT;
    double *PQ;
    int64_t n;
    double beta;
    __device__ bool setup() {
        if (!st->running) return false;
        beta = st->beta;
        return true;
    }
    __device__ void operator()(int64_t i) { PQ[i] = (i < n ? -RU[i] : -TT[i]) + beta * PQ[i]; }
};

// ---- GMRES family --------------------------------------------------------------------------
// Start of a GMRES cycle / DQGMRES init:
//   V1 = w(1:n); Q1 = (restart ? y : 0) - w(n+1:N); residNorm = sqrt(dot(u,V1) + dot(t,Q1))
struct ArnoldiStart {
    DState *st;
    const double *w, *ut, *xy;
    double *v1;
    int64_t n;
    int restart_cycle;  // outer > 1 (cpgmres.m:166-171)
    int dq;             // DQGMRES: dot(u, V1) only (cpdqgmres.m:157)
    int first;          // first cycle: sets stopTol and pushes the history
    __device__ bool setup() { return true; }
    template <class A>
    __device__ void operator()(int64_t i, A *acc) {
        double v;
        if (i < n) {
            v = w[i];
            dadd(acc[0], ut[i], v);
        } else {
            v = restart_cycle ? xy[i] - w[i] : -w[i];
            if (!dq) dadd(acc[1], ut[i], v);
        }
        v1[i] = v;
    }
    __device__ void fin(const double *tot) {
        const double rn2 = tot[0] + tot[1];
        st->k = 0;
        st->running = 0;
        if (rn2 < 0) {
            st->err = 4, st->err_val = rn2, st->err_iter = 0, st->stop = 1;
            return;
        }
        st->residNorm = sqrt(rn2);
        if (first) {
            st->stopTol = st->atol + st->rtol * st->residNorm;
            push(st->hist, st->nh, st->hcap, st->residNorm);
        }
        st->g[0] = st->residNorm;
        const int64_t lim = dq ? st->itmax : st->restart;
        st->stop = !(st->residNorm > st->stopTol && 0 < lim);
    }
};

// Restart residual: u = b - A*x (rows < n of TMP = blkdiag(A,C)*xy), t = C*y   (cpgmres.m:167-168)
struct GmresRestartRhs {
    const double *b, *tmp;
    double *ut;
    int64_t n;
    __device__ bool setup() { return true; }
    __device__ void operator()(int64_t i) { ut[i] = i < n ? b[i] - tmp[i] : tmp[i]; }
};

// The Arnoldi window of iteration kk: GMRES j = 1..kk at column j-1;
// DQGMRES j = max(1, kk-mem+1)..kk at ring slot (j-1) % (mem+1).
struct Window {
    int64_t kk, jlo, nv, ring;
    __device__ int64_t slot(int64_t j) const { return ring ? (j - 1) % ring : (j - 1); }
};
__device__ inline Window window(const DState *st, int64_t ring) {
    Window w;
    w.kk = st->k;
    w.ring = ring;
    w.jlo = ring ? max((int64_t)1, w.kk - st->mem + 1) : 1;
    w.nv = w.kk - w.jlo + 1;
    return w;
}
// H storage: GMRES column-major (restart+1) x restart; DQGMRES ring of (mem+2) rows, width mem+2,
// indexed by the reference's (j, kk) with kk the diagonal-compressed column.
__device__ inline double &Hg(DState *st, int64_t i1, int64_t j1) {  // H(i1, j1), 1-based
    return st->H[(i1 - 1) + (j1 - 1) * (st->restart + 1)];
}
__device__ inline double &Hd(DState *st, int64_t j, int64_t kk) {  // H(j, kk), 1-based
    const int64_t W = st->mem + 2;
    return st->H[(j % W) * W + (kk - 1)];
}

// V(:,k+1) = w(1:n) ; Q(:,k+1) = Q(:,k) - w(n+1:N) ; H(j,k) = dot(V_j,u) + dot(Q_j,t) for the window
// (cpgmres.m:212-215, cpdqgmres.m:208-213).  All window dots in one streaming pass.
#ifndef CPK_DOT_GROUP
#define CPK_DOT_GROUP 8
#endif
#ifndef CPK_DOT_TILE
#define CPK_DOT_TILE 3
#endif
constexpr int kDotGroup = CPK_DOT_GROUP;
constexpr int kDotTile = CPK_DOT_TILE;  // elements per thread per step, kBlock apart
__global__ __launch_bounds__(kBlock) void arnoldi_dots_kernel(DState *st, double *V, const double *w,
                                                              const double *ut, int64_t n, int64_t N, int64_t ring,
                                                              int64_t maxv, RedBuf rb) {
    if (!st->running) return;
    const Window win = window(st, ring);
    const int64_t kk = win.kk;
    double *vnew = V + (ring ? (kk % ring) : kk) * N;
    const double *vk = V + win.slot(kk) * N;
    // phase 0: new basis vector (fused with the first dot group).  A thread's indices grow, so
    // it meets the [x; y] boundary at most once: one accumulator per vector, whose x-part
    // sum is parked in accn when the thread crosses into the y-part (same additions, same
    // order as separate x/y accumulators).
    for (int64_t g0 = 0; g0 < win.nv; g0 += kDotGroup) {
        double acc[kDotGroup], accn[kDotGroup];
#pragma unroll
        for (int j = 0; j < kDotGroup; j++) acc[j] = 0.0, accn[j] = 0.0;
        const double *vj[kDotGroup];
#pragma unroll
        for (int j = 0; j < kDotGroup; j++) vj[j] = (g0 + j < win.nv) ? V + win.slot(win.jlo + g0 + j) * N : nullptr;
        bool crossed = false;
        if (kDotTile == 1) {
            for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < N; i += (int64_t)gridDim.x * kBlock) {
                if (!crossed && i >= n) {
#pragma unroll
                    for (int j = 0; j < kDotGroup; j++) accn[j] = acc[j], acc[j] = 0.0;
                    crossed = true;
                }
                const double u = ut[i];
                if (g0 == 0) vnew[i] = i < n ? w[i] : vk[i] - w[i];
#pragma unroll
                for (int j = 0; j < kDotGroup; j++)
                    if (vj[j]) dadd(acc[j], vj[j][i], u);
            }
        } else {
            for (int64_t i0 = blockIdx.x * (int64_t)kBlock * kDotTile + threadIdx.x; i0 < N;
                 i0 += (int64_t)gridDim.x * kBlock * kDotTile) {
                double u[kDotTile], x[kDotTile][kDotGroup];
#pragma unroll
                for (int e = 0; e < kDotTile; e++) {
                    const int64_t i = min(i0 + e * kBlock, N - 1);  // clamped: loads need no predicate
                    u[e] = ut[i];
#pragma unroll
                    for (int j = 0; j < kDotGroup; j++) x[e][j] = vj[j] ? vj[j][i] : 0.0;
                }
#pragma unroll
                for (int e = 0; e < kDotTile; e++) {
                    const int64_t i = i0 + e * kBlock;
                    if (i >= N) break;
                    if (!crossed && i >= n) {
#pragma unroll
                        for (int j = 0; j < kDotGroup; j++) accn[j] = acc[j], acc[j] = 0.0;
                        crossed = true;
                    }
                    if (g0 == 0) vnew[i] = i < n ? w[i] : vk[i] - w[i];
#pragma unroll
                    for (int j = 0; j < kDotGroup; j++)
                        if (vj[j]) dadd(acc[j], x[e][j], u[e]);
                }
            }
        }
        if (!crossed) {
#pragma unroll
            for (int j = 0; j < kDotGroup; j++) accn[j] = acc[j], acc[j] = 0.0;
        }
        double red[2 * kDotGroup];
#pragma unroll
        for (int j = 0; j < kDotGroup; j++) red[2 * j] = accn[j], red[2 * j + 1] = acc[j];
        block_sum<2 * kDotGroup>(red);
        if (threadIdx.x == 0)
            for (int j = 0; j < 2 * kDotGroup && 2 * g0 + j < 2 * win.nv; j++)
                st_agent(rb.partials + (size_t)blockIdx.x * 2 * maxv + 2 * g0 + j, red[j]);
    }
    __shared__ int s_last;
    if (threadIdx.x == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        s_last = arrive_last(rb.counter);
    }
    __syncthreads();
    if (!s_last) return;
    // the last workgroup sums the 2 * nv window sums over the grid's partials, kDotGroup sums at
    // a time (an even count: a window pair stays in one group) with every partial load of a thread in flight (per sum: thread-strided over the
    // workgroups, then the block tree -- the same order for every sum)
    __shared__ double hv[kDotGroup];
    if (!rb.defer && ring && threadIdx.x == 0)  // fresh ring row for H(kk, .)
        for (int64_t c = 1; c <= st->mem + 2; c++) Hd(st, kk, c) = 0.0;
    for (int64_t j0 = 0; j0 < 2 * win.nv; j0 += kDotGroup) {
        double a[kDotGroup];
#pragma unroll
        for (int q = 0; q < kDotGroup; q++) a[q] = 0.0;
        for (unsigned b = threadIdx.x; b < gridDim.x; b += blockDim.x) {
            double t[kDotGroup];
#pragma unroll
            for (int q = 0; q < kDotGroup; q++)
                t[q] = j0 + q < 2 * win.nv ? ld_agent(rb.partials + (size_t)b * 2 * maxv + j0 + q) : 0.0;
#pragma unroll
            for (int q = 0; q < kDotGroup; q++) a[q] += t[q];
        }
        block_sum<kDotGroup>(a);
        if (threadIdx.x == 0)
#pragma unroll
            for (int q = 0; q < kDotGroup; q++) hv[q] = a[q];
        __syncthreads();
        if (threadIdx.x == 0)
            for (int64_t q = 0; q < kDotGroup && j0 + q < 2 * win.nv; q++) {
                const int64_t j = j0 + q;
                if (rb.defer) {  // distributed mode: local window sums out; arnoldi_fin_kernel after the allreduce
                    rb.defer[j] = hv[q];
                } else if (j & 1) {
                    const int64_t jj = win.jlo + j / 2;
                    const double h = hv[q - 1] + hv[q];
                    if (ring) Hd(st, jj, 2 + kk - jj) = h;
                    else Hg(st, jj, kk) = h;
                }
            }
        __syncthreads();
    }
}

// exact_dots: the same window sums, each exact (xacc.hpp).  One streaming pass per group of
// kXDotGroup window vectors (an x-part and a y-part expansion per vector: 24 doubles at 4), the
// workgroup's expansions deposited after each group, and the last workgroup rounds the 2 * nv
// sums in chunks of 16 (an even count: a window pair stays in one chunk).  Sum index
// 2 * (window position) + (0: x-part, 1: y-part) of 2 * maxv per launch.
constexpr int kXDotGroup = 4;
__global__ __launch_bounds__(kBlock) void arnoldi_dots_exact_kernel(DState *st, double *V, const double *w,
                                                                    const double *ut, int64_t n, int64_t N,
                                                                    int64_t ring, int64_t maxv, RedBuf rb) {
    if (!st->running) return;
    const Window win = window(st, ring);
    const int64_t kk = win.kk;
    double *vnew = V + (ring ? (kk % ring) : kk) * N;
    const double *vk = V + win.slot(kk) * N;
    const int nsum = (int)(2 * maxv);
    for (int64_t g0 = 0; g0 < win.nv; g0 += kXDotGroup) {
        XAcc acc[2 * kXDotGroup];  // [2q]: x-part of window vector g0 + q, [2q + 1]: y-part
        const double *vj[kXDotGroup];
#pragma unroll
        for (int q = 0; q < kXDotGroup; q++) {
            acc_init(acc[2 * q], rb.xsub, (int)(2 * (g0 + q)) % nsum, nsum);
            acc_init(acc[2 * q + 1], rb.xsub, (int)(2 * (g0 + q) + 1) % nsum, nsum);
            vj[q] = (g0 + q < win.nv) ? V + win.slot(win.jlo + g0 + q) * N : nullptr;
        }
        for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < N; i += (int64_t)gridDim.x * kBlock) {
            const double u = ut[i];
            if (g0 == 0) vnew[i] = i < n ? w[i] : vk[i] - w[i];
#pragma unroll
            for (int q = 0; q < kXDotGroup; q++)
                if (vj[q]) {
                    if (i < n) dadd(acc[2 * q], vj[q][i], u);
                    else dadd(acc[2 * q + 1], vj[q][i], u);
                }
        }
        block_deposit<2 * kXDotGroup>(acc);  // the unused tail of the last group deposits zeros
    }
    __shared__ int s_last;
    if (threadIdx.x == 0) s_last = arrive_last(rb.counter);
    __syncthreads();
    if (!s_last) return;
    __shared__ int64_t dig[16][kXW];
    __shared__ double hv[16];
    if (!rb.xdefer && ring && threadIdx.x == 0)  // fresh ring row for H(kk, .)
        for (int64_t c = 1; c <= st->mem + 2; c++) Hd(st, kk, c) = 0.0;
    for (int j0 = 0; j0 < 2 * win.nv; j0 += 16) {
        const int ns = (int)min((int64_t)16, 2 * win.nv - j0);
        gather_digits(rb.xsub, nsum, j0, ns, dig, rb.xdefer);
        if (rb.xdefer) continue;
        if (threadIdx.x < ns) hv[threadIdx.x] = xround(dig[threadIdx.x]);
        __syncthreads();
        if (threadIdx.x == 0)
            for (int q = 1; q < ns; q += 2) {
                const int64_t jj = win.jlo + (j0 + q) / 2;
                const double h = hv[q - 1] + hv[q];
                if (ring) Hd(st, jj, 2 + kk - jj) = h;
                else Hg(st, jj, kk) = h;
            }
        __syncthreads();
    }
}

// distributed mode: H(j, k) from the allreduced window sums (same additions as above)
__global__ void arnoldi_fin_kernel(DState *st, int64_t ring, const double *tot) {
    if (threadIdx.x || blockIdx.x || !st->running) return;
    const Window win = window(st, ring);
    const int64_t kk = win.kk;
    if (ring)
        for (int64_t c = 1; c <= st->mem + 2; c++) Hd(st, kk, c) = 0.0;
    for (int64_t j = 0; j < win.nv; j++) {
        const int64_t jj = win.jlo + j;
        const double h = tot[2 * j] + tot[2 * j + 1];
        if (ring) Hd(st, jj, 2 + kk - jj) = h;
        else Hg(st, jj, kk) = h;
    }
}

// the window dots of one Arnoldi step (with the distributed allreduce when needed)
static void launch_arnoldi_dots(Ctx &c, DState *st, double *V, const double *w, const double *ut, int64_t n, int64_t N,
                                int64_t ring, int64_t maxv) {
    const bool dist = c.dist();
    if (dist && (size_t)(2 * maxv) > c.red.n) throw Error(CPK_ERR_UNSUPPORTED, "Arnoldi window too wide for the distributed reduction buffer");
    // at most the resident workgroups (occupancy x CUs): a trailing partial wave of workgroups
    // would double the pass's tail (cf. spmv_grid)
    static const int resident = [] {
        int occ = 0, dev = 0, cus = 256;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void *)arnoldi_dots_kernel, kBlock, 0) != hipSuccess ||
            occ < 1)
            occ = 1;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        return occ * cus;
    }();
    const int grid = std::min(ew_grid(N), resident);
    if (c.exact())
        hipLaunchKernelGGL(arnoldi_dots_exact_kernel, dim3(grid), dim3(kBlock), 0, c.stream, st, V, w, ut, n, N, ring,
                           maxv, red_buf(c));
    else
        hipLaunchKernelGGL(arnoldi_dots_kernel, dim3(grid), dim3(kBlock), 0, c.stream, st, V, w, ut, n, N, ring, maxv,
                           red_buf(c));
    if (dist) {
        allreduce_red(c, (int)(2 * maxv));
        hipLaunchKernelGGL(arnoldi_fin_kernel, dim3(1), dim3(64), 0, c.stream, st, ring, (const double *)c.red.p);
    }
}

// V(:,k+1) -= H(j,k) V(:,j) for the window in order; H(k+1,k) = sqrt(dot(u,V_{k+1}) + dot(t,Q_{k+1}));
// then rotations, SymGivens and the g update (cpgmres.m:214-247, cpdqgmres.m:214-250).
// Window coefficients and basis pointers of one step, tabulated in LDS once per workgroup:
// the per-element loops then read (h_j, V_j) from LDS instead of recomputing ring slots and
// H indices (64-bit divisions) for every element.
constexpr int kWinTab = 1024;
struct WinTab {
    const double *const *p;
    const double *h;
    int nv;
};

struct ArnoldiOrth {
    DState *st;
    double *V;
    const double *ut;
    int64_t n, N, ring;
    Window win;
    double *vnew;
    WinTab tab;
    __device__ bool setup() {
        if (!st->running) return false;
        win = window(st, ring);
        vnew = V + (ring ? (win.kk % ring) : win.kk) * N;
        __shared__ const double *tp[kWinTab];
        __shared__ double th[kWinTab];
        tab.nv = win.nv <= kWinTab ? (int)win.nv : -1;
        for (int j = threadIdx.x; j < tab.nv; j += blockDim.x) {
            tp[j] = V + win.slot(win.jlo + j) * N;
            th[j] = h(win.jlo + j);
        }
        __syncthreads();
        tab.p = tp, tab.h = th;
        return true;
    }
    __device__ double h(int64_t j) const {
        return ring ? Hd(st, j, 2 + win.kk - j) : Hg(st, j, win.kk);
    }
    template <class A>
    __device__ void operator()(int64_t i, A *acc) {
        double v = vnew[i];
        if (tab.nv >= 0) {
#pragma unroll 8
            for (int j = 0; j < tab.nv; j++) v = v - tab.h[j] * tab.p[j][i];
        } else {
            for (int64_t j = win.jlo; j <= win.kk; j++) v = v - h(j) * V[win.slot(j) * N + i];
        }
        vnew[i] = v;
        if (i < n) dadd(acc[0], ut[i], v);  // (no dynamic index: an XAcc array stays in registers)
        else dadd(acc[1], ut[i], v);
    }
    // kTile elements i0 + e * kBlock (ewtred_kernel): the same operations per element; the
    // thread's partial sums take its elements in this tiled order (deterministic)
    template <class A>
    __device__ void tile(int64_t i0, int64_t Nn, A *acc) {
        if (tab.nv < 0 || i0 + (kTile - 1) * kBlock >= Nn) {
            for (int e = 0; e < kTile; e++)
                if (i0 + e * kBlock < Nn) (*this)(i0 + e * kBlock, acc);
            return;
        }
        double v[kTile];
#pragma unroll
        for (int e = 0; e < kTile; e++) v[e] = vnew[i0 + e * kBlock];
#pragma unroll 4
        for (int j = 0; j < tab.nv; j++) {
            const double hj = tab.h[j];
            const double *pj = tab.p[j] + i0;
#pragma unroll
            for (int e = 0; e < kTile; e++) v[e] = v[e] - hj * pj[e * kBlock];
        }
#pragma unroll
        for (int e = 0; e < kTile; e++) {
            const int64_t i = i0 + e * kBlock;
            vnew[i] = v[e];
            if (i < n) dadd(acc[0], ut[i], v[e]);
            else dadd(acc[1], ut[i], v[e]);
        }
    }
    __device__ void fin(const double *tot) {
        const int64_t kk = win.kk;
        const double hn2 = tot[0] + tot[1];
        if (hn2 < 0) {
            st->err = 4, st->err_val = hn2, st->err_iter = kk, st->stop = 1;
            return;
        }
        const double hk1 = sqrt(hn2);
        st->hk1 = hk1;
        if (!ring) {  // cpgmres.m:219-247
            Hg(st, kk + 1, kk) = hk1;
            for (int64_t j = 1; j <= kk - 1; j++) {
                const double Hjk = st->c[j - 1] * Hg(st, j, kk) + st->s[j - 1] * Hg(st, j + 1, kk);
                Hg(st, j + 1, kk) = st->s[j - 1] * Hg(st, j, kk) - st->c[j - 1] * Hg(st, j + 1, kk);
                Hg(st, j, kk) = Hjk;
            }
            double c, s, d;
            sym_givens(Hg(st, kk, kk), Hg(st, kk + 1, kk), c, s, d);
            st->c[kk - 1] = c, st->s[kk - 1] = s, Hg(st, kk, kk) = d;
            Hg(st, kk + 1, kk) = 0;
            st->g[kk] = s * st->g[kk - 1];
            st->g[kk - 1] = c * st->g[kk - 1];
            st->residNorm = fabs(st->g[kk]);
            push(st->hist, st->nh, st->hcap, st->residNorm);
            st->stop = !(st->residNorm > st->stopTol && kk < st->restart);
        } else {  // cpdqgmres.m:218-269
            const int64_t mem = st->mem, M1 = mem + 1;
            const int64_t kpos = (kk - 1) % M1, kp1pos = kk % M1, rotpos = (kk - 1) % mem;
            Hd(st, kk, 1) = hk1;
            for (int64_t j = max((int64_t)1, kk - mem); j <= kk - 1; j++) {
                const int64_t jr = (j - 1) % mem, k1 = kk - j + 1, k2 = k1 + 1;
                const double Hjk = st->c[jr] * Hd(st, j, k2) + st->s[jr] * Hd(st, j + 1, k1);
                Hd(st, j + 1, k1) = st->s[jr] * Hd(st, j, k2) - st->c[jr] * Hd(st, j + 1, k1);
                Hd(st, j, k2) = Hjk;
            }
            double c, s, d;
            sym_givens(Hd(st, kk, 2), Hd(st, kk, 1), c, s, d);
            st->c[rotpos] = c, st->s[rotpos] = s, Hd(st, kk, 2) = d;
            Hd(st, kk, 1) = 0;
            st->g[kp1pos] = s * st->g[kpos];
            st->g[kpos] = c * st->g[kpos];
            st->residNorm = fabs(st->g[kp1pos]);
            push(st->hist, st->nh, st->hcap, st->residNorm);
            st->stop = !(st->residNorm > st->stopTol && kk < st->itmax);
        }
    }
};

// GMRES: V(:,k+1) /= H(k+1,k) (lucky breakdown if 0)
struct GmresNormalize {
    DState *st;
    double *V;
    int64_t N;
    double h;
    double *v;
    __device__ bool setup() {
        if (!st->running) return false;
        h = st->hk1;
        v = V + st->k * N;
        return true;
    }
    __device__ void operator()(int64_t i) {
        if (h != 0) v[i] = v[i] / h;
    }
};

// DQGMRES: normalise V(:,kp1pos); PV(:,kpos) = (V(:,kpos) - sum H(j,kk) PV(:,jpos)) / H(k,2);
// x = x + g(kpos)*PV(:,kpos); y = y - g(kpos)*PQ(:,kpos)   (cpdqgmres.m:222-265)
struct DqgmresDirection {
    DState *st;
    double *V, *PV, *xy;
    int64_t n, N;
    int64_t kk, mem, M1, kpos, jlo;
    double h, hkk, gk;
    double *vn, *pk;
    const double *vk;
    WinTab tab;
    __device__ bool setup() {
        if (!st->running) return false;
        kk = st->k, mem = st->mem, M1 = mem + 1;
        kpos = (kk - 1) % M1;
        jlo = max((int64_t)1, kk - mem);
        h = st->hk1;
        hkk = Hd(st, kk, 2);
        gk = st->g[kpos];
        vn = V + (kk % M1) * N, vk = V + kpos * N, pk = PV + kpos * N;
        __shared__ const double *tp[kWinTab];
        __shared__ double th[kWinTab];
        const int64_t nv = kk - jlo;
        tab.nv = nv <= kWinTab ? (int)nv : -1;
        for (int j = threadIdx.x; j < tab.nv; j += blockDim.x) {
            const int64_t jj = jlo + j;
            tp[j] = PV + ((jj - 1) % M1) * N;
            th[j] = Hd(st, jj, 2 + kk - jj);
        }
        __syncthreads();
        tab.p = tp, tab.h = th;
        return true;
    }
    __device__ void operator()(int64_t i) {
        if (h != 0) vn[i] = vn[i] / h;
        double pv = vk[i];
        if (tab.nv >= 0) {
#pragma unroll 8
            for (int j = 0; j < tab.nv; j++) pv = pv - tab.h[j] * tab.p[j][i];
        } else {
            for (int64_t j = jlo; j <= kk - 1; j++) pv = pv - Hd(st, j, 2 + kk - j) * PV[((j - 1) % M1) * N + i];
        }
        pv = pv / hkk;
        pk[i] = pv;
        xy[i] = i < n ? xy[i] + gk * pv : xy[i] - gk * pv;
    }
    __device__ void tile(int64_t i0, int64_t Nn) {
        if (tab.nv < 0 || i0 + (kTile - 1) * kBlock >= Nn) {
            for (int e = 0; e < kTile; e++)
                if (i0 + e * kBlock < Nn) (*this)(i0 + e * kBlock);
            return;
        }
        double pv[kTile];
#pragma unroll
        for (int e = 0; e < kTile; e++) {
            const int64_t i = i0 + e * kBlock;
            if (h != 0) vn[i] = vn[i] / h;
            pv[e] = vk[i];
        }
#pragma unroll 4
        for (int j = 0; j < tab.nv; j++) {
            const double hj = tab.h[j];
            const double *pj = tab.p[j] + i0;
#pragma unroll
            for (int e = 0; e < kTile; e++) pv[e] = pv[e] - hj * pj[e * kBlock];
        }
#pragma unroll
        for (int e = 0; e < kTile; e++) {
            const int64_t i = i0 + e * kBlock;
            const double q = pv[e] / hkk;
            pk[i] = q;
            xy[i] = i < n ? xy[i] + gk * q : xy[i] - gk * q;
        }
    }
};

// z = H(1:k,1:k) \ g(1:k): column-oriented back substitution (cpgmres.m:257)
struct GmresBackSolve {
    DState *st;
    __device__ void operator()() {
        const int64_t k = st->k;
        for (int64_t i = 0; i < k; i++) st->z[i] = st->g[i];
        for (int64_t j = k; j >= 1; j--) {
            st->z[j - 1] = st->z[j - 1] / Hg(st, j, j);
            for (int64_t i = 1; i < j; i++) st->z[i - 1] = st->z[i - 1] - st->z[j - 1] * Hg(st, i, j);
        }
    }
};
// x = x + V(:,1:k)*z ; q = 0 + Q(:,1:k)*z ; y = y - q   (cpgmres.m:258-260)
struct GmresUpdateX {
    DState *st;
    const double *V;
    double *xy;
    int64_t n, N, k;
    __device__ bool setup() {
        k = st->k;
        return true;
    }
    __device__ void operator()(int64_t i) {
        double t = 0.0;
        for (int64_t j = 0; j < k; j++) t = t + V[j * N + i] * st->z[j];
        if (i < n) xy[i] = xy[i] + t;
        else xy[i] = xy[i] - (0.0 + t);
    }
};

// reg_cpkrylov.m:157 : b1 = b(1:n) - A*xy0(1:n) - B'*xy0(n+1:N)
struct ShiftRhs {
    const double *b, *t1, *t2;
    double *b1;
    __device__ bool setup() { return true; }
    __device__ void operator()(int64_t i) { b1[i] = b[i] - t1[i] - t2[i]; }
};
// x = [xy0(1:n) + dx; xy0(n+1:N) + dy]
struct Recover {
    const double *xy0, *dxy;
    double *x;
    __device__ bool setup() { return true; }
    __device__ void operator()(int64_t i) { x[i] = xy0[i] + dxy[i]; }
};
struct AnyNonzero {  // any(b(n+1:n+m))
    const double *b;
    int64_t n;
    int *out;
    __device__ bool setup() { return true; }
    template <class A>
    __device__ void operator()(int64_t i, A *acc) {
        if (b[n + i] != 0) dadd(acc[0], 1.0, 1.0);  // a count: nonzero iff any
    }
    __device__ void fin(const double *tot) { *out = tot[0] != 0 ? 1 : 0; }
};
struct Copy {
    const double *src;
    double *dst;
    __device__ bool setup() { return true; }
    __device__ void operator()(int64_t i) { dst[i] = src[i]; }
};

}  // namespace

// ==============================================================================================
// host driver
// ==============================================================================================
// A SolveCore is kept by the preconditioner between calls with the same method, operators,
// vectors and captured properties (solver_key): its workspace and the captured iteration
// graphs are reused, so a repeated solve costs its kernels plus one state upload.
struct SolveCore {
    Ctx &c;
    Precond &M;
    const DMat &AC;
    int64_t n, m, N;
    int method;
    bool print = true;
    double atol = 1e-6, rtol = 1e-6, btol = 0, itmax = 0, restart = 50, mem = 50;
    DBuf<DState> dst;
    DState h{};
    DBuf<double> hist, hist2, hist3, aux, H, cvec, svec, gvec, zvec;
    std::vector<DBuf<double>> vecs;
    int64_t printed = 0;
    int batch = 16;
    bool use_graph = true;
    // reused across calls
    std::vector<DBuf<double>> rings;
    size_t ring_next = 0;
    std::vector<std::pair<hipGraph_t, hipGraphExec_t>> graphs;  // one per loop site

    SolveCore(Ctx &cc, Precond &MM, const DMat &ACm, int meth, const cpk_opts *o)
        : c(cc), M(MM), AC(ACm), n(MM.n), m(MM.m), N(MM.N), method(meth) {
        reset(o);
    }
    ~SolveCore() {
        for (auto &g : graphs) {
            if (g.second) (void)hipGraphExecDestroy(g.second);
            if (g.first) (void)hipGraphDestroy(g.first);
        }
    }
    // per-call options (they only reach the device through DState, not through captured kernels)
    void reset(const cpk_opts *o) {
        // defaults use the global sizes (size(A,1) in the reference), identical on every rank
        itmax = (method == CPK_GMRES || method == CPK_DQGMRES) ? (double)(M.gn + M.gm) : (double)M.gn;
        atol = 1e-6, rtol = 1e-6, btol = 0, restart = 50, mem = 50, print = true;
        if (o) {
            if (o->has_atol) atol = o->atol;
            if (o->has_rtol) rtol = o->rtol;
            if (o->has_btol) btol = o->btol;
            if (o->has_itmax) itmax = o->itmax;
            if (o->has_restart) restart = o->restart;
            if (o->has_mem) mem = std::max(1.0, o->mem);  // cpdqgmres.m:116-118
            if (o->has_print) print = o->print != 0;
        }
        use_graph = !c.opts.no_graph;
        if (c.dist() && !(c.comm->capturable() && c.opts.dist_graph)) use_graph = false;
        if (c.rank != 0) print = false;
        batch = c.opts.batch > 0 ? c.opts.batch : 16;
        printed = 0;
        ring_next = 0;
    }

    double *vec(size_t i) {
        while (vecs.size() <= i) {
            vecs.emplace_back();
            vecs.back().alloc(std::max<size_t>((size_t)N, 1));  // a rank may own no rows
        }
        return vecs[i].p;
    }
    // the ring_next-th contiguous allocation of `count` N-vectors (slot rings, Arnoldi bases)
    double *ring(size_t count) {
        if (ring_next == rings.size()) rings.emplace_back();
        DBuf<double> &r = rings[ring_next++];
        const size_t want = std::max<size_t>(count * (size_t)N, 1);  // a rank may own no rows
        if (r.n != want) r.alloc(want);
        return r.p;
    }
    template <class T>
    static void ensure(DBuf<T> &b, size_t count) {
        if (b.n != count) b.alloc(count);
    }

    void setup_state(int64_t hcap, int64_t maxv) {
        ensure(dst, 1);
        std::memset(&h, 0, sizeof h);
        h.itmax = (int64_t)std::min(itmax, 9.0e15);
        if (h.itmax < 0) h.itmax = 0;
        h.atol = atol, h.rtol = rtol, h.btol = btol;
        h.hcap = hcap;
        h.exact = c.exact() ? 1 : 0;
        ensure(hist, hcap);
        ensure(hist2, hcap);
        ensure(hist3, hcap);
        ensure(aux, 3 * hcap);
        h.hist = hist.p, h.hist2 = hist2.p, h.hist3 = hist3.p, h.aux = aux.p;
        h.restart = (int64_t)restart;
        h.mem = (int64_t)mem;
        if (maxv > 0) {
            const int64_t R = h.restart, Mm = h.mem;
            if (method == CPK_GMRES) {
                ensure(H, (R + 1) * R);
                ensure(cvec, R), ensure(svec, R), ensure(gvec, R + 1), ensure(zvec, R);
            } else {
                ensure(H, (Mm + 2) * (Mm + 2));
                ensure(cvec, Mm), ensure(svec, Mm), ensure(gvec, Mm + 1), ensure(zvec, 1);
            }
            H.zero(c.stream), cvec.zero(c.stream), svec.zero(c.stream), gvec.zero(c.stream);
            h.H = H.p, h.c = cvec.p, h.s = svec.p, h.g = gvec.p, h.z = zvec.p;
        }
        CPK_HIP(hipMemcpyAsync(dst.p, &h, sizeof h, hipMemcpyHostToDevice, c.stream));
        size_t need = std::max<size_t>((size_t)AC.nblk * 2, (size_t)M.dKp.nblk * 2);
        const size_t ewg = (size_t)std::max<int64_t>(kEwGrid, ewt_grid(N));
        need = std::max<size_t>(need, ewg * 2);
        need = std::max<size_t>(need, ewg * 2 * std::max<int64_t>(maxv, 1));
        c.ensure_partials(need);
        if (c.exact()) c.ensure_xacc((size_t)std::max<int64_t>(2 * maxv, 4));
    }

    void pull() {
        CPK_HIP(hipMemcpyAsync(&h, dst.p, sizeof h, hipMemcpyDeviceToHost, c.stream));
        CPK_HIP(hipStreamSynchronize(c.stream));
    }

    // ---- the distributed solve's status agreement -------------------------------------------
    // At each agreement point every rank contributes a status word (0, or its error code and
    // rank: solve_status_kernel, which also reads every sweep chain's device error word), the
    // ranks take the maximum (Comm::allreduce_max_i64), and if it is not 0 every rank throws:
    // the failing rank its own error, the others the same code naming that rank.  Points: before
    // the solve's first collective (method_solve_device) and after every graph batch, where the
    // host synchronises anyway (the word travels with the state read-back).  A failure between
    // collectives of a batch enqueued eagerly cannot be contained this way (the other ranks are
    // already inside that batch's collectives); a captured batch fails before it starts.
    DBuf<int64_t> status;
    int64_t status_h = 0;
    int64_t nbatch = 0;
    bool agreeing() const { return c.dist() && c.comm->has_peers(); }
    int64_t status_word(int code) const { return code ? ((int64_t)code << 16) | (0xffff - (c.rank & 0xffff)) : 0; }
    // engine option fail_inject "R:site[:K]" (test hook): does this rank fail at `site` / batch k?
    int injected(const char *site, int64_t k = 0) const {
        if (c.opts.fail_inject.empty()) return 0;
        int r = -1, kk = 0;
        char st[16] = {0};
        if (sscanf(c.opts.fail_inject.c_str(), "%d:%15[a-z]:%d", &r, st, &kk) < 2 || r != c.rank) return 0;
        if (std::string(st) != site) return 0;
        return (std::string(site) == "setup" || kk == k) ? CPK_ERR_HIP : 0;
    }
    void status_enqueue(int code) {
        ensure(status, 1);
        const DFactor *fs[2] = {&M.dF, &M.sep.tsw};
        launch_solve_status(c, fs, 2, status_word(code), status_word(CPK_ERR_HIP), status.p);
        c.comm->allreduce_max_i64(status.p, 1, c.stream);
        CPK_HIP(hipMemcpyAsync(&status_h, status.p, sizeof status_h, hipMemcpyDeviceToHost, c.stream));
    }
    void status_check(std::exception_ptr local) {  // after the stream synchronised
        if (!status_h) return;
        const int code = (int)(status_h >> 16), who = 0xffff - (int)(status_h & 0xffff);
        // the chains' error words are read (and cleared) by check_chain on the rank that set them
        try {
            check_chain(M.dF);
            check_chain(M.sep.tsw);
        } catch (const Error &) {
            if (!local) local = std::current_exception();
        }
        if (local) std::rethrow_exception(local);
        throw Error(code, "distributed solve stopped: rank " + std::to_string(who) + " failed (status " +
                              std::to_string(code) + "); every rank returns its error");
    }
    // the agreement before the solve's first collective
    void agree_setup(std::exception_ptr local, int code) {
        status_enqueue(code);
        CPK_HIP(hipStreamSynchronize(c.stream));
        status_check(local);
    }

    // replay `body` (one iteration) in batches until the device sets `stop`.  A batch is a
    // captured graph of b iterations (b a power of two <= batch), captured once per loop site
    // and size and replayed by later calls with the same key.  After the first batch the size
    // follows the observed convergence rate, so the batch that crosses the tolerance carries
    // few no-op iterations (every kernel tests the device-side `running` flag, so the size
    // only affects time, never results).
    hipGraphExec_t graph_for(size_t site, int b, const std::function<void()> &body) {
        const size_t slot = site * 8 + (size_t)__builtin_ctz((unsigned)b);
        if (graphs.size() <= slot) graphs.resize(slot + 1, {nullptr, nullptr});
        if (!graphs[slot].second) {
            hipGraph_t graph = nullptr;
            try {
                CPK_HIP(hipStreamBeginCapture(c.stream, hipStreamCaptureModeThreadLocal));
                for (int i = 0; i < b; i++) body();
                CPK_HIP(hipStreamEndCapture(c.stream, &graph));
                graphs[slot].first = graph;
                CPK_HIP(hipGraphInstantiate(&graphs[slot].second, graph, nullptr, nullptr, 0));
            } catch (const Error &e) {
                // a transport that cannot be captured (deterministic, so every rank lands here):
                // end the capture, drop the graph and run this solver's batches eagerly
                hipGraph_t g2 = nullptr;
                (void)hipStreamEndCapture(c.stream, &g2);
                if (g2) (void)hipGraphDestroy(g2);
                if (graph && graph != g2) (void)hipGraphDestroy(graph);
                graphs[slot] = {nullptr, nullptr};
                (void)hipGetLastError();
                if (!c.dist()) throw;
                fprintf(stderr, "cpk: iteration-graph capture failed (%s); running batches eagerly\n", e.what());
                use_graph = false;
                return nullptr;
            }
        }
        return graphs[slot].second;
    }

    static int pow2_at_least(double v, int cap) {
        int b = 1;
        while (b < cap && b < v) b <<= 1;
        return b;
    }

    void loop(const std::function<void()> &body, const std::function<void()> &printer, size_t site = 0) {
        pull();
        if (h.stop) return;
        const int64_t guard = h.k + (int64_t)std::min(itmax, 4.0e9) + 2 * batch + 2;
        int b = pow2_at_least(batch, 64);
        const bool adapt = c.opts.batch <= 0;
        for (;;) {
            const double res0 = h.residNorm;
            const int64_t k0 = h.k;
            // distributed: a rank-local failure of this batch (a host error, a sweep chain's
            // timed-out wait) joins the batch's status agreement instead of leaving the other
            // ranks in the next collective (kernels/cpminres.m:195-199: the caller sees the error)
            std::exception_ptr local;
            int code = 0;
            try {
                hipGraphExec_t exec = use_graph ? graph_for(site, b, body) : nullptr;
                if (exec) CPK_HIP(hipGraphLaunch(exec, c.stream));
                else
                    for (int i = 0; i < b; i++) body();
                nbatch++;
                code = injected("batch", nbatch);
                if (injected("chain", nbatch) && !debug_set_chain_error(c, M.dF) && !debug_set_chain_error(c, M.sep.tsw))
                    code = CPK_ERR_HIP;  // no chain to fail: the host error instead
                if (code) throw Error(code, "fail_inject: rank " + std::to_string(c.rank) + " failed after batch " +
                                                std::to_string(nbatch));
            } catch (const Error &e) {
                local = std::current_exception(), code = e.code;
            } catch (...) {
                local = std::current_exception(), code = CPK_ERR_HIP;
            }
            if (!agreeing()) {
                if (local) std::rethrow_exception(local);
            } else {
                status_enqueue(code);
            }
            pull();
            if (agreeing()) status_check(local);
            if (print && printer) printer();
            if (h.stop) break;
            if (h.k > guard) throw Error(CPK_ERR_HIP, "solver loop did not terminate");
            b = pow2_at_least(batch, 64);
            const double res = h.residNorm, tol = h.stopTol;
            if (adapt && h.k > k0 && res > 0 && res0 > res && tol > 0 && tol < res) {
                // geometric model of the residual over the last batch: iterations still needed
                const double rate = std::log(res / res0) / (double)(h.k - k0);
                const double rem = std::log(tol / res) / rate;
                if (rem > 0 && rem < 1e6) b = pow2_at_least(std::ceil(rem), b);
            }
            if (itmax - (double)h.k < b) b = pow2_at_least(std::max(1.0, itmax - (double)h.k), b);
        }
    }

    std::vector<double> fetch(const DBuf<double> &d, int64_t len) {
        std::vector<double> v(std::max<int64_t>(len, 0));
        if (len > 0) CPK_HIP(hipMemcpy(v.data(), d.p, len * sizeof(double), hipMemcpyDeviceToHost));
        return v;
    }

    void print_hist_lines(const char *fmt, int64_t offset = 0) {
        if (h.nh <= printed) return;
        auto v = fetch(hist, std::min(h.nh, h.hcap));
        for (int64_t i = printed; i < (int64_t)v.size(); i++) printf(fmt, (long long)(i + offset), v[i]);
        printed = (int64_t)v.size();
        fflush(stdout);
    }

    void raise_error() {
        char buf[256];
        if (h.err == 1) {
            if (method == CPK_CGLANCZOS)
                snprintf(buf, sizeof buf,
                         "CPCGLanczos:IndefiniteError: Iter %lld, beta (before sqrt) = %g : preconditioner not second-order sufficient",
                         (long long)h.err_iter, h.err_val);
            else
                snprintf(buf, sizeof buf,
                         "Iter %lld, beta (before sqrt) = %g : preconditioner does not behave as a spd matrix.",
                         (long long)h.err_iter, h.err_val);
        } else if (h.err == 3) {
            snprintf(buf, sizeof buf,
                     "Iter 0, 2nd Lanczos vec, beta (before sqrt) = %g : preconditioner does not behave as a spd matrix.",
                     h.err_val);
        } else if (h.err == 2) {
            snprintf(buf, sizeof buf, "Iter %lld, residNorm2 = %g < 0: complex residual norm", (long long)h.err_iter,
                     h.err_val);
        } else {
            snprintf(buf, sizeof buf, "Iter %lld: negative squared norm %g (complex square root)",
                     (long long)h.err_iter, h.err_val);
        }
        throw Error(CPK_ERR_INDEFINITE, buf);
    }

    // ------------------------------------------------------------------------------------------
    void minres_like(int kind, const double *b, double *xy, cpk_stats *stats);
    void cg(const double *b, double *xy, cpk_stats *stats);
    void gmres(const double *b, double *xy, cpk_stats *stats);
    void dqgmres(const double *b, double *xy, cpk_stats *stats);

    void finish_stats(cpk_stats *stats) {
        if (!stats) return;
        stats->niters = h.k;
        stats->status = 0;
        auto cp = [&](double *dstp, const DBuf<double> &src, int64_t len, int64_t *outlen, int prefix, double pv) {
            *outlen = len + (prefix ? 1 : 0);
            if (!dstp) return;
            if (*outlen > stats->hist_cap) throw Error(CPK_ERR_ARGS, "history buffer too small");
            int64_t off = 0;
            if (prefix) dstp[0] = pv, off = 1;
            if (len > 0) CPK_HIP(hipMemcpy(dstp + off, src.p, len * sizeof(double), hipMemcpyDeviceToHost));
        };
        if (method == CPK_SYMMLQ) {
            const int prefix = h.flag != 2;  // cgresidHistory = [beta1; cgresidHistory]
            cp(stats->hist, hist, std::min(h.nh, h.hcap), &stats->hist_len, prefix, h.beta1);
            cp(stats->hist_lq, hist2, std::min(h.nh2, h.hcap), &stats->lq_len, 0, 0);
            cp(stats->hist_qr, hist3, std::min(h.nh3, h.hcap), &stats->qr_len, 0, 0);
        } else {
            cp(stats->hist, hist, std::min(h.nh, h.hcap), &stats->hist_len, 0, 0);
            stats->lq_len = stats->qr_len = 0;
        }
    }
};

// ---- cpminres / cpcglanczos / cpsymmlq ------------------------------------------------------
void SolveCore::minres_like(int kind, const double *b, double *xy, cpk_stats *stats) {
    const int64_t hcap = (int64_t)std::min(itmax, 1.0e8) + 4;
    setup_state(hcap, 0);
    DState *st = dst.p;
    double *VQ = ring(3);  // Lanczos vectors [vk; qk] for k-1, k, k+1
    double *W = ring(3);   // [wv; wq] (3 slots for minres, 1 for the others)
    double *UT = vec(0), *VPREC = vec(1);
    // vprec = M * [u; t] with u = b, t = 0
    launch_set_concat(c, UT, b, n, m);
    M.apply(UT, N, VPREC, nullptr);
    // cpminres, fused update (below): v1 unnormalised in RAW as well, for the first product
    double *RAW = kind == 0 && !c.opts.no_minres_fuse ? vec(2) : nullptr;
    if (kind == 0)
        launch_ewred<1>(c, N, InitLanczos<0>{st, VPREC, b, VQ + N, VQ, W + 2 * N, xy, n});
    else if (kind == 1)
        launch_ewred<1>(c, N, InitLanczos<1>{st, VPREC, b, VQ + N, VQ, nullptr, xy, n});
    else
        launch_ewred<1>(c, N, InitLanczos<2>{st, VPREC, b, VQ + N, VQ, W, xy, n});
    if (RAW) CPK_HIP(hipMemcpyAsync(RAW, VQ + N, sizeof(double) * N, hipMemcpyDeviceToDevice, c.stream));
    launch_ew(c, N, NormalizeCopy{st, VQ + N, kind == 2 ? nullptr : W, 0, 0.0});
    CPK_HIP(hipGetLastError());
    pull();
    if (h.err) raise_error();
    if (kind == 0) {
        if (print) {
            printf("\n**** Constraint-preconditioned version of MINRES ****\n\n");
            printf("stopTol = %e\n", h.stopTol);
            printf("%5s  %9s\n", "iter", "|resid|");
        }
        // distributed: vprec = M*[u; -t] does not depend on alpha (cpminres.m:187-190), so alpha's
        // partials ride in the preconditioner's first separator allgather instead of an allreduce
        // exact mode: alpha's and beta's digits take their own int64 allreduce (no piggyback)
        const bool piggy = c.dist() && M.piggyback_ok() && !c.opts.no_piggy && !c.exact();
        // and beta's partials ride in the next Lanczos vector's halo exchange (spare slots)
        const bool hmerge = piggy && AC.halo() && AC.kstride >= AC.kmax + 2 && !c.opts.no_halo_merge;
        // fused update: the Lanczos step leaves the new vector unnormalised in RAW and makes the
        // previous iteration's w/x update; the Krylov product normalises (no MinresUpdate pass)
        auto iterate = [&](const auto &pol) {
            if (hmerge) launch_krylov_halo(c, AC, st, pol);  // v1's halo, before the first iteration
            auto body = [&]() {
                if (piggy) {
                    launch_krylov_spmv(c, AC, st, UT, n, pol, true, hmerge);
                    M.apply(UT, n, VPREC, &st->running, c.red.p);
                    if (!hmerge) launch_krylov_fin_sep(c, M.sep, st, pol);  // else in the Lanczos step
                } else {
                    launch_krylov_spmv(c, AC, st, UT, n, pol);
                    M.apply(UT, n, VPREC, &st->running);
                }
                LanczosStep<0> ls{st, VQ, VPREC, UT, xy, W, n, N, 0, 2, 1};
                ls.raw = RAW;
                if (hmerge) {
                    ls.sep = M.sep.rbuf.p, ls.sep_ranks = c.nranks, ls.sep_kt = M.sep.kt, ls.sep_data = M.sep.kt_data;
                    launch_lanczos_step_halo(c, AC, st, N, ls);
                } else {
                    launch_ewtred<2>(c, N, ls);
                }
                if (!RAW) launch_ewt(c, N, MinresUpdate{st, VQ, W, xy, n, N});
            };
            if (print) print_hist_lines("%5lld  %9.2e\n");
            loop(body, [&]() { print_hist_lines("%5lld  %9.2e\n"); });
        };
        if (RAW)
            iterate(PolLanczosSpmv<0, true>{VQ, N, 0, RAW});
        else
            iterate(PolLanczosSpmv<0>{VQ, N, 0});
        if (RAW) launch_ewt(c, N, MinresUpdate{st, VQ, W, xy, n, N, true});
        if (h.err) raise_error();
        if (print) printf("\n");
        if (stats) stats->solved = h.residNorm <= h.stopTol;
    } else if (kind == 1) {
        if (print) {
            printf("\n**** Constraint-preconditioned version of CP-CGLanczos ****\n\n");
            printf("stopTol = %e, bstopTol = %e\n", h.stopTol, h.bstopTol);
            printf("%5s  %9s", "iter", "|resid|");
            if (btol > 0) printf("  %9s  %9s  %9s", "bkerr", "|op|", "|x|");
            printf("\n");
        }
        auto pr = [&]() {
            if (h.nh <= printed) return;
            auto v = fetch(hist, std::min(h.nh, h.hcap));
            auto a = fetch(aux, 3 * std::min(h.nh, h.hcap));
            for (int64_t i = printed; i < (int64_t)v.size(); i++) {
                printf("%5lld  %9.2e", (long long)i, v[i]);
                if (btol > 0)
                    printf("  %9.2e  %9.2e  %9.2e", i ? v[i] / a[3 * (i - 1)] : 0.0, i ? a[3 * (i - 1) + 1] : 0.0,
                           i ? a[3 * (i - 1) + 2] : 0.0);
                printf("\n");
            }
            printed = (int64_t)v.size();
        };
        auto body = [&]() {
            launch_krylov_spmv(c, AC, st, UT, n, PolLanczosSpmv<1>{VQ, N, 0});
            M.apply(UT, n, VPREC, &st->running);
            launch_ewred<2>(c, N, LanczosStep<1>{st, VQ, VPREC, UT, xy, W, n, N, 0, 2, 1});
            launch_ew(c, N, CglUpdate{st, VQ, W, N});
        };
        if (print) pr();
        loop(body, pr);
        if (h.err) raise_error();
        if (print) printf("\n");
        if (stats) {
            stats->solved = 0, stats->status = 0;
            if (h.residNorm <= h.stopTol) stats->solved = 1, stats->status = 1;
            if (btol > 0 && h.residNorm <= h.bstopTol) stats->solved = 1, stats->status = 2;
        }
        finish_stats(stats);
        if (stats) {
            stats->solved = 0, stats->status = 0;
            if (h.residNorm <= h.stopTol) stats->solved = 1, stats->status = 1;
            if (btol > 0 && h.residNorm <= h.bstopTol) stats->solved = 1, stats->status = 2;
        }
        return;
    } else {
        // cpsymmlq: the cpsymmlq.m:182 `printf` quirk is not reproduced
        if (print) {
            printf("\n**** Constraint-preconditioned version of SYMMLQ ****\n\n");
            printf("the printed |cgresid| is one iter ahead, unless the solver\nstops at iter = 0\n\n");
            printf("stopTol = %e\n", h.stopTol);
            printf("%5s   %9s   %9s   %9s\n", "iter", "|cgresid|", "|lqresid|", "|qrresid|");
        }
        if (h.flag != 2) {
            // pre-step: second Lanczos vector (cpsymmlq.m:193-225), vk = VQ[1], vkp1 -> VQ[2]
            launch_krylov_spmv(c, AC, st, UT, n, PolPlainSpmv{VQ + N});
            M.apply(UT, n, VPREC, nullptr);
            launch_ewred<2>(c, N, SymmlqPre{st, VQ + N, VPREC, UT, VQ + 2 * N, n});
            launch_ew(c, N, NormalizeCopy{st, VQ + 2 * N, nullptr, 0, 0.0});
            CPK_HIP(hipGetLastError());
            pull();
            if (h.err) raise_error();
            auto pr = [&]() {
                if (h.nh <= printed) return;
                auto cgv = fetch(hist, std::min(h.nh, h.hcap));
                auto lq = fetch(hist2, std::min(h.nh2, h.hcap));
                auto qr = fetch(hist3, std::min(h.nh3, h.hcap));
                for (int64_t i = printed; i < (int64_t)cgv.size(); i++)
                    printf("%5lld  %9.2e   %9.2e    %9.2e\n", (long long)i, cgv[i], lq[i], qr[i]);
                printed = (int64_t)cgv.size();
            };
            auto body = [&]() {
                launch_krylov_spmv(c, AC, st, UT, n, PolLanczosSpmv<2>{VQ, N, 1});
                M.apply(UT, n, VPREC, &st->running);
                launch_ewred<2>(c, N, LanczosStep<2>{st, VQ, VPREC, UT, xy, W, n, N, 1, 0, 2});
                launch_ew(c, N, SymmlqUpdate{st, VQ, W, xy, n, N});
            };
            loop(body, pr);
            if (h.err) raise_error();
            launch_scalar(c, SymmlqPostScalar{st});
            launch_ew(c, N, SymmlqMoveCg{st, xy, W, n});
            launch_set_concat(c, UT, b, n, m);
            M.apply(UT, N, VPREC, nullptr);
            launch_ew(c, N, SymmlqFirstStep{st, xy, VPREC, n});
            CPK_HIP(hipGetLastError());
            pull();
            if (print) printf("%5lld     ---      %9.2e    %9.2e\n\n", (long long)h.k, h.lqresid, h.qrresid);
        } else if (print) {
            printf("%5lld  %9.2e   %9.2e    %9.2e\n", 0LL, h.cgresid, h.lqresid, h.qrresid);
        }
        if (stats) stats->solved = h.cgresid <= h.stopTol;
    }
    finish_stats(stats);
}

// ---- cpcg -------------------------------------------------------------------------------------
void SolveCore::cg(const double *b, double *xy, cpk_stats *stats) {
    const int64_t hcap = (int64_t)std::min(itmax, 1.0e8) + 4;
    setup_state(hcap, 0);
    DState *st = dst.p;
    double *GW = vec(0), *PQ = vec(1), *APCQ = vec(2), *RU = vec(3), *TT = vec(4);
    double *XA = xy;
    launch_ew(c, N, CgInit0{b, GW, XA, n});
    M.apply(GW, N, RU, nullptr);
    launch_ewred<1>(c, N, CgInit1{st, RU, GW, PQ, n});
    CPK_HIP(hipGetLastError());
    pull();
    if (h.err) raise_error();
    if (print) {
        printf("\n**** Constraint-preconditioned version of CG ****\n\n");
        printf("stopTol = %e\n", h.stopTol);
        printf("%5s  %9s  %9s  %9s  %9s\n", "iter", "resid", "pr-curv", "du-curv", "steplen");
        printf("%5d  %9.2e  ", 0, h.residNorm);
        printed = 1;
    }
    auto pr = [&]() {
        if (h.nh <= printed) return;
        auto v = fetch(hist, std::min(h.nh, h.hcap));
        auto a = fetch(aux, 3 * std::min(h.nh, h.hcap));
        for (int64_t i = printed; i < (int64_t)v.size(); i++) {
            printf("%9.2e  %9.2e  %9.2e\n", a[3 * (i - 1)], a[3 * (i - 1) + 1], a[3 * (i - 1) + 2]);
            printf("%5lld  %9.2e  ", (long long)i, v[i]);
        }
        printed = (int64_t)v.size();
    };
    auto body = [&]() {
        launch_krylov_spmv(c, AC, st, APCQ, n, PolCgSpmv{PQ});
        launch_ew(c, N, CgStep{st, XA, GW, PQ, APCQ});
        M.apply(GW, N, RU, &st->running);
        launch_ewred<2>(c, N, CgResid{st, XA, RU, GW, TT, n});
        launch_ew(c, N, CgDir{st, RU, TT, PQ, n});
    };
    loop(body, pr);
    if (h.err) raise_error();
    if (print) printf("\n\n");
    if (stats) stats->solved = h.residNorm <= h.stopTol;
    finish_stats(stats);
}

// ---- cpgmres ----------------------------------------------------------------------------------
void SolveCore::gmres(const double *b, double *xy, cpk_stats *stats) {
    const int64_t R = (int64_t)restart;
    if (R < 1) throw Error(CPK_ERR_ARGS, "restart must be >= 1");
    // the cycles can overrun itmax by up to restart-1 iterations (cpgmres.m:148,203)
    const int64_t hcap = (int64_t)(std::ceil(std::min(itmax, 1.0e8) / (double)R) * R) + 4;
    setup_state(hcap, R);
    DState *st = dst.p;
    double *V = ring((size_t)(R + 1));
    double *UT = vec(0), *Wv = vec(1), *TMP = vec(2);
    CPK_HIP(hipMemsetAsync(xy, 0, N * sizeof(double), c.stream));
    const double outermax = std::ceil(itmax / (double)R);
    int64_t outer = 0;
    bool finished = false;
    if (print) printf("\n**** Constraint-preconditioned version of GMRES(%lld) ****\n\n", (long long)R);
    while (!finished && outer < outermax) {
        outer++;
        if (outer == 1) {
            launch_set_concat(c, UT, b, n, m);  // u = b, t = 0
            M.apply(UT, n, Wv, nullptr);        // M * [u; -t]
        } else {
            launch_spmv(c, AC, xy, TMP, nullptr);  // [A*x; C*y]
            launch_ew(c, N, GmresRestartRhs{b, TMP, UT, n});
            M.apply(UT, n, Wv, nullptr);
        }
        launch_ewred<2>(c, N, ArnoldiStart{st, Wv, UT, xy, V, n, outer > 1 ? 1 : 0, 0, outer == 1 ? 1 : 0});
        launch_ew(c, N, NormalizeCopy{st, V, nullptr, 1, 0.0});
        CPK_HIP(hipGetLastError());
        pull();
        if (h.err) raise_error();
        if (print && outer == 1) {
            printf("stopTol = %e\n", h.stopTol);
            printf("%5s  %9s\n", "iter", "|resid|");
            print_hist_lines("%5lld  %14.7e\n");
        }
        const int64_t base = (outer - 1) * R, hist0 = h.nh;
        auto body = [&]() {
            launch_krylov_spmv(c, AC, st, UT, n, PolArnoldiSpmv{V, N, 0});
            M.apply(UT, n, Wv, &st->running);
            launch_arnoldi_dots(c, st, V, Wv, UT, n, N, 0, R);
            launch_ewtred<2>(c, N, ArnoldiOrth{st, V, UT, n, N, 0, Window{}, nullptr});
            launch_ew(c, N, GmresNormalize{st, V, N});
        };
        loop(body, [&]() {  // printed iteration = (outer - 1) * restart + k  (cpgmres.m:252)
            if (h.nh <= printed) return;
            auto v = fetch(hist, std::min(h.nh, h.hcap));
            for (int64_t i = std::max(printed, hist0); i < (int64_t)v.size(); i++)
                printf("%5lld  %14.7e\n", (long long)(base + (i - hist0) + 1), v[i]);
            printed = (int64_t)v.size();
        });
        if (h.err) raise_error();
        launch_scalar(c, GmresBackSolve{st});
        launch_ew(c, N, GmresUpdateX{st, V, xy, n, N, 0});
        CPK_HIP(hipGetLastError());
        pull();
        finished = h.residNorm <= h.stopTol;
    }
    if (stats) {
        finish_stats(stats);
        stats->niters = (outer - 1) * R + h.k;
        stats->solved = h.residNorm <= h.stopTol;
    }
}

// ---- cpdqgmres --------------------------------------------------------------------------------
void SolveCore::dqgmres(const double *b, double *xy, cpk_stats *stats) {
    const double memd = std::min(mem, itmax);  // cpdqgmres.m:125
    mem = std::max(1.0, memd);
    const int64_t Mm = (int64_t)mem, M1 = Mm + 1;
    const int64_t hcap = (int64_t)std::min(itmax, 1.0e8) + 4;
    setup_state(hcap, Mm);
    DState *st = dst.p;
    double *V = ring((size_t)M1), *PV = ring((size_t)M1);
    double *UT = vec(0), *Wv = vec(1);
    CPK_HIP(hipMemsetAsync(xy, 0, N * sizeof(double), c.stream));
    if (print) printf("\n**** Constraint-preconditioned version of DQGMRES - mem = %lld ****\n\n", (long long)Mm);
    launch_set_concat(c, UT, b, n, m);
    M.apply(UT, N, Wv, nullptr);  // M * [u; t], t = 0 (cpdqgmres.m:154)
    launch_ewred<2>(c, N, ArnoldiStart{st, Wv, UT, xy, V, n, 0, 1, 1});
    launch_ew(c, N, NormalizeCopy{st, V, nullptr, 1, 0.0});
    CPK_HIP(hipGetLastError());
    pull();
    if (h.err) {
        char buf[160];
        snprintf(buf, sizeof buf, "Undefined variable k (dot(u,V1) = %g < 0, cpdqgmres.m:158-160)", h.err_val);
        throw Error(CPK_ERR_INDEFINITE, buf);
    }
    if (print) {
        printf("stopTol = %e\n", h.stopTol);
        printf("%5s  %9s\n", "iter", "|resid|");
    }
    // profile_passes (diagnostic): events between the passes of every iteration, eager batches
    const bool prof = c.opts.profile_passes;
    std::vector<hipEvent_t> evs;
    size_t ev_used = 0;
    const int64_t k_start = h.k;
    int64_t kh = h.k;  // the host's copy of the iteration counter (window sizes of the byte model)
    std::vector<double> wdots, wdir;
    auto mark = [&]() {
        if (ev_used == evs.size()) {
            hipEvent_t e;
            CPK_HIP(hipEventCreate(&e));
            evs.push_back(e);
        }
        CPK_HIP(hipEventRecord(evs[ev_used++], c.stream));
    };
    if (prof) use_graph = false;
    auto body = [&]() {
        if (prof) mark();
        launch_krylov_spmv(c, AC, st, UT, n, PolArnoldiSpmv{V, N, M1});
        if (prof) mark();
        M.apply(UT, n, Wv, &st->running);
        if (prof) mark();
        launch_arnoldi_dots(c, st, V, Wv, UT, n, N, M1, Mm);
        if (prof) mark();
        launch_ewtred<2>(c, N, ArnoldiOrth{st, V, UT, n, N, M1, Window{}, nullptr});
        if (prof) mark();
        launch_ewt(c, N, DqgmresDirection{st, V, PV, xy, n, N});
        if (prof) {
            mark();
            // window sizes of this iteration (kernels: window(st, M1) and DqgmresDirection::setup)
            const int64_t kk = kh + 1, mem_ = (int64_t)h.mem;
            wdots.push_back((double)(kk - std::max<int64_t>(1, kk - mem_ + 1) + 1));
            wdir.push_back((double)(kk - std::max<int64_t>(1, kk - mem_)));
            kh++;
        }
    };
    if (print) print_hist_lines("%5lld  %14.7e\n");
    loop(body, [&]() { print_hist_lines("%5lld  %14.7e\n"); });
    if (prof) {
        CPK_HIP(hipStreamSynchronize(c.stream));
        // the iterations that ran (a batch's no-op iterations past the stop are not counted)
        const size_t its = (size_t)std::min<int64_t>(std::max<int64_t>(h.k - k_start, 0), (int64_t)(ev_used / 6));
        double ms[5] = {0, 0, 0, 0, 0}, wd = 0, wr = 0;
        for (size_t it = 0; it < its; it++) {
            for (int q = 0; q < 5; q++) {
                float t = 0;
                CPK_HIP(hipEventElapsedTime(&t, evs[6 * it + q], evs[6 * it + q + 1]));
                ms[q] += t;
            }
            wd += wdots[it], wr += wdir[it];
        }
        c.pass_ms[0] = (double)its;
        for (int q = 0; q < 5; q++) c.pass_ms[1 + q] = ms[q];
        c.pass_ms[6] = wd, c.pass_ms[7] = wr;
        for (hipEvent_t e : evs) (void)hipEventDestroy(e);
    }
    if (h.err) raise_error();
    if (stats) stats->solved = h.residNorm <= h.stopTol;
    finish_stats(stats);
}

// ==============================================================================================
// The cached solver of (method, operators, vectors, captured properties); see SolveCore.
static std::string solver_key(const Ctx &c, const Precond &M, const DMat &AC, int method, const cpk_opts *o,
                              const double *d_b, const double *d_xy) {
    char buf[512];
    const double restart = o && o->has_restart ? o->restart : 50, mem = o && o->has_mem ? o->mem : 50;
    const double itmax = o && o->has_itmax ? o->itmax : -1;
    // the context's engine options enter through their hash (graphs captured under one set of
    // options are not replayed under another)
    snprintf(buf, sizeof buf, "%d|%llu|%p|%p|%p|%p|%p|%.17g|%.17g|%.17g|%d|%.17g|%.17g|%.17g|%llx", method,
             (unsigned long long)AC.gen, (const void *)d_b, (const void *)d_xy, (const void *)c.partials.p,
             (const void *)c.counter.p, (const void *)c.red.p, M.nitref, M.force_itref, M.itref_tol,
             (M.residual_update != 0 && M.handle) ? 1 : 0, restart, mem,
             method == CPK_DQGMRES ? itmax : 0.0, (unsigned long long)engine_opts_hash(c.opts));
    return buf;
}

static SolveCore &solver_for(Ctx &c, Precond &M, const DMat &AC, int method, const cpk_opts *opts,
                             const double *d_b = nullptr, const double *d_xy = nullptr) {
    const std::string key = solver_key(c, M, AC, method, opts, d_b, d_xy);
    for (auto &e : M.solvers)
        if (e.first == key) {
            auto *s = static_cast<SolveCore *>(e.second.get());
            s->reset(opts);
            return *s;
        }
    if (M.solvers.size() >= 4) M.solvers.erase(M.solvers.begin());  // bounded: oldest out
    std::shared_ptr<void> sp(new SolveCore(c, M, AC, method, opts));
    M.solvers.emplace_back(key, sp);
    return *static_cast<SolveCore *>(sp.get());
}

void method_solve_device(Ctx &c, int method, const double *d_b, const DMat &AC, Precond &M, const cpk_opts *opts,
                         double *d_xy, cpk_stats *stats) {
    if (method < CPK_CG || method > CPK_DQGMRES) throw Error(CPK_ERR_ARGS, "unknown method");
    CPK_HIP(hipEventRecord(c.ev0, c.stream));
    SolveCore &s = solver_for(c, M, AC, method, opts, d_b, d_xy);
    s.nbatch = 0;
    if (s.agreeing()) {  // a rank that fails before the solve's first collective stops every rank
        std::exception_ptr local;
        int code = s.injected("setup");
        if (code) {
            try {
                throw Error(code, "fail_inject: rank " + std::to_string(c.rank) + " failed at the solve's setup");
            } catch (const Error &) {
                local = std::current_exception();
            }
        }
        s.agree_setup(local, code);
    }
    switch (method) {
    case CPK_MINRES: s.minres_like(0, d_b, d_xy, stats); break;
    case CPK_CGLANCZOS: s.minres_like(1, d_b, d_xy, stats); break;
    case CPK_SYMMLQ: s.minres_like(2, d_b, d_xy, stats); break;
    case CPK_CG: s.cg(d_b, d_xy, stats); break;
    case CPK_GMRES: s.gmres(d_b, d_xy, stats); break;
    case CPK_DQGMRES: s.dqgmres(d_b, d_xy, stats); break;
    }
    CPK_HIP(hipEventRecord(c.ev1, c.stream));
    CPK_HIP(hipEventSynchronize(c.ev1));
    check_chain(M.dF);
    check_chain(M.sep.tsw);
    if (stats) {
        float ms = 0;
        CPK_HIP(hipEventElapsedTime(&ms, c.ev0, c.ev1));
        stats->loop_ms = ms;
        stats->bytes_moved = method_bytes(method, AC, M, stats->niters, opts);
    }
}

int reg_shift_device(Ctx &c, const double *d_b, const DMat &Arows, const DMat &Btrows, int64_t bt_colmin, Precond &M,
                     double *d_b1, double *d_xy0) {
    const int64_t n = M.n, m = M.m, N = M.N;
    DBuf<int> flag;
    flag.alloc(1);
    int shift = 0;
    if (M.gm > 0) {  // any(b(n+1:n+m)) over all ranks
        c.ensure_partials((size_t)kEwGrid);
        CPK_HIP(hipMemsetAsync(flag.p, 0, sizeof(int), c.stream));
        launch_ewred<1>(c, m, AnyNonzero{d_b, n, flag.p});
        CPK_HIP(hipMemcpyAsync(&shift, flag.p, sizeof(int), hipMemcpyDeviceToHost, c.stream));
        CPK_HIP(hipStreamSynchronize(c.stream));
    }
    if (shift) {
        DBuf<double> t1, t2;
        t1.alloc(std::max<int64_t>(N, 1)), t2.alloc(std::max<int64_t>(N, 1));
        // xy0 = M * [zeros(n,1); b(n+1:n+m)]   (reg_cpkrylov.m:156)
        if (n) CPK_HIP(hipMemsetAsync(t1.p, 0, n * sizeof(double), c.stream));
        if (m) CPK_HIP(hipMemcpyAsync(t1.p + n, d_b + n, m * sizeof(double), hipMemcpyDeviceToDevice, c.stream));
        M.apply(t1.p, N, d_xy0, nullptr);
        launch_spmv(c, Arows, d_xy0, t1.p, nullptr);                     // rows < n: A*xy0(1:n)
        launch_spmv_colmask(c, Btrows, bt_colmin, d_xy0, t2.p, nullptr);  // rows < n: B'*xy0(n+1:N)
        launch_ew(c, n, ShiftRhs{d_b, t1.p, t2.p, d_b1});  // b1 = b(1:n) - A*xy0(1:n) - B'*xy0(n+1:N)
        CPK_HIP(hipStreamSynchronize(c.stream));
    } else {
        if (n) CPK_HIP(hipMemcpyAsync(d_b1, d_b, n * sizeof(double), hipMemcpyDeviceToDevice, c.stream));
        if (N) CPK_HIP(hipMemsetAsync(d_xy0, 0, N * sizeof(double), c.stream));
    }
    return shift;
}

void reg_solve_device(Ctx &c, int method, const double *d_b, const DMat &AC, const DMat &Arows, const DMat &Btrows,
                      int64_t bt_colmin, Precond &M, const cpk_opts *opts, double *d_x, cpk_stats *stats) {
    const int64_t n = M.n, N = M.N;
    auto t0 = std::chrono::steady_clock::now();
    DBuf<double> xy0, b1, dxy;
    xy0.alloc(std::max<int64_t>(N, 1)), b1.alloc(std::max<int64_t>(n, 1)), dxy.alloc(std::max<int64_t>(N, 1));
    const int shift = reg_shift_device(c, d_b, Arows, Btrows, bt_colmin, M, b1.p, xy0.p);
    method_solve_device(c, method, b1.p, AC, M, opts, shift ? dxy.p : d_x, stats);
    if (shift) launch_ew(c, N, Recover{xy0.p, dxy.p, d_x});  // x = [xy0(1:n) + dx; xy0(n+1:N) + dy]
    CPK_HIP(hipStreamSynchronize(c.stream));
    if (stats) stats->stime = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

void profile_kernels(Ctx &c, const DMat &AC, Precond &M, int reps, cpk_profile *out) {
    const int64_t N = M.N;
    const int64_t NW = std::max<int64_t>(std::max<int64_t>(N, M.nsub + M.sep.nT), 1);  // distributed work vectors
    reps = std::max(reps, 1);
    DBuf<double> x, y, z;
    x.alloc(NW), y.alloc(NW), z.alloc(NW);
    CPK_HIP(hipMemsetAsync(y.p, 0, NW * sizeof(double), c.stream));
    std::vector<double> h(NW);
    for (int64_t i = 0; i < NW; i++) h[i] = 1.0 + 1e-3 * (double)(i % 1000);
    CPK_HIP(hipMemcpy(x.p, h.data(), NW * sizeof(double), hipMemcpyHostToDevice));
    auto timeit = [&](const std::function<void()> &f) {
        f();  // warm
        CPK_HIP(hipEventRecord(c.ev0, c.stream));
        for (int r = 0; r < reps; r++) f();
        CPK_HIP(hipEventRecord(c.ev1, c.stream));
        CPK_HIP(hipEventSynchronize(c.ev1));
        float ms = 0;
        CPK_HIP(hipEventElapsedTime(&ms, c.ev0, c.ev1));
        return (double)ms / reps;
    };
    const double Nn = (double)N, l = (double)M.dF.nnz;
    out->spmv_ms = timeit([&]() { launch_spmv(c, AC, x.p, y.p, nullptr); });
    out->spmv_bytes = 12.0 * AC.nnz + 4.0 * (Nn + 1) + 8.0 * Nn + 8.0 * Nn;
    if (M.sched_path() && M.xs.n) {  // the refinement residual the apply runs: Kp, x and y in schedule order
        out->resid_ms = timeit([&]() { launch_spmv_resid_sched(c, M.dKps, nullptr, x.p, 0, y.p, z.p, nullptr); });
        out->resid_bytes = 12.0 * M.dKps.nnz + 4.0 * (Nn + 1) + 8.0 * Nn /*y*/ + 8.0 * Nn /*x*/ + 8.0 * Nn /*r*/;
    } else if (M.sched_path()) {  // x through perm
        out->resid_ms = timeit([&]() { launch_spmv_resid_sched(c, M.dKps, M.dF.perm.p, x.p, M.n, y.p, z.p, nullptr); });
        out->resid_bytes = 12.0 * M.dKps.nnz + 4.0 * (Nn + 1) + 8.0 * Nn /*y*/ + 12.0 * Nn /*x, perm*/ + 8.0 * Nn /*r*/;
    } else {
        out->resid_ms = timeit([&]() { launch_spmv_resid(c, M.dKp, x.p, M.n, y.p, z.p, nullptr, nullptr); });
        out->resid_bytes = 12.0 * M.dKp.nnz + 4.0 * (Nn + 1) + 8.0 * Nn /*y*/ + 8.0 * Nn /*x*/ + 8.0 * Nn /*r*/;
    }
    // one LDL solve as the apply runs it: the forward sweep (its last round deferred when fused),
    // then the pair forward + backward; the backward's time is the pair's minus the forward's.
    // Launch order (bench.py's PMC parser): (1 + reps) forward sweeps, (1 + reps) pairs
    // profile_fwd_sched (diagnostic): the forward reads x as if it were the signed input in schedule
    // order (no perm gather; the values are meaningless, the time and traffic are not)
    FwdIn last;
    const bool fsched = c.opts.profile_fwd_sched;
    out->fwd_ms = timeit([&]() { launch_sptrsv_fwd(c, M.dF, x.p, M.n, M.w.p, nullptr, nullptr, fsched, nullptr, &last); });
    out->fwd_bytes = 12.0 * l - 2.0 * (double)M.dF.nnz16 + 4.0 * (Nn + 1) + 4.0 * Nn /*perm*/ + 8.0 * Nn /*x*/ + 8.0 * Nn /*w*/;
    const double pair_ms = timeit([&]() {
        launch_sptrsv_fwd(c, M.dF, x.p, M.n, M.w.p, nullptr, nullptr, fsched, nullptr, &last);
        launch_sptrsv_bwd(c, M.dF, M.w.p, z.p, false, nullptr, nullptr, nullptr, &last, nullptr, true);
    });
    out->bwd_ms = pair_ms - out->fwd_ms;
    // w out: the upper rounds' rows only (wdead: round 0, the last round, writes y and not w)
    out->bwd_bytes = 12.0 * l + 4.0 * (Nn + 1) + 4.0 * Nn + 8.0 * Nn /*D*/ + 8.0 * Nn /*w in*/ +
                     8.0 * (Nn - (double)M.dF.bwd_dead_w_rows()) /*w out*/ + 8.0 * Nn /*y*/;
    out->bwd_dead_store_bytes = 8.0 * (double)M.dF.bwd_dead_w_rows();
    out->apply_ms = timeit([&]() { M.apply(x.p, M.n, z.p, nullptr); });
    out->apply_bytes = M.apply_bytes();
    out->fwd_launches = out->bwd_launches = (int64_t)M.dF.round_ptr.size() - 1;
    if (last.valid) {  // the deferred rounds (the last one; with the sweep chain every upper round)
        // run as one launch inside the backward count
        out->fwd_launches = last.from;
        out->bwd_launches = last.from + 1;
        // its forward half runs in the backward launch: its bytes move with it, so
        // fwd / bwd each pair time and bytes of the same launches (the sum is unchanged)
        const DFactor &F = M.dF;
        double rows = 0, ents = 0;
        for (int64_t b = F.round_ptr[last.from]; b < F.round_ptr.back(); b++) {
            const int32_t *m = &F.hmeta[(size_t)b * 8];
            rows += m[1] - m[0], ents += m[5] - m[4];
        }
        const double fl = 12.0 * ents + 4.0 * (rows + 1) + 4.0 * rows + 8.0 * rows + 8.0 * rows;
        out->fwd_bytes -= fl, out->bwd_bytes += fl;
    }
    out->fwd_resid_ms = out->fwd_resid_bytes = 0;
    // the fused refinement input: one GPU on Kps, distributed (schedule order) on the rank's Kpsl
    const DMat &Ks = M.dist ? M.dKpsl : M.dKps;
    if ((M.sched_path() || M.dsched) && M.xs.n && M.fused_resid &&
        launch_sptrsv_fwd_resid(c, M.dF, Ks, x.p, y.p, z.p, nullptr)) {
        out->fwd_resid_ms = timeit([&]() { launch_sptrsv_fwd_resid(c, M.dF, Ks, x.p, y.p, z.p, nullptr); });
        // Kps, y, xs (the residual's reads) + the factor and w (the sweep's); r never goes to HBM
        // for round 0 (the tail rows' r write and read are < 1 % and not counted)
        const double Nr = (double)M.dF.N;
        out->fwd_resid_bytes = 12.0 * Ks.nnz + 4.0 * (Nr + 1) + 8.0 * Nr /*y*/ + 8.0 * Nr /*xs*/ + 12.0 * l -
                               2.0 * (double)M.dF.nnz16 + 4.0 * (Nr + 1) + 8.0 * Nr /*w*/;
    }
}

// Algorithmic HBM bytes of one method call: per iteration the Krylov SpMV,
// the preconditioner apply and the streaming vector kernels, counted as ideal single touches.
double method_bytes(int method, const DMat &AC, const Precond &M, int64_t iters, const cpk_opts *opts) {
    const double N = (double)M.N;
    const double spmv = 12.0 * AC.nnz + 4.0 * (N + 1) + 8.0 * N /*x*/ + 8.0 * N /*y*/;
    const double mapply = M.apply_bytes();
    double vec = 0;
    switch (method) {
    case CPK_MINRES:  // lanczos step (5 streams) + update (8 streams); fused: the step with the update
        // (10 streams) and the normalised vector the Krylov product stores (1)
        vec = 8 * N * (M.ctx && !M.ctx->opts.no_minres_fuse ? 10 + 1 : 5 + 8);
        break;
    case CPK_CGLANCZOS: vec = 8 * N * (7 + 4); break;
    case CPK_SYMMLQ: vec = 8 * N * (5 + 7); break;
    case CPK_CG: vec = 8 * N * (6 + 5 + 4); break;
    case CPK_GMRES:
    case CPK_DQGMRES: {
        double w = 50;
        if (opts && method == CPK_GMRES && opts->has_restart) w = opts->restart;
        if (opts && method == CPK_DQGMRES && opts->has_mem) w = opts->mem;
        vec = 8 * N * (3 + w / 2 + w / 2 + 3);
        break;
    }
    }
    return (double)iters * (spmv + mapply + vec);
}

}  // namespace cpk
