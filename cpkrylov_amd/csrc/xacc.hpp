// xacc.hpp -- exact, order-independent inner products on the device (engine option exact_dots).
//
// The reference's dot/norm go to MKL, whose summation order is unknown, so
// the default reductions (devutil.hpp: fixed per device and grid) match the oracle only to
// rounding.  In exact mode every inner product is the correctly rounded value of the EXACT sum
// of its TwoProd pairs p = a*b, e = fma(a, b, -p) (p + e = a*b unless a product under- or
// overflows): a single, summation-order-free definition, so a history is the same bits on any
// grid, any rank count and in the oracle (orc_set_exact, which computes it its own way).
//
// Representation.  A thread accumulates into a floating-point expansion of kXK doubles (a TwoSum
// cascade: every step is error-free, so the expansion plus whatever it deposits holds the exact
// sum); the rare error term that outlives the cascade is deposited into the workgroup's digits.
// At the end of the kernel the 64 lanes of a wave merge their expansions by shuffles, the waves
// of the workgroup through LDS, and one lane deposits the workgroup's kXK terms as fixed-point
// digits: value = sum d[i] * 2^(32 i - 1074), one signed 32-bit chunk per int64 word (every
// double is an integer multiple of 2^-1074; words kXW - 1 counts non-finite terms).  Workgroups
// add their digits into kXSub sub-accumulators (agent-scope 8-byte atomic adds: exact and
// commutative) chosen by blockIdx, so no address sees more than 1/kXSub of the grid; the last
// workgroup (the arrival ticket of devutil.hpp) sums the sub-accumulators, zeroes them for the
// next launch and rounds each sum once, to nearest even.  Distributed: it hands the digits to
// an int64 allreduce instead, and xround_kernel rounds the global sums on every rank.
// Hand-off protocol: MI355X_MICROARCH.md "Valid forms", {8-B agent atomics both sides}: every
// depositing wave drains with s_waitcnt vmcnt(0) before the workgroup barrier that precedes its
// ticket, and the last workgroup reads the digits with agent-scope atomic loads.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "dev.hpp"
#include "devutil.hpp"

namespace cpk {

constexpr int kXK = 3;     // doubles of a thread's expansion
constexpr int kXW = 68;    // int64 words of a superaccumulator (67 digits + the non-finite count)
constexpr int kXSub = 16;  // sub-accumulators per sum a launch spreads its workgroups over

__device__ __forceinline__ int64_t ld_agent64(const int64_t *p) {
    return __hip_atomic_load(const_cast<int64_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent64(int64_t *p, int64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void add_agent64(int64_t *p, int64_t v) {
    if (v) __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the digits of x added into d[0..kXW) (agent-scope atomics; d is a sub-accumulator in HBM)
__device__ inline void xdeposit(int64_t *d, double x) {
    if (x == 0) return;
    const uint64_t bits = (uint64_t)__double_as_longlong(x);
    const int E = (int)((bits >> 52) & 0x7ff);
    if (E == 0x7ff) {  // inf / nan: the sum is NaN
        add_agent64(d + kXW - 1, 1);
        return;
    }
    uint64_t mant = bits & ((1ull << 52) - 1);
    int off = 0;
    if (E) mant |= 1ull << 52, off = E - 1;
    const int i = off >> 5, sh = off & 31;
    const uint64_t lo = mant << sh, hi = sh ? mant >> (64 - sh) : 0;
    int64_t c0 = (int64_t)(lo & 0xffffffffu), c1 = (int64_t)(lo >> 32), c2 = (int64_t)hi;
    if (bits >> 63) c0 = -c0, c1 = -c1, c2 = -c2;
    add_agent64(d + i, c0);
    add_agent64(d + i + 1, c1);
    add_agent64(d + i + 2, c2);
}

// A thread's exact accumulator: the expansion, and where its overflow goes (this workgroup's
// sub-accumulator of the sum: uniform across the wave, so the compiler keeps it in SGPRs)
struct XAcc {
    double t[kXK];
    int64_t *ovf;
    __device__ __forceinline__ void init(int64_t *o) {
#pragma unroll
        for (int k = 0; k < kXK; k++) t[k] = 0.0;
        ovf = o;
    }
    __device__ __forceinline__ void add(double x) {
#pragma unroll
        for (int k = 0; k < kXK; k++) {  // TwoSum cascade (no FMA contraction: -ffp-contract=off)
            const double s = t[k] + x, bb = s - t[k];
            x = (t[k] - (s - bb)) + (x - bb);
            t[k] = s;
        }
        if (x != 0) xdeposit(ovf, x);  // beyond the expansion's reach (and every non-finite term)
    }
    __device__ __forceinline__ void add_prod(double a, double b) {
        const double p = a * b;
        add(p);
        add(fma(a, b, -p));
    }
};

// the accumulation step of the reducing functors: one definition per accumulator kind
__device__ __forceinline__ void dadd(double &acc, double a, double b) { acc += a * b; }
__device__ __forceinline__ void dadd(XAcc &acc, double a, double b) { acc.add_prod(a, b); }

// a reducing kernel's accumulators: 0.0, or an empty expansion bound to this workgroup's
// sub-accumulator of sum j (of nv)
__device__ __forceinline__ void acc_init(double &a, int64_t *, int, int) { a = 0.0; }
__device__ __forceinline__ void acc_init(XAcc &a, int64_t *xsub, int j, int nv) {
    a.init(xsub + ((size_t)(blockIdx.x % kXSub) * nv + j) * kXW);
}

// bits [lo, lo + 64) of the normalised magnitude digits u[0..nd) (each in [0, 2^32)), lo >= 0
__device__ inline uint64_t xbits64(const int64_t *u, int nd, int lo) {
    const int i = lo >> 5, sh = lo & 31;
    const uint64_t w0 = i < nd ? (uint64_t)u[i] : 0, w1 = i + 1 < nd ? (uint64_t)u[i + 1] : 0,
                   w2 = i + 2 < nd ? (uint64_t)u[i + 2] : 0;
    uint64_t r = (w0 | (w1 << 32)) >> sh;
    if (sh) r |= w2 << (64 - sh);
    return r;
}

// the double nearest the digits' value (ties to even).  d: kXW summed (un-normalised) words,
// normalised in place (LDS or global: no private array, so the kernels need no scratch)
__device__ inline double xround(int64_t *d) {
    if (d[kXW - 1]) return __longlong_as_double(0x7ff8000000000000ll);
    constexpr int ND = kXW - 1;
    constexpr int64_t kM32 = 0xffffffffll;
    int64_t carry = 0;
#pragma unroll 1
    for (int i = 0; i < ND; i++) {  // digits into [0, 2^32), the sign left in the carry
        const int64_t t = d[i] + carry;
        d[i] = t & kM32;
        carry = t >> 32;
    }
    const bool neg = carry < 0;
    const uint64_t sign = neg ? (1ull << 63) : 0;
    const double inf = __longlong_as_double((long long)(sign | (0x7ffull << 52)));
    if (neg) {  // magnitude = 2^(32 ND) - value: invert the digits and add one
        if (carry != -1) return inf;
        int64_t c2 = 1;
#pragma unroll 1
        for (int i = 0; i < ND; i++) {
            const int64_t t = (kM32 - d[i]) + c2;
            d[i] = t & kM32;
            c2 = t >> 32;
        }
        if (c2) return inf;
    } else if (carry != 0) {
        return inf;
    }
    int top = ND - 1;
#pragma unroll 1
    while (top >= 0 && d[top] == 0) top--;
    if (top < 0) return 0.0;
    const int b = 32 * top + (32 - __clz((unsigned)d[top]));  // bit length of the magnitude
    uint64_t rb;
    if (b <= 53) {  // exactly representable: V * 2^-1074 with V < 2^53
        const uint64_t V = xbits64(d, ND, 0) & ((1ull << 53) - 1);
        rb = V < (1ull << 52) ? V : ((1ull << 52) | (V & ((1ull << 52) - 1)));
    } else {
        int sh = b - 53;
        uint64_t M = xbits64(d, ND, sh) & ((1ull << 53) - 1);
        const int guard = (int)(xbits64(d, ND, sh - 1) & 1);
        const int lo = sh - 1;  // sticky: any bit in [0, lo)
        bool sticky = false;
#pragma unroll 1
        for (int i = 0; i < (lo >> 5) && !sticky; i++) sticky = d[i] != 0;
        if (!sticky && (lo & 31)) sticky = (d[lo >> 5] & ((1ll << (lo & 31)) - 1)) != 0;
        if (guard && (sticky || (M & 1))) {
            M++;
            if (M == (1ull << 53)) M >>= 1, sh++;
        }
        const int ef = sh - 1074 + 52 + 1023;  // biased exponent of M * 2^(sh - 1074)
        if (ef >= 2047) return inf;
        rb = ((uint64_t)ef << 52) | (M & ((1ull << 52) - 1));
    }
    return __longlong_as_double((long long)(sign | rb));
}

// norm([a b]) of the exact mode (cpminres.m:218, cpsymmlq.m:239,291,324): one operation
// sequence shared with the oracle (cpk_oracle.c xnorm2) instead of two libm hypots -- a power-
// of-two scaling, a^2 + b^2 as a double-double (TwoProd by FMA, TwoSum), its square root and
// one Newton correction.  Every step is an IEEE-rounded basic operation, so both sides agree.
__device__ inline double xnorm2(double a, double b) {
    a = fabs(a), b = fabs(b);
    if (a < b) {
        const double t = a;
        a = b, b = t;
    }
    if (!(b > 0) || !isfinite(a)) return a + b;
    double sc = 1.0, us = 1.0;
    if (a > 0x1p500) sc = 0x1p-600, us = 0x1p600;
    else if (a < 0x1p-500) sc = 0x1p600, us = 0x1p-600;
    a = a * sc, b = b * sc;
    const double p1 = a * a, e1 = fma(a, a, -p1);
    const double p2 = b * b, e2 = fma(b, b, -p2);
    const double s = p1 + p2, bb = s - p1, t = (p1 - (s - bb)) + (p2 - bb);
    double lo = t + (e1 + e2);
    const double hi = s + lo;
    lo = lo - (hi - s);
    const double r = sqrt(hi);
    const double res = fma(-r, r, hi) + lo;
    return (r + res / (2.0 * r)) * us;
}

// A workgroup's exact sums deposited into their sub-accumulators (v[j].ovf): the 64 lanes of a
// wave merge by shuffles, the waves through LDS, and thread 0 deposits the merged expansions.
// On return every wave has drained its deposits (s_waitcnt vmcnt(0)) and thread 0 its own:
// a ticket taken by thread 0 after the final barrier follows every deposit of the workgroup.
template <int NV>
__device__ __forceinline__ void block_deposit(XAcc (&v)[NV]) {
    __shared__ double xs[kBlock / kWave][NV][kXK];
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
#pragma unroll
    for (int j = 0; j < NV; j++)  // wave merge, one sum at a time: lane 0 ends with the wave's sum
#pragma unroll
        for (int off = kWave / 2; off > 0; off >>= 1) {
            double o[kXK];
#pragma unroll
            for (int k = 0; k < kXK; k++) o[k] = __shfl_down(v[j].t[k], off, kWave);
            if (lane < off)
#pragma unroll
                for (int k = 0; k < kXK; k++) v[j].add(o[k]);
        }
    if (lane == 0)
#pragma unroll
        for (int j = 0; j < NV; j++)
#pragma unroll
            for (int k = 0; k < kXK; k++) xs[wid][j][k] = v[j].t[k];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's overflow deposits done
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll 1
        for (int w = 1; w < (int)(blockDim.x / kWave); w++)
#pragma unroll
            for (int j = 0; j < NV; j++)
#pragma unroll
                for (int k = 0; k < kXK; k++) v[j].add(xs[w][j][k]);
#pragma unroll
        for (int j = 0; j < NV; j++)
#pragma unroll
            for (int k = 0; k < kXK; k++) xdeposit(v[j].ovf, v[j].t[k]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();  // xs[] free for the caller's next deposit
}

// The last workgroup's half: the digits of sums [s0, s0 + ns) of a launch of nv sums, summed
// over the sub-accumulators into dig[ns][kXW] (LDS), which are zeroed for the next launch;
// xdefer (optional) also receives them at [s0 + j]
__device__ __forceinline__ void gather_digits(int64_t *xsub, int nv, int s0, int ns, int64_t (*dig)[kXW], int64_t *xdefer) {
    const unsigned G = gridDim.x < kXSub ? gridDim.x : kXSub;
#pragma unroll 1
    for (int c = threadIdx.x; c < ns * kXW; c += blockDim.x) {
        int64_t s = 0;
        for (unsigned g = 0; g < G; g++) {
            int64_t *p = xsub + ((size_t)g * nv + s0) * kXW + c;
            s += ld_agent64(p);
            st_agent64(p, 0);
        }
        dig[c / kXW][c % kXW] = s;
        if (xdefer) xdefer[(size_t)s0 * kXW + c] = s;
    }
    __syncthreads();
}

// Exact grid reduction of NV sums (the XAcc form of devutil.hpp grid_sum, same contract):
// true in every thread of the last-arriving workgroup, where tot[] (thread 0) holds the
// rounded sums; distributed (rb.xdefer) the digits go there and it returns false.
template <int NV>
__device__ bool grid_sum(XAcc (&v)[NV], RedBuf rb, double (&tot)[NV], bool *was_last = nullptr) {
    __shared__ int64_t dig[NV][kXW];
    __shared__ double rt[NV];
    __shared__ int s_last;
    block_deposit<NV>(v);
    if (threadIdx.x == 0) s_last = arrive_last(rb.counter);
    __syncthreads();
    if (was_last) *was_last = s_last != 0;
    if (!s_last) return false;
    gather_digits(rb.xsub, NV, 0, NV, dig, rb.xdefer);
    if (rb.xdefer) return false;
    if (threadIdx.x < NV) rt[threadIdx.x] = xround(dig[threadIdx.x]);
    __syncthreads();
    if (threadIdx.x == 0)
#pragma unroll
        for (int j = 0; j < NV; j++) tot[j] = rt[j];
    return true;
}

// the reduction buffers of a launch: the partials and tickets, the distributed deferral, and in
// exact mode the sub-accumulators and the digit deferral (Ctx::ensure_partials / ensure_xacc
// sized them before any capture)
inline RedBuf red_buf(Ctx &c) {
    const bool dist = c.dist(), ex = c.exact();
    return RedBuf{c.partials.p, c.counter.p, dist && !ex ? c.red.p : nullptr, ex ? c.xsub.p : nullptr,
                  dist && ex ? c.xred.p : nullptr};
}
// distributed mode: the local sums the reduction deferred (c.red, or c.xred's digits in exact
// mode) summed over the ranks into c.red -- the exact digits by an int64 allreduce and then
// rounded on every rank (xround_kernel), so every rank holds the same bits
void allreduce_red(Ctx &c, int nv);
}  // namespace cpk
