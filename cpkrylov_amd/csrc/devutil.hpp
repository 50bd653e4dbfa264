// devutil.hpp -- device helpers shared by the HIP translation units (gfx950, wave64).
//
// Reductions are deterministic: each workgroup reduces in a fixed tree (wave shuffles, then
// LDS), publishes its partial, and the LAST workgroup to arrive (one agent-scope atomic
// ticket) sums the partials in a fixed order and runs the scalar epilogue.  The hand-off
// follows MI355X_MICROARCH.md "Valid forms", row 1: partials are stored with 8-byte
// agent-scope atomic stores (sc1 write-through), every storing wave drains with
// s_waitcnt vmcnt(0) before the ticket add, and the last workgroup reads the partials with
// agent-scope atomic loads (sc1), so no release/acquire cache fences are needed.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace cpk {

constexpr int kWave = 64;
constexpr int kBlock = 256;  // threads per workgroup of the streaming kernels

struct RedBuf {
    double *partials;   // [grid][NV]
    unsigned *counter;  // zero between launches (the last workgroup resets it)
    double *defer = nullptr;  // distributed mode: the last workgroup stores the local sums here
                              // instead of running the epilogue (it runs after the allreduce)
    // exact mode (xacc.hpp, engine option exact_dots): the sums' sub-accumulators
    // [kXSub][NV][kXW] (zero between launches), and the distributed mode's digit output [NV][kXW]
    int64_t *xsub = nullptr;
    int64_t *xdefer = nullptr;
};

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) v += __shfl_down(v, off, kWave);
    return v;
}

// Block-wide sum of NV values; result valid in thread 0.  Fixed tree => deterministic.
template <int NV>
__device__ __forceinline__ void block_sum(double (&v)[NV]) {
    __shared__ double red[kBlock / kWave][NV];
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
#pragma unroll
    for (int j = 0; j < NV; j++) v[j] = wave_sum(v[j]);
    if (lane == 0)
#pragma unroll
        for (int j = 0; j < NV; j++) red[wid][j] = v[j];
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int j = 0; j < NV; j++) {
            double s = red[0][j];
            for (int w = 1; w < (int)(blockDim.x / kWave); w++) s += red[w][j];
            v[j] = s;
        }
    }
    __syncthreads();
}

__device__ __forceinline__ void st_agent(double *p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_agent(const double *p) {
    return __hip_atomic_load(const_cast<double *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Arrival ticket of a grid reduction (thread 0 of each workgroup, after its partials have been
// stored and drained).  Workgroups first count in on one of 16 group tickets, each on its own
// cache line, and only the last of a group counts in on the global ticket: same-address
// atomics per ticket drop from gridDim.x to ~gridDim.x/16, which is what bounds the tail of a
// reduction over thousands of workgroups.  Tickets are reset by their last arrival.
constexpr unsigned kTicketGroups = 16, kTicketStride = 16;  // 64-byte lines
constexpr size_t kTicketWords = kTicketStride * (1 + kTicketGroups);
__device__ __forceinline__ bool arrive_last(unsigned *counter) {
    const unsigned G = gridDim.x, g = blockIdx.x % kTicketGroups;
    const unsigned ngroups = G < kTicketGroups ? G : kTicketGroups;
    const unsigned gsize = (G - g + kTicketGroups - 1) / kTicketGroups;
    unsigned *cg = counter + kTicketStride * (1 + g);
    if (__hip_atomic_fetch_add(cg, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != gsize - 1) return false;
    __hip_atomic_store(cg, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (__hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != ngroups - 1) return false;
    __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
}

// Reduce v over the whole grid.  Returns true in every thread of the last-arriving
// workgroup, where tot[] (thread 0) holds the grid-wide sums in a fixed summation order.
template <int NV>
__device__ __forceinline__ bool grid_sum(double (&v)[NV], RedBuf rb, double (&tot)[NV], bool *was_last = nullptr) {
    __shared__ int s_last;
    block_sum<NV>(v);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int j = 0; j < NV; j++) st_agent(rb.partials + (size_t)blockIdx.x * NV + j, v[j]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        s_last = arrive_last(rb.counter);
    }
    __syncthreads();
    if (was_last) *was_last = s_last != 0;
    if (!s_last) return false;
    double acc[NV];
#pragma unroll
    for (int j = 0; j < NV; j++) acc[j] = 0.0;
    constexpr int kTail = 8;  // grids up to 8 * blockDim: every partial load in flight at once
    if (gridDim.x <= kTail * blockDim.x) {
        double t[kTail][NV];
#pragma unroll
        for (int q = 0; q < kTail; q++) {
            const unsigned b = threadIdx.x + q * blockDim.x;
#pragma unroll
            for (int j = 0; j < NV; j++) t[q][j] = b < gridDim.x ? ld_agent(rb.partials + (size_t)b * NV + j) : 0.0;
        }
#pragma unroll
        for (int q = 0; q < kTail; q++)
            if (threadIdx.x + q * blockDim.x < gridDim.x)
#pragma unroll
                for (int j = 0; j < NV; j++) acc[j] += t[q][j];  // same additions, same order
    } else {
        for (unsigned b = threadIdx.x; b < gridDim.x; b += blockDim.x)
#pragma unroll
            for (int j = 0; j < NV; j++) acc[j] += ld_agent(rb.partials + (size_t)b * NV + j);
    }
    block_sum<NV>(acc);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int j = 0; j < NV; j++) tot[j] = acc[j];
        if (rb.defer)
#pragma unroll
            for (int j = 0; j < NV; j++) rb.defer[j] = acc[j];
    }
    return rb.defer == nullptr;
}

// Predicate shared by every solver-loop kernel: run only while the iteration is live.
__device__ __forceinline__ bool skip(const int *run_flag, const int *active_flag) {
    return (run_flag && *run_flag == 0) || (active_flag && *active_flag == 0);
}

}  // namespace cpk
