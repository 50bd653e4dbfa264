// spmv.hpp -- LDS-staged streaming CSR SpMV (gfx950) with a pluggable row epilogue.
//
// Each workgroup owns a precomputed row range whose nonzeros (<= kSpmvCap) are contiguous in
// HBM.  Phase 1 streams (val, col) coalesced -- consecutive lanes read consecutive entries --
// forms the products val*x[col] and stages them in LDS.  Phase 2 gives each thread whole rows
// and sums that row's products in column order from 0.0 (no FMA), which is the accumulation
// order of MATLAB's sparse mtimes, so results are bit-identical to the CPU restatement.
// A row longer than kSpmvCap sits alone in its workgroup and is summed chunk by chunk.
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "dev.hpp"
#include "devutil.hpp"

namespace cpk {

// HALO: distributed rows (DistCsr); column c >= nloc reads the allgathered halo xg[c - nloc].
// A workgroup handles row blocks blockIdx.x, blockIdx.x + gridDim.x, ... (grid: spmv_grid).
// a gathered input value as the epilogue wants it: Epi::xl where it has one (EpiKrylov's
// normalise-on-read), else as stored.  Halo values arrive already transformed.
template <class E, class = void>
struct HasXl : std::false_type {};
template <class E>
struct HasXl<E, std::void_t<decltype(&E::xl)>> : std::true_type {};
template <class Epi>
__device__ __forceinline__ double gathered(const Epi &e, double v) {
    if constexpr (HasXl<Epi>::value) return e.xl(v);
    return v;
}

// x[c], or for a ghost column (c >= nloc) the allgathered halo value xg[c - nloc]: ONE load from
// a selected base (two predicated loads per entry made the distributed SpMV 23 % slower than the
// single-GPU one at P = 1, r05); local values through the epilogue's transform, halo values as
// they arrived (already transformed by their owner)
template <bool HALO, class Epi>
__device__ __forceinline__ double halo_gather(const Epi &epi, const double *x, const double *xg, int64_t nloc,
                                              int32_t c) {
    if constexpr (!HALO) return gathered(epi, x[c]);
    const bool loc = c < nloc;
    // a selected base and a selected index (no pointer before xg is ever formed)
    const double *base = loc ? x : xg;
    const int64_t k = loc ? (int64_t)c : (int64_t)c - nloc;
    const double v = base[k];
    return loc ? gathered(epi, v) : v;
}

// Epi::kWaves where the epilogue sets one (EpiKrylov's normalise-on-read needs more registers)
template <class E, class = void>
struct SpmvWaves : std::integral_constant<int, CPK_SPMV_WAVES> {};
template <class E>
struct SpmvWaves<E, std::void_t<decltype(E::kWaves)>> : std::integral_constant<int, E::kWaves> {};

template <class Epi, bool HALO = false>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(SpmvWaves<Epi>::value))) void spmv_stream(const uint32_t *__restrict__ ptr,
                                                      const int32_t *__restrict__ col,
                                                      const double *__restrict__ val,
                                                      const int32_t *__restrict__ blk, int64_t nblk,
                                                      const double *x, int64_t col_min, Epi epi,
                                                      const double *xg, int64_t nloc) {
    __shared__ double prod[kSpmvCap];
    if (epi.skip()) return;
    x = epi.xvec(x);
    const int tid = threadIdx.x;
    for (int64_t b = blockIdx.x; b < nblk; b += gridDim.x) {
    if (b != blockIdx.x) __syncthreads();  // prod[] of the previous block fully consumed
    const int64_t r0 = blk[b], r1 = blk[b + 1];
    const uint32_t e0 = ptr[r0], e1 = ptr[r1];
    if (e1 - e0 <= (uint32_t)kSpmvCap) {
        // phase 1, fully unrolled so every load of a thread is in flight at once: the (col, val)
        // stream and this thread's row pointers first, then the dependent x gathers
        constexpr int EPT = kSpmvCap / kBlock, RPT = kSpmvMaxRows / kBlock;
        int32_t cc[EPT];
        double vv[EPT], xv[EPT];
        uint32_t pa[RPT], pb[RPT];
        double pr[RPT];  // the epilogue's per-row operand (e.g. x(i) of r = x - A*y), prefetched
#pragma unroll
        for (int j = 0; j < EPT; j++) {
            const uint32_t e = e0 + tid + j * kBlock;
            // the matrix is streamed once per launch: non-temporal, so it does not evict the
            // gathered vector from L2
            cc[j] = e < e1 ? __builtin_nontemporal_load(col + e) : 0;
            vv[j] = e < e1 ? __builtin_nontemporal_load(val + e) : 0.0;
        }
#pragma unroll
        for (int j = 0; j < RPT; j++) {
            const int64_t r = r0 + tid + j * kBlock;
            if (r < r1) pa[j] = ptr[r], pb[j] = ptr[r + 1], pr[j] = epi.pre(r);
        }
#pragma unroll
        for (int j = 0; j < EPT; j++) {
            const int32_t c = cc[j];
            xv[j] = halo_gather<HALO>(epi, x, xg, nloc, c);
        }
#pragma unroll
        for (int j = 0; j < EPT; j++) {
            const uint32_t e = e0 + tid + j * kBlock;
            if (e < e1) prod[e - e0] = (cc[j] >= col_min) ? vv[j] * xv[j] : 0.0;
        }
        __syncthreads();
        // phase 2: whole rows per thread, summed in column order from 0.0
#pragma unroll
        for (int j = 0; j < RPT; j++) {
            const int64_t r = r0 + tid + j * kBlock;
            if (r < r1) {
                double acc = 0.0;
                for (uint32_t e = pa[j] - e0; e < pb[j] - e0; e++) acc += prod[e];
                epi.row(r, acc, pr[j]);
            }
        }
    } else {
        double acc = 0.0;  // one long row (r1 == r0 + 1)
        for (uint32_t c0 = e0; c0 < e1; c0 += kSpmvCap) {
            const uint32_t c1 = min(e1, c0 + (uint32_t)kSpmvCap);
            for (uint32_t e = c0 + tid; e < c1; e += kBlock) {
                const int32_t c = col[e];
                const double xv = halo_gather<HALO>(epi, x, xg, nloc, c);
                prod[e - c0] = (c >= col_min) ? val[e] * xv : 0.0;
            }
            __syncthreads();
            if (tid == 0)
                for (uint32_t e = 0; e < c1 - c0; e++) acc += prod[e];
            __syncthreads();
        }
        if (tid == 0) epi.row(r0, acc, epi.pre(r0));
    }
    }
    epi.finish();
}

// Grid of a launch: exactly the workgroups that are resident at once (occupancy x CUs: 6 x 256
// = 1536 on MI355X), each walking every 1536th row block, so no second, partial wave of
// workgroups trails the launch.  Measured at S10: the Krylov SpMV (reducing) 123 us with a
// 2048 grid at 5 waves per SIMD, 93-97 us; the residual SpMV (one workgroup per row block
// before) 125 -> 120 us.  Deterministic for a given device: the grid fixes which partials each
// inner product sums.
template <class Epi, bool HALO>
inline unsigned spmv_grid(int64_t nblk) {
    static const int64_t resident = [] {
        int occ = 0, dev = 0, cus = 256;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void *)spmv_stream<Epi, HALO>, kBlock, 0) !=
                hipSuccess ||
            occ < 1)
            occ = 1;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        return (int64_t)occ * cus;
    }();
    return (unsigned)std::max<int64_t>(1, std::min<int64_t>(nblk, resident));
}

}  // namespace cpk
