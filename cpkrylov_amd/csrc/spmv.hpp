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

#include "dev.hpp"
#include "devutil.hpp"

namespace cpk {

// HALO: distributed rows (DistCsr); column c >= nloc reads the allgathered halo xg[c - nloc].
template <class Epi, bool HALO = false>
__global__ __launch_bounds__(kBlock) void spmv_stream(const uint32_t *__restrict__ ptr,
                                                      const int32_t *__restrict__ col,
                                                      const double *__restrict__ val,
                                                      const int32_t *__restrict__ blk,
                                                      const double *x, int64_t col_min, Epi epi,
                                                      const double *xg, int64_t nloc) {
    __shared__ double prod[kSpmvCap];
    if (epi.skip()) return;
    x = epi.xvec(x);
    const int64_t r0 = blk[blockIdx.x], r1 = blk[blockIdx.x + 1];
    const uint32_t e0 = ptr[r0], e1 = ptr[r1];
    const int tid = threadIdx.x;
    if (e1 - e0 <= (uint32_t)kSpmvCap) {
        for (uint32_t e = e0 + tid; e < e1; e += kBlock) {
            const int32_t c = col[e];
            const double xv = (!HALO || c < nloc) ? x[c] : xg[c - nloc];
            prod[e - e0] = (c >= col_min) ? val[e] * xv : 0.0;
        }
        __syncthreads();
        for (int64_t r = r0 + tid; r < r1; r += kBlock) {
            double acc = 0.0;
            const uint32_t a = ptr[r] - e0, b = ptr[r + 1] - e0;
            for (uint32_t e = a; e < b; e++) acc += prod[e];
            epi.row(r, acc);
        }
    } else {
        double acc = 0.0;  // one long row (r1 == r0 + 1)
        for (uint32_t c0 = e0; c0 < e1; c0 += kSpmvCap) {
            const uint32_t c1 = min(e1, c0 + (uint32_t)kSpmvCap);
            for (uint32_t e = c0 + tid; e < c1; e += kBlock) {
                const int32_t c = col[e];
                const double xv = (!HALO || c < nloc) ? x[c] : xg[c - nloc];
                prod[e - c0] = (c >= col_min) ? val[e] * xv : 0.0;
            }
            __syncthreads();
            if (tid == 0)
                for (uint32_t e = 0; e < c1 - c0; e++) acc += prod[e];
            __syncthreads();
        }
        if (tid == 0) epi.row(r0, acc);
    }
    epi.finish();
}

}  // namespace cpk
