// Where do the waves of 256-thread workgroups land?  Every wave records its SIMD, CU, shader
// array / engine, XCC and LDS base (s_getreg, read only) for a grid of workgroups whose dynamic
// LDS allows 5 per CU (the +-64 window's first upper round).  Prints, per (CU, SIMD), how many
// "wave 0"s landed there: if every workgroup's wave 0 shares one SIMD, a kernel that runs its
// serial phase on wave 0 leaves three SIMDs idle.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <vector>

__global__ void probe(unsigned *out, int spin) {
    extern __shared__ char lds[];
    unsigned hw, xcc, la;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_LDS_ALLOC)" : "=s"(la));
    lds[threadIdx.x] = (char)hw;
    // stay resident long enough that the whole grid's first wave of workgroups co-resides
    long long t0 = clock64();
    while (clock64() - t0 < spin) __builtin_amdgcn_s_sleep(1);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        const int w = threadIdx.x >> 6;
        unsigned *o = out + ((size_t)blockIdx.x * 4 + w) * 3;
        o[0] = hw, o[1] = xcc, o[2] = la + (unsigned)lds[0] * 0u;
    }
}

int main() {
    const int G = 1280, lds = 32 * 1024;
    unsigned *d;
    hipMalloc(&d, (size_t)G * 4 * 3 * sizeof(unsigned));
    hipLaunchKernelGGL(probe, dim3(G), dim3(256), lds, 0, d, 2000000);
    hipDeviceSynchronize();
    std::vector<unsigned> h((size_t)G * 12);
    hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    // HW_ID (gfx9): wave_id [3:0], simd_id [5:4], pipe [7:6], cu_id [11:8], sh_id [12], se_id [15:13]
    std::map<std::pair<unsigned, unsigned>, int> w0;  // (cu key, simd) -> wave-0 count
    std::map<unsigned, int> percu, simdhist[4];
    int same = 0, distinct4 = 0;
    for (int b = 0; b < G; b++) {
        unsigned simds = 0;
        for (int w = 0; w < 4; w++) simds |= 1u << ((h[(b * 4 + w) * 3] >> 4) & 3);
        distinct4 += simds == 15;
        const unsigned hw = h[b * 12], key = (h[b * 12 + 1] << 16) | (hw >> 8 & 0xff);
        w0[{key, (hw >> 4) & 3}]++;
        percu[key]++;
        for (int w = 0; w < 4; w++) simdhist[w][(h[(b * 4 + w) * 3] >> 4) & 3]++;
        (void)same;
    }
    printf("workgroups %d, CUs seen %zu, workgroups with 4 waves on 4 distinct SIMDs: %d\n", G, percu.size(), distinct4);
    for (int w = 0; w < 4; w++)
        printf("wave %d by SIMD: %d %d %d %d\n", w, simdhist[w][0], simdhist[w][1], simdhist[w][2], simdhist[w][3]);
    int maxw0 = 0;
    std::map<int, int> hist;
    for (auto &kv : percu) {
        int m = 0;
        for (unsigned s = 0; s < 4; s++) { auto it = w0.find({kv.first, s}); m = std::max(m, it == w0.end() ? 0 : it->second); }
        hist[m]++;
        maxw0 = std::max(maxw0, m);
    }
    printf("per CU: most wave-0s on one SIMD -> number of CUs:");
    for (auto &kv : hist) printf(" %d:%d", kv.first, kv.second);
    printf("\nfirst 8 workgroups (xcc, hw_id per wave, lds_alloc):\n");
    for (int b = 0; b < 8; b++)
        printf("  wg %d xcc %u simd %u %u %u %u cu %u lds %08x\n", b, h[b * 12 + 1], h[b * 12] >> 4 & 3, h[b * 12 + 3] >> 4 & 3,
               h[b * 12 + 6] >> 4 & 3, h[b * 12 + 9] >> 4 & 3, h[b * 12] >> 8 & 15, h[b * 12 + 2]);
    hipFree(d);
    return 0;
}
