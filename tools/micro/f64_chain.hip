// Dependent-latency microbenchmark (diagnostic): cycles per dependent v_add_f64 / v_fma_f64 /
// v_add_f32 on one wave, and per DPP-shift + add step, timed with s_memtime.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void chain(const double *in, double *out, long long *cyc, int n) {
    double a = in[threadIdx.x], b = in[threadIdx.x + 64];
    float af = (float)a, bf = (float)b;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++) {
#pragma unroll
        for (int k = 0; k < 16; k++) a = a - b;
    }
    asm volatile("" :: "v"(a));
    long long t1 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; i++) {
#pragma unroll
        for (int k = 0; k < 16; k++) af = af - bf;
    }
    asm volatile("" :: "v"(af));
    long long t2 = __builtin_amdgcn_s_memtime();
    double x = b;
    for (int i = 0; i < n; i++) {
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), 0x130, 0xf, 0xf, true);
            const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), 0x130, 0xf, 0xf, true);
            x = __hiloint2double(hi, lo);
            a -= x;
        }
    }
    asm volatile("" :: "v"(a));
    long long t3 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[0] = t1 - t0, cyc[1] = t2 - t1, cyc[2] = t3 - t2;
    out[threadIdx.x] = a + af;
}
int main() {
    double *in, *out;
    long long *cyc;
    hipMalloc(&in, 128 * 8), hipMalloc(&out, 64 * 8), hipMalloc(&cyc, 64);
    hipMemset(in, 0, 128 * 8);
    const int n = 1000;
    for (int rep = 0; rep < 3; rep++) {
        hipLaunchKernelGGL(chain, dim3(1), dim3(64), 0, 0, in, out, cyc, n);
        long long h[3];
        hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
        printf("cycles per dependent op: add_f64 %.1f  add_f32 %.1f  dpp-shift+add_f64 %.1f\n", h[0] / (16.0 * n),
               h[1] / (16.0 * n), h[2] / (16.0 * n));
    }
    return 0;
}
