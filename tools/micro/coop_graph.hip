// Can a cooperative launch (grid-wide barrier) be captured into a hipGraph on this stack, and
// what does one grid barrier cost?  Each phase p: every workgroup adds its id to slot p, grid
// barrier, then workgroup 0 checks the previous phase's sum.  Build:
//   hipcc -O2 --offload-arch=gfx950 tools/micro/coop_graph.hip -o build/coop_graph
#include <hip/hip_runtime.h>
#include <hip/hip_cooperative_groups.h>
#include <chrono>
#include <cstdio>
#include <vector>

namespace cg = cooperative_groups;

__global__ void phases_kernel(int nphase, unsigned long long *sums, int *bad) {
    cg::grid_group grid = cg::this_grid();
    for (int p = 0; p < nphase; p++) {
        if (threadIdx.x == 0) atomicAdd(&sums[p], (unsigned long long)blockIdx.x + 1);
        grid.sync();
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            const unsigned long long g = gridDim.x, want = g * (g + 1) / 2;
            if (sums[p] != want) atomicAdd(bad, 1);
        }
    }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s -> %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
    int dev = 0, coop = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev));
    printf("cooperative launch supported: %d\n", coop);
    int per_cu = 0, cus = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void *)phases_kernel, 512, 0));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    printf("co-resident workgroups: %d per CU x %d CUs\n", per_cu, cus);
    const int G = 96, NP = 6;
    unsigned long long *sums;
    int *bad;
    CK(hipMalloc(&sums, NP * sizeof(unsigned long long)));
    CK(hipMalloc(&bad, sizeof(int)));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int np = NP;
    void *args[] = {&np, &sums, &bad};
    // 1) direct cooperative launch
    CK(hipMemsetAsync(sums, 0, NP * sizeof(unsigned long long), s));
    CK(hipMemsetAsync(bad, 0, sizeof(int), s));
    CK(hipLaunchCooperativeKernel((const void *)phases_kernel, dim3(G), dim3(512), args, 0, s));
    CK(hipStreamSynchronize(s));
    int hbad = -1;
    CK(hipMemcpy(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost));
    printf("direct: bad = %d\n", hbad);
    // 2) captured into a graph
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    hipError_t le = hipLaunchCooperativeKernel((const void *)phases_kernel, dim3(G), dim3(512), args, 0, s);
    hipError_t ce = hipStreamEndCapture(s, &g);
    printf("capture: launch %s, end %s\n", hipGetErrorString(le), hipGetErrorString(ce));
    if (le != hipSuccess || ce != hipSuccess) return 2;
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int rep = 0; rep < 3; rep++) {
        CK(hipMemsetAsync(sums, 0, NP * sizeof(unsigned long long), s));
        CK(hipMemsetAsync(bad, 0, sizeof(int), s));
        CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost));
        printf("graph run %d: bad = %d\n", rep, hbad);
    }
    // 3) cost: NP barriers vs 1 (event-timed, 50 launches each)
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int nphase : {1, 2, 7}) {
        np = nphase;
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < 50; i++) CK(hipLaunchCooperativeKernel((const void *)phases_kernel, dim3(G), dim3(512), args, 0, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("phases %d: %.2f us per launch\n", nphase, ms * 1e3f / 50);
    }
    return 0;
}
