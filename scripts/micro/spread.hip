// Diagnostic (not product code): how fast does the dispatcher start the
// waves of a 1024-wave grid, as a function of the kernel's VGPR and LDS
// footprint and block size?  Each wave stamps s_memrealtime at entry; we
// report the spread (first -> last wave start) and the kernel time.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                          \
    do {                                                               \
        hipError_t e = (x);                                            \
        if (e != hipSuccess) {                                         \
            printf("%s: %s\n", #x, hipGetErrorString(e));              \
            return 1;                                                  \
        }                                                              \
    } while (0)

template <int LDS_FLOATS, bool BIGV>
__global__ void probe(unsigned long long *st, float *sink) {
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    const unsigned w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if ((threadIdx.x & 63) == 0) st[w] = t;
    if constexpr (LDS_FLOATS > 0) {
        __shared__ float sh[LDS_FLOATS];
        sh[threadIdx.x] = (float)t;
        __syncthreads();
        if (sh[(threadIdx.x + 1) % blockDim.x] == 12345.f) sink[0] = 1;
    }
    if constexpr (BIGV) {
        // force a ~110-VGPR allocation without spilling
        asm volatile("v_mov_b32 v109, 0" ::: "v109");
    }
}

template <int LDS_FLOATS, bool BIGV>
int run(const char *name, int block, int waves) {
    unsigned long long *st;
    float *sink;
    CK(hipMalloc(&st, waves * 8));
    CK(hipMalloc(&sink, 4));
    const int grid = waves * 64 / block;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<double> spreads, times;
    for (int r = 0; r < 20; ++r) {
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(a, 0));
        hipLaunchKernelGGL((probe<LDS_FLOATS, BIGV>), dim3(grid), dim3(block), 0, 0, st, sink);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        std::vector<unsigned long long> h(waves);
        CK(hipMemcpy(h.data(), st, waves * 8, hipMemcpyDeviceToHost));
        auto mm = std::minmax_element(h.begin(), h.end());
        if (r >= 5) {
            spreads.push_back((*mm.second - *mm.first) * 0.01);
            times.push_back(ms * 1000);
        }
    }
    std::sort(spreads.begin(), spreads.end());
    std::sort(times.begin(), times.end());
    printf("%-28s block %4d grid %5d: start spread p50 %.2f us, event time p50 %.2f us\n", name,
           block, grid, spreads[spreads.size() / 2], times[times.size() / 2]);
    CK(hipFree(st));
    CK(hipFree(sink));
    return 0;
}

int main() {
    for (int block : {64, 256}) {
        run<0, false>("plain", block, 1024);
        run<0, true>("vgpr110", block, 1024);
        run<3840, false>("lds15KB", block, 1024);
        run<3840, true>("lds15KB+vgpr110", block, 1024);
    }
    run<0, false>("plain 4096 waves", 256, 4096);
    run<3840, true>("lds+vgpr 4096 waves", 256, 4096);
    return 0;
}
