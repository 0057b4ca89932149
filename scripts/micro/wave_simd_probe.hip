// Where do a 256-thread block's four waves run?  HW_ID (SIMD / CU / SE) and
// XCC_ID of every wave of a 1,024-block launch shaped like ppo_head_kernel's
// (40 KB of LDS per block, so 4 blocks per CU are resident as with the head
// kernel's 126 VGPRs), each wave spinning ~50 us so the grid is co-resident;
// then, per (XCC, SE, CU, SIMD), how many of its waves are wave 0-1 of their
// block (the head kernel's policy role) under the role maps tried.
//   hipcc --offload-arch=gfx950 -O2 -o build/wave_simd_probe wave_simd_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <tuple>
#include <vector>

__global__ __launch_bounds__(256) void probe(unsigned *out, int spin) {
    extern __shared__ float lds[];
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);     // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);   // HW_REG_XCC_ID
    float x = threadIdx.x;
    for (int i = 0; i < spin; ++i) x = x * 0.999f + 1.0f;
    lds[threadIdx.x] = x;
    if ((threadIdx.x & 63) == 0) {
        const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
        out[3 * w] = hw;
        out[3 * w + 1] = xcc;
        out[3 * w + 2] = (unsigned)lds[threadIdx.x] & 1;
    }
}

int main() {
    const int nb = 1024;
    unsigned *d;
    hipMalloc(&d, nb * 4 * 3 * 4);
    hipLaunchKernelGGL(probe, dim3(nb), dim3(256), 40 * 1024, 0, d, 200000);
    std::vector<unsigned> h(nb * 4 * 3);
    hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    // role maps: 0 = waves 0-1 policy (current); 1 = (wid>>1) ^ (b & 1); 2 = (wid>>1) ^ ((b>>8)&1)
    for (int map = 0; map < 3; ++map) {
        std::map<std::tuple<int, int, int, int>, std::pair<int, int>> cnt;
        for (int b = 0; b < nb; ++b)
            for (int w = 0; w < 4; ++w) {
                const unsigned hw = h[3 * (4 * b + w)], xcc = h[3 * (4 * b + w) + 1];
                const int simd = (hw >> 4) & 3, cu = (hw >> 8) & 15, sh = (hw >> 12) & 1,
                          se = (hw >> 13) & 7;
                int pol = (w >> 1) == 0;
                if (map == 1) pol = (((w >> 1) ^ (b & 1)) == 0);
                if (map == 2) pol = (((w >> 1) ^ ((b >> 8) & 1)) == 0);
                auto &c = cnt[{(int)(xcc & 15), se * 2 + sh, cu, simd}];
                c.first += pol;
                c.second += 1;
            }
        std::map<std::pair<int, int>, int> hist;   // (policy waves, waves) per SIMD
        for (auto &kv : cnt) hist[kv.second]++;
        printf("map %d: %zu SIMDs;", map, cnt.size());
        for (auto &kv : hist) printf(" %d/%d x%d", kv.first.first, kv.first.second, kv.second);
        printf("\n");
    }
    // the first 8 blocks' placement
    for (int b = 0; b < 8; ++b) {
        printf("block %d:", b);
        for (int w = 0; w < 4; ++w) {
            const unsigned hw = h[3 * (4 * b + w)];
            printf(" w%d xcc%u se%u cu%u simd%u", w, h[3 * (4 * b + w) + 1] & 15, (hw >> 13) & 7,
                   (hw >> 8) & 15, (hw >> 4) & 3);
        }
        printf("\n");
    }
    return 0;
}
