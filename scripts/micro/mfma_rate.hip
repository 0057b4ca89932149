// Calibration: the x6 GEMM's MFMA stream alone (no memory), 2 waves/SIMD.
// hipcc -O3 --offload-arch=gfx950 mfma_rate.hip -o build/mfma_rate
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
template <int MODE>
__global__ __launch_bounds__(512) void k(float *out, int iters, float seed) {
    __shared__ char pad[100000];
    bf16x8_t a[2][3], b[2][3];
    for (int i = 0; i < 2; ++i)
        for (int p = 0; p < 3; ++p)
            for (int e = 0; e < 8; ++e) {
                // hashed (random-looking) operands: toggling bits set the power
                unsigned hsh = (threadIdx.x * 2654435761u) ^ ((e * 8 + p * 2 + i) * 40503u) ^
                               (unsigned)(seed * 977.f);
                hsh ^= hsh >> 13; hsh *= 0x5bd1e995u; hsh ^= hsh >> 15;
                a[i][p][e] = (__bf16)(((hsh & 0xffff) / 32768.f - 1.f));
                b[i][p][e] = (__bf16)((((hsh >> 16) & 0xffff) / 32768.f - 1.f) * 0.06f);
            }
    f32x16_t h[2][2] = {}, l[2][2] = {};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                if (MODE == 0) {   // x6: 1 hi + 5 dependent lo
                    h[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j][0], a[i][0], h[i][j], 0, 0, 0);
                    f32x16_t t = l[i][j];
                    t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j][1], a[i][0], t, 0, 0, 0);
                    t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j][0], a[i][1], t, 0, 0, 0);
                    t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j][2], a[i][0], t, 0, 0, 0);
                    t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j][0], a[i][2], t, 0, 0, 0);
                    t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j][1], a[i][1], t, 0, 0, 0);
                    l[i][j] = t;
                } else {           // 6 independent-ish: spread over h and l alternately
                    for (int r = 0; r < 3; ++r) {
                        h[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j][r], a[i][0], h[i][j], 0, 0, 0);
                        l[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[j][0], a[i][r], l[i][j], 0, 0, 0);
                    }
                }
            }
    }
    float s = 0.f;
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j)
            for (int r = 0; r < 16; ++r) s += h[i][j][r] + l[i][j][r];
    pad[threadIdx.x] = (char)s;
    __syncthreads();
    out[blockIdx.x * 512 + threadIdx.x] = s + pad[(threadIdx.x + 1) & 511];
}
int main() {
    float *o;
    hipMalloc(&o, 256 * 512 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 64;   // 64 x 24 = 1536 MFMAs per wave (the GEMM's count at m = 65,536)
    for (int mode = 0; mode < 2; ++mode) {
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(e0);
            for (int r = 0; r < 20; ++r) {
                if (mode == 0) k<0><<<256, 512>>>(o, iters, 1.0f + r);
                else k<1><<<256, 512>>>(o, iters, 1.0f + r);
            }
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double us = ms * 1e3 / 20;
            const double fl = 256.0 * 8 * iters * 24 * 32768;
            printf("mode %d: %.1f us per launch, %.0f TF/s bf16 (ideal at 2.4 GHz: %.1f us)\n",
                   mode, us, fl / us / 1e6, iters * 24 * 32 * 2 / 2.4e3);
        }
    }
    return 0;
}
