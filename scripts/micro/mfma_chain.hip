// Cycles per v_mfma_f32_32x32x16_bf16 at ONE wave per SIMD, by accumulator
// placement and dependency pattern (s_memtime around the loop, per wave).
// hipcc -O3 --offload-arch=gfx950 mfma_chain.hip -o /tmp/mfma_chain
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
#define MV(d, x, w) asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(d) : "v"(x), "v"(w))
#define MA(d, x, w) asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(d) : "v"(x), "v"(w))
template <int MODE>
__global__ __launch_bounds__(256, 1) void k(float *out, unsigned long long *cyc, int iters) {
    __shared__ char pad[150000];
    bf16x8_t x, w;
    for (int e = 0; e < 8; ++e) {
        unsigned h = (threadIdx.x * 2654435761u) ^ (e * 40503u);
        h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
        x[e] = (__bf16)((h & 0xffff) / 32768.f - 1.f);
        w[e] = (__bf16)(((h >> 16) & 0xffff) / 32768.f - 1.f);
    }
    f32x16_t a0 = {}, a1 = {}, a2 = {}, a3 = {};
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
        if (MODE == 0) {          // builtin, 4 accumulators round robin
            a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, w, a0, 0, 0, 0);
            a1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, w, a1, 0, 0, 0);
            a2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, w, a2, 0, 0, 0);
            a3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, w, a3, 0, 0, 0);
        } else if (MODE == 1) {   // builtin, one chain
            a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, w, a0, 0, 0, 0);
            a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, w, a0, 0, 0, 0);
            a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, w, a0, 0, 0, 0);
            a0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(x, w, a0, 0, 0, 0);
        } else if (MODE == 2) {   // asm, VGPR accumulator, one chain
            MV(a0, x, w); MV(a0, x, w); MV(a0, x, w); MV(a0, x, w);
        } else if (MODE == 3) {   // asm, VGPR accumulators, 2 chains interleaved
            MV(a0, x, w); MV(a1, x, w); MV(a0, x, w); MV(a1, x, w);
        } else if (MODE == 4) {   // asm, VGPR accumulators, 4 chains
            MV(a0, x, w); MV(a1, x, w); MV(a2, x, w); MV(a3, x, w);
        } else if (MODE == 5) {   // asm, AGPR accumulator, one chain
            MA(a0, x, w); MA(a0, x, w); MA(a0, x, w); MA(a0, x, w);
        } else if (MODE == 6) {   // asm, AGPR accumulators, 4 chains
            MA(a0, x, w); MA(a1, x, w); MA(a2, x, w); MA(a3, x, w);
        } else if (MODE == 7) {   // one asm block: VGPR chain, 2 VALU between dependent MFMAs
            float f0 = x[0], f1 = x[1];
            asm volatile(
                "v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0\n\t"
                "v_add_f32 %3, %3, %4\n\tv_add_f32 %4, %4, %3\n\t"
                "v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0\n\t"
                "v_add_f32 %3, %3, %4\n\tv_add_f32 %4, %4, %3\n\t"
                "v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0\n\t"
                "v_add_f32 %3, %3, %4\n\tv_add_f32 %4, %4, %3\n\t"
                "v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0"
                : "+v"(a0) : "v"(x), "v"(w), "v"(f0), "v"(f1));
        } else if (MODE == 8) {   // one asm block: VGPR chain, back to back
            asm volatile(
                "v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0\n\t"
                "v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0\n\t"
                "v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0\n\t"
                "v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0"
                : "+v"(a0) : "v"(x), "v"(w));
        } else if (MODE == 9) {   // one asm block: 2 VGPR chains alternating, 2 VALU between
            float f0 = x[0], f1 = x[1];
            asm volatile(
                "v_mfma_f32_32x32x16_bf16 %0, %2, %3, %0\n\t"
                "v_add_f32 %4, %4, %5\n\tv_add_f32 %5, %5, %4\n\t"
                "v_mfma_f32_32x32x16_bf16 %1, %2, %3, %1\n\t"
                "v_add_f32 %4, %4, %5\n\tv_add_f32 %5, %5, %4\n\t"
                "v_mfma_f32_32x32x16_bf16 %0, %2, %3, %0\n\t"
                "v_add_f32 %4, %4, %5\n\tv_add_f32 %5, %5, %4\n\t"
                "v_mfma_f32_32x32x16_bf16 %1, %2, %3, %1"
                : "+v"(a0), "+v"(a1) : "v"(x), "v"(w), "v"(f0), "v"(f1));
        } else if (MODE == 10) {  // one asm block: VGPR chain, one ds_read between
            int adr = threadIdx.x * 16;
            float4 r;
            asm volatile(
                "v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0\n\t"
                "ds_read_b128 %3, %4\n\t"
                "v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0\n\t"
                "ds_read_b128 %3, %4 offset:4096\n\t"
                "v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0\n\t"
                "ds_read_b128 %3, %4 offset:8192\n\t"
                "v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0\n\t"
                "s_waitcnt lgkmcnt(0)"
                : "+v"(a0), "=&v"(r) : "v"(x), "v"(w), "v"(adr) : "memory");
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
    float s = 0.f;
    for (int r = 0; r < 16; ++r) s += a0[r] + a1[r] + a2[r] + a3[r];
    pad[threadIdx.x] = (char)s;
    __syncthreads();
    out[blockIdx.x * 256 + threadIdx.x] = s + pad[(threadIdx.x + 1) & 255];
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}
template <int MODE>
void run(float *o, unsigned long long *c, const char *name) {
    const int iters = 1024;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(k<MODE>, dim3(256), dim3(256), 0, 0, o, c, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        unsigned long long h[1024];
        hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost);
        double avg = 0;
        for (int i = 0; i < 1024; ++i) avg += h[i];
        avg /= 1024;
        printf("%-40s rep %d: %.1f us, %.2f cycles/MFMA (s_memtime), %.2f GHz\n", name, rep,
               ms * 1e3, avg / (4.0 * iters), avg / (ms * 1e-3) / 1e9);
    }
}
int main() {
    float *o;
    unsigned long long *c;
    hipMalloc(&o, 256 * 256 * 4);
    hipMalloc(&c, 1024 * 8);
    run<0>(o, c, "builtin, 4 accumulators");
    run<1>(o, c, "builtin, 1 chain");
    run<2>(o, c, "asm VGPR acc, 1 chain");
    run<3>(o, c, "asm VGPR acc, 2 chains");
    run<4>(o, c, "asm VGPR acc, 4 chains");
    run<5>(o, c, "asm AGPR acc, 1 chain");
    run<6>(o, c, "asm AGPR acc, 4 chains");
    run<7>(o, c, "asm block, chain, 2 VALU between");
    run<8>(o, c, "asm block, chain back to back");
    run<9>(o, c, "asm block, 2 chains alt, 2 VALU between");
    run<10>(o, c, "asm block, chain, ds_read between");
    return 0;
}
