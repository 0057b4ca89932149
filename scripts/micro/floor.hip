// Diagnostic microbenchmark (not product code): the memory/launch floor of
// the env step's access pattern on MI355X, to separate "physics cost" from
// "moving 305 B per env through one small launch".
//   empty      : 256 x 256-thread blocks, no memory
//   copy4      : float4 stream copy, B bytes in + B bytes out
//   skel       : the step kernel's exact loads/stores (15 f64 SoA + float4 +
//                i32 in; 12 f64 + i32 + LDS-staged (N,15) f32 obs + f32 + u8
//                out), no physics
//   skel_nt    : skel with non-temporal stores
//   skel2      : skel with 2 envs per thread (16-B f64 loads)
// Build/run:  hipcc -O3 --offload-arch=gfx950 floor.hip -o floor && ./floor
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e = (x);                                                   \
        if (e != hipSuccess) {                                                \
            printf("%s: %s\n", #x, hipGetErrorString(e));                     \
            exit(1);                                                          \
        }                                                                     \
    } while (0)

__global__ void empty_k() {}

__global__ void copy4_k(const float4 *__restrict__ a, float4 *__restrict__ b, int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) b[i] = a[i];
}

template <bool NT>
__global__ __launch_bounds__(256) void skel_k(double *f, int64_t stride, int32_t *step,
                                              const float4 *act, float *obs, float *rew,
                                              uint8_t *done, int64_t n) {
    __shared__ float sh[256 * 15];
    int64_t base = (int64_t)blockIdx.x * 256, i = base + threadIdx.x;
    float ob[15];
    if (i < n) {
        double s[15];
#pragma unroll
        for (int k = 0; k < 15; ++k) s[k] = f[k * stride + i];
        float4 a = act[i];
        int st = step[i] + 1;
#pragma unroll
        for (int k = 0; k < 12; ++k) {
            double x = s[k] + (double)a.x * 1e-30;
            if (NT)
                __builtin_nontemporal_store(x, &f[k * stride + i]);
            else
                f[k * stride + i] = x;
            ob[k] = (float)x;
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) ob[12 + k] = (float)(s[12 + k] - s[k]);
        step[i] = st;
        rew[i] = a.y;
        done[i] = st > 1000000;
    } else {
        for (int k = 0; k < 15; ++k) ob[k] = 0;
    }
    for (int k = 0; k < 15; ++k) sh[threadIdx.x * 15 + k] = ob[k];
    __syncthreads();
    float4 *d4 = reinterpret_cast<float4 *>(obs + base * 15);
    const float4 *s4 = reinterpret_cast<const float4 *>(sh);
    if (base + 256 <= n)
        for (int q = threadIdx.x; q < 960; q += 256) {
            if (NT) {
                typedef float nf4 __attribute__((ext_vector_type(4)));
                nf4 v = {s4[q].x, s4[q].y, s4[q].z, s4[q].w};
                __builtin_nontemporal_store(v, reinterpret_cast<nf4 *>(&d4[q]));
            } else {
                d4[q] = s4[q];
            }
        }
}

__global__ __launch_bounds__(256) void skel2_k(double *f, int64_t stride, int32_t *step,
                                               const float4 *act, float *obs, float *rew,
                                               uint8_t *done, int64_t n) {
    __shared__ float sh[512 * 15];
    int64_t base = (int64_t)blockIdx.x * 512, i = base + 2 * threadIdx.x;
    float ob[2][15];
    if (i < n) {
        double2 s[15];
#pragma unroll
        for (int k = 0; k < 15; ++k) s[k] = *reinterpret_cast<const double2 *>(&f[k * stride + i]);
        float4 a0 = act[i], a1 = act[i + 1];
        int2 st = *reinterpret_cast<const int2 *>(&step[i]);
#pragma unroll
        for (int k = 0; k < 12; ++k) {
            double2 x = make_double2(s[k].x + a0.x * 1e-30, s[k].y + a1.x * 1e-30);
            *reinterpret_cast<double2 *>(&f[k * stride + i]) = x;
            ob[0][k] = (float)x.x;
            ob[1][k] = (float)x.y;
        }
        for (int k = 0; k < 3; ++k) {
            ob[0][12 + k] = (float)(s[12 + k].x - s[k].x);
            ob[1][12 + k] = (float)(s[12 + k].y - s[k].y);
        }
        *reinterpret_cast<int2 *>(&step[i]) = make_int2(st.x + 1, st.y + 1);
        *reinterpret_cast<float2 *>(&rew[i]) = make_float2(a0.y, a1.y);
        done[i] = 0;
        done[i + 1] = 0;
    }
    for (int e = 0; e < 2; ++e)
        for (int k = 0; k < 15; ++k) sh[(2 * threadIdx.x + e) * 15 + k] = ob[e][k];
    __syncthreads();
    float4 *d4 = reinterpret_cast<float4 *>(obs + base * 15);
    const float4 *s4 = reinterpret_cast<const float4 *>(sh);
    if (base + 512 <= n)
        for (int q = threadIdx.x; q < 1920; q += 256) d4[q] = s4[q];
}

template <typename F>
float time_graph(F launch, int reps) {
    hipStream_t s;
    CK(hipStreamCreate(&s));
    for (int i = 0; i < 10; ++i) launch(s);
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int i = 0; i < reps; ++i) launch(s);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, s));
    CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    CK(hipStreamDestroy(s));
    return ms * 1000.f / reps;
}

int main() {
    const int reps = 500;
    printf("empty 256x256: %.3f us\n",
           time_graph([](hipStream_t s) { empty_k<<<256, 256, 0, s>>>(); }, reps));
    for (int64_t n : {65536LL, 262144LL, 1048576LL, 4194304LL}) {
        const int64_t stride = n;
        double *f;
        int32_t *step;
        float4 *act;
        float *obs, *rew;
        uint8_t *done;
        CK(hipMalloc(&f, 15 * n * 8));
        CK(hipMalloc(&step, n * 4));
        CK(hipMalloc(&act, n * 16));
        CK(hipMalloc(&obs, n * 60));
        CK(hipMalloc(&rew, n * 4));
        CK(hipMalloc(&done, n));
        CK(hipMemset(f, 0, 15 * n * 8));
        CK(hipMemset(step, 0, n * 4));
        CK(hipMemset(act, 0, n * 16));
        const double bytes = 305.0 * n;
        unsigned g1 = (unsigned)((n + 255) / 256), g2 = (unsigned)((n + 511) / 512);
        float t0 = time_graph([&](hipStream_t s) {
            skel_k<false><<<g1, 256, 0, s>>>(f, stride, step, act, obs, rew, done, n);
        }, reps);
        float t1 = time_graph([&](hipStream_t s) {
            skel_k<true><<<g1, 256, 0, s>>>(f, stride, step, act, obs, rew, done, n);
        }, reps);
        float t2 = time_graph([&](hipStream_t s) {
            skel2_k<<<g2, 256, 0, s>>>(f, stride, step, act, obs, rew, done, n);
        }, reps);
        // float4 copy moving the same total bytes (half read, half write)
        const int64_t n4 = (int64_t)(bytes / 2 / 16);
        float4 *ca, *cb;
        CK(hipMalloc(&ca, n4 * 16));
        CK(hipMalloc(&cb, n4 * 16));
        CK(hipMemset(ca, 0, n4 * 16));
        float t3 = time_graph([&](hipStream_t s) {
            copy4_k<<<(unsigned)((n4 + 255) / 256), 256, 0, s>>>(ca, cb, n4);
        }, reps);
        printf("n=%8lld  skel %.3f us (%.0f GB/s)  skel_nt %.3f us (%.0f GB/s)  skel2 %.3f us (%.0f GB/s)  copy4 %.3f us (%.0f GB/s)\n",
               (long long)n, t0, bytes / t0 / 1e3, t1, bytes / t1 / 1e3, t2, bytes / t2 / 1e3, t3,
               bytes / t3 / 1e3);
        CK(hipFree(f)); CK(hipFree(step)); CK(hipFree(act)); CK(hipFree(obs));
        CK(hipFree(rew)); CK(hipFree(done)); CK(hipFree(ca)); CK(hipFree(cb));
    }
    return 0;
}
