// Shared helpers for libdronerl.so (gfx950): error plumbing, Philox4x32-10,
// launch geometry.  Internal header; the public ABI is include/dronerl.h.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../../include/dronerl.h"

namespace dr {

// Nontemporal (streaming) stores: written through to memory as the kernel
// runs instead of staying dirty in L2 until the end-of-kernel writeback.
template <typename T>
__device__ inline void store_nt(T *p, T x) {
    __builtin_nontemporal_store(x, p);
}
__device__ inline void store_nt(float4 *p, float4 x) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store(f4v{x.x, x.y, x.z, x.w}, reinterpret_cast<f4v *>(p));
}

// ----------------------------------------------------------------------------
// Errors: a per-thread message for handle-less calls, a per-handle one else.
// ----------------------------------------------------------------------------
void set_global_error(const std::string &msg);
const char *global_error();

#define DR_HIP_CHECK_RET(expr, errsink)                                       \
    do {                                                                      \
        hipError_t e__ = (expr);                                              \
        if (e__ != hipSuccess) {                                              \
            errsink(std::string(#expr) + ": " + hipGetErrorString(e__));      \
            return DR_ERR_HIP;                                                \
        }                                                                     \
    } while (0)

// RAII device switch: entry points run on the handle's device and restore
// the caller's current device on exit.
struct DeviceGuard {
    int prev = -1;
    bool switched = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) == hipSuccess && prev != dev) {
            switched = (hipSetDevice(dev) == hipSuccess);
        }
    }
    ~DeviceGuard() {
        if (switched) (void)hipSetDevice(prev);
    }
};

// ----------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al., SC'11), counter-based: every (key, counter)
// pair gives an independent 128-bit block, so env i's draws never depend on
// how many other envs reset or in which order.
// ----------------------------------------------------------------------------
struct u32x4 {
    uint32_t x, y, z, w;
};

__host__ __device__ inline u32x4 philox4x32_10(u32x4 c, uint32_t k0,
                                               uint32_t k1) {
    constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    constexpr uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)M0 * c.x;
        const uint64_t p1 = (uint64_t)M1 * c.z;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += W0;
        k1 += W1;
    }
    return c;
}

// 53-bit uniform double in [0,1) from two words (numpy's construction:
// (a >> 5) * 2^26 + (b >> 6), scaled by 2^-53).
__host__ __device__ inline double u01_f64(uint32_t a, uint32_t b) {
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) *
           (1.0 / 9007199254740992.0);
}

// Uniform double in [0,1) with 32 random bits (exact: w * 2^-32).
__host__ __device__ inline double u01_w32(uint32_t w) {
    return (double)w * (1.0 / 4294967296.0);
}

// 24-bit uniform float in [0,1).
__host__ __device__ inline float u01_f32(uint32_t a) {
    return (float)(a >> 8) * (1.0f / 16777216.0f);
}

// Stream tags (counter word w) so that different consumers of one key never
// share a counter.
enum : uint32_t {
    TAG_RESET = 0x52000000u,    // env reset uniforms, block index in low bits
    TAG_ACTION = 0x41000000u,   // synthetic random policy
    TAG_NORMAL = 0x4E000000u,   // Gaussian policy noise
    TAG_PERM = 0x50000000u      // minibatch permutation keys
};

// The network's tanh (every kernel that applies it calls tanh_fast / tanh4,
// so all paths agree bitwise).  DR_TANH_RAT 1 (default since round 3): the
// rational form below, measured faster (linear_tanh 34.6 vs 37.9 us, the
// head kernel 58.0 vs 61.5 us, PPO 5.84-5.85 vs 5.76-5.77 updates/s, same
// box, scripts/micro/round3_y.sh); 0: the two-form evaluation (<= 2 ulp).
#ifndef DR_TANH_RAT
#define DR_TANH_RAT 1
#endif
// Rational f32 tanh: x P(x^2) / Q(x^2) on x clamped to +-7.905 (odd degree-13
// / even degree-6 minimax set, as in Eigen's generic_fast_tanh_float), one
// hardware rcp; <= 6 ulp from the correctly rounded tanh (4.6 ulp with an
// exact quotient, scripts/micro/tanh_rat.py), half the VALU of the two-form
// evaluation.  The clamp is NaN-propagating (IEEE maximum / minimum), so NaN
// stays NaN; +-inf -> +-tanh(7.905) (1 - 3 ulp).
__device__ inline float tanh_rat(float x) {
    const float c = 7.90531110763549805f;
    const float xc = __builtin_elementwise_minimum(__builtin_elementwise_maximum(x, -c), c);
    const float s = xc * xc;
    float p = fmaf(s, -2.76076847742355e-16f, 2.00018790482477e-13f);
    p = fmaf(s, p, -8.60467152213735e-11f);
    p = fmaf(s, p, 5.12229709037114e-08f);
    p = fmaf(s, p, 1.48572235717979e-05f);
    p = fmaf(s, p, 6.37261928875436e-04f);
    p = fmaf(s, p, 4.89352455891786e-03f);
    float q = fmaf(s, 1.19825839466702e-06f, 1.18534705686654e-04f);
    q = fmaf(s, q, 2.26843463243900e-03f);
    q = fmaf(s, q, 4.89352518554385e-03f);
    return (xc * p) * __builtin_amdgcn_rcpf(q);
}

// tanh_rat on a pair, written on 2-wide vectors so that the polynomials and
// products issue as packed f32 (v_pk_fma_f32 / v_pk_mul_f32); per component
// bitwise tanh_rat.
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ inline f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) {
    return __builtin_elementwise_fma(a, b, c);
}
__device__ inline f32x2 tanh_rat2(f32x2 x) {
    const f32x2 c = {7.90531110763549805f, 7.90531110763549805f};
    const f32x2 xc = __builtin_elementwise_minimum(__builtin_elementwise_maximum(x, -c), c);
    const f32x2 s = xc * xc;
    auto k = [](float v) { return f32x2{v, v}; };
    f32x2 p = pk_fma(s, k(-2.76076847742355e-16f), k(2.00018790482477e-13f));
    p = pk_fma(s, p, k(-8.60467152213735e-11f));
    p = pk_fma(s, p, k(5.12229709037114e-08f));
    p = pk_fma(s, p, k(1.48572235717979e-05f));
    p = pk_fma(s, p, k(6.37261928875436e-04f));
    p = pk_fma(s, p, k(4.89352455891786e-03f));
    f32x2 q = pk_fma(s, k(1.19825839466702e-06f), k(1.18534705686654e-04f));
    q = pk_fma(s, q, k(2.26843463243900e-03f));
    q = pk_fma(s, q, k(4.89352518554385e-03f));
    const f32x2 r = {__builtin_amdgcn_rcpf(q.x), __builtin_amdgcn_rcpf(q.y)};
    return (xc * p) * r;
}

// tanh_fast with DR_TANH_RAT 0: a branch-free f32 tanh (<= 2 ulp): odd Taylor polynomial through x^15 for
// |x| < 0.55 (truncation < 0.5 ulp there), 1 - 2 / (e^{2|x|} + 1) above
// (hardware exp2 / rcp, the cancellation costs <= 2 ulp at the switch),
// sign restored; NaN propagates, +-inf -> +-1.  The device library's tanhf
// branches per element, which costs ~3x the instructions in a wave.
__device__ inline float tanh_fast(float x) {
#if DR_TANH_RAT
    return tanh_rat(x);
#else
    const float ax = fabsf(x);
    const float z = ax * ax;
    float p = fmaf(z, -929569.0f / 638512875.0f, 21844.0f / 6081075.0f);
    p = fmaf(z, p, -1382.0f / 155925.0f);
    p = fmaf(z, p, 62.0f / 2835.0f);
    p = fmaf(z, p, -17.0f / 315.0f);
    p = fmaf(z, p, 2.0f / 15.0f);
    p = fmaf(z, p, -1.0f / 3.0f);
    const float small = fmaf(ax * z, p, ax);
    const float e = __builtin_amdgcn_exp2f(ax * 2.8853900817779268f);  // e^{2|x|}
    const float large = fmaf(-2.0f, __builtin_amdgcn_rcpf(e + 1.0f), 1.0f);
    return copysignf(ax < 0.55f ? small : large, x);
#endif
}

// Compute units of the current device, looked up once per device index (a
// process may drive handles on several GPUs).
inline int device_cu_count() {
    static int cache[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    if (cache[dev] == 0) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            n < 1)
            n = 256;
        cache[dev] = n;
    }
    return cache[dev];
}

constexpr int kBlock = 256;   // 4 waves of 64

inline unsigned grid_for(int64_t n, int per_block = kBlock) {
    return (unsigned)((n + per_block - 1) / per_block);
}

}  // namespace dr
