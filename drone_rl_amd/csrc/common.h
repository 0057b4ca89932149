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

// Branch-free f32 tanh (<= 2 ulp): odd Taylor polynomial through x^15 for
// |x| < 0.55 (truncation < 0.5 ulp there), 1 - 2 / (e^{2|x|} + 1) above
// (hardware exp2 / rcp, the cancellation costs <= 2 ulp at the switch),
// sign restored; NaN propagates, +-inf -> +-1.  The device library's tanhf
// branches per element, which costs ~3x the instructions in a wave.
__device__ inline float tanh_fast(float x) {
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
}

constexpr int kBlock = 256;   // 4 waves of 64

inline unsigned grid_for(int64_t n, int per_block = kBlock) {
    return (unsigned)((n + per_block - 1) / per_block);
}

}  // namespace dr
