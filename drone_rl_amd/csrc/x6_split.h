// Exact three-plane bf16 split of f32 values for the bf16 matrix cores (the
// x6 GEMM scheme of gemm_x6.hip: x = h + m + l, each plane RNE of the
// remainder, x - h and (x - h) - m exact in f32, the last remainder a bf16),
// used by the weight-image split, the weight-gradient GEMM's operands and the
// fused first-layer backward's grad_z1 / observation planes (all in
// gemm_x6.hip).
#pragma once

#include <cstdint>

namespace dr {

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

__device__ inline uint32_t pk_bf16(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){a, b}, bf16x2_t));
}
__device__ inline float lo_f(uint32_t p) { return __uint_as_float(p << 16); }
__device__ inline float hi_f(uint32_t p) { return __uint_as_float(p & 0xffff0000u); }

// x[0..7] = h + m + l exactly, packed as 8 bf16 per plane (element j in
// bits 16j of the 128-bit value).
__device__ inline void split8(const float x[8], u32x4_t &h, u32x4_t &m, u32x4_t &l) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float a = x[2 * q], b = x[2 * q + 1];
        const uint32_t ph = pk_bf16(a, b);
        const float ra = a - lo_f(ph), rb = b - hi_f(ph);
        const uint32_t pm = pk_bf16(ra, rb);
        const float sa = ra - lo_f(pm), sb = rb - hi_f(pm);
        h[q] = ph;
        m[q] = pm;
        l[q] = pk_bf16(sa, sb);
    }
}

}  // namespace dr
