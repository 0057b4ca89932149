// Exact three-plane bf16 split of f32 values for the bf16 matrix cores (the
// x6 GEMM scheme of gemm_x6.hip: x = h + m + l, each plane RNE of the
// remainder, x - h and (x - h) - m exact in f32, the last remainder a bf16),
// used by the weight-image split, the weight-gradient GEMM's operands and the
// fused first-layer backward's grad_z1 / observation planes (gemm_x6.hip),
// and the operand images below (also built by ppo_kernels.hip).
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

// ---------------------------------------------------------------------------
// Operand images of the x6 GEMMs (gemm_x6.hip), built by split_weights_kernel
// / split_x_kernel and by the first-layer forward's auxiliary blocks
// (ppo_kernels.hip linear_tanh_kernel<K, true>): the same items, so every
// producer writes the same bytes.
constexpr int XK = 256;                 // reduction length (hidden width)
constexpr int XN = 256;                 // output columns
constexpr int X6_RS = 32;               // rows per row step of the GEMM kernels
constexpr int64_t W_IMG = (int64_t)3 * XN * XK * 2;   // 384 KB per net: 3 bf16 planes
constexpr int64_t W_FRAG = 64 * 16;     // one plane fragment: 1 KB

// Weight image of `batch` nets in the weight-stationary kernel's register
// order: img[b][w][ct][s][p][lane][16 B] is the v_mfma_f32_16x16x32_bf16 B
// fragment of plane p of Bt (= W for transpose 0, W^T for transpose 1; W
// (256, 256) row-major per net) for wave w's column tile ct and k32 step s:
// lane = c + 16 q holds Bt[n = 64 w + 16 ct + c][k = 32 s + 8 q .. + 7], so
// each fragment is one coalesced 1-KB load.
__host__ __device__ inline int64_t wimg_off(int n, int k0) {
    const int w = n >> 6, ct = (n >> 4) & 3, c = n & 15, s = k0 >> 5, q = (k0 >> 3) & 3;
    return ((int64_t)((w * 4 + ct) * 8 + s) * 3 * 64 + c + 16 * q) * 16;
}

// Item t (b, n, 8-k chunk) of the weight image; transpose 2 builds both forms
// (y 0: the W^T form at img, y 1: the W form after it).
__device__ inline void split_weights_item(const float *__restrict__ w, int transpose, int batch,
                                          uint8_t *__restrict__ img, int t, int y) {
    if (t >= batch * XN * (XK / 8)) return;
    if (transpose == 2) {
        transpose = y;
        img += (int64_t)y * batch * W_IMG;
    }
    const int c = t & 31, n = (t >> 5) & (XN - 1), b = t >> 13;
    const float *wb = w + (int64_t)b * XN * XK;
    const int k0 = c * 8;
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
        x[j] = transpose ? wb[(int64_t)(k0 + j) * XN + n] : wb[(int64_t)n * XK + k0 + j];
    u32x4_t h, m, l;
    split8(x, h, m, l);
    uint8_t *base = img + (int64_t)b * W_IMG + wimg_off(n, k0);
    *reinterpret_cast<u32x4_t *>(base) = h;
    *reinterpret_cast<u32x4_t *>(base + W_FRAG) = m;
    *reinterpret_cast<u32x4_t *>(base + 2 * W_FRAG) = l;
}

// The first-layer observation image of the fused input-gradient GEMM
// (gemm_x6_fl_kernel): per row step a record of X^T's A fragments.
constexpr int FL_F = 16;                                // 15 features + the bias column
// One v_mfma_f32_16x16x32_bf16 A fragment
// per plane and row step, K = the step's 32 rows: lane L = f + 16 q holds
// feature f of rows 4 q + e (e < 4, row tile 0) and 16 + 4 q + e - 4 (e >= 4,
// row tile 1) -- the rows the main GEMM's 16 x 16 accumulators of the two
// row tiles hold in lane (column, q), registers e & 3.
constexpr int XREC = 3 * 64 * 16;                       // 3,072 B per row step
__host__ __device__ inline int xrec_off(int p, int lane) { return (p * 64 + lane) * 16; }

__device__ inline void split_x_item(const float *__restrict__ x, const int32_t *__restrict__ rows,
                                    int64_t m, int k, uint8_t *__restrict__ img, int64_t t) {
    const int64_t g = t >> 6;
    if (g >= m / X6_RS) return;
    const int L = (int)(t & 63), f = L & 15, q = L >> 4;
    uint8_t *rec = img + g * XREC;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int64_t row = g * X6_RS + (e < 4 ? 4 * q + e : 16 + 4 * q + (e - 4));
        const int64_t src = rows ? (int64_t)rows[row] : row;
        v[e] = f < k ? x[src * k + f] : (f == FL_F - 1 ? 1.0f : 0.0f);
    }
    u32x4_t h, mm, l;
    split8(v, h, mm, l);
    *reinterpret_cast<u32x4_t *>(rec + xrec_off(0, L)) = h;
    *reinterpret_cast<u32x4_t *>(rec + xrec_off(1, L)) = mm;
    *reinterpret_cast<u32x4_t *>(rec + xrec_off(2, L)) = l;
}

}  // namespace dr
