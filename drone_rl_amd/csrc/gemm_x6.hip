// fp32-accurate GEMM on the bf16 matrix cores for the PPO MLP's 256 x 256
// layer (MI355X, gfx950).
//
// gfx950 has no xf32 MFMA and its f32-input MFMA runs at 1/16 of the bf16
// rate, so the hipBLASLt fp32 GEMMs of the 256 x 256 layer cap at 157 TF/s.
// These kernels keep fp32 accuracy on the bf16 MFMA instead:
//
//   * every fp32 operand x is split EXACTLY into three bf16 planes,
//     x = h + m + l (8 + 8 + 8 significant bits, RNE at each level: x - h
//     and (x - h) - m are exact in fp32, and the last remainder fits a bf16);
//   * a product a*b is formed from the six plane products whose weight is
//     >= 2^-16 of the leading one (h*h, h*m, m*h, h*l, l*h, m*m), each exact
//     in the MFMA; the three dropped ones (m*l, l*m, l*l) are <= 2^-23 of
//     |a*b| together -- below one fp32 rounding of the product;
//   * h*h accumulates in its own fp32 accumulator and the five small
//     products in a second one, added once at the end, so the small terms'
//     roundings are 2^-8 smaller than the leading chain's.
//
// Measured against an f64 GEMM on the same inputs this is slightly MORE
// accurate than the f32 MFMA chain (tests/test_gemm_x6_gpu.py), at 6 bf16
// MFMAs per product: 2.67x the f32 MFMA rate in peak terms.
//
// Every kernel runs on v_mfma_f32_16x16x32_bf16 (round 6).  The chip holds
// its clock down under these MFMA-dense loops (DVFS give-back), and at equal
// cycles per FLOP the 16x16x32 shape holds a higher clock than 32x32x16
// (MI355X_MICROARCH.md, DVFS give-back item 7); same-box A/B against the
// round-5 32x32x16 kernels (profiles/r06_x6_shape_ab*.json): forward 82-84
// vs 85-86 us, the fused input gradient 113 vs 120 us, PPO 7.64-7.65 vs
// 7.41-7.43 updates/s.
//
// Shape: C[b] = A[b] . B[b]^T, b < batch (the pi and vf MLPs), A (m, 256) f32
// row-major, B given as a pre-split image (dr_gemm_x6_split_weights: the
// layer weight W for the forward z = h W^T, or W^T for grad_h = grad_z W),
// C (m, 256) f32: gemm_x6_ws16_kernel, weight-stationary (the weights in
// registers, A streamed once); the weight gradient dW = G^T H by
// gemm_x6_wgrad16_kernel (split-K over row chunks); the input gradient with
// the first layer's backward in its epilogue by gemm_x6_fl16_kernel.
//
// Reference: the MLP layers of SB3's ActorCriticPolicy (MlpExtractor,
// net_arch [256, 256], /root/reference/train.py:36-43) -- torch fp32 Linear.

#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "x6_split.h"

#pragma clang fp contract(off)
// glds16_s clobbers m0 (reserved: the compiler sets it before each own use)
#pragma clang diagnostic ignored "-Winline-asm"

namespace dr {
namespace {

#define X6_S2(x) #x
#define X6_S(x) X6_S2(x)
constexpr int XWAVES = 8;               // waves of the weight-gradient kernel
constexpr int XTHREADS = 64 * XWAVES;

// the weight image (wimg_off, x6_split.h), one thread per (b, n, 8-k chunk)
__global__ __launch_bounds__(256) void split_weights_kernel(const float *__restrict__ w,
                                                            int transpose, int batch,
                                                            uint8_t *__restrict__ img) {
    split_weights_item(w, transpose, batch, img, blockIdx.x * 256 + threadIdx.x, blockIdx.y);
}

// global_load_lds_dwordx4 by inline asm (the saddr form: a wave-uniform
// 64-bit base in SGPRs and a 32-bit per-lane byte offset, so a loop of these
// keeps one offset VGPR): lane l's 16 bytes land at LDS byte lds_base + 16 l.
// Issued by hand because hipcc's waitcnt pass drains every pending LDS DMA
// (vmcnt(0)) before any ds_read it cannot prove disjoint from it; the waits
// are counted by hand.
__device__ inline void glds16_s(const void *sbase, uint32_t voff, uint32_t lds_base) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
                 ::"v"(voff), "s"(sbase), "s"(lds_base)
                 : "memory", "m0");
}
__device__ inline uint32_t lds_addr(const uint8_t *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t *)p;
}

// ---------------------------------------------------------------------------
// dr_gemm_x6: weight-stationary.  A 256-thread block (one wave per SIMD, 512
// registers) holds its net's three weight planes in registers for the whole
// launch -- wave w the 64 output columns 64 w .. + 63 as 4 column tiles of
// 16 x 8 k32 steps x 3 planes of MFMA B fragments = 384 registers, the h and
// m planes in AGPRs (read there by inline-asm MFMAs: hipcc's MFMA builtin
// copies AGPR operands back to VGPRs before every use), the l plane in VGPRs
// -- and streams only the activations: per 32-row step each wave moves its 8
// rows of f32 by LDS-DMA into a private staging slot (no other wave reads
// them, so no barrier orders them), splits them into the block's
// double-buffered plane image and runs 384 MFMAs on the block's 32 rows; one
// barrier per row step publishes the planes.
//
// LDS: planes 2 x 48 KB (32 rows x 256 k x 3 planes, stored chunk-major:
// the 16-B chunk c (8 k) of row r at c * 512 + 16 r, so a fragment read's
// 16-lane group (16 consecutive rows of one chunk) is 256 contiguous bytes,
// and every address is a per-lane base plus an immediate; the split writes'
// 16-lane groups (8 rows of two adjacent chunks) are conflict-free because
// the odd chunk's lanes write the other 8-B half of their slots) + f32
// staging 2 x 32 KB (wave w's 8 KB: piece i holds split chunks 4 i .. + 3 of
// its 8 rows, slot 32 h + 8 c' + r = row r, chunk 4 i + c', float4 h) =
// 160 KB.
constexpr int WS_RS = X6_RS;                         // rows per row step
constexpr int WS_PLANE = WS_RS * XK * 2;             // 16 KB: one plane of a row step
constexpr int WS_PSTAGE = 3 * WS_PLANE;              // 48 KB
constexpr int WS_FSLOT = WS_RS * XK * 4;             // 32 KB: f32 rows of a row step
constexpr int WS_LDS_F = 2 * WS_PSTAGE;              // staging after the two plane stages
constexpr int WS_LDS = 2 * WS_PSTAGE + 2 * WS_FSLOT; // 160 KB
constexpr int WS_THREADS = 256;
// fragment sets in flight (read two k32 steps ahead)
constexpr int WS_NF = 3;
// The 16-row A fragments of v_mfma_f32_16x16x32_bf16 let a phase be a ROW
// tile: phase t runs rows 16 t .. + 15 of the row step against all four of
// the wave's 16-column tiles, so each activation fragment is read from LDS
// once per row step (48 ds_read_b128; the round-5 32x32x16 kernel re-read
// them per column tile, 96).  The weights come in the image order of
// wimg_off: wave w's column tile ct, k32 step s.  Per SIMD and row step:
// 384 MFMAs of 16 cycles (6,144 pipe cycles, 3,072 of issue), 48 fragment
// reads, 32 stores, 8 DMA pieces.  Accumulators D[m][n] of a 16 x 16 tile:
// column n = lane & 15, row m = 4 (lane >> 4) + r, r = 0..3.
typedef float f32x4_t __attribute__((ext_vector_type(4)));

__device__ inline void mfma16_a(f32x4_t &d, const bf16x8_t &x, const bf16x8_t &w) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(d) : "v"(x), "a"(w));
}
__device__ inline void mfma16_v(f32x4_t &d, const bf16x8_t &x, const bf16x8_t &w) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(d) : "v"(x), "v"(w));
}
__device__ inline void mfma16_first(f32x4_t &d, const bf16x8_t &x, const bf16x8_t &w) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=&v"(d) : "v"(x), "a"(w));
}

// The split of one staged half-unit (a, b, c, d -> the h, m, l planes of the
// pairs (a, b), (c, d)) as 12 pieces of at most two VALU instructions, each
// issued as its own asm statement right behind one of a k32 step's MFMAs, so
// that it runs in that MFMA's issue shadow (an MFMA holds the SIMD's vector
// issue for 8 of its 16 cycles; two 4-cycle VALU fit the rest,
// MI355X_MICROARCH.md cycle constants) instead of as one block between MFMA
// groups.  Bitwise the C++ split (pk_bf16 = v_cvt_pk_bf16_f32, lo_f / hi_f
// = shift / mask, plain f32 subtractions).  Round 6, with the memory
// instructions likewise spread one per MFMA slot: forward 85.7 -> 81.7 us,
// the fused kernel 113.7-116.4 -> 103.8-107.8 us (alternating A/Bs, the
// same output bytes).
struct SplitHU {
    float a, b, c, d;
    uint32_t h0, h1, m0, m1, l0, l1;
};
__device__ inline void sp_cvt(uint32_t &o, float i0, float i1) {
    asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(o) : "v"(i0), "v"(i1));
}
__device__ inline void sp_cvt2(uint32_t &o0, uint32_t &o1, float i0, float i1, float i2,
                               float i3) {
    asm volatile("v_cvt_pk_bf16_f32 %0, %2, %3\n\tv_cvt_pk_bf16_f32 %1, %4, %5"
                 : "=&v"(o0), "=v"(o1)
                 : "v"(i0), "v"(i1), "v"(i2), "v"(i3));
}
__device__ inline void sp_sublo(float &r, uint32_t h) {     // r -= lo_f(h)
    uint32_t t;
    asm volatile("v_lshlrev_b32 %1, 16, %2\n\tv_sub_f32 %0, %0, %1"
                 : "+v"(r), "=&v"(t)
                 : "v"(h));
}
__device__ inline void sp_subhi(float &r, uint32_t h) {     // r -= hi_f(h)
    uint32_t t;
    asm volatile("v_and_b32 %1, 0xffff0000, %2\n\tv_sub_f32 %0, %0, %1"
                 : "+v"(r), "=&v"(t)
                 : "v"(h));
}
__device__ inline void split_piece(SplitHU &u, int i) {
    switch (i) {
    case 0: sp_cvt(u.h0, u.a, u.b); break;
    case 1: sp_cvt(u.h1, u.c, u.d); break;
    case 2: sp_sublo(u.a, u.h0); break;
    case 3: sp_subhi(u.b, u.h0); break;
    case 4: sp_sublo(u.c, u.h1); break;
    case 5: sp_subhi(u.d, u.h1); break;
    case 6: sp_cvt2(u.m0, u.m1, u.a, u.b, u.c, u.d); break;
    case 7: sp_sublo(u.a, u.m0); break;
    case 8: sp_subhi(u.b, u.m0); break;
    case 9: sp_sublo(u.c, u.m1); break;
    case 10: sp_subhi(u.d, u.m1); break;
    case 11: sp_cvt2(u.l0, u.l1, u.a, u.b, u.c, u.d); break;
    default: break;
    }
}

__global__ __launch_bounds__(WS_THREADS, 1) void gemm_x6_ws16_kernel(
    const float *__restrict__ A, const uint8_t *__restrict__ img, float *__restrict__ C,
    int64_t m, int batch) {
    __shared__ __attribute__((aligned(16))) uint8_t sh[WS_LDS];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int b = (int)blockIdx.x % batch;
    const int per = (int)gridDim.x / batch;
    const int j0 = (int)blockIdx.x / batch;
    const int steps_net = (int)(m / WS_RS);
    const int R = (steps_net - j0 + per - 1) / per;
    const float *Ab = A + (int64_t)b * m * XK;
    float *Cb = C + (int64_t)b * m * XN;
    const int fc = lane & 15, fq = lane >> 4;

    // the weights: wave w's 4 column tiles x 8 k32 steps x 3 planes as B
    // fragments (lane: column 64 w + 16 ct + fc, k 32 s + 8 fq .. + 7); h, m
    // planes in AGPRs (read there by the asm MFMAs), l in VGPRs
    bf16x8_t Wa[4][8][2], Wv[4][8];
    {
        const uint8_t *ib = img + (int64_t)b * W_IMG + lane * 16;
#pragma unroll
        for (int ct = 0; ct < 4; ++ct)
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                const uint8_t *src = ib + ((w * 4 + ct) * 8 + s) * 3 * W_FRAG;
                Wa[ct][s][0] = *reinterpret_cast<const bf16x8_t *>(src);
                Wa[ct][s][1] = *reinterpret_cast<const bf16x8_t *>(src + W_FRAG);
                Wv[ct][s] = *reinterpret_cast<const bf16x8_t *>(src + 2 * W_FRAG);
            }
    }

    // staging: wave w's 8 rows of row step k in its 8 KB of slot k & 1.  Piece
    // i: lane L = 32 h + 8 c' + r loads float4 h of split chunk 4 i + c' of
    // row r (each row contributes 128 contiguous bytes per piece).  Odd
    // chunks are staged with their two float4 halves swapped, so that the
    // lanes splitting an odd chunk process its halves in the opposite order
    // to their even-chunk neighbours (the conflict-free split writes)
    const int sr = lane & 7, sc = (lane >> 3) & 3, shf = lane >> 5;
    const uint32_t voff_f = (uint32_t)(sr * 1024 + 32 * sc + 16 * (shf ^ (sc & 1)));
    auto issue_rows = [&](int k) {
        const float *r0 = Ab + ((int64_t)(j0 + k * per) * WS_RS + 8 * w) * XK;
        uint8_t *dst = sh + WS_LDS_F + (k & 1) * WS_FSLOT + w * 8 * 1024;
#pragma unroll
        for (int i = 0; i < 8; ++i) glds16_s(r0 + 32 * i, voff_f, lds_addr(dst + i * 1024));
    };
    const int rd_base = WS_LDS_F + w * 8 * 1024 + (lane >> 5) * 1024 + (lane & 31) * 16;
    auto split_read = [&](int k, int u, int hf, float4 &v) {
        v = *reinterpret_cast<const float4 *>(sh + rd_base + (k & 1) * WS_FSLOT + u * 2048 +
                                              hf * 512);
    };
    const int wr_base = (lane >> 3) * 512 + (8 * w + sr) * 16;
    const int wr_odd = (lane >> 3) & 1;
    const int wr_half[2] = {wr_base + 8 * wr_odd, wr_base + 8 * (wr_odd ^ 1)};
    auto split_store = [&](int k, int u, int hf, uint32_t h0, uint32_t h1, uint32_t m0,
                           uint32_t m1, uint32_t l0, uint32_t l1) {
        uint8_t *dst = sh + (k & 1) * WS_PSTAGE + wr_half[hf] + u * 8 * 512;
        typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
        *reinterpret_cast<u32x2_t *>(dst) = (u32x2_t){h0, h1};
        *reinterpret_cast<u32x2_t *>(dst + WS_PLANE) = (u32x2_t){m0, m1};
        *reinterpret_cast<u32x2_t *>(dst + 2 * WS_PLANE) = (u32x2_t){l0, l1};
    };
    auto split_rw = [&](int k, int u, int hf) {
        float4 v;
        split_read(k, u, hf, v);
        const uint32_t h0 = pk_bf16(v.x, v.y);
        float ra = v.x - lo_f(h0), rb = v.y - hi_f(h0);
        const uint32_t m0 = pk_bf16(ra, rb);
        const uint32_t l0 = pk_bf16(ra - lo_f(m0), rb - hi_f(m0));
        const uint32_t h1 = pk_bf16(v.z, v.w);
        ra = v.z - lo_f(h1), rb = v.w - hi_f(h1);
        const uint32_t m1 = pk_bf16(ra, rb);
        const uint32_t l1 = pk_bf16(ra - lo_f(m1), rb - hi_f(m1));
        split_store(k, u, hf, h0, h1, m0, m1, l0, l1);
    };
    // activation fragments of global k32 step g of a row step (row tile
    // g >> 3, k32 step g & 7; MFMA A operand): row 16 (g >> 3) + fc, k
    // 32 (g & 7) + 8 fq .. + 7 = chunk 4 (g & 7) + fq.  A 16-lane group
    // reads 16 consecutive rows of one chunk: 256 contiguous bytes
    typedef bf16x8_t AFrag[3];
    const int fr_base = fq * 512 + fc * 16;
    auto read_frag = [&](int k, int g, AFrag &f) {
        const uint8_t *src = sh + (k & 1) * WS_PSTAGE + fr_base + (g >> 3) * 256 + (g & 7) * 2048;
#pragma unroll
        for (int p = 0; p < 3; ++p) f[p] = *reinterpret_cast<const bf16x8_t *>(src + p * WS_PLANE);
    };
    auto read_frag_plane = [&](int k, int g, AFrag &f, int p) {
        const uint8_t *src = sh + (k & 1) * WS_PSTAGE + fr_base + (g >> 3) * 256 + (g & 7) * 2048;
        f[p] = *reinterpret_cast<const bf16x8_t *>(src + p * WS_PLANE);
    };
    // accumulators [row tile][column tile]: hi (h.h) and lo (the five small
    // products)
    f32x4_t acc_h[2][4], acc_l[2][4];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) acc_h[t][ct] = acc_l[t][ct] = (f32x4_t){};
    // output i = 4 ct + r of row tile t: row 16 t + 4 fq + r, column
    // 64 w + 16 ct + fc (four 64-B row segments per store)
    const int st_off = (4 * fq * XN + fc) * 4;
    auto store_one = [&](int k, int t, int i) {
        const int ct = i >> 2, r = i & 3;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            Cb + (int64_t)(j0 + k * per) * WS_RS * XN, 0, k < 0 ? 0 : WS_RS * XN * 4,
            0x00020000);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc_h[t][ct][r]), rs, st_off,
                                              ((16 * t + r) * XN + 64 * w + 16 * ct) * 4, 0);
    };
    // the accumulators are operands of the wait-state pad, so the compiler
    // cannot hoist the adds above it (next to the MFMAs that write them)
    auto finish_tile = [&](int t) {
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7"
                     : "+v"(acc_h[t][0]), "+v"(acc_h[t][1]), "+v"(acc_h[t][2]),
                       "+v"(acc_h[t][3]), "+v"(acc_l[t][0]), "+v"(acc_l[t][1]),
                       "+v"(acc_l[t][2]), "+v"(acc_l[t][3])::"memory");
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) acc_h[t][ct] = acc_h[t][ct] + acc_l[t][ct];
    };
    // the six products of row tile t, k32 step s, for the four column tiles
    // (h += xh.wh; l += xh.wm, xm.wh, xh.wl, xl.wh, xm.wm: per output the
    // order of every x6 kernel), interleaved over the column tiles
    // extra(i) runs behind MFMA i of the 24 (the split pieces, the step's
    // fragment reads and stores)
    auto mfma_group = [&](bool first, int t, int s, const AFrag &x, auto &&extra) {
        auto piece = [&](int i) { extra(i); };
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) {
            if (first) mfma16_first(acc_h[t][ct], x[0], Wa[ct][s][0]);
            else mfma16_a(acc_h[t][ct], x[0], Wa[ct][s][0]);
            piece(ct);
        }
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) {
            if (first) mfma16_first(acc_l[t][ct], x[0], Wa[ct][s][1]);
            else mfma16_a(acc_l[t][ct], x[0], Wa[ct][s][1]);
            piece(4 + ct);
        }
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) {
            mfma16_a(acc_l[t][ct], x[1], Wa[ct][s][0]);
            piece(8 + ct);
        }
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) {
            mfma16_v(acc_l[t][ct], x[0], Wv[ct][s]);
            piece(12 + ct);
        }
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) {
            mfma16_a(acc_l[t][ct], x[2], Wa[ct][s][0]);
            piece(16 + ct);
        }
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) {
            mfma16_a(acc_l[t][ct], x[1], Wa[ct][s][1]);
            piece(20 + ct);
        }
    };

    if (R > 0) issue_rows(0);
    if (R > 1) issue_rows(1);
    __builtin_amdgcn_sched_barrier(0);
    if (R > 1)
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");     // weights + rows of step 0
    else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int q = 0; q < 8; ++q) split_rw(0, q >> 1, q & 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");       // staging slot 0 read
    issue_rows(R > 2 ? 2 : R - 1);                           // clamped: never split
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");         // step 1's staging
    asm volatile("s_barrier" ::: "memory");                  // planes of step 0
    AFrag fb[WS_NF];
    read_frag(0, 0, fb[0]);
    read_frag(0, 1, fb[1]);
    // Row step k, per wave: phase t = row tile t's 8 k32 steps (4 column
    // tiles x 6 products = 24 MFMAs each) with the other row tile's 16
    // output stores beside them (t = 0: row tile 1 of step k - 1); fragments
    // two k32 steps ahead; split half-unit q = 4 t + (s >> 1) of row step
    // k + 1 read at even s, split and written at odd s, and behind each
    // unit's second half the DMA of its two staging pieces for step k + 3;
    // then lgkmcnt(0) + barrier.  No data-dependent branch (round 4: 99-100
    // vs 105-106 us with branches around the first and last steps' work):
    // row step 0's phase-0 stores go through a 0-byte buffer range, the last
    // steps split their successor's clamped staging into the unused plane
    // buffer.  Branches would also risk the compiler copying an accumulator
    // between asm MFMA groups, a VALU read inside an MFMA's wait states
    // (tests/test_x6_asm_hazards.py).
    // unit u's staging pieces, consumed by the split of half-units 2 u and
    // 2 u + 1, refilled with step k + 3 (clamped: such rows are never split)
    auto dma_piece = [&](int k, int u, int i) {
        const int k3 = k + 3 >= R ? R - 1 : k + 3;
        const float *r0 = Ab + ((int64_t)(j0 + k3 * per) * WS_RS + 8 * w) * XK;
        uint8_t *dst = sh + WS_LDS_F + ((k + 3) & 1) * WS_FSLOT + w * 8 * 1024;
        glds16_s(r0 + 32 * (2 * u + i), voff_f, lds_addr(dst + (2 * u + i) * 1024));
    };
    auto split_store_plane = [&](int k, int u, int hf, int p, const SplitHU &x) {
        uint8_t *dst = sh + (k & 1) * WS_PSTAGE + wr_half[hf] + u * 8 * 512 + p * WS_PLANE;
        typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
        const uint32_t lo = p == 0 ? x.h0 : p == 1 ? x.m0 : x.l0;
        const uint32_t hi = p == 0 ? x.h1 : p == 1 ? x.m1 : x.l1;
        *reinterpret_cast<u32x2_t *>(dst) = (u32x2_t){lo, hi};
    };
    float4 v;
    SplitHU pu{};           // the previous odd step's planes (pq >= 0)
    int pq = -1;
    auto row_step = [&](int k) {
        // the staging of step k + 1 (issued in step k - 2): every vector
        // memory op of step k - 1 (32 stores + 8 DMA pieces) is younger;
        // for k = 0 the prologue waited
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        pq = -1;            // (a compile-time value at every use below)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int ko = t == 1 ? k : k - 1;
            finish_tile(1 - t);
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                const int g = 8 * t + s;
                constexpr int D = WS_NF - 1;
                const int q = 4 * t + (s >> 1);
                SplitHU u{v.x, v.y, v.z, v.w, 0u, 0u, 0u, 0u, 0u, 0u};
                // behind the odd MFMAs the split pieces (odd s) or the
                // previous odd step's plane stores and staging DMA (even
                // s), behind the even ones one memory instruction each, all
                // pinned by scheduling barriers: the three fragment reads
                // of k32 step g + D, the two output stores, the staging read
                auto extra = [&](int i) {
                    if ((s & 1) && (i & 1)) split_piece(u, i >> 1);
                    if (!(s & 1) && (i & 1) && pq >= 0 && (i >> 1) < 5) {
                        const int j = i >> 1;
                        __builtin_amdgcn_sched_barrier(0);
                        if (j < 3) split_store_plane(k + 1, pq >> 1, pq & 1, j, pu);
                        else if (pq & 1) dma_piece(k, pq >> 1, j - 3);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                    if (!(i & 1)) {
                        const int j = i >> 1;
                        __builtin_amdgcn_sched_barrier(0);
                        if (j < 3 && g + D < 16) read_frag_plane(k, g + D, fb[(g + D) % WS_NF], j);
                        if (j == 3) store_one(ko, 1 - t, 2 * s);
                        if (j == 4) store_one(ko, 1 - t, 2 * s + 1);
                        if (j == 5 && (s & 1) == 0) split_read(k + 1, q >> 1, q & 1, v);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                };
                mfma_group(s == 0, t, s, fb[g % WS_NF], extra);
                if ((s & 1) == 0) {
                    pq = -1;                    // stored in this step's slots
                } else if (t == 1 && s == 7) {
                    // the row step's last split: its planes before the barrier
                    split_store(k + 1, q >> 1, q & 1, u.h0, u.h1, u.m0, u.m1, u.l0, u.l1);
                    dma_piece(k, q >> 1, 0);
                    dma_piece(k, q >> 1, 1);
                } else {
                    pu = u;                     // stored in the next step's slots
                    pq = q;
                }
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        read_frag(k + 1, 0, fb[0]);          // after the last step: unused
        read_frag(k + 1, 1, fb[1]);
    };
    for (int k = 0; k < R; ++k) row_step(k);
    if (R > 0) {
        finish_tile(1);
#pragma unroll
        for (int i = 0; i < 16; ++i) store_one(R - 1, 1, i);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// Weight gradient of the same layer, dW[b] = G[b]^T H[b] (G = grad_z, H = the
// layer input, both (m, 256) f32 row-major), split over C row chunks: block
// (b, n-half, chunk) writes the 128 x 256 partial ws[b][chunk][n][k] of its
// (m / C)-row chunk; the chunk sum is left to the caller (the trainer's
// deferred finish sums C = 64 chunks in a fixed order).  8 waves as 2 (n) x
// 4 (k) of 64 x 64 outputs, the same split hi/lo accumulation as the forward.
//
// Both operands are reduced over rows, so an MFMA fragment holds ROWS of one
// column.  Each 32-row stage is split ONCE: every thread loads 6 float4 of
// the stage (2 of G's 32 x 128 half, 4 of H's 32 x 256) into registers one
// stage ahead, splits them and writes the three bf16 planes ROW-major into
// LDS; the fragments come back column-major through gfx950's transposing
// read ds_read_b64_tr_b16 (two per fragment).
constexpr int TW_BM = 32;                          // rows per stage
constexpr int TW_PLANE_ROW = (128 + 256) * 2;      // 768 B: one plane of one row

typedef short i16x4_t __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// gemm_x6_wgrad16_kernel: a stage's 32 rows are ONE k32 step: each wave's
// 64 x 64 outputs are 4 x 4 tiles of 16 x 16 (the same 128 accumulator
// registers), 96 MFMAs of 16 cycles per stage (the same 1,536 pipe cycles).
// Fragments come from the same row-major plane image through two
// transposed reads each; K (the rows) is permuted so the two reads of a
// 32-lane half cover 8 distinct rows: A/B lane L = i + 16 g holds column i
// of rows 4 g + e (e < 4) and 16 + 4 g + e - 4 (e >= 4) -- the same
// permutation in both operands, so the products are the same.  The row
// stride is 2,336 B (== 32 mod 256): rows 0..7 of a half fall in distinct
// 8-bank groups, conflict-free.  Per wave and stage: 24 split elements (~130
// VALU), 18 ds_write_b64, 48 transposed reads, 96 MFMAs, one barrier.  The
// round-5 32x32x16 form ran 116.7 us vs 114.2 for this one at 65,536 rows,
// 64 chunks (scripts/micro/gemm_x6_bench.py, one box).
constexpr int TW16_ROW = 3 * TW_PLANE_ROW + 32;    // 2,336 B
constexpr int TW16_STAGE = TW_BM * TW16_ROW;       // 74,752 B
constexpr int TW16_LDS = 2 * TW16_STAGE;           // 149,504 B

__device__ inline bf16x8_t tr16_frag(const uint8_t *p) {
    typedef __attribute__((address_space(3))) i16x4_t lds_i16x4;
    const i16x4_t a = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_i16x4 *)(uintptr_t)lds_addr(p));
    const i16x4_t c = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_i16x4 *)(uintptr_t)lds_addr(p + 16 * TW16_ROW));
    return __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(a, c, 0, 1, 2, 3, 4, 5, 6, 7));
}

__global__ __launch_bounds__(XTHREADS) void gemm_x6_wgrad16_kernel(
    const float *__restrict__ Gm, const float *__restrict__ Hm, float *__restrict__ ws,
    int64_t m, int chunks) {
    __shared__ __attribute__((aligned(16))) uint8_t sh[TW16_LDS];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wn = wid >> 2, wk = wid & 3;
    const int chunk = (int)(blockIdx.x % chunks);
    const int nh = (int)((blockIdx.x / chunks) & 1);
    const int b = (int)(blockIdx.x / chunks / 2);
    const int64_t rows = m / chunks;
    const int G_ = (int)(rows / TW_BM);
    const float *Gb = Gm + ((int64_t)b * m + (int64_t)chunk * rows) * 256 + nh * 128;
    const float *Hb = Hm + ((int64_t)b * m + (int64_t)chunk * rows) * 256;

    int ld_src[6], ld_dst[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const int q = tid + 512 * (i < 2 ? i : i - 2);
        const int r = i < 2 ? q >> 5 : q >> 6;
        const int c = i < 2 ? (q & 31) * 4 : (q & 63) * 4;
        ld_src[i] = r * 256 + c;
        ld_dst[i] = r * TW16_ROW + (i < 2 ? c : 128 + c) * 2;
    }
    f32x4_t ld[6];
    auto load = [&](int g) {
        const int64_t r0 = (int64_t)g * TW_BM * 256;
#pragma unroll
        for (int i = 0; i < 6; ++i)
            ld[i] = *reinterpret_cast<const f32x4_t *>((i < 2 ? Gb : Hb) + r0 + ld_src[i]);
    };
    auto split_store = [&](int buf) {
        uint8_t *S = sh + buf * TW16_STAGE;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const f32x4_t x = ld[i];
            uint32_t h[2], mm[2], l[2];
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const float a = x[2 * q], c = x[2 * q + 1];
                const uint32_t ph = pk_bf16(a, c);
                const float ra = a - lo_f(ph), rc = c - hi_f(ph);
                const uint32_t pm = pk_bf16(ra, rc);
                h[q] = ph;
                mm[q] = pm;
                l[q] = pk_bf16(ra - lo_f(pm), rc - hi_f(pm));
            }
            uint8_t *d = S + ld_dst[i];
            *reinterpret_cast<uint2 *>(d) = make_uint2(h[0], h[1]);
            *reinterpret_cast<uint2 *>(d + TW_PLANE_ROW) = make_uint2(mm[0], mm[1]);
            *reinterpret_cast<uint2 *>(d + 2 * TW_PLANE_ROW) = make_uint2(l[0], l[1]);
        }
    };
    // transposed-read lane address (T10): lane 4 q + p of 16-lane group g
    // supplies row 4 g + q, columns 4 p .. 4 p + 3 of the tile's 16 columns
    const int li = lane & 15, gq = lane >> 4;
    const int fbase = (4 * gq + (li >> 2)) * TW16_ROW + 8 * (li & 3);
    const int gcol = (wn * 64) * 2, hcol = (128 + wk * 64) * 2;

    f32x4_t acc_h[4][4], acc_l[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc_h[i][j] = acc_l[i][j] = (f32x4_t){};

    // the stage's fragments: G tile i (columns wn 64 + 16 i ..), H tile j
    auto read_g = [&](int g, int i, bf16x8_t (&f)[3]) {
        const uint8_t *S = sh + (g & 1) * TW16_STAGE + fbase + gcol + 32 * i;
#pragma unroll
        for (int p = 0; p < 3; ++p) f[p] = tr16_frag(S + p * TW_PLANE_ROW);
    };
    auto read_h = [&](int g, int j, bf16x8_t (&f)[3]) {
        const uint8_t *S = sh + (g & 1) * TW16_STAGE + fbase + hcol + 32 * j;
#pragma unroll
        for (int p = 0; p < 3; ++p) f[p] = tr16_frag(S + p * TW_PLANE_ROW);
    };
    auto mfma6 = [&](int i, int j, const bf16x8_t (&a)[3], const bf16x8_t (&c)[3]) {
        acc_h[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], c[0], acc_h[i][j], 0, 0, 0);
        f32x4_t t = acc_l[i][j];
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], c[1], t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], c[0], t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], c[2], t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], c[0], t, 0, 0, 0);
        t = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], c[1], t, 0, 0, 0);
        acc_l[i][j] = t;
    };

    load(0);
    split_store(0);
    load(G_ > 1 ? 1 : 0);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    // Stage g, per wave: the G fragments of its 4 tiles, then per H tile
    // j its fragments and the 4 x 6 MFMAs of column j (the next tile's
    // reads behind them), the split of stage g + 1 after the second H tile,
    // lgkmcnt(0) + barrier at the end, the loads of stage g + 2 behind the
    // split.  The last iteration re-splits the last stage (no branch).
    bf16x8_t fg[4][3], fh[2][3];
    for (int g = 0; g < G_; ++g) {
#pragma unroll
        for (int i = 0; i < 4; ++i) read_g(g, i, fg[i]);
        read_h(g, 0, fh[0]);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (j + 1 < 4) read_h(g, j + 1, fh[(j + 1) & 1]);
#pragma unroll
            for (int i = 0; i < 4; ++i) mfma6(i, j, fg[i], fh[j & 1]);
            if (j == 1) {
                split_store((g + 1) & 1);
                load(g + 2 < G_ ? g + 2 : G_ - 1);
            }
        }
        // the scheduler's MFMA / LDS-read interleave (iglp_opt(0)): 100-103
        // vs 105-107 us per call, bitwise the same partials (alternating
        // A/B, scripts/micro/r6_sessions.sh m, r6_sessions.sh n; a hand-written
        // sched_group_barrier pipeline and the two waves of a SIMD splitting
        // at different points of the stage measured equal or slower)
        __builtin_amdgcn_iglp_opt(0);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    // D[n][k] of tile (i, j): column k = 16 j + (lane & 15), row n =
    // 16 i + 4 (lane >> 4) + r
    const int fc = lane & 15, fq = lane >> 4;
    float *out = ws + ((int64_t)b * chunks + chunk) * 256 * 256 + (int64_t)(nh * 128) * 256;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const f32x4_t v = acc_h[i][j] + acc_l[i][j];
            float *c = out + (int64_t)(wn * 64 + 16 * i + 4 * fq) * 256 + wk * 64 + 16 * j + fc;
#pragma unroll
            for (int r = 0; r < 4; ++r) c[r * 256] = v[r];
        }
}

// ---------------------------------------------------------------------------
// dr_gemm_x6_bwd_first (round 5): the 256 x 256 layer's input gradient with
// the first layer's backward fused into its epilogue.  The unfused step wrote
// grad_h1 = grad_z2 W1 (134 MB for both nets at 65,536 rows) and
// first_layer_bwd_kernel read it back with h1 (268 MB) to form
// grad_z1 = grad_h1 (1 - h1^2), the 256 x 15 weight gradient grad_z1^T x and
// the bias gradient.  Here each output tile's grad_h1 stays in registers:
// the epilogue loads h1 (the only extra traffic, 134 MB), forms grad_z1,
// splits it exactly into three bf16 planes (the x6 scheme) and accumulates
// D2 = X^T grad_z1 on the matrix cores, X the minibatch observations with a
// constant 1 as a 16th feature (so D2's feature-15 row is the bias gradient).
// A block writes its D2 once, as one partial row of first_layer_bwd_kernel's
// partial layout, and the step's existing level-1 / level-2 sums finish it.
//
// D2 orientation: the MFMA's A operand is X^T (M = feature, K = rows), its B
// operand is grad_z1 (K = rows, N = columns).  The main GEMM's accumulator
// layout gives lane (fr, fh) column fr and rows 8 (r >> 2) + 4 fh + (r & 3),
// r = 0..15: registers 8 j .. 8 j + 7 are exactly the B fragment of K step j
// (K index 8 fh + e <-> row 16 j + 4 fh + (e & 3) + 8 (e >> 2)), so grad_z1
// needs no data movement.  The two column tiles of a wave share one
// 32 x 32 accumulator: tile 0's features in D2 rows 0..15, tile 1's in rows
// 16..31 (each tile's A fragment is zero in the other half), 16 registers for
// the wave's 64 columns x 16 features.
//
// Registers: the weights' h and m planes stay in AGPRs as in
// gemm_x6_ws16_kernel, but the l plane is streamed from L2 (two 1-KB
// fragments per k32 step, six fragments ahead: every vector-memory wait is
// in issue order, so a fragment load queued behind the h1 / staging loads
// from HBM waits for them too -- round 5: 2 ahead 127 us per call, 6 ahead
// 118) to make room for the epilogue, and the activation rows are
// register-staged by compiler-tracked loads four split half-units ahead
// (no LDS-DMA staging: every vector memory op is visible to the compiler's
// waitcnt pass).  LDS holds only the double-buffered planes.
// the X planes image (xrec_off, x6_split.h)
__global__ __launch_bounds__(256) void split_x_kernel(const float *__restrict__ x, int64_t m,
                                                      int k, uint8_t *__restrict__ img) {
    split_x_item(x, nullptr, m, k, img, (int64_t)blockIdx.x * 256 + threadIdx.x);
}

// ---------------------------------------------------------------------------
// gemm_x6_fl16_kernel: phase t of a row step runs the wave's column
// tiles 2 t, 2 t + 1 (16 columns each) for both 16-row tiles -- per k32
// step 2 row tiles x 2 column tiles x 6 products = 24 MFMAs, the same 192
// per phase and 6,144 pipe cycles per row step as the forward -- and
// the epilogue of the other phase's four tiles.  The l plane of the weights
// is streamed from L2 as before (two 1-KB fragments per k32 step).
//
// D2 = X^T grad_z1 runs on the same shape with K = the row step's 32 rows:
// the B fragment of column tile ct is registers 0..3 of row tile 0's
// accumulator and 0..3 of row tile 1's (K index 8 q + e <-> row 4 q + e and
// 16 + 4 q + e - 4, q = lane >> 4), the A fragment is the record of
// x6_split.h (split_x_item), so no lane ever holds a zero half: 12 MFMAs of
// 16 cycles per phase (the round-5 32x32x16 kernel: 12 of 32, half of each
// A fragment zero).
__global__ __launch_bounds__(WS_THREADS, 1) void gemm_x6_fl16_kernel(
    const float *__restrict__ A, const uint8_t *__restrict__ img, const float *__restrict__ H,
    const uint8_t *__restrict__ ximg, float *__restrict__ part, int64_t m, int batch) {
    __shared__ __attribute__((aligned(16))) uint8_t sh[2 * WS_PSTAGE];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int b = (int)blockIdx.x % batch;
    const int per = (int)gridDim.x / batch;
    const int j0 = (int)blockIdx.x / batch;
    const int steps_net = (int)(m / WS_RS);
    const int R = (steps_net - j0 + per - 1) / per;
    const float *Ab = A + (int64_t)b * m * XK;
    const float *Hb = H + (int64_t)b * m * XN;
    const int fc = lane & 15, fq = lane >> 4;

    constexpr int kBufFlags = 0x00020000;
    const __amdgpu_buffer_rsrc_t wrs =
        __builtin_amdgcn_make_buffer_rsrc((void *)(img + (int64_t)b * W_IMG), 0, (int)W_IMG,
                                          kBufFlags);
    const int lane16 = lane * 16;
    auto wfrag = [&](int ct, int s, int p) {
        return __builtin_bit_cast(
            bf16x8_t, __builtin_amdgcn_raw_buffer_load_b128(
                          wrs, lane16, (((w * 4 + ct) * 8 + s) * 3 + p) * W_FRAG, 0));
    };
    // the weights' h and m planes in AGPRs (wimg_off's order)
    bf16x8_t Wa[4][8][2];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int s = 0; s < 8; ++s) {
            Wa[ct][s][0] = wfrag(ct, s, 0);
            Wa[ct][s][1] = wfrag(ct, s, 1);
        }
    // the l plane: fragment u of a row step (k32 step g = u >> 1 of the row
    // step's 16, g = 8 t + s, column tile 2 t + (u & 1)), loaded WLA ahead
    auto wl_load = [&](int u) {
        const int g = (u >> 1) & 15;
        return wfrag(2 * (g >> 3) + (u & 1), g & 7, 2);
    };
    constexpr int WLA = 6, WLR = 8;
    bf16x8_t wl[WLR];
#pragma unroll
    for (int u = 0; u < WLA; ++u) wl[u] = wl_load(u);

    // activation staging: lane L splits row L & 7 of the wave's 8 rows,
    // chunk 8 u + (L >> 3), half hf ^ (chunk & 1) (the conflict-free split
    // writes of gemm_x6_ws16_kernel), as a float4 register loaded four split
    // half-units ahead; half-unit q = 2 u + hf of row step k (clamped to the
    // last step: such rows are split into the unused plane buffer, never read)
    const int sr = lane & 7, sch = lane >> 3, sodd = sch & 1;
    const int soff[2] = {sr * 1024 + 32 * sch + 16 * sodd, sr * 1024 + 32 * sch + 16 * (sodd ^ 1)};
    auto stage_load = [&](int k, int q) {
        const int kk = k < R ? k : R - 1;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(Ab + ((int64_t)(j0 + kk * per) * WS_RS + 8 * w) * XK), 0, 8 * XK * 4,
            kBufFlags);
        return __builtin_bit_cast(
            float4, __builtin_amdgcn_raw_buffer_load_b128(rs, soff[q & 1], 256 * (q >> 1), 0));
    };
    const int wr_base = sch * 512 + (8 * w + sr) * 16;
    const int wr_half[2] = {wr_base + 8 * sodd, wr_base + 8 * (sodd ^ 1)};
    auto split_store = [&](int k, int q, const float4 &v) {
        uint32_t h[2], mm[2], l[2];
        const float x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const float a = x[2 * p], c = x[2 * p + 1];
            const uint32_t ph = pk_bf16(a, c);
            const float ra = a - lo_f(ph), rc = c - hi_f(ph);
            const uint32_t pm = pk_bf16(ra, rc);
            h[p] = ph;
            mm[p] = pm;
            l[p] = pk_bf16(ra - lo_f(pm), rc - hi_f(pm));
        }
        uint8_t *dst = sh + (k & 1) * WS_PSTAGE + wr_half[q & 1] + (q >> 1) * 8 * 512;
        typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
        *reinterpret_cast<u32x2_t *>(dst) = (u32x2_t){h[0], h[1]};
        *reinterpret_cast<u32x2_t *>(dst + WS_PLANE) = (u32x2_t){mm[0], mm[1]};
        *reinterpret_cast<u32x2_t *>(dst + 2 * WS_PLANE) = (u32x2_t){l[0], l[1]};
    };
    // A fragments of k32 step s for both row tiles (gemm_x6_ws16_kernel's
    // addressing): row 16 rt + fc, chunk 4 s + fq
    typedef bf16x8_t AFrag[2][3];
    const int fr_base = fq * 512 + fc * 16;
    auto read_frag = [&](int k, int s, AFrag &f) {
        const uint8_t *src = sh + (k & 1) * WS_PSTAGE + fr_base + s * 2048;
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int p = 0; p < 3; ++p)
                f[rt][p] = *reinterpret_cast<const bf16x8_t *>(src + rt * 256 + p * WS_PLANE);
    };
    auto read_frag_one = [&](int k, int s, AFrag &f, int rt, int p) {
        const uint8_t *src = sh + (k & 1) * WS_PSTAGE + fr_base + s * 2048;
        f[rt][p] = *reinterpret_cast<const bf16x8_t *>(src + rt * 256 + p * WS_PLANE);
    };
    auto split_store_u = [&](int k, int q, const SplitHU &u) {
        uint8_t *dst = sh + (k & 1) * WS_PSTAGE + wr_half[q & 1] + (q >> 1) * 8 * 512;
        typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
        *reinterpret_cast<u32x2_t *>(dst) = (u32x2_t){u.h0, u.h1};
        *reinterpret_cast<u32x2_t *>(dst + WS_PLANE) = (u32x2_t){u.m0, u.m1};
        *reinterpret_cast<u32x2_t *>(dst + 2 * WS_PLANE) = (u32x2_t){u.l0, u.l1};
    };
    // accumulators [phase][row tile][column tile of the phase]
    f32x4_t acc_h[2][2][2], acc_l[2][2][2];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc_h[t][rt][j] = acc_l[t][rt][j] = (f32x4_t){};
    auto finish_tiles = [&](int t) {
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7"
                     : "+v"(acc_h[t][0][0]), "+v"(acc_h[t][0][1]), "+v"(acc_h[t][1][0]),
                       "+v"(acc_h[t][1][1]), "+v"(acc_l[t][0][0]), "+v"(acc_l[t][0][1]),
                       "+v"(acc_l[t][1][0]), "+v"(acc_l[t][1][1])::"memory");
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc_h[t][rt][j] = acc_h[t][rt][j] + acc_l[t][rt][j];
    };
    // the six products of k32 step s for phase t's 2 x 2 tiles, interleaved
    // over the tiles (per output gemm_x6_ws16_kernel's order)
    // extra(i) runs behind MFMA i of the 24 (split pieces, memory ops)
    auto mfma_group = [&](bool first, int t, int s, const AFrag &x, const bf16x8_t &wl0,
                          const bf16x8_t &wl1, auto &&extra) {
        int i = 0;
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                if (first) mfma16_first(acc_h[t][rt][j], x[rt][0], Wa[2 * t + j][s][0]);
                else mfma16_a(acc_h[t][rt][j], x[rt][0], Wa[2 * t + j][s][0]);
                extra(i++);
            }
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                if (first) mfma16_first(acc_l[t][rt][j], x[rt][0], Wa[2 * t + j][s][1]);
                else mfma16_a(acc_l[t][rt][j], x[rt][0], Wa[2 * t + j][s][1]);
                extra(i++);
            }
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                mfma16_a(acc_l[t][rt][j], x[rt][1], Wa[2 * t + j][s][0]);
                extra(i++);
            }
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                mfma16_v(acc_l[t][rt][j], x[rt][0], j ? wl1 : wl0);
                extra(i++);
            }
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                mfma16_a(acc_l[t][rt][j], x[rt][2], Wa[2 * t + j][s][0]);
                extra(i++);
            }
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                mfma16_a(acc_l[t][rt][j], x[rt][1], Wa[2 * t + j][s][1]);
                extra(i++);
            }
    };

    // ---- the epilogue: grad_z1 of phase tt's tiles of row step kk into D2
    f32x4_t d2[4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) d2[ct] = (f32x4_t){};
    // h1 of (row tile rt, column tile j of phase tt, register r): row
    // 16 rt + 4 fq + r, column 64 w + 16 (2 tt + j) + fc
    float hb[2][2][4];
    const int hoff = (4 * fq * XN + 64 * w + fc) * 4;
    auto h_load = [&](int kk, int tt, int i) {
        const int rt = i >> 3, j = (i >> 2) & 1, r = i & 3;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(Hb + (int64_t)(j0 + kk * per) * WS_RS * XN), 0, WS_RS * XN * 4, kBufFlags);
        hb[rt][j][r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
            rs, hoff, ((16 * rt + r) * XN + 16 * (2 * tt + j)) * 4, 0));
    };
    const int xoff = xrec_off(0, lane);
    auto x_frag = [&](int kk, bf16x8_t (&xf)[3]) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(ximg + (int64_t)(j0 + kk * per) * XREC), 0, XREC, kBufFlags);
#pragma unroll
        for (int p = 0; p < 3; ++p)
            xf[p] = __builtin_bit_cast(bf16x8_t, __builtin_amdgcn_raw_buffer_load_b128(
                                                     rs, xoff, p * 1024, 0));
    };
    // the six D2 products of phase tt's column tile j: one asm statement,
    // so D2 stays in VGPRs (the builtin's accumulator took AGPRs, evicting a
    // weight fragment with a copy back before each use, round 5) and no
    // compiler VALU lands between the MFMAs; s_nop 4 covers the VALU writes
    // of bh, bm, bl -> SrcB reads
    auto d2_mfma = [&](int tt, int j, const bf16x8_t (&xf)[3], const bf16x8_t &bh,
                       const bf16x8_t &bm, const bf16x8_t &bl) {
        f32x4_t &d = d2[2 * tt + j];
        asm volatile("s_nop 4\n\t"
                     "v_mfma_f32_16x16x32_bf16 %0, %1, %4, %0\n\t"
                     "v_mfma_f32_16x16x32_bf16 %0, %1, %5, %0\n\t"
                     "v_mfma_f32_16x16x32_bf16 %0, %2, %4, %0\n\t"
                     "v_mfma_f32_16x16x32_bf16 %0, %1, %6, %0\n\t"
                     "v_mfma_f32_16x16x32_bf16 %0, %3, %4, %0\n\t"
                     "v_mfma_f32_16x16x32_bf16 %0, %2, %5, %0"
                     : "+v"(d)
                     : "v"(xf[0]), "v"(xf[1]), "v"(xf[2]), "v"(bh), "v"(bm), "v"(bl));
    };
    // grad_z1 = grad_h1 (1 - h1^2) of phase tt's column tile j (both row
    // tiles: the B fragment's 8 K values), split, and the six products.
    // (Round 6: the same VALU as asm pieces spread over the MFMA slots of
    // k32 steps 4 / 6 measured 128-131 vs 106-108 us per call; not taken.)
    auto d2_tile = [&](int tt, int j, const bf16x8_t (&xf)[3]) {
        float gz[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const float y = hb[e >> 2][j][e & 3];
            gz[e] = acc_h[tt][e >> 2][j][e & 3] * (1.0f - y * y);
        }
        u32x4_t gh, gm, gl;
        split8(gz, gh, gm, gl);
        d2_mfma(tt, j, xf, __builtin_bit_cast(bf16x8_t, gh), __builtin_bit_cast(bf16x8_t, gm),
                __builtin_bit_cast(bf16x8_t, gl));
    };
    // ---- prologue: step 0's planes, the staging ring for step 1 ----
    {
        float4 v0[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v0[q] = stage_load(0, q);
#pragma unroll
        for (int q = 0; q < 8; ++q) split_store(0, q, v0[q]);
    }
    float4 stg[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) stg[q] = stage_load(1, q);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    AFrag fb[2];
    read_frag(0, 0, fb[0]);
    bf16x8_t xf[3];

    // Row step k, per wave: phase t = column tiles 2 t, 2 t + 1 over the 8
    // k32 steps (24 MFMAs each) and the epilogue of phase tt = 1 - t's
    // tiles (row step k - 1 in phase 0, k in phase 1): h1 loads at k32
    // steps 0..3 (four each), the X fragment at 1, D2 of tile 0 at 5 and of
    // tile 1 at 7; A fragments one k32 step ahead; split half-unit q = 4 t +
    // (s >> 1) of step k + 1 at odd s, with the staging load of q + 4 behind
    // it.  Step 0's phase-0 epilogue is of the zeroed phase-1 tiles: D2 += 0.
    auto row_step = [&](int k) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int tt = 1 - t;
            const int kk = t == 0 ? (k > 0 ? k - 1 : 0) : k;
            finish_tiles(tt);
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                const int g = 8 * t + s;
                const int q = 4 * t + (s >> 1);
                // the step's memory instructions, one per MFMA slot (pinned
                // between scheduling barriers): 6 A-fragment reads of k32
                // step g + 1, 2 l-plane loads, 4 h1 loads (s < 4), the X
                // fragment's 3 loads (s = 2; D2 at s = 5, 7), the staging
                // load behind odd steps' split
                auto mem_op = [&](int op) {
                    if (op < 6) {
                        if (g + 1 < 16) read_frag_one(k, (g + 1) & 7, fb[(g + 1) & 1], op / 3, op % 3);
                    } else if (op < 8) {
                        const int u = 2 * g + (op - 6) + WLA;
                        wl[u % WLR] = wl_load(u);
                    } else if (op < 12) {
                        if (s < 4) h_load(kk, tt, 4 * s + (op - 8));
                    } else if (op == 12 && (s & 1)) {
                        stg[q & 3] = stage_load(q + 4 < 8 ? k + 1 : k + 2, (q + 4) & 7);
                    } else if (op >= 12 && op < 15 && s == 2) {
                        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                            (void *)(ximg + (int64_t)(j0 + kk * per) * XREC), 0, XREC,
                            kBufFlags);
                        xf[op - 12] = __builtin_bit_cast(
                            bf16x8_t,
                            __builtin_amdgcn_raw_buffer_load_b128(rs, xoff, (op - 12) * 1024, 0));
                    }
                };
                SplitHU u{stg[q & 3].x, stg[q & 3].y, stg[q & 3].z, stg[q & 3].w,
                          0u, 0u, 0u, 0u, 0u, 0u};
                auto extra = [&](int i) {
                    if ((s & 1) && (i & 1)) split_piece(u, i >> 1);
                    int op = -1;
                    if (!(i & 1)) op = i >> 1;
                    else if (!(s & 1)) op = 12 + (i >> 1);
                    else if (i == 23) op = 12;
                    if (op >= 0) {
                        __builtin_amdgcn_sched_barrier(0);
                        mem_op(op);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                };
                mfma_group(s == 0, t, s, fb[g & 1], wl[(2 * g) % WLR], wl[(2 * g + 1) % WLR],
                           extra);
                if (s == 5) d2_tile(tt, 0, xf);
                if (s == 7) d2_tile(tt, 1, xf);
                if (s & 1) split_store_u(k + 1, q, u);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        read_frag(k + 1, 0, fb[0]);
    };
    for (int k = 0; k < R; ++k) row_step(k);
    // phase 1's tiles of the last row step
    if (R > 0) {
        finish_tiles(1);
#pragma unroll
        for (int i = 0; i < 16; ++i) h_load(R - 1, 1, i);
        x_frag(R - 1, xf);
        d2_tile(1, 0, xf);
        d2_tile(1, 1, xf);
    }
    // D2 -> this block's partial row (first_layer_bwd_kernel's layout:
    // [feature * 256 + column], row j0 * batch + b): tile ct, lane (fc, fq),
    // register r = feature 4 fq + r, column 64 w + 16 ct + fc
    float *out = part + ((int64_t)j0 * batch + b) * (FL_F * XN);
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7"
                 : "+v"(d2[0]), "+v"(d2[1]), "+v"(d2[2]), "+v"(d2[3])::"memory");
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int r = 0; r < 4; ++r) out[(4 * fq + r) * XN + 64 * w + 16 * ct + fc] = d2[ct][r];
}

int fail_g(int code, const std::string &msg) {
    set_global_error(msg);
    return code;
}

}  // namespace

// Launchers of the fused input-gradient + first-layer backward (the C ABI
// entry dr_gemm_x6_bwd_first in ppo_kernels.hip adds the level-1 partial sum
// in the first-layer workspace layout).
size_t gemm_x6_x_bytes(int64_t m) { return m < WS_RS ? 0 : (size_t)(m / WS_RS) * XREC; }

int gemm_x6_split_x_launch(int64_t m, int k, const float *x, void *ximg, hipStream_t st) {
    const int64_t threads = (m / WS_RS) * 64;
    hipLaunchKernelGGL(split_x_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st,
                       x, m, k, static_cast<uint8_t *>(ximg));
    return hipGetLastError() == hipSuccess ? DR_OK : DR_ERR_HIP;
}

// returns the blocks per net (the partial rows written), or -1
// blocks per net of gemm_x6_fl16_kernel at m rows (its partial rows)
int gemm_x6_fl_rows(int batch, int64_t m) {
    const int n_cu = device_cu_count();
    const int units = (int)(batch * (m / WS_RS));
    int grid = units < n_cu ? units : n_cu;
    grid -= grid % batch;
    return grid / batch;
}

int gemm_x6_fl_launch(int batch, int64_t m, const float *gz, const void *img, const float *h,
                      const void *ximg, float *part, hipStream_t st) {
    const int grid = gemm_x6_fl_rows(batch, m) * batch;
    hipLaunchKernelGGL(gemm_x6_fl16_kernel, dim3(grid), dim3(WS_THREADS), 0, st, gz,
                       static_cast<const uint8_t *>(img), h, static_cast<const uint8_t *>(ximg),
                       part, m, batch);
    return hipGetLastError() == hipSuccess ? grid / batch : -1;
}

}  // namespace dr

using namespace dr;

extern "C" {

size_t dr_gemm_x6_weights_bytes(int64_t batch) {
    return batch < 1 ? 0 : (size_t)(batch * W_IMG);
}

int dr_gemm_x6_split_weights(int64_t batch, const float *w, int transpose, void *img,
                             void *stream) {
    if (batch < 1 || batch > 2 || !w || !img || transpose < 0 || transpose > 2 ||
        (((uintptr_t)img) & 15))
        return fail_g(DR_ERR_INVALID, "dr_gemm_x6_split_weights: bad arguments");
    const int threads = (int)batch * XN * (XK / 8);
    // transpose 2: both images in one launch (W^T form at img, W form after it)
    hipLaunchKernelGGL(split_weights_kernel, dim3((threads + 255) / 256, transpose == 2 ? 2 : 1),
                       dim3(256), 0, static_cast<hipStream_t>(stream), w, transpose, (int)batch,
                       static_cast<uint8_t *>(img));
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? DR_OK
                           : fail_g(DR_ERR_HIP, std::string("split_weights_kernel: ") +
                                                    hipGetErrorString(e));
}

int dr_gemm_x6(int64_t batch, int64_t m, const float *a, const void *img, float *c,
               void *stream) {
    if (batch < 1 || batch > 2 || m < 128 || m % 128 || m > (int64_t(1) << 26) || !a ||
        !img || !c || (((uintptr_t)a) & 15) || (((uintptr_t)img) & 15) ||
        (((uintptr_t)c) & 15))
        return fail_g(DR_ERR_INVALID,
                      "dr_gemm_x6: bad arguments (m must be a positive multiple of 128, "
                      "pointers 16-byte aligned)");
    // one 160-KB block per CU, the same number of blocks per net
    const int n_cu = device_cu_count();
    const int units = (int)(batch * (m / WS_RS));
    int grid = units < n_cu ? units : n_cu;
    grid -= grid % (int)batch;
    // plain stores: the next kernel reads C back from the Infinity Cache
    // (round 5: the streamed-l-plane form of the fused kernel without its
    // epilogue, 112-113 vs 103-109 us for this kernel, bitwise the same C)
    hipLaunchKernelGGL(gemm_x6_ws16_kernel, dim3(grid),
                       dim3(WS_THREADS), 0,
                       static_cast<hipStream_t>(stream), a, static_cast<const uint8_t *>(img), c,
                       m, (int)batch);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess
               ? DR_OK
               : fail_g(DR_ERR_HIP, std::string("dr_gemm_x6: ") + hipGetErrorString(e));
}

int dr_gemm_x6_wgrad(int64_t batch, int64_t m, int64_t chunks, const float *g, const float *h,
                     float *ws, void *stream) {
    if (batch < 1 || batch > 2 || chunks < 1 || m < 1 || m % chunks ||
        (m / chunks) % TW_BM || m > (int64_t(1) << 26) || !g || !h ||
        !ws || (((uintptr_t)g) & 15) || (((uintptr_t)h) & 15) || (((uintptr_t)ws) & 15))
        return fail_g(DR_ERR_INVALID,
                      "dr_gemm_x6_wgrad: bad arguments (m / chunks a positive multiple of 32; "
                      "pointers 16-byte aligned)");
    hipLaunchKernelGGL(gemm_x6_wgrad16_kernel, dim3((unsigned)(batch * 2 * chunks)),
                       dim3(XTHREADS), 0, static_cast<hipStream_t>(stream), g, h, ws, m,
                       (int)chunks);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? DR_OK
                           : fail_g(DR_ERR_HIP, std::string("gemm_x6_wgrad16_kernel: ") +
                                                    hipGetErrorString(e));
}

}  // extern "C"
