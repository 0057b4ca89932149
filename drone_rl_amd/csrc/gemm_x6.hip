// fp32-accurate GEMM on the bf16 matrix cores for the PPO MLP's 256 x 256
// layer (MI355X, gfx950).
//
// gfx950 has no xf32 MFMA and its f32-input MFMA runs at 1/16 of the bf16
// rate, so the hipBLASLt fp32 GEMMs of the 256 x 256 layer cap at 157 TF/s.
// This kernel keeps fp32 accuracy on the bf16 MFMA instead:
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
// Shape: C[b] = A[b] . B[b]^T, b < batch (the pi and vf MLPs), A (m, 256) f32
// row-major, B given as a pre-split image (dr_gemm_x6_split_weights: the
// layer weight W for the forward z = h W^T, or W^T for grad_h = grad_z W),
// C (m, 256) f32.  One 512-thread block owns 128 full rows (all 256
// columns), so A is read from HBM exactly once; the weight image (384 KB per
// net) streams from L2.
//
// Pipeline per 32-deep k stage (two LDS stages of 72 KB): the weight image
// arrives by global_load_lds (the global image is stored in the LDS layout,
// 1 KB per wave-instruction, lane-linear), A is loaded as f32 into
// registers, split by VALU and written to LDS as three bf16 planes while the
// waves run the previous stage's MFMAs.  8 waves as 2 (rows) x 4 (columns),
// each owning a 64 x 64 output tile = 2 x 2 v_mfma_f32_32x32x16_bf16 tiles.
//
// LDS image of a plane: rows of 32 k (64 B = four 16-B chunks), chunk c of
// row r stored at chunk c ^ ((r >> 2) & 3): the 16 lanes of every
// ds_read_b128 lane group then hit 16 distinct 16-B bank slots.
//
// Reference: the MLP layers of SB3's ActorCriticPolicy (MlpExtractor,
// net_arch [256, 256], /root/reference/train.py:36-43) -- torch fp32 Linear.

#include <cstdlib>
#include <type_traits>

#include "common.h"

#pragma clang fp contract(off)
// glds16 clobbers m0 (reserved: the compiler sets it before each own use)
#pragma clang diagnostic ignored "-Winline-asm"

namespace dr {
namespace {

// DR_X6_ABL (diagnostic builds only, scripts/micro/gemm_x6_ablate.sh; results
// are wrong by construction): 1 = no split (raw f32 bits as bf16), 2 = no
// fragment reads in the k loop, 3 = no global_load_lds in the k loop.
#ifndef DR_X6_ABL
#define DR_X6_ABL 0
#endif
// DR_X6_STAMPS (diagnostic builds only): s_memtime at four points of every
// stage for the waves of blocks 0-7, read back by dr_x6_diag_stamps
// (scripts/micro/gemm_x6_stamps.py); no output depends on a stamp.
#ifndef DR_X6_STAMPS
#define DR_X6_STAMPS 0
#endif
// 1: the f32 A fragments of a k16 step are split into bf16 planes as soon as
// they are read (during the previous step's MFMAs), not at the step's start
#ifndef DR_X6_EARLY
#define DR_X6_EARLY 0
#endif
// 1 (A/B knob): one accumulator per tile; each k16 step's five small
// products go into a zero-started temporary that is added to it (64 fewer
// accumulator registers, 16 f32 adds per tile and step)
#ifndef DR_X6_ACC1
#define DR_X6_ACC1 0
#endif
// 1 (A/B knob): the next stages' global_load_lds are issued after the
// step-1 MFMAs instead of right after the barrier
#ifndef DR_X6_LATEISSUE
#define DR_X6_LATEISSUE 0
#endif
// 1 (A/B knob): waves 4-7 split their step-1 fragments before the barrier,
// so after it they start with MFMAs while waves 0-3 start with the split
// (a stagger of the SIMD partners, MI355X_MICROARCH.md two-waves item 9)
#ifndef DR_X6_STAGGER
#define DR_X6_STAGGER 0
#endif
// 1: raise the wave's issue priority around its MFMA cluster; 2: static
// s_setprio 1 for waves 4-7 (the arbitration losers) before the loop
// (A/B knob)
// DR_X6_NOCOMP (diagnostic, wrong by construction): L1 without forming A
#ifndef DR_X6_NOCOMP
#define DR_X6_NOCOMP 0
#endif
// 1: in the first-layer-fused form the SIMD partners form the next A stage on
// either side of their MFMAs (see the L1 loop); 0: both before
#ifndef DR_X6_L1_SPLIT
#define DR_X6_L1_SPLIT 1
#endif
#ifndef DR_X6_PRIO
#define DR_X6_PRIO 0
#endif
// 1 (A/B knob, the round-3 form): the next stage's step-0 fragments read only
// when that stage exists (path-dependent LDS count: lgkmcnt(0) before step 1)
#ifndef DR_X6_CONDREAD
#define DR_X6_CONDREAD 0
#endif
// 1 (A/B knob): a scheduling fence right after step 1's fragment reads
#ifndef DR_X6_F1EARLY
#define DR_X6_F1EARLY 0
#endif

constexpr int XK = 256;                 // reduction length (hidden width)
constexpr int XN = 256;                 // output columns
constexpr int XBM = 128;                // rows per block
constexpr int XBK = 32;                 // k per LDS stage
constexpr int XKC = XK / XBK;           // 8 stages
// waves per block: 8 (2 x 4 waves of 64 x 64 outputs, 2 waves per SIMD) or
// 4 (1 x 4 waves of 128 x 64 outputs, one wave per SIMD with 512 registers)
#ifndef DR_X6_WAVES
#define DR_X6_WAVES 8
#endif
#if DR_X6_WAVES == 8
#define X6_NA 2      // A-row global_load_lds per wave per stage
#define X6_NA_NST 18 // + the 16 float4 stores of a finished tile
#define X6_NST 16
#define X6_PRO 10    // prologue: younger than stage 0's loads (A1 + B1 + A2)
#elif DR_X6_WAVES == 4
#define X6_NA 4
#define X6_NA_NST 36
#define X6_NST 32
#define X6_PRO 20
#else
#error "DR_X6_WAVES must be 4 or 8"
#endif
#define X6_S2(x) #x
#define X6_S(x) X6_S2(x)
constexpr int XWAVES = DR_X6_WAVES;
constexpr int XMT = 16 / XWAVES;        // 32-row tiles per wave
constexpr int XTHREADS = 64 * XWAVES;
constexpr int B_PLANE = XN * 64;        // 16 KB: 256 rows x 32 bf16
constexpr int B_STAGE = 3 * B_PLANE;    // 48 KB
constexpr int64_t W_IMG = (int64_t)XKC * B_STAGE;  // 384 KB per net

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

__device__ inline int swz(int row, int chunk) {
    return row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4);
}

// Weight image of `batch` nets: img[b][kc][plane][n][64 B] holds
// Bt[n][kc*32 .. +32) with Bt = W (transpose 0) or W^T (transpose 1),
// W (256, 256) row-major per net.  One thread per (b, kc, n, chunk).
__global__ __launch_bounds__(256) void split_weights_kernel(const float *__restrict__ w,
                                                            int transpose, int batch,
                                                            uint8_t *__restrict__ img) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= batch * XKC * XN * 4) return;
    if (transpose == 2) {      // both images: blockIdx.y 0 -> W^T form, 1 -> W form
        transpose = (int)blockIdx.y;
        img += (int64_t)blockIdx.y * batch * W_IMG;
    }
    const int c = t & 3, n = (t >> 2) & (XN - 1), kc = (t >> 10) & (XKC - 1), b = t >> 13;
    const float *wb = w + (int64_t)b * XN * XK;
    const int k0 = kc * XBK + c * 8;
    float x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
        x[j] = transpose ? wb[(int64_t)(k0 + j) * XN + n] : wb[(int64_t)n * XK + k0 + j];
    u32x4_t h, m, l;
    split8(x, h, m, l);
    uint8_t *base = img + (int64_t)b * W_IMG + (int64_t)kc * B_STAGE + swz(n, c);
    *reinterpret_cast<u32x4_t *>(base) = h;
    *reinterpret_cast<u32x4_t *>(base + B_PLANE) = m;
    *reinterpret_cast<u32x4_t *>(base + 2 * B_PLANE) = l;
}

typedef __attribute__((address_space(3))) void lds_void;

#if DR_X6_STAMPS
constexpr int kStG = 64;   // stages recorded per wave
__device__ unsigned long long g_x6_st[8 * XWAVES * kStG * 4];
#define X6_STAMP(g, k)                                                                 \
    do {                                                                               \
        __builtin_amdgcn_sched_barrier(0);                                             \
        const unsigned long long t__ = __builtin_amdgcn_s_memtime();                   \
        if (blockIdx.x < 8 && (g) < kStG && (threadIdx.x & 63) == 0)                    \
            g_x6_st[((blockIdx.x * XWAVES + (threadIdx.x >> 6)) * kStG + (g)) * 4 + (k)] = t__; \
        __builtin_amdgcn_sched_barrier(0);                                             \
    } while (0)
#else
#define X6_STAMP(g, k) \
    do {               \
    } while (0)
#endif

// LDS: weight image stages WB[2] (48 KB each, bf16 planes), A stages A32[3]
// (16 KB each, f32 rows of 32 k: 128 B, 16-B chunk c of row r at c ^ ((r >>
// 1) & 7), conflict-free for the fragment reads).  144 KB: one block per CU.
constexpr int A32_STAGE = XBM * XBK * 4;             // 16 KB
constexpr int LDS_WB = 0;
constexpr int LDS_A32 = 2 * B_STAGE;
constexpr int LDS_TOTAL = 2 * B_STAGE + 3 * A32_STAGE;
// First-layer-fused form (L1): the A stages are computed in the kernel, two
// stages ahead into a 2-stage ring, from the tile's observation rows (16
// floats per row, the 16th zero), staged per tile by LDS-DMA into a 2-tile
// ring after it: 96 + 32 + 16 = 144 KB.
constexpr int OBS_TILE = XBM * 16 * 4;               // 8 KB
constexpr int LDS_OBS = 2 * B_STAGE + 2 * A32_STAGE;

// global_load_lds_dwordx4 by inline asm: lane l's 16 bytes land at LDS
// byte lds_base + 16 l.  Issued by hand because hipcc's waitcnt pass drains
// every pending LDS DMA (vmcnt(0)) before any ds_read it cannot prove
// disjoint from it -- once per stage here; the waits are counted by hand.
__device__ inline void glds16(const void *gptr, uint32_t lds_base) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                 ::"v"(gptr), "s"(lds_base)
                 : "memory", "m0");
}
// The same with the global address split into a wave-uniform 64-bit base
// (SGPRs) and a 32-bit per-lane byte offset (the saddr form): a loop of
// these keeps one offset VGPR instead of a 64-bit address per instruction.
__device__ inline void glds16_s(const void *sbase, uint32_t voff, uint32_t lds_base) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
                 ::"v"(voff), "s"(sbase), "s"(lds_base)
                 : "memory", "m0");
}
__device__ inline uint32_t lds_addr(const uint8_t *p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint8_t *)p;
}

__device__ inline int swz32(int row, int chunk) {
    return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}

// Persistent: block blockIdx.x owns tiles blockIdx.x, + gridDim.x, ...; its
// (tile, stage) pairs form ONE stream of stages g = 0 .. 8 * tiles - 1, so
// the loads of the next tile's first stages overlap the current tile's last
// MFMAs and its output stores (no per-tile pipeline fill / drain).  Both
// operands arrive by global_load_lds: stage g's weight image one stage ahead
// (from L2), its A rows (f32, from HBM) two stages ahead.  Each wave splits
// the f32 A fragments it reads from LDS into the three bf16 planes in
// registers, right before its MFMAs.  Waits are counted by hand (vmcnt
// retires in issue order), with a raw s_barrier per stage.
// L1 (first-layer fusion): A = tanh(obs W0^T + b0) is not read but formed
// here, with linear_tanh_kernel's exact arithmetic (acc = 0, fmaf over the 15
// inputs in order, + bias, tanh_fast), so the result is bitwise that of
// dr_linear_tanh2 followed by dr_gemm_x6; it is also written to h1 when
// non-null (the weight gradient and the first-layer backward read it).
//   l1_obs16 (m, 16) rows: the 15 observations, then 0
//   l1_w0p   (batch, 256, 16): W0 row k (15 floats), then b0[k] (restrict:
//            read-only in the kernel, so its wave-uniform loads are scalar)
//   l1_h1    (batch, m, 256) side output, nullable
template <bool L1>
__global__ __launch_bounds__(XTHREADS) void gemm_x6_kernel(
    const float *__restrict__ A, const uint8_t *__restrict__ img, float *__restrict__ C,
    int64_t m, int ntiles, int nt, const float *__restrict__ l1_obs16,
    const float *__restrict__ l1_w0p, float *__restrict__ l1_h1) {
    __shared__ __attribute__((aligned(16))) uint8_t sh[LDS_TOTAL];
    constexpr int NA = L1 ? 2 : 3;          // A-stage ring depth
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = XWAVES == 8 ? wid >> 2 : 0, wn = wid & 3;
    const int tiles_per_net = (int)(m / XBM);
    const int nmine = (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
    const int G = nmine * XKC;

    auto tile_of = [&](int g) { return (int)blockIdx.x + (g >> 3) * (int)gridDim.x; };
    auto net_of = [&](int t) { return t / tiles_per_net; };
    auto issue_b = [&](int g) {
        const uint8_t *src = img + (int64_t)net_of(tile_of(g)) * W_IMG + (g & 7) * B_STAGE;
        uint8_t *dst = sh + LDS_WB + (g & 1) * B_STAGE;
#pragma unroll
        for (int i = 0; i < B_STAGE / 1024 / XWAVES; ++i) {
            const int ins = wid + XWAVES * i;
            glds16(src + ins * 1024 + lane * 16, lds_addr(dst + ins * 1024));
        }
    };
    // A stage: 16 wave-instructions of 1 KB = 8 rows each; lane L fills LDS
    // chunk L & 7 of row 8 ins + (L >> 3), i.e. global chunk (L & 7) ^ swizzle
    const int a_row_l = lane >> 3, a_chk_l = lane & 7;
    auto issue_a = [&](int g) {
        const int t = tile_of(g), b = net_of(t);
        const float *src = A + ((int64_t)b * m + (int64_t)(t - b * tiles_per_net) * XBM) * XK +
                           (g & 7) * XBK;
        uint8_t *dst = sh + LDS_A32 + (g % NA) * A32_STAGE;
#pragma unroll
        for (int i = 0; i < A32_STAGE / 1024 / XWAVES; ++i) {
            const int ins = wid + XWAVES * i;
            const int row = ins * 8 + a_row_l;
            const int chunk = a_chk_l ^ ((row >> 1) & 7);
            glds16(src + (int64_t)row * XK + chunk * 4, lds_addr(dst + ins * 1024));
        }
    };

    // L1: the observation rows of a tile (128 x 64 B) by LDS-DMA, one 1-KB
    // wave-instruction per wave into obs buffer j & 1 for the block's j-th
    // tile; lane L fills the 16-B slot (row L >> 2, chunk L & 3) with global
    // chunk (L & 3) ^ (row & 3) of that row (the reads below are then
    // conflict-free: 16 consecutive rows hit 16 distinct bank quads)
    auto issue_obs = [&](int j) {
        const int t = (int)blockIdx.x + j * (int)gridDim.x, b = net_of(t);
        const int row = wid * 16 + (lane >> 2), chunk = (lane & 3) ^ (row & 3);
        const float *src = l1_obs16 + ((int64_t)(t - b * tiles_per_net) * XBM + row) * 16 +
                           chunk * 4;
        glds16(src, lds_addr(sh + LDS_OBS + (j & 1) * OBS_TILE + wid * 1024));
    };
    // L1: stage s of A = tanh(obs W0^T + b0): wave w forms the 4 columns
    // k = 32 (s & 7) + 4 w .. + 3 (weights wave-uniform: scalar loads) of
    // tile rows lane and lane + 64; each row's 4 values are one 16-B LDS
    // chunk of the A stage (and one 16-B store of h1)
    auto compute_a = [&](int s_) {
        const int t = tile_of(s_), b = net_of(t), j = s_ >> 3;
        const int k0 = (s_ & 7) * XBK + 4 * wid;
        const float *obs_t = reinterpret_cast<const float *>(sh + LDS_OBS + (j & 1) * OBS_TILE);
        uint8_t *dst = sh + LDS_A32 + (s_ % NA) * A32_STAGE;
        const float *wq = l1_w0p + ((int64_t)b * XN + k0) * 16;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int r = lane + 64 * h;
            // two columns at a time (their 32 weights in SGPRs), the 15
            // inputs one 16-B LDS chunk at a time; each column keeps
            // linear_tanh's fmaf order i = 0 .. 14
            float o[4];
#pragma unroll
            for (int qp = 0; qp < 4; qp += 2) {
                float acc[2] = {0.f, 0.f};
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const float4 v = *reinterpret_cast<const float4 *>(obs_t + r * 16 +
                                                                        ((c ^ (r & 3)) << 2));
                    const float xc[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int i = 4 * c + u;
                        if (i < 15) {
#pragma unroll
                            for (int q = 0; q < 2; ++q)
                                acc[q] = fmaf(xc[u], wq[(qp + q) * 16 + i], acc[q]);
                        }
                    }
                }
#pragma unroll
                for (int q = 0; q < 2; ++q) o[qp + q] = tanh_fast(acc[q] + wq[(qp + q) * 16 + 15]);
                __builtin_amdgcn_sched_barrier(0);
            }
            const float4 ov = make_float4(o[0], o[1], o[2], o[3]);
            *reinterpret_cast<float4 *>(dst + swz32(r, wid)) = ov;
            if (l1_h1)
                *reinterpret_cast<float4 *>(
                    l1_h1 + ((int64_t)b * m + (int64_t)(t - b * tiles_per_net) * XBM + r) * XK +
                    k0) = ov;
            // one row at a time: the register file is nearly full here (the
            // next step's fragments and 128 accumulators are live)
            __builtin_amdgcn_sched_barrier(0);
        }
    };

    // fragment offsets: tile row fr = lane & 31, k half fh = lane >> 5
    const int fr = lane & 31, fh = lane >> 5;
    int a_off[XMT][2][2], b_off[2][2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int i = 0; i < XMT; ++i) {
            // 8 consecutive k of A row r: chunks 4s + 2fh and 4s + 2fh + 1
            a_off[i][s][0] = swz32(wm * 64 + i * 32 + fr, 4 * s + 2 * fh);
            a_off[i][s][1] = swz32(wm * 64 + i * 32 + fr, 4 * s + 2 * fh + 1);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) b_off[j][s] = swz(wn * 64 + j * 32 + fr, 2 * s + fh);
    }

    // Raw fragments of one k16 step: the f32 A rows (split later) and the
    // three weight planes.
    struct Frag {
        float4 a[XMT][2];
        bf16x8_t b[2][3];
        bf16x8_t a3[XMT][3];   // the split A planes
    };
    auto read_frag = [&](int g, int s, Frag &f) {
        if (DR_X6_ABL == 2 && g > 0) {
            f.a[0][0].x += 1.0f;
            return;
        }
        const uint8_t *SA = sh + LDS_A32 + (g % NA) * A32_STAGE;
        const uint8_t *SB = sh + LDS_WB + (g & 1) * B_STAGE;
#pragma unroll
        for (int i = 0; i < XMT; ++i) {
            f.a[i][0] = *reinterpret_cast<const float4 *>(SA + a_off[i][s][0]);
            f.a[i][1] = *reinterpret_cast<const float4 *>(SA + a_off[i][s][1]);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int p = 0; p < 3; ++p)
                f.b[j][p] = *reinterpret_cast<const bf16x8_t *>(SB + p * B_PLANE + b_off[j][s]);
    };

    // Accumulators hold the TRANSPOSED tile, D[n][m] = sum_k Bt[n][k] A[m][k]
    // (the weight fragment is the MFMA's A operand): a lane then owns 4
    // consecutive output columns per register quad, stored as one float4.
    f32x16_t acc_h[XMT][2], acc_l[XMT][2];   // [A row tile i][weight tile j]
    auto zero_acc = [&]() {
#pragma unroll
        for (int i = 0; i < XMT; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                acc_h[i][j] = (f32x16_t){};
                acc_l[i][j] = (f32x16_t){};
            }
    };
    auto split_frag = [&](Frag &f) {
#pragma unroll
        for (int i = 0; i < XMT; ++i) {
            const float x[8] = {f.a[i][0].x, f.a[i][0].y, f.a[i][0].z, f.a[i][0].w,
                                f.a[i][1].x, f.a[i][1].y, f.a[i][1].z, f.a[i][1].w};
            u32x4_t h, mm, l;
            if (DR_X6_ABL == 1) {
                h = (u32x4_t){__float_as_uint(x[0]), __float_as_uint(x[1]), __float_as_uint(x[2]),
                              __float_as_uint(x[3])};
                mm = (u32x4_t){__float_as_uint(x[4]), __float_as_uint(x[5]), __float_as_uint(x[6]),
                               __float_as_uint(x[7])};
                l = h ^ mm;
            } else {
                split8(x, h, mm, l);
            }
            f.a3[i][0] = __builtin_bit_cast(bf16x8_t, h);
            f.a3[i][1] = __builtin_bit_cast(bf16x8_t, mm);
            f.a3[i][2] = __builtin_bit_cast(bf16x8_t, l);
        }
    };
    auto mfma_step = [&](Frag &f, bool presplit = false) {
        if (!DR_X6_EARLY && !presplit) split_frag(f);
        const bf16x8_t(&fa)[XMT][3] = f.a3;
        if (DR_X6_PRIO == 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < XMT; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const bf16x8_t *w = f.b[j];
                acc_h[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], fa[i][0],
                                                                      acc_h[i][j], 0, 0, 0);
                f32x16_t t = DR_X6_ACC1 ? (f32x16_t){} : acc_l[i][j];
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[1], fa[i][0], t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], fa[i][1], t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[2], fa[i][0], t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], fa[i][2], t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[1], fa[i][1], t, 0, 0, 0);
                if (DR_X6_ACC1) {
#pragma unroll
                    for (int r = 0; r < 16; ++r) acc_h[i][j][r] = acc_h[i][j][r] + t[r];
                } else {
                    acc_l[i][j] = t;
                }
            }
        if (DR_X6_PRIO == 1) __builtin_amdgcn_s_setprio(0);
    };
    // D[n][m] map: m = fr (the lane), n = 8 (r >> 2) + 4 fh + (r & 3): the
    // register quad q holds columns n0 + 8q + 4fh .. +4 of row m -> float4.
    auto epilogue = [&](int g) {
        const int t = tile_of(g), b = net_of(t);
        float *Cb = C + ((int64_t)b * m + (int64_t)(t - b * tiles_per_net) * XBM) * XN;
#pragma unroll
        for (int i = 0; i < XMT; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const f32x16_t v = acc_h[i][j] + acc_l[i][j];
                float *c = Cb + (int64_t)(wm * 64 + i * 32 + fr) * XN + wn * 64 + j * 32 + 4 * fh;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 o = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
                    if (nt)
                        store_nt(reinterpret_cast<float4 *>(c + 8 * q), o);
                    else
                        *reinterpret_cast<float4 *>(c + 8 * q) = o;
                }
            }
    };

    // Stage g's schedule (per wave): MFMAs of k16 step 0 while the step-1
    // fragments are read; wait for stage g + 1's operands + barrier; issue
    // the image of g + 2 and the A rows of g + 3 into stage g's (now free)
    // buffers; read stage g + 1's step-0 fragments during step 1's MFMAs.
    // VMEM ops per wave: 6 image + 2 A loads per stage, 16 stores per tile.
    if constexpr (L1) {
        // Per wave and iteration g after the barrier: the image of g + 2 (6
        // LDS-DMA), at a tile's first iteration the next tile's observation
        // rows (1), the 2 h1 stores of stage g + 2 (h1 non-null), and after
        // a tile's last MFMAs its 16 output stores.  The barrier of g needs
        // the image of g + 1: everything older than iteration g - 1's
        // observation load, h1 stores and output stores.
        const bool h1s = l1_h1 != nullptr;
        auto wait_bar = [&](int n) {
            __builtin_amdgcn_sched_barrier(0);
            switch (n) {
                case 1: asm volatile("s_waitcnt vmcnt(1) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
                case 2: asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
                case 3: asm volatile("s_waitcnt vmcnt(3) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
                case 16: asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
                case 18: asm volatile("s_waitcnt vmcnt(18) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
                default: asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
            }
        };
        zero_acc();
        issue_b(0);
        issue_b(1);                               // G >= 8
        issue_obs(0);
        wait_bar(0);                              // tile 0's observations visible
        compute_a(0);
        compute_a(1);
        wait_bar(0);                              // A stages 0, 1 visible
        Frag f0, f1;
        read_frag(0, 0, f0);
        for (int g = 0; g < G; ++g) {
            read_frag(g, 1, f1);
            mfma_step(f0);
            int n = 0;
            if (g > 0 && g + 1 < G) {
                const int p = g - 1;              // what iteration g - 1 issued after its image load
                n = (h1s && p + 2 < G ? 2 : 0) +
                    ((p & 7) == 0 && (p >> 3) + 1 < nmine ? 1 : 0) + ((p & 7) == 7 ? 16 : 0);
            }
            wait_bar(n);
            if (g + 2 < G) issue_b(g + 2);
            if ((g & 7) == 0 && (g >> 3) + 1 < nmine) issue_obs((g >> 3) + 1);
            // The SIMD partners (waves w and w + 4) form the next A stage at
            // different times: waves 0-3 before this half-stage's MFMAs,
            // waves 4-7 after them, so one partner's VALU runs beside the
            // other's MFMAs (DR_X6_L1_SPLIT=0: every wave before)
            const bool early = !DR_X6_L1_SPLIT || wid < XWAVES / 2;
            __builtin_amdgcn_sched_barrier(0);
            if (early && g + 2 < G && !DR_X6_NOCOMP) compute_a(g + 2);
            __builtin_amdgcn_sched_barrier(0);
            if (DR_X6_CONDREAD) {
                if (g + 1 < G) read_frag(g + 1, 0, f0);
            } else {
                read_frag(g + 1 < G ? g + 1 : g, 0, f0);   // see the L1 = false loop
            }
            __builtin_amdgcn_sched_barrier(0);
            mfma_step(f1);
            __builtin_amdgcn_sched_barrier(0);
            if (!early && g + 2 < G && !DR_X6_NOCOMP) compute_a(g + 2);
            __builtin_amdgcn_sched_barrier(0);
            if ((g & 7) == 7) {
                epilogue(g);
                zero_acc();
            }
        }
        return;
    }
    zero_acc();
    issue_b(0);
    issue_a(0);
    issue_a(1);
    issue_b(1);
    issue_a(2);                                   // G >= 8
    asm volatile("s_waitcnt vmcnt(" X6_S(X6_PRO) ")\n\ts_barrier" ::: "memory");
    if (DR_X6_PRIO == 2 && wid >= 4) __builtin_amdgcn_s_setprio(1);
    Frag f0, f1;
    read_frag(0, 0, f0);
    if (DR_X6_EARLY) split_frag(f0);
    for (int g = 0; g < G; ++g) {
        X6_STAMP(g, 0);
        read_frag(g, 1, f1);
        // DR_X6_F1EARLY: keep step 1's reads ahead of step 0's split and
        // MFMAs (the scheduler otherwise sinks them to the step's end)
        if (DR_X6_F1EARLY) __builtin_amdgcn_sched_barrier(0);
        mfma_step(f0);
        const bool pre1 = DR_X6_STAGGER && wid >= 4;
        if (DR_X6_EARLY || pre1) split_frag(f1);
        X6_STAMP(g, 1);
        // stage g + 1's image and A rows have landed; younger VMEM ops: the
        // A rows of g + 2 (issued one stage ago) and the previous tile's
        // 16 stores
        const bool a2 = g + 2 < G, epi_prev = (g & 7) == 0 && g > 0;
        __builtin_amdgcn_sched_barrier(0);
        if (a2 && epi_prev)
            asm volatile("s_waitcnt vmcnt(" X6_S(X6_NA_NST) ") lgkmcnt(0)\n\ts_barrier" ::: "memory");
        else if (epi_prev)
            asm volatile("s_waitcnt vmcnt(" X6_S(X6_NST) ") lgkmcnt(0)\n\ts_barrier" ::: "memory");
        else if (a2)
            asm volatile("s_waitcnt vmcnt(" X6_S(X6_NA) ") lgkmcnt(0)\n\ts_barrier" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        X6_STAMP(g, 2);
        if (!DR_X6_LATEISSUE) {
            if (g + 2 < G && DR_X6_ABL != 3) issue_b(g + 2);
            if (g + 3 < G && DR_X6_ABL != 3) issue_a(g + 3);
        }
        // unconditional (the last iteration re-reads stage g; unused): a
        // read on one path only would make the waitcnt pass merge the two
        // paths' LDS counts into an lgkmcnt(0) before step 1's split, which
        // exposes these reads' latency; counted on every path, the waits
        // below are lgkmcnt(>= 10): only step 1's reads, which the barrier
        // already drained
        if (DR_X6_CONDREAD) {
            if (g + 1 < G) read_frag(g + 1, 0, f0);
        } else {
            read_frag(g + 1 < G ? g + 1 : g, 0, f0);
        }
        __builtin_amdgcn_sched_barrier(0);
        mfma_step(f1, pre1);
        if (DR_X6_LATEISSUE) {
            __builtin_amdgcn_sched_barrier(0);
            if (g + 2 < G && DR_X6_ABL != 3) issue_b(g + 2);
            if (g + 3 < G && DR_X6_ABL != 3) issue_a(g + 3);
        }
        if (DR_X6_EARLY && g + 1 < G) split_frag(f0);
        X6_STAMP(g, 3);
        if ((g & 7) == 7) {
            epilogue(g);
            zero_acc();
        }
    }
}

// ---------------------------------------------------------------------------
// Ping-pong form of gemm_x6_kernel<false> (A/B form, DRONERL_X6_PP=1: the
// same tiles, LDS images and per-output MFMA order, so bitwise the same C;
// measured slower, 143-148 vs 121-125 us: in-kernel stamps show the MFMA
// interval at ~1,300 cycles for its 24 MFMAs, not 768 -- the partner's
// split VALU, LDS-DMA and fragment reads share the SIMD's vector issue with
// the MFMAs, so alternating the roles does not take them off the MFMA
// wave's path).
//
// The two waves of each SIMD alternate roles once per barrier interval
// (MI355X_MICROARCH.md, two waves per SIMD): while one wave issues the 24
// MFMAs of a k16 step back to back, its partner reads and splits the
// fragments of its next step (and issues LDS-DMA / output stores), so the
// matrix pipe is not left idle while a wave splits.  Group A = waves 0-3
// (tile rows 0-63), group B = waves 4-7 (rows 64-127); u = global k16 step
// (stage g = u >> 1, half s = u & 1), U = 2 G steps per block:
//   interval 2u - 1: A prep(u)       B MFMA(u - 1)
//   interval 2u    : A MFMA(u)       B prep(u)
// (interval -1: A prep(0), B idle; the last, 2U - 1: A stores its rows of
// the last tile).  Every interval ends in a barrier, the
// same count for both groups.  A wave holds ONE step's fragments (prep fills
// them, its next interval's MFMAs consume them), 48 VGPRs beside the 128
// accumulator registers.
//
// LDS: stage g (B image slot g & 1, A rows slot g % 3) is read in intervals
// 4g - 1 .. 4g + 2.  Its slots are refilled after the barrier that ends
// 4g + 2: the image of g + 2 by group A in interval 4g + 3, the A rows of
// g + 3 by group B in 4g + 4; each group waits for its own DMA at the end of
// interval 4h + 2 (h = g + 1 resp. g + 2) before the barrier that publishes
// stage h + 1 for its first read at 4h + 3.  A tile's outputs are stored by
// a group in the prep interval after its last MFMA step (A: 32T + 31, B:
// 32T + 32; B's last tile after the loop).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(XTHREADS) void gemm_x6_pp_kernel(const float *__restrict__ A,
                                                              const uint8_t *__restrict__ img,
                                                              float *__restrict__ C, int64_t m,
                                                              int ntiles, int nt) {
    static_assert(XWAVES == 8, "the ping-pong kernel pairs waves w and w + 4");
    __shared__ __attribute__((aligned(16))) uint8_t sh[LDS_TOTAL];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int grp = wid >> 2, wq = wid & 3;
    const int wm = grp, wn = wq;
    const int tiles_per_net = (int)(m / XBM);
    const int nmine = (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
    const int G = nmine * XKC;
    const int U = 2 * G;

    auto tile_of = [&](int g) { return (int)blockIdx.x + (g >> 3) * (int)gridDim.x; };
    auto net_of = [&](int t) { return t / tiles_per_net; };
    // stage g's weight image by NW waves (index w of NW); addresses as a
    // uniform base plus one per-lane offset (glds16_s)
    const uint32_t voff_b = (uint32_t)lane * 16;
    // (NW = 4 or 8: the compile-time count of waves sharing the stage)
    auto issue_b = [&](int g, int w, auto nw) {
        constexpr int NW = decltype(nw)::value;
        const uint8_t *src = img + (int64_t)net_of(tile_of(g)) * W_IMG + (g & 7) * B_STAGE;
        uint8_t *dst = sh + LDS_WB + (g & 1) * B_STAGE;
#pragma unroll
        for (int q = 0; q < B_STAGE / 1024 / NW; ++q) {
            const int ins = w + NW * q;
            glds16_s(src + ins * 1024, voff_b, lds_addr(dst + ins * 1024));
        }
    };
    // A rows: instruction ins moves rows 8 ins + (lane >> 3); lane L fills LDS
    // chunk L & 7 with global chunk (L & 7) ^ ((row >> 1) & 7), which depends
    // on ins only through its parity: two offset VGPRs
    uint32_t voff_a[2];
#pragma unroll
    for (int par = 0; par < 2; ++par) {
        const int chunk = (lane & 7) ^ (((lane >> 4) + 4 * par) & 7);
        voff_a[par] = (uint32_t)(((lane >> 3) * XK + chunk * 4) * 4);
    }
    auto issue_a = [&](int g, int w, auto nw) {
        constexpr int NW = decltype(nw)::value;
        const int t = tile_of(g), b = net_of(t);
        const float *src = A + ((int64_t)b * m + (int64_t)(t - b * tiles_per_net) * XBM) * XK +
                           (g & 7) * XBK;
        uint8_t *dst = sh + LDS_A32 + (g % 3) * A32_STAGE;
#pragma unroll
        for (int q = 0; q < A32_STAGE / 1024 / NW; ++q) {
            const int ins = w + NW * q;          // NW even: ins & 1 == w & 1
            glds16_s(src + (int64_t)ins * 8 * XK, voff_a[w & 1], lds_addr(dst + ins * 1024));
        }
    };
    using N4 = std::integral_constant<int, 4>;
    using N8 = std::integral_constant<int, 8>;

    const int fr = lane & 31, fh = lane >> 5;
    int a_off[2][2][2], b_off[2][2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            a_off[i][s][0] = swz32(wm * 64 + i * 32 + fr, 4 * s + 2 * fh);
            a_off[i][s][1] = swz32(wm * 64 + i * 32 + fr, 4 * s + 2 * fh + 1);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) b_off[j][s] = swz(wn * 64 + j * 32 + fr, 2 * s + fh);
    }
    bf16x8_t fa[2][3], fb[2][3];           // one step's split A planes and weight planes
    f32x16_t acc_h[2][2], acc_l[2][2];
    auto zero_acc = [&]() {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                acc_h[i][j] = (f32x16_t){};
                acc_l[i][j] = (f32x16_t){};
            }
    };
    // fragments of k16 step u: f32 A rows (split here) and the weight planes
    auto prep = [&](int u) {
        const int g = u >> 1, s = u & 1;
        const uint8_t *SA = sh + LDS_A32 + (g % 3) * A32_STAGE;
        const uint8_t *SB = sh + LDS_WB + (g & 1) * B_STAGE;
        float4 ra[2][2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            ra[i][0] = *reinterpret_cast<const float4 *>(SA + a_off[i][s][0]);
            ra[i][1] = *reinterpret_cast<const float4 *>(SA + a_off[i][s][1]);
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int p = 0; p < 3; ++p)
                fb[j][p] = *reinterpret_cast<const bf16x8_t *>(SB + p * B_PLANE + b_off[j][s]);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const float x[8] = {ra[i][0].x, ra[i][0].y, ra[i][0].z, ra[i][0].w,
                                ra[i][1].x, ra[i][1].y, ra[i][1].z, ra[i][1].w};
            u32x4_t h, mm, l;
            split8(x, h, mm, l);
            fa[i][0] = __builtin_bit_cast(bf16x8_t, h);
            fa[i][1] = __builtin_bit_cast(bf16x8_t, mm);
            fa[i][2] = __builtin_bit_cast(bf16x8_t, l);
        }
    };
    // the products of gemm_x6_kernel's mfma_step, in its order
    auto mfma = [&]() {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const bf16x8_t *w = fb[j];
                acc_h[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], fa[i][0],
                                                                      acc_h[i][j], 0, 0, 0);
                f32x16_t &t = acc_l[i][j];
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[1], fa[i][0], t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], fa[i][1], t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[2], fa[i][0], t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], fa[i][2], t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[1], fa[i][1], t, 0, 0, 0);
            }
    };
    // the group's rows of the tile that stage g belongs to (16 float4 per lane)
    auto epilogue = [&](int g) {
        const int t = tile_of(g), b = net_of(t);
        float *Cb = C + ((int64_t)b * m + (int64_t)(t - b * tiles_per_net) * XBM) * XN;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const f32x16_t v = acc_h[i][j] + acc_l[i][j];
                float *c = Cb + (int64_t)(wm * 64 + i * 32 + fr) * XN + wn * 64 + j * 32 + 4 * fh;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 o = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2],
                                                 v[4 * q + 3]);
                    if (nt)
                        store_nt(reinterpret_cast<float4 *>(c + 8 * q), o);
                    else
                        *reinterpret_cast<float4 *>(c + 8 * q) = o;
                }
            }
    };
    auto bar = [&]() {
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
    };

    // prologue: stages 0, 1 (image and A rows) and the A rows of 2, by all
    // eight waves, all landed
    issue_b(0, wid, N8{});
    issue_a(0, wid, N8{});
    issue_b(1, wid, N8{});
    issue_a(1, wid, N8{});
    issue_a(2, wid, N8{});
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    zero_acc();
    bar();
    // Each group runs its own straight-line loop (one k16 step u per
    // iteration: a prep interval and an MFMA interval), so the register
    // allocator sees one fragment set and one accumulator set per path; both
    // loops end 2U + 1 intervals after the prologue barrier.
    if (grp == 0) {
        for (int u = 0; u < U; ++u) {
            X6_STAMP(u, 0);
            // interval 2u - 1: the image of stage u/2 + 1 (u even >= 2, i.e.
            // 4g + 3 with g = u/2 - 1), this step's fragments, then the
            // stores of a tile whose last step was u - 1
            if ((u & 1) == 0 && u >= 2 && (u >> 1) + 1 < G) issue_b((u >> 1) + 1, wq, N4{});
            prep(u);
            if (u >= 16 && (u & 15) == 0) {
                epilogue((u - 1) >> 1);
                zero_acc();
            }
            X6_STAMP(u, 1);
            bar();
            X6_STAMP(u, 2);
            // interval 2u: MFMA(u); for odd u = 2h + 1 it is interval 4h + 2:
            // wait for the image of stage h + 1 (issued in iteration 2h;
            // younger: that iteration's tile stores, h % 8 == 0, h >= 8)
            mfma();
            if (u & 1) {
                const int h = (u - 1) >> 1;
                __builtin_amdgcn_sched_barrier(0);
                if (h >= 8 && (h & 7) == 0)
                    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
                else
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            X6_STAMP(u, 3);
            bar();
        }
        // interval 2U - 1: the last tile's rows
        epilogue(G - 1);
        bar();
    } else {
        bar();                                   // interval -1
        for (int u = 0; u < U; ++u) {
            X6_STAMP(u, 0);
            // interval 2u: the A rows of stage u/2 + 2 (u even >= 2, i.e.
            // 4g + 4 with g = u/2 - 1), this step's fragments, a finished
            // tile's stores
            if ((u & 1) == 0 && u >= 2 && (u >> 1) + 2 < G) issue_a((u >> 1) + 2, wq, N4{});
            prep(u);
            if (u >= 16 && (u & 15) == 0) {
                epilogue((u - 1) >> 1);
                zero_acc();
            }
            if (u & 1) {
                // interval 4h + 2 (u = 2h + 1): wait for the A rows of stage
                // h + 1 (issued in iteration 2h - 2); younger: the A rows of
                // iteration 2h (stage h + 2, h >= 1) and the tile stores of
                // iteration 2h - 2 (h % 8 == 1, h >= 9) or 2h (h % 8 == 0, h >= 8)
                const int h = (u - 1) >> 1;
                const bool st = (h >= 9 && (h & 7) == 1) || (h >= 8 && (h & 7) == 0);
                const bool a2 = h >= 1 && h + 2 < G;
                __builtin_amdgcn_sched_barrier(0);
                if (st && a2)
                    asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
                else if (st)
                    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
                else if (a2)
                    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                else
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            X6_STAMP(u, 1);
            bar();
            X6_STAMP(u, 2);
            mfma();                              // interval 2u + 1
            X6_STAMP(u, 3);
            bar();
        }
        epilogue(G - 1);
    }
}

// ---------------------------------------------------------------------------
// Cooperative-split form of gemm_x6_kernel<false> (dr_gemm_x6's default;
// DRONERL_X6_CS=0 restores gemm_x6_kernel).  The same tiles, weight image and
// per-output MFMA order, so bitwise the same C.
//
// In gemm_x6_kernel every wave splits the f32 A fragments it reads, and the
// four waves that share a row half split the same values: 176 VALU per wave
// and stage beside its 48 MFMAs, on a SIMD whose vector issue the MFMAs, the
// LDS-DMA and the fragment reads also need (the stamps of the ping-pong form
// above).  Here the block splits each A stage once: every wave moves 16 rows
// of the f32 stage by LDS-DMA into its own part of one 16-KB A32 buffer and
// splits exactly those rows (8 k per lane), writing the three planes into a
// double-buffered plane image in the weight image's layout (row r, 16-B
// chunk c at swz(r, c)); the waves then read bf16 plane fragments (6
// ds_read_b128 per k16 step instead of 4 f32 reads and 88 VALU).  No wave
// reads another wave's A32 rows, so that buffer needs no barrier: the wave's
// own vmcnt orders its reads behind its DMA.  LDS: the image ring (2 x 48
// KB) + the plane ring (2 x 24 KB) + A32 (16 KB) = 160 KB.
//
// Iteration g (stage g), per wave:
//   1. split stage g + 1 (its A rows issued in iteration g - 1, waited by a
//      hand count) into planes (g + 1) & 1, read by nobody since the barrier
//      that ended iteration g - 1 (they held stage g - 1)
//   2. fragments of step 1 of stage g; MFMAs of step 0
//   3. wait: image g + 1 landed; plane writes and fragment reads done;
//      barrier B_g
//   4. LDS-DMA: A rows of stage g + 2, then image g + 2 into slot g & 1
//   5. fragments of step 0 of stage g + 1; MFMAs of step 1 of stage g
//   6. after a tile's last stage: its 16 float4 stores
// Measured: 117-121 vs 124-128 us for both nets at 65,536 rows.
// ---------------------------------------------------------------------------
constexpr int CS_PLANE = XBM * 64;                   // 8 KB: 128 rows x 32 bf16
constexpr int CS_STAGE = 3 * CS_PLANE;               // 24 KB
constexpr int CS_LDS_AP = 2 * B_STAGE;               // the plane ring after the image ring
constexpr int CS_LDS_A32 = 2 * B_STAGE + 2 * CS_STAGE;  // one f32 A stage (16 KB) after it
constexpr int CS_LDS = CS_LDS_A32 + A32_STAGE;       // 160 KB: all of the CU's LDS

__global__ __launch_bounds__(XTHREADS) void gemm_x6_cs_kernel(const float *__restrict__ A,
                                                              const uint8_t *__restrict__ img,
                                                              float *__restrict__ C, int64_t m,
                                                              int ntiles, int nt) {
    static_assert(XWAVES == 8, "512-thread blocks: one split unit (row, 8 k) per thread");
    __shared__ __attribute__((aligned(16))) uint8_t sh[CS_LDS];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid >> 2, wn = wid & 3;
    const int tiles_per_net = (int)(m / XBM);
    const int nmine = (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
    const int G = nmine * XKC;

    auto tile_of = [&](int g) { return (int)blockIdx.x + (g >> 3) * (int)gridDim.x; };
    auto net_of = [&](int t) { return t / tiles_per_net; };
    const uint32_t voff_b = (uint32_t)lane * 16;
    auto issue_b = [&](int g) {
        const uint8_t *src = img + (int64_t)net_of(tile_of(g)) * W_IMG + (g & 7) * B_STAGE;
        uint8_t *dst = sh + LDS_WB + (g & 1) * B_STAGE;
#pragma unroll
        for (int q = 0; q < B_STAGE / 1024 / XWAVES; ++q) {
            const int ins = wid + XWAVES * q;
            glds16_s(src + ins * 1024, voff_b, lds_addr(dst + ins * 1024));
        }
    };
    // A: each wave moves 16 rows of the f32 stage by LDS-DMA (pieces wid and
    // wid + 8: rows 8 wid .. + 7 and 64 + 8 wid .. + 7, the A32 layout of
    // gemm_x6_kernel) into the one A32 buffer and splits exactly those rows,
    // so no other wave reads them: its own vmcnt orders its reads behind its
    // own DMA, no barrier.  Lane L: row sr (L < 32: the first piece), k
    // chunk sc (8 k = f32 chunks 2 sc, 2 sc + 1).
    const int sr = (lane < 32 ? 8 * wid : 64 + 8 * wid) + ((lane & 31) >> 2), sc = lane & 3;
    uint32_t voff_a[2];
#pragma unroll
    for (int par = 0; par < 2; ++par) {
        const int chunk = (lane & 7) ^ (((lane >> 4) + 4 * par) & 7);
        voff_a[par] = (uint32_t)(((lane >> 3) * XK + chunk * 4) * 4);
    }
    auto issue_a = [&](int g) {
        const int t = tile_of(g), b = net_of(t);
        const float *src = A + ((int64_t)b * m + (int64_t)(t - b * tiles_per_net) * XBM) * XK +
                           (g & 7) * XBK;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int ins = wid + XWAVES * q;
            glds16_s(src + (int64_t)ins * 8 * XK, voff_a[ins & 1],
                     lds_addr(sh + CS_LDS_A32 + ins * 1024));
        }
    };
    auto split_stage = [&](int g) {
        const uint8_t *SA = sh + CS_LDS_A32;
        const float4 v0 = *reinterpret_cast<const float4 *>(SA + swz32(sr, 2 * sc));
        const float4 v1 = *reinterpret_cast<const float4 *>(SA + swz32(sr, 2 * sc + 1));
        const float x[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
        u32x4_t h, mm, l;
        split8(x, h, mm, l);
        uint8_t *dst = sh + CS_LDS_AP + (g & 1) * CS_STAGE + swz(sr, sc);
        *reinterpret_cast<u32x4_t *>(dst) = h;
        *reinterpret_cast<u32x4_t *>(dst + CS_PLANE) = mm;
        *reinterpret_cast<u32x4_t *>(dst + 2 * CS_PLANE) = l;
    };

    const int fr = lane & 31, fh = lane >> 5;
    int a_off[2][2], b_off[2][2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
        for (int i = 0; i < 2; ++i) a_off[i][s] = swz(wm * 64 + i * 32 + fr, 2 * s + fh);
#pragma unroll
        for (int j = 0; j < 2; ++j) b_off[j][s] = swz(wn * 64 + j * 32 + fr, 2 * s + fh);
    }
    struct Frag {
        bf16x8_t a[2][3];
        bf16x8_t b[2][3];
    };
    auto read_frag = [&](int g, int s, Frag &f) {
        const uint8_t *SA = sh + CS_LDS_AP + (g & 1) * CS_STAGE;
        const uint8_t *SB = sh + LDS_WB + (g & 1) * B_STAGE;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int p = 0; p < 3; ++p)
                f.a[i][p] = *reinterpret_cast<const bf16x8_t *>(SA + p * CS_PLANE + a_off[i][s]);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int p = 0; p < 3; ++p)
                f.b[j][p] = *reinterpret_cast<const bf16x8_t *>(SB + p * B_PLANE + b_off[j][s]);
    };
    f32x16_t acc_h[2][2], acc_l[2][2];
    auto zero_acc = [&]() {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                acc_h[i][j] = (f32x16_t){};
                acc_l[i][j] = (f32x16_t){};
            }
    };
    auto mfma_step = [&](const Frag &f) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const bf16x8_t *w = f.b[j];
                const bf16x8_t *fa = f.a[i];
                acc_h[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], fa[0], acc_h[i][j],
                                                                      0, 0, 0);
                f32x16_t t = acc_l[i][j];
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[1], fa[0], t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], fa[1], t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[2], fa[0], t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], fa[2], t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[1], fa[1], t, 0, 0, 0);
                acc_l[i][j] = t;
            }
    };
    auto epilogue = [&](int g) {
        const int t = tile_of(g), b = net_of(t);
        float *Cb = C + ((int64_t)b * m + (int64_t)(t - b * tiles_per_net) * XBM) * XN;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const f32x16_t v = acc_h[i][j] + acc_l[i][j];
                float *c = Cb + (int64_t)(wm * 64 + i * 32 + fr) * XN + wn * 64 + j * 32 + 4 * fh;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 o = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2],
                                                 v[4 * q + 3]);
                    if (nt)
                        store_nt(reinterpret_cast<float4 *>(c + 8 * q), o);
                    else
                        *reinterpret_cast<float4 *>(c + 8 * q) = o;
                }
            }
    };

    // prologue: A(0), images 0 and 1; split stage 0; A(1); image 0 and
    // planes 0 visible
    issue_a(0);
    issue_b(0);
    issue_b(1);
    asm volatile("s_waitcnt vmcnt(12)" ::: "memory");     // A(0): younger 2 x 6 image
    split_stage(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");    // A32 read before A(1) lands
    issue_a(1);
    asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)\n\ts_barrier" ::: "memory");   // image 0
    zero_acc();
    Frag f0, f1;
    read_frag(0, 0, f0);
    for (int g = 0; g < G; ++g) {
        // split first (only f0 live beside the accumulators).  This wave's
        // A(g + 1) pieces were issued in iteration g - 1 right after its
        // barrier, before image g + 1 (6) and that iteration's tile stores
        // (16 after a tile's last stage); in the prologue after everything
        if (g + 1 < G) {
            const bool epi_prev = (g & 7) == 0 && g > 0;
            __builtin_amdgcn_sched_barrier(0);
            if (g == 0)
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            else if (epi_prev)
                asm volatile("s_waitcnt vmcnt(22)" ::: "memory");
            else
                asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
            split_stage(g + 1);
        }
        __builtin_amdgcn_sched_barrier(0);
        read_frag(g, 1, f1);
        mfma_step(f0);
        // image g + 1 (issued in iteration g - 1 after A(g + 1)); younger:
        // that iteration's tile stores (16 after a tile's last stage).  The
        // lgkmcnt(0) also retires this wave's A32 reads before its next DMA
        const bool epi_prev = (g & 7) == 0 && g > 0;
        __builtin_amdgcn_sched_barrier(0);
        if (epi_prev)
            asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (g + 2 < G) issue_a(g + 2);
        if (g + 2 < G) issue_b(g + 2);
        read_frag(g + 1 < G ? g + 1 : g, 0, f0);
        __builtin_amdgcn_sched_barrier(0);
        mfma_step(f1);
        if ((g & 7) == 7) {
            epilogue(g);
            zero_acc();
        }
    }
}

// ---------------------------------------------------------------------------
// Half-width variant: 256-thread blocks own 128 rows x 128 columns (one
// column half of the output), 80 KB of LDS, so TWO blocks share a CU and the
// two waves on each SIMD come from different blocks: no common barrier keeps
// them in lockstep (in the 512-thread kernel a SIMD's two waves reach their
// VALU / LDS phases together, stamps in DESIGN.md section 12).  Both operand
// rings are two stages deep (A and the image of stage g + 2 issued after
// stage g's barrier); the A rows of a row tile are read by both column-half
// blocks (the second read mostly from L2 / the Infinity Cache).
constexpr int HX_WAVES = 4;
constexpr int HX_THREADS = 64 * HX_WAVES;
constexpr int HX_BPLANE = 128 * 64;                  // 8 KB
constexpr int HX_BSTAGE = 3 * HX_BPLANE;             // 24 KB
constexpr int HX_LDS_A = 2 * HX_BSTAGE;              // A32 ring after the image ring
constexpr int HX_LDS = 2 * HX_BSTAGE + 2 * A32_STAGE; // 80 KB
#define HX_NLOAD 10                                  // 6 image + 4 A per wave per stage
#define HX_NST 16                                    // float4 stores per lane per tile

__global__ __launch_bounds__(HX_THREADS) __attribute__((amdgpu_waves_per_eu(2, 2)))
void gemm_x6_half_kernel(const float *__restrict__ A, const uint8_t *__restrict__ img,
                         float *__restrict__ C, int64_t m, int ntiles) {
    __shared__ __attribute__((aligned(16))) uint8_t sh[HX_LDS];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wid >> 1, wn = wid & 1;
    const int tiles_per_net = (int)(m / XBM);
    const int nmine = (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
    const int G = nmine * XKC;
    // tile t: column half t & 1 of row tile t >> 1 (global over both nets)
    auto tile_of = [&](int g) { return (int)blockIdx.x + (g >> 3) * (int)gridDim.x; };
    auto issue = [&](int g) {
        const int t = tile_of(g), h = t & 1, rt = t >> 1, b = rt / tiles_per_net;
        const uint8_t *srcb = img + (int64_t)b * W_IMG + (g & 7) * B_STAGE + h * HX_BPLANE;
        uint8_t *dstb = sh + (g & 1) * HX_BSTAGE;
#pragma unroll
        for (int i = 0; i < HX_BSTAGE / 1024 / HX_WAVES; ++i) {
            const int ins = wid + HX_WAVES * i, p = ins >> 3;
            glds16(srcb + p * B_PLANE + (ins & 7) * 1024 + lane * 16,
                   lds_addr(dstb + ins * 1024));
        }
        const float *srca = A + ((int64_t)b * m + (int64_t)(rt - b * tiles_per_net) * XBM) * XK +
                            (g & 7) * XBK;
        uint8_t *dsta = sh + HX_LDS_A + (g & 1) * A32_STAGE;
#pragma unroll
        for (int i = 0; i < A32_STAGE / 1024 / HX_WAVES; ++i) {
            const int ins = wid + HX_WAVES * i;
            const int row = ins * 8 + (lane >> 3);
            const int chunk = (lane & 7) ^ ((row >> 1) & 7);
            glds16(srca + (int64_t)row * XK + chunk * 4, lds_addr(dsta + ins * 1024));
        }
    };
    const int fr = lane & 31, fh = lane >> 5;
    int a_off[2][2][2], b_off[2][2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            a_off[i][s2][0] = swz32(wm * 64 + i * 32 + fr, 4 * s2 + 2 * fh);
            a_off[i][s2][1] = swz32(wm * 64 + i * 32 + fr, 4 * s2 + 2 * fh + 1);
            b_off[i][s2] = swz(wn * 64 + i * 32 + fr, 2 * s2 + fh);
        }
    }
    struct Frag {
        float4 a[2][2];
        bf16x8_t b[2][3];
    };
    auto read_frag = [&](int g, int s2, Frag &f) {
        const uint8_t *SA = sh + HX_LDS_A + (g & 1) * A32_STAGE;
        const uint8_t *SB = sh + (g & 1) * HX_BSTAGE;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            f.a[i][0] = *reinterpret_cast<const float4 *>(SA + a_off[i][s2][0]);
            f.a[i][1] = *reinterpret_cast<const float4 *>(SA + a_off[i][s2][1]);
#pragma unroll
            for (int p = 0; p < 3; ++p)
                f.b[i][p] = *reinterpret_cast<const bf16x8_t *>(SB + p * HX_BPLANE + b_off[i][s2]);
        }
    };
    f32x16_t acc_h[2][2], acc_l[2][2];
    auto zero_acc = [&]() {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                acc_h[i][j] = (f32x16_t){};
                acc_l[i][j] = (f32x16_t){};
            }
    };
    auto mfma_step = [&](const Frag &f) {
        bf16x8_t fa[2][3];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const float x[8] = {f.a[i][0].x, f.a[i][0].y, f.a[i][0].z, f.a[i][0].w,
                                f.a[i][1].x, f.a[i][1].y, f.a[i][1].z, f.a[i][1].w};
            u32x4_t h, mm, l;
            split8(x, h, mm, l);
            fa[i][0] = __builtin_bit_cast(bf16x8_t, h);
            fa[i][1] = __builtin_bit_cast(bf16x8_t, mm);
            fa[i][2] = __builtin_bit_cast(bf16x8_t, l);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const bf16x8_t *w = f.b[j];
                acc_h[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], fa[i][0],
                                                                      acc_h[i][j], 0, 0, 0);
                f32x16_t t = acc_l[i][j];
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[1], fa[i][0], t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], fa[i][1], t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[2], fa[i][0], t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[0], fa[i][2], t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w[1], fa[i][1], t, 0, 0, 0);
                acc_l[i][j] = t;
            }
    };
    auto epilogue = [&](int g) {
        const int t = tile_of(g), h = t & 1, rt = t >> 1, b = rt / tiles_per_net;
        float *Cb = C + ((int64_t)b * m + (int64_t)(rt - b * tiles_per_net) * XBM) * XN + h * 128;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const f32x16_t v = acc_h[i][j] + acc_l[i][j];
                float *c = Cb + (int64_t)(wm * 64 + i * 32 + fr) * XN + wn * 64 + j * 32 + 4 * fh;
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    *reinterpret_cast<float4 *>(c + 8 * q) =
                        make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
            }
    };

    zero_acc();
    issue(0);
    issue(1);                                     // G >= 8
    asm volatile("s_waitcnt vmcnt(" X6_S(HX_NLOAD) ")\n\ts_barrier" ::: "memory");
    Frag f0, f1;
    read_frag(0, 0, f0);
    for (int g = 0; g < G; ++g) {
        read_frag(g, 1, f1);
        mfma_step(f0);
        // stage g + 1 has landed (issued a stage ago; younger: the previous
        // tile's stores) and every wave's reads of stage g are done
        __builtin_amdgcn_sched_barrier(0);
        if ((g & 7) == 0 && g > 0)
            asm volatile("s_waitcnt vmcnt(" X6_S(HX_NST) ") lgkmcnt(0)\n\ts_barrier" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (g + 2 < G) issue(g + 2);
        if (g + 1 < G) read_frag(g + 1, 0, f0);
        __builtin_amdgcn_sched_barrier(0);
        mfma_step(f1);
        if ((g & 7) == 7) {
            epilogue(g);
            zero_acc();
        }
    }
}

// ---------------------------------------------------------------------------
// Weight gradient of the same layer, dW[b] = G[b]^T H[b] (G = grad_z, H = the
// layer input, both (m, 256) f32 row-major), split over C row chunks: block
// (b, n-half, chunk) writes the 128 x 256 partial ws[b][chunk][n][k] of its
// (m / C)-row chunk; the chunk sum is left to the caller (the
// trainer's deferred finish sums C = 64 chunks in a fixed order).  Both
// operands are reduced over rows, so a fragment needs 8 consecutive ROWS of
// one column: each lane gathers them with ds_read_b32 from the f32 stage
// images (rows of 128 / 256 floats, consecutive lanes on consecutive columns:
// conflict-free) and splits them into the three bf16 planes in registers.
// Stages of 32 rows arrive by global_load_lds two stages ahead (three
// buffers); 8 waves as 2 (n) x 4 (k) of 64 x 64, the same split hi/lo
// accumulation as gemm_x6_kernel.
constexpr int TN_BM = 32;                          // rows per stage
constexpr int TN_G = TN_BM * 128 * 4;              // 16 KB: G stage (128 n)
constexpr int TN_H = TN_BM * 256 * 4;              // 32 KB: H stage (256 k)
constexpr int TN_STAGE = TN_G + TN_H;              // 48 KB
constexpr int TN_LDS = 3 * TN_STAGE;               // 144 KB
constexpr int TN_NG = TN_G / 1024 / XWAVES;        // 2 glds per wave per stage
constexpr int TN_NH = TN_H / 1024 / XWAVES;        // 4
#define TN_VM_YOUNG 6                              // TN_NG + TN_NH
#define TN_VM_PRO 12

__global__ __launch_bounds__(XTHREADS) void gemm_x6_wgrad_kernel(
    const float *__restrict__ Gm, const float *__restrict__ Hm, float *__restrict__ ws,
    int64_t m, int chunks) {
    __shared__ __attribute__((aligned(16))) uint8_t sh[TN_LDS];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wn = wid >> 2, wk = wid & 3;
    const int chunk = (int)(blockIdx.x % chunks);
    const int nh = (int)((blockIdx.x / chunks) & 1);
    const int b = (int)(blockIdx.x / chunks / 2);
    const int64_t rows = m / chunks;
    const int G_ = (int)(rows / TN_BM);
    const float *Gb = Gm + ((int64_t)b * m + (int64_t)chunk * rows) * 256 + nh * 128;
    const float *Hb = Hm + ((int64_t)b * m + (int64_t)chunk * rows) * 256;

    // stage g -> buffer g % 3; a G wave-instruction moves 2 rows x 512 B, an H
    // one 1 row x 1 KB (lane-linear, no swizzle: the b32 reads below are
    // conflict-free on plain rows)
    auto issue = [&](int g) {
        uint8_t *dst = sh + (g % 3) * TN_STAGE;
        const int64_t r0 = (int64_t)g * TN_BM;
#pragma unroll
        for (int i = 0; i < TN_NG; ++i) {
            const int ins = wid + XWAVES * i;                 // rows 2 ins, 2 ins + 1
            const int row = 2 * ins + (lane >> 5);
            glds16(Gb + (r0 + row) * 256 + (lane & 31) * 4, lds_addr(dst + ins * 1024));
        }
#pragma unroll
        for (int i = 0; i < TN_NH; ++i) {
            const int ins = wid + XWAVES * i;                 // row ins
            glds16(Hb + (r0 + ins) * 256 + lane * 4, lds_addr(dst + TN_G + ins * 1024));
        }
    };

    const int fr = lane & 31, fh = lane >> 5;
    // fragment of k16 step s: rows 16 s + 8 fh + j (j = 0..7) of one column
    int g_off[2][2], h_off[2][2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            g_off[i][s2] = (16 * s2 + 8 * fh) * 512 + (wn * 64 + i * 32 + fr) * 4;
            h_off[i][s2] = TN_G + (16 * s2 + 8 * fh) * 1024 + (wk * 64 + i * 32 + fr) * 4;
        }
    struct RawFrag {
        float g[2][8];
        float h[2][8];
    };
    auto read_frag = [&](int g, int s2, RawFrag &f) {
        const uint8_t *S = sh + (g % 3) * TN_STAGE;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                f.g[i][j] = *reinterpret_cast<const float *>(S + g_off[i][s2] + j * 512);
                f.h[i][j] = *reinterpret_cast<const float *>(S + h_off[i][s2] + j * 1024);
            }
    };
    f32x16_t acc_h[2][2], acc_l[2][2];                    // [n tile i][k tile j]
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            acc_h[i][j] = (f32x16_t){};
            acc_l[i][j] = (f32x16_t){};
        }
    auto mfma_step = [&](const RawFrag &f) {
        bf16x8_t fg[2][3], fhp[2][3];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            u32x4_t a0, a1, a2, c0, c1, c2;
            split8(f.g[i], a0, a1, a2);
            split8(f.h[i], c0, c1, c2);
            fg[i][0] = __builtin_bit_cast(bf16x8_t, a0);
            fg[i][1] = __builtin_bit_cast(bf16x8_t, a1);
            fg[i][2] = __builtin_bit_cast(bf16x8_t, a2);
            fhp[i][0] = __builtin_bit_cast(bf16x8_t, c0);
            fhp[i][1] = __builtin_bit_cast(bf16x8_t, c1);
            fhp[i][2] = __builtin_bit_cast(bf16x8_t, c2);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const bf16x8_t *a = fg[i], *c = fhp[j];
                acc_h[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], c[0], acc_h[i][j],
                                                                      0, 0, 0);
                f32x16_t t = acc_l[i][j];
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], c[1], t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], c[0], t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], c[2], t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], c[0], t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], c[1], t, 0, 0, 0);
                acc_l[i][j] = t;
            }
    };

    issue(0);
    issue(1);
    issue(2);                                      // G_ >= 3 (checked by the host)
    asm volatile("s_waitcnt vmcnt(" X6_S(TN_VM_PRO) ")\n\ts_barrier" ::: "memory");
    RawFrag f0, f1;
    read_frag(0, 0, f0);
    for (int g = 0; g < G_; ++g) {
        read_frag(g, 1, f1);
        mfma_step(f0);
        // stage g + 1 has landed (the loads of g + 2 may be in flight), and
        // every wave's reads of stage g are done
        __builtin_amdgcn_sched_barrier(0);
        if (g + 2 < G_)
            asm volatile("s_waitcnt vmcnt(" X6_S(TN_VM_YOUNG) ") lgkmcnt(0)\n\ts_barrier" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (g + 3 < G_) issue(g + 3);
        if (DR_X6_CONDREAD) {
            if (g + 1 < G_) read_frag(g + 1, 0, f0);
        } else {
            read_frag(g + 1 < G_ ? g + 1 : g, 0, f0);   // see gemm_x6_kernel
        }
        __builtin_amdgcn_sched_barrier(0);
        mfma_step(f1);
    }
    // D[n][k]: column k = fr, row n = (r & 3) + 8 (r >> 2) + 4 fh
    float *out = ws + ((int64_t)b * chunks + chunk) * 256 * 256 + (int64_t)(nh * 128) * 256;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const f32x16_t v = acc_h[i][j] + acc_l[i][j];
            float *c = out + (int64_t)(wn * 64 + i * 32 + 4 * fh) * 256 + wk * 64 + j * 32 + fr;
#pragma unroll
            for (int r = 0; r < 16; ++r) c[((r & 3) + 8 * (r >> 2)) * 256] = v[r];
        }
}

// ---------------------------------------------------------------------------
// Cooperative-split form of gemm_x6_wgrad_kernel (A/B form, DRONERL_X6_WCS=1;
// measured slower: 157 vs 137 us at 65,536 rows, 64 chunks -- the 16-row
// stages need a barrier per k16 step, and each step's fragment reads wait
// for that barrier).  The same blocks, output layout and per-output MFMA
// order (the same six products of the same bf16 planes), so bitwise the
// same workspace (tests/test_gemm_x6_gpu.py).
//
// gemm_x6_wgrad_kernel gathers each fragment with 8 ds_read_b32 and splits it
// in registers: 32 reads and 176 split VALU per wave and k16 step, each G
// value split by the four waves of its n half and each H value by two.  Here
// the block splits every value once, per 16-row stage, into a transposed
// plane image in the MFMA fragment order (per column: the 16 rows as two
// 16-B chunks of 8 bf16, the chunks of columns 8-15 mod 16 swapped: reads
// and writes free of bank conflicts); the waves read 12 ds_read_b128 of
// planes per step.  A split unit is 8 rows x 1 column (one split8): 768 per
// stage (128 G + 256 H columns x 2 row groups).  Wave w owns row group
// w & 1 and 96 of the 384 columns (w >> 1): it moves exactly those f32 values
// (8 rows x 96 columns, 3 KB: three LDS-DMA pieces) into its own slot of a
// 2-deep staging ring and splits them (lane L: columns L and, below 32,
// 64 + L), so no other wave reads its staging: its own vmcnt orders its
// reads behind its DMA.  LDS: planes 2 x 36 KB + staging 2 x 24 KB = 120 KB.
//
// Iteration g (16-row stage g), per wave: fragments of stage g (planes
// g & 1); split stage g + 1 (its DMA, issued in iteration g - 1, is the only
// vector-memory op in flight: vmcnt(0)) into planes (g + 1) & 1, which held
// stage g - 1, read before the barrier that ended iteration g - 1; MFMAs of
// stage g; lgkmcnt(0) + barrier; LDS-DMA stage g + 2 into staging g & 1
// (its stage-g values were split in iteration g - 1).
// ---------------------------------------------------------------------------
constexpr int WC_BM = 16;                            // rows per stage
constexpr int WC_GP = 128 * WC_BM * 2;               // 4 KB: one G plane (128 n x 16 rows)
constexpr int WC_HP = 256 * WC_BM * 2;               // 8 KB: one H plane (256 k x 16 rows)
constexpr int WC_PSTAGE = 3 * WC_GP + 3 * WC_HP;     // 36 KB of planes per stage
constexpr int WC_SSLOT = 8 * 96 * 4;                 // 3 KB: one wave's staging slot
constexpr int WC_SSTAGE = XWAVES * WC_SSLOT;         // 24 KB
constexpr int WC_LDS_S = 2 * WC_PSTAGE;              // staging ring after the plane ring
constexpr int WC_LDS = 2 * WC_PSTAGE + 2 * WC_SSTAGE;  // 120 KB

// byte offset of column c's row chunk q (0: rows 0-7, 1: rows 8-15) in a plane
__device__ inline int wc_off(int c, int q) { return c * 32 + ((q ^ ((c >> 3) & 1)) << 4); }

__global__ __launch_bounds__(XTHREADS) void gemm_x6_wgrad_cs_kernel(
    const float *__restrict__ Gm, const float *__restrict__ Hm, float *__restrict__ ws,
    int64_t m, int chunks) {
    __shared__ __attribute__((aligned(16))) uint8_t sh[WC_LDS];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wn = wid >> 2, wk = wid & 3;
    const int chunk = (int)(blockIdx.x % chunks);
    const int nh = (int)((blockIdx.x / chunks) & 1);
    const int b = (int)(blockIdx.x / chunks / 2);
    const int64_t rows = m / chunks;
    const int G_ = (int)(rows / WC_BM);
    const float *Gb = Gm + ((int64_t)b * m + (int64_t)chunk * rows) * 256 + nh * 128;
    const float *Hb = Hm + ((int64_t)b * m + (int64_t)chunk * rows) * 256;

    // this wave's split share: row group rg, global columns 96 q .. + 95
    // (0-127: G column, 128-383: H column - 128)
    const int rg = wid & 1, q0 = 96 * (wid >> 1);
    // DMA: piece p moves the wave's local floats 256 p .. + 255 (8 rows x 96
    // columns, row-major); lane L's 16 B = local row r, columns j .. j + 3
    const float *src_p[3];
#pragma unroll
    for (int p = 0; p < 3; ++p) {
        const int f = 256 * p + 4 * lane, r = f / 96, j = f % 96, cg = q0 + j;
        src_p[p] = cg < 128 ? Gb + (int64_t)(8 * rg + r) * 256 + cg
                            : Hb + (int64_t)(8 * rg + r) * 256 + (cg - 128);
    }
    auto issue = [&](int g) {
        const int64_t off = (int64_t)g * WC_BM * 256;      // WC_BM rows of 256 floats
        uint8_t *dst = sh + WC_LDS_S + (g & 1) * WC_SSTAGE + wid * WC_SSLOT;
#pragma unroll
        for (int p = 0; p < 3; ++p) glds16(src_p[p] + off, lds_addr(dst + p * 1024));
    };
    // split unit u (0: column q0 + lane; 1: column q0 + 64 + lane, lanes < 32)
    auto split_unit = [&](int g, int jl) {
        const float *S = reinterpret_cast<const float *>(sh + WC_LDS_S + (g & 1) * WC_SSTAGE +
                                                         wid * WC_SSLOT);
        float x[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) x[r] = S[r * 96 + jl];
        u32x4_t h, mm, l;
        split8(x, h, mm, l);
        const int cg = q0 + jl;
        uint8_t *P = sh + (g & 1) * WC_PSTAGE;
        uint8_t *dst = cg < 128 ? P + wc_off(cg, rg) : P + 3 * WC_GP + wc_off(cg - 128, rg);
        const int pl = cg < 128 ? WC_GP : WC_HP;
        *reinterpret_cast<u32x4_t *>(dst) = h;
        *reinterpret_cast<u32x4_t *>(dst + pl) = mm;
        *reinterpret_cast<u32x4_t *>(dst + 2 * pl) = l;
    };
    auto split_stage = [&](int g) {
        split_unit(g, lane);
        if (lane < 32) split_unit(g, 64 + lane);
    };

    const int fr = lane & 31, fh = lane >> 5;
    int g_off[2], h_off[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        g_off[i] = wc_off(wn * 64 + i * 32 + fr, fh);
        h_off[i] = 3 * WC_GP + wc_off(wk * 64 + i * 32 + fr, fh);
    }
    struct Frag {
        bf16x8_t g[2][3];
        bf16x8_t h[2][3];
    };
    auto read_frag = [&](int g, Frag &f) {
        const uint8_t *P = sh + (g & 1) * WC_PSTAGE;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                f.g[i][p] = *reinterpret_cast<const bf16x8_t *>(P + g_off[i] + p * WC_GP);
                f.h[i][p] = *reinterpret_cast<const bf16x8_t *>(P + h_off[i] + p * WC_HP);
            }
    };
    f32x16_t acc_h[2][2], acc_l[2][2];                    // [n tile i][k tile j]
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            acc_h[i][j] = (f32x16_t){};
            acc_l[i][j] = (f32x16_t){};
        }
    // gemm_x6_wgrad_kernel's products, in its order
    auto mfma_step = [&](const Frag &f) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const bf16x8_t *a = f.g[i], *c = f.h[j];
                acc_h[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], c[0], acc_h[i][j],
                                                                      0, 0, 0);
                f32x16_t t = acc_l[i][j];
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], c[1], t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], c[0], t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], c[2], t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], c[0], t, 0, 0, 0);
                t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], c[1], t, 0, 0, 0);
                acc_l[i][j] = t;
            }
    };

    issue(0);
    issue(1);                                      // G_ >= 2 (checked by the host)
    asm volatile("s_waitcnt vmcnt(3)" ::: "memory");  // this wave's stage-0 pieces
    split_stage(0);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    Frag f;
    for (int g = 0; g < G_; ++g) {
        read_frag(g, f);
        if (g + 1 < G_) {
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // stage g + 1's pieces
            split_stage(g + 1);
        }
        __builtin_amdgcn_sched_barrier(0);
        mfma_step(f);
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (g + 2 < G_) issue(g + 2);
    }
    // D[n][k]: column k = fr, row n = (r & 3) + 8 (r >> 2) + 4 fh
    float *out = ws + ((int64_t)b * chunks + chunk) * 256 * 256 + (int64_t)(nh * 128) * 256;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const f32x16_t v = acc_h[i][j] + acc_l[i][j];
            float *c = out + (int64_t)(wn * 64 + i * 32 + 4 * fh) * 256 + wk * 64 + j * 32 + fr;
#pragma unroll
            for (int r = 0; r < 16; ++r) c[((r & 3) + 8 * (r >> 2)) * 256] = v[r];
        }
}

// The L1 operands: w0p[b][k] = (W0[b][k][0..15), b0[b][k]) and, when obs is
// given, obs16[r] = (obs[r][0..15), 0).  One thread per 16-float row.
__global__ __launch_bounds__(256) void pack_first_kernel(int batch, const float *__restrict__ w0,
                                                         const float *__restrict__ b0,
                                                         float *__restrict__ w0p, int64_t m,
                                                         const float *__restrict__ obs,
                                                         float *__restrict__ obs16) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t nw = (int64_t)batch * XN;
    if (t < nw) {
        float r[16];
#pragma unroll
        for (int i = 0; i < 15; ++i) r[i] = w0[t * 15 + i];
        r[15] = b0[t];
#pragma unroll
        for (int q = 0; q < 4; ++q)
            reinterpret_cast<float4 *>(w0p + t * 16)[q] =
                make_float4(r[4 * q], r[4 * q + 1], r[4 * q + 2], r[4 * q + 3]);
    } else if (obs && t - nw < m) {
        const int64_t i = t - nw;
        float r[16];
#pragma unroll
        for (int c = 0; c < 15; ++c) r[c] = obs[i * 15 + c];
        r[15] = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q)
            reinterpret_cast<float4 *>(obs16 + i * 16)[q] =
                make_float4(r[4 * q], r[4 * q + 1], r[4 * q + 2], r[4 * q + 3]);
    }
}

int fail_g(int code, const std::string &msg) {
    set_global_error(msg);
    return code;
}

}  // namespace
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
    const int threads = (int)batch * XKC * XN * 4;
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
    if (batch < 1 || batch > 2 || m < XBM || m % XBM || m > (int64_t(1) << 26) || !a ||
        !img || !c || (((uintptr_t)a) & 15) || (((uintptr_t)img) & 15) ||
        (((uintptr_t)c) & 15))
        return fail_g(DR_ERR_INVALID,
                      "dr_gemm_x6: bad arguments (m must be a positive multiple of 128, "
                      "pointers 16-byte aligned)");
    static int n_cu = 0;
    if (n_cu == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            n_cu < 1)
            n_cu = 256;
    }
    // DRONERL_X6_HALF=1: the half-width kernel (two 80-KB blocks per CU)
    static const int half = [] {
        const char *e = getenv("DRONERL_X6_HALF");
        return e && e[0] == '1' ? 1 : 0;
    }();
    if (half) {
        const int nt2 = (int)(batch * (m / XBM) * 2);
        const int grid2 = nt2 < 2 * n_cu ? nt2 : 2 * n_cu;
        hipLaunchKernelGGL(gemm_x6_half_kernel, dim3(grid2), dim3(HX_THREADS), 0,
                           static_cast<hipStream_t>(stream), a,
                           static_cast<const uint8_t *>(img), c, m, nt2);
        const hipError_t e2 = hipGetLastError();
        return e2 == hipSuccess ? DR_OK
                                : fail_g(DR_ERR_HIP, std::string("gemm_x6_half_kernel: ") +
                                                         hipGetErrorString(e2));
    }
    const int ntiles = (int)(batch * (m / XBM));
    const int grid = ntiles < n_cu ? ntiles : n_cu;       // one 144-KB block per CU
    // DRONERL_X6_NT=1 (A/B knob, read once): nontemporal output stores --
    // measured 4.76 vs 5.74 updates/s: the next GEMM reads these rows back
    // from the Infinity Cache when they are stored plainly
    static const int nt = [] {
        const char *e = getenv("DRONERL_X6_NT");
        return e && e[0] == '1' ? 1 : 0;
    }();
    // DRONERL_X6_PP=1 (A/B knob, read once): the ping-pong schedule
    // (measured slower: 143-148 vs 121-125 us)
    static const int pp = [] {
        const char *e = getenv("DRONERL_X6_PP");
        return e && e[0] == '1' ? 1 : 0;
    }();
    // the cooperative-split form unless DRONERL_X6_CS=0 (A/B knob, read
    // once): 117-121 vs 124-128 us at 65,536 rows (scripts/micro/gemm_x6_bench.py)
    static const int cs = [] {
        const char *e = getenv("DRONERL_X6_CS");
        return e && e[0] == '0' ? 0 : 1;
    }();
    if (cs)
        hipLaunchKernelGGL(gemm_x6_cs_kernel, dim3(grid), dim3(XTHREADS), 0,
                           static_cast<hipStream_t>(stream), a,
                           static_cast<const uint8_t *>(img), c, m, ntiles, nt);
    else if (pp)
        hipLaunchKernelGGL(gemm_x6_pp_kernel, dim3(grid), dim3(XTHREADS), 0,
                           static_cast<hipStream_t>(stream), a,
                           static_cast<const uint8_t *>(img), c, m, ntiles, nt);
    else
        hipLaunchKernelGGL(gemm_x6_kernel<false>, dim3(grid), dim3(XTHREADS), 0,
                           static_cast<hipStream_t>(stream), a,
                           static_cast<const uint8_t *>(img), c, m, ntiles, nt, nullptr,
                           nullptr, nullptr);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess
               ? DR_OK
               : fail_g(DR_ERR_HIP, std::string("gemm_x6_kernel: ") + hipGetErrorString(e));
}

int dr_gemm_x6_l1_pack(int64_t batch, const float *w0, const float *b0, float *w0p, int64_t m,
                       const float *obs, float *obs16, void *stream) {
    if (batch < 1 || batch > 2 || !w0 || !b0 || !w0p || (((uintptr_t)w0p) & 15) ||
        (obs && (m < 1 || !obs16 || (((uintptr_t)obs16) & 15))))
        return fail_g(DR_ERR_INVALID, "dr_gemm_x6_l1_pack: bad arguments");
    const int64_t n = batch * XN + (obs ? m : 0);
    hipLaunchKernelGGL(pack_first_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), (int)batch, w0, b0, w0p, m, obs, obs16);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? DR_OK
                           : fail_g(DR_ERR_HIP, std::string("pack_first_kernel: ") +
                                                    hipGetErrorString(e));
}

int dr_gemm_x6_l1(int64_t batch, int64_t m, const float *obs16, const float *w0p, const void *img,
                  float *c, float *h1, void *stream) {
    if (batch < 1 || batch > 2 || m < XBM || m % XBM || m > (int64_t(1) << 26) || !obs16 ||
        !w0p || !img || !c || ((((uintptr_t)obs16) | ((uintptr_t)w0p) | ((uintptr_t)img) |
                                ((uintptr_t)c) | ((uintptr_t)h1)) & 15))
        return fail_g(DR_ERR_INVALID,
                      "dr_gemm_x6_l1: bad arguments (m must be a positive multiple of 128, "
                      "pointers 16-byte aligned)");
    int dev = 0, n_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n_cu < 1)
        n_cu = 256;
    const int ntiles = (int)(batch * (m / XBM));
    const int grid = ntiles < n_cu ? ntiles : n_cu;
    hipLaunchKernelGGL(gemm_x6_kernel<true>, dim3(grid), dim3(XTHREADS), 0,
                       static_cast<hipStream_t>(stream), nullptr,
                       static_cast<const uint8_t *>(img), c, m, ntiles, 0, obs16, w0p, h1);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? DR_OK
                           : fail_g(DR_ERR_HIP, std::string("gemm_x6_kernel<L1>: ") +
                                                    hipGetErrorString(e));
}

int dr_gemm_x6_wgrad(int64_t batch, int64_t m, int64_t chunks, const float *g, const float *h,
                     float *ws, void *stream) {
    if (batch < 1 || batch > 2 || chunks < 1 || m < 1 || m % chunks ||
        (m / chunks) % TN_BM || m / chunks < 3 * TN_BM || m > (int64_t(1) << 26) || !g || !h ||
        !ws || (((uintptr_t)g) & 15) || (((uintptr_t)h) & 15) || (((uintptr_t)ws) & 15))
        return fail_g(DR_ERR_INVALID,
                      "dr_gemm_x6_wgrad: bad arguments (m / chunks a multiple of 32, >= 96; "
                      "pointers 16-byte aligned)");
    // DRONERL_X6_WCS=1 (A/B knob, read once): the cooperative-split form
    // (bitwise the same; measured slower, 157 vs 137 us)
    static const int wcs = [] {
        const char *e = getenv("DRONERL_X6_WCS");
        return e && e[0] == '1' ? 1 : 0;
    }();
    if (wcs)
        hipLaunchKernelGGL(gemm_x6_wgrad_cs_kernel, dim3((unsigned)(batch * 2 * chunks)),
                           dim3(XTHREADS), 0, static_cast<hipStream_t>(stream), g, h, ws, m,
                           (int)chunks);
    else
        hipLaunchKernelGGL(gemm_x6_wgrad_kernel, dim3((unsigned)(batch * 2 * chunks)),
                           dim3(XTHREADS), 0, static_cast<hipStream_t>(stream), g, h, ws, m,
                           (int)chunks);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? DR_OK
                           : fail_g(DR_ERR_HIP, std::string("gemm_x6_wgrad_kernel: ") +
                                                    hipGetErrorString(e));
}

#if DR_X6_STAMPS
int dr_x6_diag_stamps(void *host_out, size_t bytes) {
    if (bytes < sizeof(g_x6_st)) return DR_ERR_INVALID;
    return hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_x6_st), sizeof(g_x6_st)) == hipSuccess
               ? DR_OK
               : DR_ERR_HIP;
}
#endif

}  // extern "C"
