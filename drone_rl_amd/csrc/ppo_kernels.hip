// PPO arithmetic for MI355X (gfx950): GAE scan, Gaussian policy sampling,
// minibatch permutation and gather, fused clipped-surrogate loss + head
// gradients, fused grad-norm clip + Adam.
//
// Restates stable-baselines3 PPO (not vendored in the reference; called at
// /root/reference/train.py:36-43 and 63-68).  The SB3 algorithm is recalled
// in SURVEY.md Appendix C; its results are pinned by this build's own CPU
// restatement (oracle/ppo_ref.py), not by reference vectors ("parity
// unpinned").  Every kernel here is HBM-bound elementwise / scan / reduction
// work; only the MLP GEMMs (torch, hipBLASLt -> MFMA) are matrix-shaped.
//
// Reductions are deterministic: fixed per-block partials, then a fixed-order
// combine (no float atomics), so a rerun reproduces every bit.

#include <cmath>
#include <cstdlib>
#include <string>

#include "common.h"
#include "x6_split.h"

#pragma clang fp contract(off)

// DR_LOSS_RCP 1 (default since round 5): the Gaussian log-prob's and the PPO
// row's divisions by var, 2 var and the advantage std are products with
// reciprocals formed once per thread (an IEEE f32 division is ~10 VALU, and
// the policy rows run on 4 lanes of 64 in the head kernel: the issue cost is
// the whole wave's; its loss block 244 -> 120 VALU per 4-row tile); each term
// within an ulp or so of the quotient.  7.19-7.21 vs 7.14-7.15 PPO updates/s,
// three alternating pairs on one box (profiles/r05_loss_rcp_ab.json).  0: the
// quotients (round 1-4 bits).
#ifndef DR_LOSS_RCP
#define DR_LOSS_RCP 1
#endif

namespace dr {
namespace {

constexpr float kLogSqrt2Pi = 0.91893853320467274178f;  // log(sqrt(2*pi))

int fail0(int code, const std::string &msg) {
    set_global_error(msg);
    return code;
}

int check_launch(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return fail0(DR_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
    return DR_OK;
}

inline hipStream_t as_stream(void *s) { return static_cast<hipStream_t>(s); }

// ---------------------------------------------------------------------------
// GAE (RolloutBuffer.compute_returns_and_advantage).  One thread per env,
// reverse scan over T; (T,N) layout keeps each step's loads coalesced.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void gae_kernel(
    int64_t T, int64_t N, const float *__restrict__ rew,
    const float *__restrict__ val, const uint8_t *__restrict__ starts,
    const float *__restrict__ last_val, const uint8_t *__restrict__ last_done,
    float gamma, float gl, float *__restrict__ adv, float *__restrict__ ret) {
    const int64_t n = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (n >= N) return;
    float last = 0.f;
    float next_v = last_val[n];
    float nnt = 1.0f - (float)last_done[n];
    for (int64_t t = T - 1; t >= 0; --t) {
        const int64_t o = t * N + n;
        const float v = val[o];
        const float delta = (rew[o] + (gamma * next_v) * nnt) - v;
        last = delta + (gl * nnt) * last;
        adv[o] = last;
        ret[o] = last + v;
        next_v = v;
        nnt = 1.0f - (float)starts[o];
    }
}

// Box-Muller on two 24-bit uniforms (u1 in (0,1]).
__device__ inline void box_muller(uint32_t a, uint32_t b, float &z0, float &z1) {
    const float u1 = ((float)(a >> 8) + 1.0f) * (1.0f / 16777216.0f);
    const float u2 = (float)(b >> 8) * (1.0f / 16777216.0f);
    const float r = sqrtf(-2.0f * logf(u1));
    float s, c;
    sincosf(6.2831853071795864769f * u2, &s, &c);
    z0 = r * c;
    z1 = r * s;
}

// a = mean + std * z; logp = sum_j Normal(mean_j, std_j).log_prob(a_j)
// (torch: -((a-mu)^2)/(2 var) - log(std) - log(sqrt(2 pi))); clip for env.
__global__ __launch_bounds__(kBlock) void policy_sample_kernel(
    int64_t n, const float4 *__restrict__ mean, const float *__restrict__ log_std,
    uint32_t k0, uint32_t k1, uint64_t counter, const uint64_t *__restrict__ counter_base,
    float lo, float hi, float4 *__restrict__ a_raw, float4 *__restrict__ a_clip,
    float *__restrict__ logp) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    // device-resident counter base: a captured rollout graph replays with
    // fresh noise each PPO iteration (the base advances outside the graph)
    if (counter_base) counter += *counter_base;
    const float ls[4] = {log_std[0], log_std[1], log_std[2], log_std[3]};
    const float4 mu = mean[i];
    const u32x4 r = philox4x32_10(
        u32x4{(uint32_t)i, (uint32_t)((uint64_t)i >> 32), (uint32_t)counter,
              TAG_NORMAL ^ (uint32_t)(counter >> 32)},
        k0, k1);
    float z[4];
    box_muller(r.x, r.y, z[0], z[1]);
    box_muller(r.z, r.w, z[2], z[3]);
    const float m[4] = {mu.x, mu.y, mu.z, mu.w};
    float a[4], lp = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float sd = expf(ls[j]);
        a[j] = m[j] + sd * z[j];
        const float d = a[j] - m[j];
        const float var = sd * sd;
#if DR_LOSS_RCP  // the same reciprocal as RowLossConst::inv_2var (the first epoch's ratio stays 1)
        lp += (-(d * d) * (1.0f / (2.0f * var)) - logf(sd)) - kLogSqrt2Pi;
#else
        lp += (-(d * d) / (2.0f * var) - logf(sd)) - kLogSqrt2Pi;
#endif
    }
    if (a_raw) a_raw[i] = make_float4(a[0], a[1], a[2], a[3]);
    if (a_clip)
        a_clip[i] = make_float4(fminf(fmaxf(a[0], lo), hi), fminf(fmaxf(a[1], lo), hi),
                                fminf(fmaxf(a[2], lo), hi), fminf(fmaxf(a[3], lo), hi));
    if (logp) logp[i] = lp;
}

// ---------------------------------------------------------------------------
// Minibatch permutation (RolloutBuffer.get's np.random.permutation): element
// i gets the 64-bit Philox key K_i = (r.x << 32) | r.y of counter (i,
// counter); the permutation is the order of (K_i, i), i.e. the stable argsort
// of the keys.  Built from four kernels that keep no state across launches
// (so a hipGraph replay is a fresh sort; rocPRIM's onesweep radix sort,
// used before, faulted on the second replay of a captured graph):
//   1. perm_hist:    B = 2^lgB buckets on the top lgB key bits (at most 1024
//                    elements per bucket on average); per-tile bucket counts
//                    (LDS histogram), keys written out;
//   2. perm_scan:    per bucket, the running count over tiles (exclusive)
//                    and the total; then one block scans the B totals;
//   3. perm_scatter: element ids to their bucket's range (a tile's slots
//                    of one bucket are claimed in any order -- step 4 fixes
//                    the order);
//   4. perm_sort:    one block per bucket sorts (key, id) with an
//                    all-ascending bitonic network in LDS (buckets above
//                    kPermCap elements -- probability ~e^-330 at the mean
//                    of 1024 -- sort in global scratch with the same code).
// Bucket order is key order, so the result is exactly the stable argsort.
// ---------------------------------------------------------------------------
constexpr int kPermCap = 2048;          // elements per bucket sorted in LDS
constexpr int kPermMaxLgB = 14;         // B <= 16384 (64 KB LDS histogram)

struct PermGeom {
    int64_t n, B, tile, T;
    int lgB;
};

PermGeom perm_geom(int64_t n) {
    PermGeom g{};
    g.n = n;
    g.lgB = 0;
    while (g.lgB < kPermMaxLgB && ((int64_t)1024 << g.lgB) < n) ++g.lgB;
    g.B = (int64_t)1 << g.lgB;
    g.tile = g.B * 4 > 4096 ? g.B * 4 : 4096;
    g.T = (n + g.tile - 1) / g.tile;
    return g;
}

__device__ inline uint64_t perm_key(int64_t i, uint32_t k0, uint32_t k1, uint64_t counter) {
    const u32x4 r = philox4x32_10(
        u32x4{(uint32_t)i, (uint32_t)((uint64_t)i >> 32), (uint32_t)counter,
              TAG_PERM ^ (uint32_t)(counter >> 32)},
        k0, k1);
    return ((uint64_t)r.x << 32) | r.y;
}

__device__ inline uint32_t perm_bucket(uint64_t key, int lgB) {
    return lgB ? (uint32_t)(key >> (64 - lgB)) : 0u;
}

__global__ __launch_bounds__(kBlock) void perm_hist_kernel(
    PermGeom g, uint32_t k0, uint32_t k1, uint64_t counter,
    const uint64_t *__restrict__ counter_base, uint64_t *__restrict__ keys,
    uint32_t *__restrict__ hist) {
    extern __shared__ uint32_t sh_cnt[];
    if (counter_base) counter += *counter_base;     // device-resident base (graphs)
    for (int64_t b = threadIdx.x; b < g.B; b += kBlock) sh_cnt[b] = 0;
    __syncthreads();
    const int64_t lo = (int64_t)blockIdx.x * g.tile;
    const int64_t hi = lo + g.tile < g.n ? lo + g.tile : g.n;
    for (int64_t i = lo + threadIdx.x; i < hi; i += kBlock) {
        const uint64_t key = perm_key(i, k0, k1, counter);
        keys[i] = key;
        atomicAdd(&sh_cnt[perm_bucket(key, g.lgB)], 1u);   // counts: order-free
    }
    __syncthreads();
    uint32_t *row = hist + (int64_t)blockIdx.x * g.B;
    for (int64_t b = threadIdx.x; b < g.B; b += kBlock) row[b] = sh_cnt[b];
}

// hist[t][b] -> exclusive running count over t; total[b].  A block owns 64
// buckets (coalesced 256 B rows of hist) and splits the tiles four ways; each
// thread reads its counts in chunks of 16 independent loads (the in-place
// rewrite would otherwise serialise every load behind the previous store).
constexpr int kScanChunk = 16;
__global__ __launch_bounds__(kBlock) void perm_scan_tiles_kernel(PermGeom g,
                                                                 uint32_t *__restrict__ hist,
                                                                 uint32_t *__restrict__ total) {
    __shared__ uint32_t part[4][64];
    const int bl = threadIdx.x & 63, grp = threadIdx.x >> 6;
    const int64_t b = (int64_t)blockIdx.x * 64 + bl;
    const int64_t tg = (g.T + 3) / 4;
    const int64_t t0 = grp * tg, t1 = t0 + tg < g.T ? t0 + tg : g.T;
    const bool ok = b < g.B;
    uint32_t s = 0;
    for (int64_t t = t0; t < t1; t += kScanChunk) {
        uint32_t c[kScanChunk];
#pragma unroll
        for (int q = 0; q < kScanChunk; ++q)
            c[q] = (ok && t + q < t1) ? hist[(t + q) * g.B + b] : 0u;
#pragma unroll
        for (int q = 0; q < kScanChunk; ++q) s += c[q];
    }
    part[grp][bl] = s;
    __syncthreads();
    uint32_t run = 0;
    for (int q = 0; q < grp; ++q) run += part[q][bl];
    if (ok && grp == 3) total[b] = run + s;
    for (int64_t t = t0; t < t1; t += kScanChunk) {
        uint32_t c[kScanChunk];
#pragma unroll
        for (int q = 0; q < kScanChunk; ++q)
            c[q] = (ok && t + q < t1) ? hist[(t + q) * g.B + b] : 0u;
#pragma unroll
        for (int q = 0; q < kScanChunk; ++q) {
            if (ok && t + q < t1) hist[(t + q) * g.B + b] = run;
            run += c[q];
        }
    }
}

// start[b] = exclusive scan of total, start[B] = n (one block of 1024)
__global__ __launch_bounds__(1024) void perm_scan_buckets_kernel(PermGeom g,
                                                                 const uint32_t *__restrict__ total,
                                                                 uint32_t *__restrict__ start) {
    __shared__ uint32_t part[1024];
    const int t = threadIdx.x;
    const int64_t per = (g.B + 1023) / 1024;
    const int64_t lo = t * per, hi = lo + per < g.B ? lo + per : g.B;
    uint32_t s = 0;
    for (int64_t b = lo; b < hi; ++b) s += total[b];
    part[t] = s;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {          // inclusive Hillis-Steele
        const uint32_t v = t >= off ? part[t - off] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint32_t run = part[t] - s;
    for (int64_t b = lo; b < hi; ++b) {
        start[b] = run;
        run += total[b];
    }
    if (t == 1023) start[g.B] = (uint32_t)g.n;
}

__global__ __launch_bounds__(kBlock) void perm_scatter_kernel(
    PermGeom g, const uint64_t *__restrict__ keys, const uint32_t *__restrict__ hist,
    const uint32_t *__restrict__ start, int32_t *__restrict__ ids) {
    extern __shared__ uint32_t sh_cur[];
    const uint32_t *row = hist + (int64_t)blockIdx.x * g.B;
    for (int64_t b = threadIdx.x; b < g.B; b += kBlock) sh_cur[b] = start[b] + row[b];
    __syncthreads();
    const int64_t lo = (int64_t)blockIdx.x * g.tile;
    const int64_t hi = lo + g.tile < g.n ? lo + g.tile : g.n;
    for (int64_t i = lo + threadIdx.x; i < hi; i += kBlock) {
        const uint32_t pos = atomicAdd(&sh_cur[perm_bucket(keys[i], g.lgB)], 1u);
        ids[pos] = (int32_t)i;
    }
}

__device__ inline bool perm_greater(uint64_t ka, int32_t ia, uint64_t kb, int32_t ib) {
    return ka > kb || (ka == kb && ia > ib);
}

// All-ascending bitonic sort of (key, id) pairs at [0, s), padded virtually
// to the next power of two with +inf: every comparator puts the minimum at
// the lower index, so padding (the suffix) never moves and is never read.
// In LDS, the steps whose pairs stay inside aligned 64-element segments (the
// first merge step while k <= 64, every later one with j <= 32) run wave-local
// -- each wave always owns the same segments and one wave's LDS operations
// execute in order -- so only the steps that cross segments pay a workgroup
// barrier (10 of 55 at 1,024 elements).  In global scratch every step ends
// with a barrier.
template <bool LDS, typename KP, typename IP>
__device__ inline void bitonic_sort_pairs(KP key, IP id, int64_t s64) {
    // k and j are powers of two: pair indices by shifts and masks (an int64
    // division per comparator cost more than the whole comparator)
    const int s = (int)s64;
    int lp = 0;
    while ((1 << lp) < s) ++lp;
    const int P = 1 << lp;
    auto cmpswap = [&](int lk, int lj, int p) {
        int lo, hi;
        if (lj == lk - 1) {          // first merge step: mirrored pairs
            const int blk = p >> lj, off = p & ((1 << lj) - 1);
            lo = (blk << lk) + off;
            hi = (blk << lk) + (1 << lk) - 1 - off;
        } else {
            lo = ((p >> lj) << (lj + 1)) + (p & ((1 << lj) - 1));
            hi = lo + (1 << lj);
        }
        if (hi < s) {
            const uint64_t ka = key[lo], kb = key[hi];
            const int32_t ia = id[lo], ib = id[hi];
            if (perm_greater(ka, ia, kb, ib)) {
                key[lo] = kb;
                key[hi] = ka;
                id[lo] = ib;
                id[hi] = ia;
            }
        }
    };
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nseg = (P + 63) / 64, seg_pairs = P < 64 ? P / 2 : 32;
    bool pending = false;            // wave-local writes not yet seen block-wide
    for (int lk = 1; lk <= lp; ++lk) {
        for (int lj = lk - 1; lj >= 0; --lj) {
            const bool local = LDS && (lj == lk - 1 ? lk <= 6 : lj <= 5);
            if (local) {
                // wave w: segments 2w + (lane >> 5) + 8 i, one pair per lane
                for (int seg = 2 * w + (lane >> 5); seg < nseg; seg += 2 * (kBlock / 64))
                    if ((lane & 31) < seg_pairs) cmpswap(lk, lj, seg * 32 + (lane & 31));
                __builtin_amdgcn_wave_barrier();
                asm volatile("" ::: "memory");   // no LDS access moves across
                pending = true;
            } else {
                if (pending) __syncthreads();
                pending = false;
                for (int p = threadIdx.x; p < P / 2; p += kBlock) cmpswap(lk, lj, p);
                __syncthreads();
            }
        }
    }
    if (pending) __syncthreads();
}

__global__ __launch_bounds__(kBlock) void perm_sort_kernel(
    PermGeom g, uint32_t k0, uint32_t k1, uint64_t counter,
    const uint64_t *__restrict__ counter_base, const uint32_t *__restrict__ start,
    int32_t *__restrict__ ids, uint64_t *__restrict__ gkeys, int32_t *__restrict__ out,
    int lds_cap) {
    __shared__ uint64_t sk[kPermCap];
    __shared__ int32_t si[kPermCap];
    if (counter_base) counter += *counter_base;
    const int64_t b = blockIdx.x;
    const int64_t base = start[b], s = (int64_t)start[b + 1] - base;
    if (s <= lds_cap) {
        for (int64_t k = threadIdx.x; k < s; k += kBlock) {
            const int32_t e = ids[base + k];
            si[k] = e;
            sk[k] = perm_key(e, k0, k1, counter);
        }
        __syncthreads();
        bitonic_sort_pairs<true>(sk, si, s);
        for (int64_t k = threadIdx.x; k < s; k += kBlock) out[base + k] = si[k];
    } else {
        // practically unreachable: the same network over global scratch
        // (the keys array is free again after the scatter)
        uint64_t *kk = gkeys + base;
        int32_t *ii = ids + base;
        for (int64_t k = threadIdx.x; k < s; k += kBlock) kk[k] = perm_key(ii[k], k0, k1, counter);
        __syncthreads();
        bitonic_sort_pairs<false>(kk, ii, s);
        for (int64_t k = threadIdx.x; k < s; k += kBlock) out[base + k] = ii[k];
    }
}

// dst[k, j] = src[idx[k], j]; one thread per output element (coalesced
// stores, gathered 4-byte loads from rows of `width` floats).
__global__ __launch_bounds__(kBlock) void gather_rows_kernel(
    int64_t m, int64_t width, const int32_t *__restrict__ idx,
    const float *__restrict__ src, float *__restrict__ dst) {
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= m * width) return;
    const int64_t k = e / width, j = e - k * width;
    dst[e] = src[(int64_t)idx[k] * width + j];
}

// --------------------------------------------------------------------------
// Tanh backward + bias gradient.  Block b owns rows [b*R, (b+1)*R); thread t
// owns 4 columns (float4) of one of 256/(n/4) row lanes; per-thread column
// partial sums are combined across the block's row lanes in LDS, giving one
// partial row per block; a second kernel sums the partial rows.
// --------------------------------------------------------------------------
constexpr int kTanhRows = 256;

__global__ __launch_bounds__(kBlock) void tanh_bwd_kernel(
    int64_t m, int n4, const float4 *__restrict__ gh, const float4 *__restrict__ h,
    float4 *__restrict__ gz, float4 *__restrict__ part) {
    __shared__ float4 red[kBlock];
    const int lanes = kBlock / n4;               // row lanes per block
    const int c = threadIdx.x % n4, rl = threadIdx.x / n4;
    const int64_t r0 = (int64_t)blockIdx.x * kTanhRows;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    constexpr int U = 8;                         // row pairs in flight per thread
    if (rl < lanes) {
        for (int r = rl; r < kTanhRows; r += U * lanes) {
            float4 g[U], y[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t row = r0 + r + u * lanes;
                const bool ok = (r + u * lanes < kTanhRows) && row < m;
                g[u] = ok ? gh[row * n4 + c] : make_float4(0.f, 0.f, 0.f, 0.f);
                y[u] = ok ? h[row * n4 + c] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t row = r0 + r + u * lanes;
                float4 z;
                z.x = g[u].x * (1.0f - y[u].x * y[u].x);
                z.y = g[u].y * (1.0f - y[u].y * y[u].y);
                z.z = g[u].z * (1.0f - y[u].z * y[u].z);
                z.w = g[u].w * (1.0f - y[u].w * y[u].w);
                if ((r + u * lanes < kTanhRows) && row < m) gz[row * n4 + c] = z;
                acc.x += z.x;
                acc.y += z.y;
                acc.z += z.z;
                acc.w += z.w;
            }
        }
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    if (rl == 0) {
        for (int k = 1; k < lanes; ++k) {
            const float4 v = red[k * n4 + c];
            acc.x += v.x;
            acc.y += v.y;
            acc.z += v.z;
            acc.w += v.w;
        }
        part[(int64_t)blockIdx.x * n4 + c] = acc;
    }
}

__global__ void colsum_kernel(int nb, int n, const float *__restrict__ part,
                              float *__restrict__ out) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    float s = 0.f;
#pragma unroll 16
    for (int b = 0; b < nb; ++b) s += part[(int64_t)b * n + j];
    out[j] = s;
}

// --------------------------------------------------------------------------
// Block reductions (wave64 shuffles, then LDS across the 4 waves).
// --------------------------------------------------------------------------
__device__ inline float wave_sum(float x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    return x;
}

template <int K>
__device__ inline void block_sum(float (&x)[K], float *sh /* K*4 */) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < K; ++k) x[k] = wave_sum(x[k]);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) sh[k * 4 + wid] = x[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k)
        x[k] = ((sh[k * 4 + 0] + sh[k * 4 + 1]) + sh[k * 4 + 2]) + sh[k * 4 + 3];
    __syncthreads();
}

// Pass 1 of the advantage normalisation: per-block (count, mean, M2)
// (Chan et al. parallel variance) -> partials[3*b].
__global__ __launch_bounds__(kBlock) void adv_stats_kernel(
    int64_t m, const float *__restrict__ adv, int64_t stride, const int32_t *__restrict__ rows,
    float *__restrict__ part) {
    __shared__ float sh[8];
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t cnt = min((int64_t)kBlock, m - (int64_t)blockIdx.x * kBlock);
    const float ai = i < m ? adv[(rows ? (int64_t)rows[i] : i) * stride] : 0.f;
    float x[1] = {ai};
    block_sum<1>(x, sh);
    const float mean = x[0] / (float)cnt;
    float d = i < m ? ai - mean : 0.f;
    float y[1] = {d * d};
    block_sum<1>(y, sh);
    if (threadIdx.x == 0) {
        part[3 * blockIdx.x + 0] = (float)cnt;
        part[3 * blockIdx.x + 1] = mean;
        part[3 * blockIdx.x + 2] = y[0];
    }
}

// One PPO.train minibatch formed in one launch (RolloutBuffer.get's
// indexing of obs, actions and the (old_logp, advantage, return) rows):
//   blocks [0, nb_obs)            obs elements, one thread per element;
//   blocks [nb_obs, +nb_rows)     action rows, one float4 per thread;
//   blocks [.., +nb_rows)         aux rows, one row per thread, plus the
//                                 advantage (count, mean, M2) partial of the
//                                 block's 256 rows -- the same rows, values
//                                 and reduction order as adv_stats_kernel, so
//                                 the partials are bitwise the same.
__global__ __launch_bounds__(kBlock) void gather_minibatch_kernel(
    int64_t m, int obs_dim, int nb_obs, int nb_rows, const int32_t *__restrict__ idx,
    const float *__restrict__ obs, const float4 *__restrict__ act,
    const float *__restrict__ aux, float *__restrict__ obs_out, float4 *__restrict__ act_out,
    float *__restrict__ aux_out, float *__restrict__ adv_part) {
    __shared__ float sh[8];
    int b = blockIdx.x;
    if (b < nb_obs) {
        const int64_t e = (int64_t)b * kBlock + threadIdx.x;
        if (e >= m * obs_dim) return;
        if (m * obs_dim <= (int64_t)UINT32_MAX) {
            // 32-bit element index: the row division is a few VALU, not the
            // ~40 of a 64-bit one
            const uint32_t e32 = (uint32_t)e, k = e32 / (uint32_t)obs_dim;
            obs_out[e] = obs[(int64_t)idx[k] * obs_dim + (e32 - k * (uint32_t)obs_dim)];
            return;
        }
        const int64_t k = e / obs_dim, j = e - k * obs_dim;
        obs_out[e] = obs[(int64_t)idx[k] * obs_dim + j];
        return;
    }
    b -= nb_obs;
    if (b < nb_rows) {
        const int64_t i = (int64_t)b * kBlock + threadIdx.x;
        if (i < m) act_out[i] = act[idx[i]];
        return;
    }
    b -= nb_rows;
    const int64_t i = (int64_t)b * kBlock + threadIdx.x;
    const int64_t cnt = min((int64_t)kBlock, m - (int64_t)b * kBlock);
    float ai = 0.f;
    if (i < m) {
        const int64_t r = idx[i];
        const float l = aux[3 * r], a = aux[3 * r + 1], ret = aux[3 * r + 2];
        aux_out[3 * i] = l;
        aux_out[3 * i + 1] = a;
        aux_out[3 * i + 2] = ret;
        ai = a;
    }
    if (!adv_part) return;
    float x[1] = {ai};
    block_sum<1>(x, sh);
    const float mean = x[0] / (float)cnt;
    float d = i < m ? ai - mean : 0.f;
    float y[1] = {d * d};
    block_sum<1>(y, sh);
    if (threadIdx.x == 0) {
        adv_part[3 * b + 0] = (float)cnt;
        adv_part[3 * b + 1] = mean;
        adv_part[3 * b + 2] = y[0];
    }
}

// ---------------------------------------------------------------------------
// One-line rollout records (round 6, verdict r05 item 5).  gather_minibatch_
// kernel reads each random rollout row from three arrays (60-B obs, 16-B
// action, 12-B aux), each in its own 128-B lines: 3.7 TCP -> TCC requests per
// row and 5.1x the algorithmic read bytes (profiles/r05_gather_pmc.json).
// pack_records_kernel writes every rollout row once per PPO iteration as one
// aligned 128-B record -- floats 0 .. d - 1 the obs (d = obs_dim <= 24), the
// action at rec_act_off(d) = 4 ceil(d / 4) (16 for the 15-d drone obs), the
// (old log-prob, advantage, return) triple right after it, the rest zero --
// and gather_records_kernel reads ONE line per gathered row.
constexpr int kRecF = DR_RECORD_FLOATS;          // 32 floats = 128 B
constexpr int kRecMaxObs = 24;
__host__ __device__ inline int rec_act_off(int d) { return 4 * ((d + 3) / 4); }

// thread (row, float4 slot s of 8): slot s holds floats 4 s .. 4 s + 3 of
// the record; the stores are contiguous
__global__ __launch_bounds__(kBlock) void pack_records_kernel(
    int64_t n, int obs_dim, const float *__restrict__ obs, const float4 *__restrict__ act,
    const float *__restrict__ logp, const float *__restrict__ adv, const float *__restrict__ ret,
    float4 *__restrict__ rec) {
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t row = t >> 3;
    const int s = (int)(t & 7);
    if (row >= n) return;
    const int ao = rec_act_off(obs_dim);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (4 * s < ao) {
        const float *o = obs + row * obs_dim;
        const int c = 4 * s;
        if (c + 0 < obs_dim) v.x = o[c + 0];
        if (c + 1 < obs_dim) v.y = o[c + 1];
        if (c + 2 < obs_dim) v.z = o[c + 2];
        if (c + 3 < obs_dim) v.w = o[c + 3];
    } else if (4 * s == ao) {
        v = act[row];
    } else if (4 * s == ao + 4) {
        v = make_float4(logp[row], adv[row], ret[row], 0.f);
    }
    rec[row * (kRecF / 4) + s] = v;
}

// One thread per gathered row (blocks of 256 rows, as the aux blocks of
// gather_minibatch_kernel): the record's first ao / 4 + 2 float4 (one
// line), the obs rows staged in LDS and written as contiguous float4, the
// action and aux rows stored directly, and the block's advantage (count,
// mean, M2) partial -- the same rows, values and reduction order as
// gather_minibatch_kernel, so every output byte is the same.
__global__ __launch_bounds__(kBlock) void gather_records_kernel(
    int64_t m, int obs_dim, const int32_t *__restrict__ idx, const float4 *__restrict__ rec,
    float *__restrict__ obs_out, float4 *__restrict__ act_out, float *__restrict__ aux_out,
    float *__restrict__ adv_part) {
    __shared__ float so[kBlock * kRecMaxObs];
    __shared__ float sh[8];
    const int b = blockIdx.x;
    const int64_t i0 = (int64_t)b * kBlock, i = i0 + threadIdx.x;
    const int cnt = (int)min((int64_t)kBlock, m - i0);
    const int aq = rec_act_off(obs_dim) / 4;       // the action's float4 slot
    float ai = 0.f;
    if (i < m) {
        const float4 *r = rec + (int64_t)idx[i] * (kRecF / 4);
        float4 q[8];
#pragma unroll
        for (int s = 0; s < 8; ++s)
            if (s <= aq + 1) q[s] = r[s];
#pragma unroll
        for (int s = 0; s < kRecMaxObs / 4; ++s) {
            const float o4[4] = {q[s].x, q[s].y, q[s].z, q[s].w};
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (4 * s + e < obs_dim) so[threadIdx.x * obs_dim + 4 * s + e] = o4[e];
        }
        float4 a4 = q[0], x4 = q[1];
#pragma unroll
        for (int s = 1; s < 7; ++s)
            if (s == aq) {
                a4 = q[s];
                x4 = q[s + 1];
            }
        act_out[i] = a4;
        aux_out[3 * i] = x4.x;
        aux_out[3 * i + 1] = x4.y;
        aux_out[3 * i + 2] = x4.z;
        ai = x4.y;
    }
    __syncthreads();
    // the block's cnt obs rows are cnt * obs_dim contiguous floats starting
    // at 256 * obs_dim * b floats (16-byte aligned: obs_out is)
    const int nf = cnt * obs_dim;
    float *dst = obs_out + i0 * obs_dim;
    for (int q = threadIdx.x; q < nf / 4; q += kBlock)
        reinterpret_cast<float4 *>(dst)[q] =
            make_float4(so[4 * q], so[4 * q + 1], so[4 * q + 2], so[4 * q + 3]);
    for (int q = (nf / 4) * 4 + threadIdx.x; q < nf; q += kBlock) dst[q] = so[q];
    if (!adv_part) return;
    float x[1] = {ai};
    block_sum<1>(x, sh);
    const float mean = x[0] / (float)cnt;
    float d = i < m ? ai - mean : 0.f;
    float y[1] = {d * d};
    block_sum<1>(y, sh);
    if (threadIdx.x == 0) {
        adv_part[3 * b + 0] = (float)cnt;
        adv_part[3 * b + 1] = mean;
        adv_part[3 * b + 2] = y[0];
    }
}

// Chan et al. merge of (n, mean, M2) b into a.
__device__ inline void chan_merge(double &n, double &mu, double &M2, double nb_, double mb,
                                  double m2b) {
    const double tot = n + nb_;
    if (tot == 0.0) return;
    const double dl = mb - mu;
    mu += dl * nb_ / tot;
    M2 += m2b + dl * dl * n * nb_ / tot;
    n = tot;
}

// Combine the per-block (n, mean, M2) partials with the whole block: strided
// per-thread merges, then a fixed-shape tree in LDS (deterministic).  Every
// thread returns the result.  Needs blockDim.x == kBlock.
__device__ inline void merge_stats_block(const float *part, int nb, float &mean,
                                         float &m2, float &count) {
    __shared__ double sn[kBlock], smu[kBlock], sm2[kBlock];
    const int t = threadIdx.x;
    double n = 0.0, mu = 0.0, M2 = 0.0;
    for (int b = t; b < nb; b += kBlock)
        chan_merge(n, mu, M2, part[3 * b], part[3 * b + 1], part[3 * b + 2]);
    sn[t] = n;
    smu[t] = mu;
    sm2[t] = M2;
    __syncthreads();
    for (int h = kBlock / 2; h > 0; h >>= 1) {
        if (t < h) {
            double a = sn[t], am = smu[t], a2 = sm2[t];
            chan_merge(a, am, a2, sn[t + h], smu[t + h], sm2[t + h]);
            sn[t] = a;
            smu[t] = am;
            sm2[t] = a2;
        }
        __syncthreads();
    }
    mean = (float)smu[0];
    m2 = (float)sm2[0];
    count = (float)sn[0];
}

// Fused PPO loss over a minibatch: per row the Gaussian log-prob of the
// taken action, ratio, clipped surrogate, value error; writes dLoss/dmean,
// dLoss/dvalue and per-block partial sums (loss terms, dLoss/dlog_std).
// Gradient conventions follow torch autograd of PPO.train's expression:
//  - min(l1, l2): a tie sends half the gradient to each branch;
//  - clamp(r, 1-e, 1+e): gradient 1 inside the closed interval, else 0.
struct LossArgs {
    int64_t m;
    const float4 *mean;
    const float *log_std;
    const float *values;
    const float4 *actions;
    const float *old_logp;
    const float *adv;
    const float *ret;
    int64_t stride;  // element stride of old_logp / adv / ret
    float clip, ent_coef, vf_coef;
    int normalize;
    const float *adv_part;  // 3 * nb partials from adv_stats_kernel
    int nb;
    float4 *grad_mean;
    float *grad_values;
    float *part;  // 12 * nb
};

constexpr int kLossK = 9;  // pl, vl, clipcnt, kl, g_ls[4], (spare)

// Per-row PPO loss terms and gradient, shared by ppo_loss_kernel and the
// fused head kernel so both compute bit-identical rows.
struct RowLossConst {
    float var[4], logsd[4];
    float inv_var[4], inv_2var[4];
    float lo, hi, clip, inv_m, vf_coef, amean, astd, inv_astd;
    int normalize;
};

__device__ inline RowLossConst row_loss_const(const float *log_std, float clip, float vf_coef,
                                              int64_t m, int normalize, float amean,
                                              float astd) {
    RowLossConst c;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float sd = expf(log_std[j]);
        c.var[j] = sd * sd;
        c.logsd[j] = logf(sd);
        c.inv_var[j] = 1.0f / c.var[j];
        c.inv_2var[j] = 1.0f / (2.0f * c.var[j]);
    }
    c.lo = 1.0f - clip;
    c.hi = 1.0f + clip;
    c.clip = clip;
    c.inv_m = 1.0f / (float)m;
    c.vf_coef = vf_coef;
    c.amean = amean;
    c.astd = astd;
    c.inv_astd = 1.0f / (astd + 1e-8f);
    c.normalize = normalize;
    return c;
}

// acc[0..8] += (-min(l1,l2), (R-V)^2, clipped, kl term, dL/dlog_std[4]);
// gm = dL/dmean (4), gv = dL/dvalue.  Gradient conventions follow torch
// autograd of PPO.train's expression: a min() tie sends half the gradient
// to each branch; clamp passes gradient inside the closed interval.
__device__ inline void ppo_row(const RowLossConst &c, const float mu[4], const float ac[4],
                               float old_lp, float A, float R, float v, float gm[4],
                               float &gv, float acc[kLossK]) {
    float lp = 0.f, zz[4], dd[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float d = ac[j] - mu[j];
        dd[j] = d;
#if DR_LOSS_RCP
        zz[j] = d * c.inv_var[j];         // d logp / d mu_j
        lp += (-(d * d) * c.inv_2var[j] - c.logsd[j]) - kLogSqrt2Pi;
#else
        zz[j] = d / c.var[j];             // d logp / d mu_j
        lp += (-(d * d) / (2.0f * c.var[j]) - c.logsd[j]) - kLogSqrt2Pi;
#endif
    }
#if DR_LOSS_RCP
    if (c.normalize) A = (A - c.amean) * c.inv_astd;
#else
    if (c.normalize) A = (A - c.amean) / (c.astd + 1e-8f);
#endif
    const float logr = lp - old_lp;
    const float r = expf(logr);
    const float rc = fminf(fmaxf(r, c.lo), c.hi);
    const float l1 = A * r, l2 = A * rc;
    acc[0] += -fminf(l1, l2);                          // policy_loss = -mean(min)
    const float g1 = l1 < l2 ? 1.f : (l1 == l2 ? 0.5f : 0.f);
    const float g2 = l2 < l1 ? 1.f : (l1 == l2 ? 0.5f : 0.f);
    const float dclamp = (r >= c.lo && r <= c.hi) ? 1.f : 0.f;
    const float dr = -(g1 * A + g2 * A * dclamp) * c.inv_m;  // dL/dratio
    const float dlp = dr * r;                                // dL/dlogp
    const float e = R - v;                                   // vf_coef * mean((R-V)^2)
    acc[1] += e * e;
    gv = c.vf_coef * (2.0f * (v - R)) * c.inv_m;
    acc[2] += (fabsf(r - 1.0f) > c.clip) ? 1.f : 0.f;
    acc[3] += (r - 1.0f) - logr;                             // approx_kl term
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        gm[j] = dlp * zz[j];
#if DR_LOSS_RCP
        acc[4 + j] += dlp * ((dd[j] * dd[j]) * c.inv_var[j] - 1.0f);  // d/dlog_std_j
#else
        acc[4 + j] += dlp * ((dd[j] * dd[j]) / c.var[j] - 1.0f);  // d/dlog_std_j
#endif
    }
}

// ppo_row's policy part (acc 0, 2, 3, 4..7 and gm) and value part (acc 1 and
// gv), operation for operation, for kernels that evaluate them on different
// waves.
__device__ inline void ppo_row_policy(const RowLossConst &c, const float mu[4],
                                      const float ac[4], float old_lp, float A, float gm[4],
                                      float acc[kLossK]) {
    float lp = 0.f, zz[4], dd[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float d = ac[j] - mu[j];
        dd[j] = d;
#if DR_LOSS_RCP
        zz[j] = d * c.inv_var[j];
        lp += (-(d * d) * c.inv_2var[j] - c.logsd[j]) - kLogSqrt2Pi;
#else
        zz[j] = d / c.var[j];
        lp += (-(d * d) / (2.0f * c.var[j]) - c.logsd[j]) - kLogSqrt2Pi;
#endif
    }
#if DR_LOSS_RCP
    if (c.normalize) A = (A - c.amean) * c.inv_astd;
#else
    if (c.normalize) A = (A - c.amean) / (c.astd + 1e-8f);
#endif
    const float logr = lp - old_lp;
    const float r = expf(logr);
    const float rc = fminf(fmaxf(r, c.lo), c.hi);
    const float l1 = A * r, l2 = A * rc;
    acc[0] += -fminf(l1, l2);
    const float g1 = l1 < l2 ? 1.f : (l1 == l2 ? 0.5f : 0.f);
    const float g2 = l2 < l1 ? 1.f : (l1 == l2 ? 0.5f : 0.f);
    const float dclamp = (r >= c.lo && r <= c.hi) ? 1.f : 0.f;
    const float dr = -(g1 * A + g2 * A * dclamp) * c.inv_m;
    const float dlp = dr * r;
    acc[2] += (fabsf(r - 1.0f) > c.clip) ? 1.f : 0.f;
    acc[3] += (r - 1.0f) - logr;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        gm[j] = dlp * zz[j];
#if DR_LOSS_RCP
        acc[4 + j] += dlp * ((dd[j] * dd[j]) * c.inv_var[j] - 1.0f);
#else
        acc[4 + j] += dlp * ((dd[j] * dd[j]) / c.var[j] - 1.0f);
#endif
    }
}

__device__ inline void ppo_row_value(const RowLossConst &c, float R, float v, float &gv,
                                     float acc[kLossK]) {
    const float e = R - v;
    acc[1] += e * e;
    gv = c.vf_coef * (2.0f * (v - R)) * c.inv_m;
}

__global__ __launch_bounds__(kBlock) void ppo_loss_kernel(LossArgs a) {
    __shared__ float sh[kLossK * 4];
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    float amean = 0.f, astd = 1.f;
    if (a.normalize) {
        float m2, cnt;
        merge_stats_block(a.adv_part, a.nb, amean, m2, cnt);
        // torch.std: unbiased (n-1); SB3 adds 1e-8 to std
        astd = sqrtf(m2 / (cnt - 1.0f));
    }
    const RowLossConst c = row_loss_const(a.log_std, a.clip, a.vf_coef, a.m, a.normalize,
                                          amean, astd);
    float acc[kLossK] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (i < a.m) {
        const float4 mu4 = a.mean[i], ac4 = a.actions[i];
        const float mu[4] = {mu4.x, mu4.y, mu4.z, mu4.w};
        const float ac[4] = {ac4.x, ac4.y, ac4.z, ac4.w};
        float gm[4], gv;
        ppo_row(c, mu, ac, a.old_logp[i * a.stride], a.adv[i * a.stride],
                a.ret[i * a.stride], a.values[i], gm, gv, acc);
        a.grad_values[i] = gv;
        a.grad_mean[i] = make_float4(gm[0], gm[1], gm[2], gm[3]);
    }
    block_sum<kLossK>(acc, sh);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < kLossK; ++k) a.part[kLossK * blockIdx.x + k] = acc[k];
        if (blockIdx.x == 0) {
            a.part[kLossK * gridDim.x + 0] = amean;
            a.part[kLossK * gridDim.x + 1] = astd;
        }
    }
}

// Final fixed-order combine: stats[8] and grad_log_std[4].
__global__ void ppo_loss_finish_kernel(int64_t m, int nb, const float *part,
                                       const float *log_std, float ent_coef,
                                       float vf_coef, float *grad_log_std,
                                       float *stats) {
    __shared__ float sh[kLossK * 4];
    float acc[kLossK];
#pragma unroll
    for (int k = 0; k < kLossK; ++k) acc[k] = 0.f;
    for (int b = threadIdx.x; b < nb; b += blockDim.x) {
#pragma unroll
        for (int k = 0; k < kLossK; ++k) acc[k] += part[kLossK * b + k];
    }
    block_sum<kLossK>(acc, sh);
    if (threadIdx.x == 0) {
        const float inv_m = 1.0f / (float)m;
        const float pl = acc[0] * inv_m;
        const float vl = acc[1] * inv_m;
        // entropy of the diagonal Gaussian is row-independent:
        // H = sum_j (0.5 + 0.5 log(2 pi) + log_std_j); entropy_loss = -H
        float H = 0.f;
        for (int j = 0; j < 4; ++j) H += 0.5f + kLogSqrt2Pi + log_std[j];
        const float el = -H;
        for (int j = 0; j < 4; ++j) grad_log_std[j] = acc[4 + j] - ent_coef;
        stats[0] = pl + ent_coef * el + vf_coef * vl;
        stats[1] = pl;
        stats[2] = vl;
        stats[3] = el;
        stats[4] = acc[2] * inv_m;
        stats[5] = acc[3] * inv_m;
        stats[6] = part[kLossK * nb + 0];
        stats[7] = part[kLossK * nb + 1];
    }
}

// ---------------------------------------------------------------------------
// Actor-critic MLP pieces around the hidden-layer GEMMs (which stay on
// hipBLASLt / MFMA).  One wave per row, lane l owning hidden columns
// [4l, 4l+4): a row of activations is one coalesced 16 B-per-lane access.
// ---------------------------------------------------------------------------
template <int CTRL>
__device__ inline float dpp_mov(float x) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), CTRL, 0xF, 0xF, true));
}

// Sum over the 64 lanes, returned wave-uniform.  Fixed butterfly order:
// quad xor 1, quad xor 2, half-row mirror, row mirror (DPP), xor 16
// (ds_swizzle), then lane 0 + lane 32.
__device__ inline float wave_allsum(float x) {
    x = x + dpp_mov<0xB1>(x);
    x = x + dpp_mov<0x4E>(x);
    x = x + dpp_mov<0x141>(x);
    x = x + dpp_mov<0x140>(x);
    x = x + __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(x), 0x401F));
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 0)) +
           __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 32));
}

// tanh_fast: common.h (shared with the first-layer-fused GEMM, gemm_x6.hip)

__device__ inline float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }

// Activation and grad_z rows (64 MB per net per minibatch): 1 = nontemporal
// stores.  With the library GEMMs (round 1) they measured faster
// (linear_tanh 23.9 -> 21.6 us, heads+loss 68.8 -> 66.2 us, the first-layer
// backward 31.8 -> 30.3 us); with the dr_gemm_x6 GEMMs reading these rows
// back, plain stores leave them in the Infinity Cache for those GEMMs:
// 6.000 -> 6.033 / 5.999 -> 6.056 updates/s (bench.py, same box), so 0.
// Round 4 (weight-stationary GEMMs): 6.46-6.48 with NT stores against
// 6.48-6.51 without (two alternating pairs, one box).
#ifndef DR_PPO_NT
#define DR_PPO_NT 0
#endif
__device__ inline void st4(float *p, float4 x) {
    if (DR_PPO_NT) store_nt(reinterpret_cast<float4 *>(p), x);
    else *reinterpret_cast<float4 *>(p) = x;
}
__device__ inline float4 tanh4(float4 v) {
#if DR_TANH_RAT
    const f32x2 lo = tanh_rat2(f32x2{v.x, v.y}), hi = tanh_rat2(f32x2{v.z, v.w});
    return make_float4(lo.x, lo.y, hi.x, hi.y);
#else
    return make_float4(tanh_fast(v.x), tanh_fast(v.y), tanh_fast(v.z), tanh_fast(v.w));
#endif
}
// z + b, as the GEMM epilogue would have added it (z already the full dot
// product; b = 0 adds exactly nothing)
__device__ inline float4 add4(float4 a, float4 b) {
    return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ inline float dot4(float4 a, float4 b) {
    return fmaf(a.w, b.w, fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)));
}

// h = tanh(x W^T + b) for a narrow input (the first layer: K = obs_dim),
// x (m,K), W (n,K), b (n), h (m,n), n % 4 == 0, n <= 256.  Memory-bound on
// the h write; replaces an addmm + a separate tanh pass over h.
// With gridDim.y == 2 the launch covers both MLPs (pi: blockIdx.y 0, vf: 1),
// which share the input rows: one launch and one tail instead of two.
struct LayerPair {
    const float *w[2];
    const float *b[2];
    float *h[2];
};

// The x6 GEMMs' operand images built by extra blocks of the first-layer
// forward launch (linear_tanh_kernel<K, true>, its last grid row): the
// 256 x 256 layer's weight images in both forms (split_weights_kernel's
// items) and, with ximg, the minibatch observation image of the fused
// input-gradient GEMM (split_x_kernel's items) -- two launches fewer per
// optimizer step, the same bytes.
struct X6Aux {
    const float *w256;         // (2, 256, 256): both nets' weights
    uint8_t *img;              // 2 x 2 x W_IMG: W^T forms, then W forms
    uint8_t *ximg;             // nullable
};
constexpr int kAuxWBlocks = 2 * XN * (XK / 8) / kBlock;    // per weight form

__device__ inline void x6_aux_block(int bx, int64_t m, int k, const float *__restrict__ x,
                                    const int32_t *__restrict__ rows, const X6Aux &aux) {
    if (bx < 2 * kAuxWBlocks) {
        split_weights_item(aux.w256, 2, 2, aux.img, (bx % kAuxWBlocks) * kBlock + threadIdx.x,
                           bx / kAuxWBlocks);
        return;
    }
    bx -= 2 * kAuxWBlocks;
    if (aux.ximg) split_x_item(x, rows, m, k, aux.ximg, (int64_t)bx * kBlock + threadIdx.x);
}

// (round 3 A/B, removed in round 4: two rows per wave and iteration measured
// 38.1 vs 37.6-37.8 us per call; the input row through per-lane loads and
// readlanes instead of scalar loads, slower)
// (diagnostic ablations of linear_tanh_kernel and the head kernel: scripts/micro/patches/ppo_diag.patch)
// minimum rows per block (4 waves) of linear_tanh_kernel (A/B knob)
#ifndef DR_LT_RPB
#define DR_LT_RPB 64
#endif
// blocks per net of linear_tanh_kernel (A/B knob)
#ifndef DR_LT_MAXB
#define DR_LT_MAXB 1024
#endif
template <int K, bool AUX>
__global__ __launch_bounds__(kBlock) void linear_tanh_kernel(int64_t m, int n,
                                                             const float *__restrict__ x,
                                                             const int32_t *__restrict__ rows,
                                                             LayerPair lp, X6Aux aux) {
    if constexpr (AUX) {
        if (blockIdx.y == gridDim.y - 1) {
            x6_aux_block(blockIdx.x, m, K, x, rows, aux);
            return;
        }
    }
    const float *__restrict__ w = lp.w[blockIdx.y];
    const float *__restrict__ b = lp.b[blockIdx.y];
    float *__restrict__ h = lp.h[blockIdx.y];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int c0 = 4 * lane;
    const bool act = c0 < n;
    // this lane's 4 weight rows are 4K contiguous floats: K float4 loads
    // (the flat parameter layout keeps every weight 16-byte aligned; the
    // ABI checks it)
    float wr[4][K], bb[4];
    {
        const float4 *w4 = reinterpret_cast<const float4 *>(w + (act ? c0 : 0) * K);
        float flat[4 * K];
#pragma unroll
        for (int t = 0; t < K; ++t) {
            const float4 v4 = w4[t];
            flat[4 * t + 0] = v4.x;
            flat[4 * t + 1] = v4.y;
            flat[4 * t + 2] = v4.z;
            flat[4 * t + 3] = v4.w;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            bb[q] = act ? b[c0 + q] : 0.f;
#pragma unroll
            for (int k = 0; k < K; ++k) wr[q][k] = flat[q * K + k];
        }
    }
    // rows are wave-strided; row r is wave-uniform, so its K inputs are
    // scalar loads straight into SGPRs (no per-lane load + K readlanes), the
    // next row's issued before this row's arithmetic
    const int64_t stride = (int64_t)gridDim.x * 4;
    int64_t r = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(wid);
    auto xrow = [&](int64_t q) -> int64_t { return rows ? (int64_t)rows[q] : q; };
    float xn[K];
    if (r < m) {
        const float *xr = x + xrow(r) * K;
#pragma unroll
        for (int k = 0; k < K; ++k) xn[k] = xr[k];
    }
    for (; r < m; r += stride) {
        float xv[K];
#pragma unroll
        for (int k = 0; k < K; ++k) xv[k] = xn[k];
        const int64_t rn = r + stride;
        if (rn < m) {
            const float *xr = x + xrow(rn) * K;
#pragma unroll
            for (int k = 0; k < K; ++k) xn[k] = xr[k];
        }
#if DR_TANH_RAT
        // the same fmaf chain per column, written as packed pairs (columns
        // 0-1, 2-3), and the pairs' rational tanh
        f32x2 a01 = {0.f, 0.f}, a23 = {0.f, 0.f};
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const f32x2 xk = {xv[k], xv[k]};
            a01 = pk_fma(xk, f32x2{wr[0][k], wr[1][k]}, a01);
            a23 = pk_fma(xk, f32x2{wr[2][k], wr[3][k]}, a23);
        }
        if (act) {
            const f32x2 t01 = tanh_rat2(a01 + f32x2{bb[0], bb[1]});
            const f32x2 t23 = tanh_rat2(a23 + f32x2{bb[2], bb[3]});
            st4(h + r * n + c0, make_float4(t01.x, t01.y, t23.x, t23.y));
        }
        continue;
#endif
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < K; ++k) {
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[q] = fmaf(xv[k], wr[q][k], acc[q]);
        }
        if (act)
            st4(h + r * n + c0,
                make_float4(tanh_fast(acc[0] + bb[0]), tanh_fast(acc[1] + bb[1]),
                            tanh_fast(acc[2] + bb[2]), tanh_fast(acc[3] + bb[3])));
    }
}

// Policy heads for inference (rollouts): mean = h_pi Wa^T + ba (m,4),
// value = h_vf Wv^T + bv (m).
__global__ __launch_bounds__(kBlock) void policy_heads_kernel(
    int64_t m, int hd, int preact, const float *__restrict__ h_pi, const float *__restrict__ h_vf,
    const float *__restrict__ zb_pi, const float *__restrict__ zb_vf,
    const float *__restrict__ w_act, const float *__restrict__ b_act,
    const float *__restrict__ w_val, const float *__restrict__ b_val,
    float4 *__restrict__ mean, float *__restrict__ value) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int c0 = 4 * lane;
    const bool act = c0 < hd;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    // the top hidden layer's bias, when its GEMM left it out (zb_*)
    const float4 zbp = (act && zb_pi) ? ld4(zb_pi + c0) : z4;
    const float4 zbv = (act && zb_vf) ? ld4(zb_vf + c0) : z4;
    float4 wa[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) wa[j] = act ? ld4(w_act + j * hd + c0) : z4;
    const float4 wv = act ? ld4(w_val + c0) : z4;
    for (int64_t r = (int64_t)blockIdx.x * 4 + wid; r < m; r += (int64_t)gridDim.x * 4) {
        float4 hp = act ? ld4(h_pi + r * hd + c0) : z4;
        float4 hv = act ? ld4(h_vf + r * hd + c0) : z4;
        if (preact) {         // inputs are pre-activations: the layer's tanh here
            hp = tanh4(add4(hp, zbp));
            hv = tanh4(add4(hv, zbv));
        }
        float d[5];
#pragma unroll
        for (int j = 0; j < 4; ++j) d[j] = wave_allsum(dot4(hp, wa[j]));
        d[4] = wave_allsum(dot4(hv, wv));
        if (lane == 0) {
            mean[r] = make_float4(d[0] + b_act[0], d[1] + b_act[1], d[2] + b_act[2],
                                  d[3] + b_act[3]);
            value[r] = d[4] + b_val[0];
        }
    }
}

// Fused heads + PPO loss + backward through the heads and the top tanh, for
// one minibatch.  Per row (one wave): mean / value from the top hidden
// activations, the PPO row loss (ppo_row) and its gradient, then
//   gz_pi = (g_mean Wa) * (1 - h_pi^2),  gz_vf = (g_v Wv) * (1 - h_vf^2)
// written for the hidden-layer backward, and per-block partial sums of every
// head parameter gradient, the top hidden biases and the loss terms.
// Partial layout per block (P = 14 + 7 h floats):
//   [0,9) loss terms, [9,13) d b_act, 13 d b_val, then d b_pi (h),
//   d b_vf (h), d W_act (4h, row-major), d W_val (h).
constexpr int kHeadFixed = 14;

struct HeadArgs {
    int64_t m;
    int hd;
    int preact;  // h_pi / h_vf are pre-activations z; the top tanh is applied here
    const float *h_pi, *h_vf;
    const float *zb_pi, *zb_vf;  // nullable: top-layer bias added to z before the tanh
    const float *w_act, *b_act, *w_val, *b_val, *log_std;
    const float4 *actions;
    const float *aux;  // (m,3): old_logp, advantage, return
    const int32_t *rows;  // nullable: minibatch row r reads actions / aux row rows[r]
    float clip, ent_coef, vf_coef;
    int normalize;
    const float *adv_part;
    int adv_nb;
    float *gz_pi, *gz_vf;
    float *part;
    int P;
};

// Roles: waves 0-1 of a block run the policy head (4 mean outputs, the
// clipped-surrogate terms, log_std), waves 2-3 the value head, each over its
// own net's top activations only (the two heads share no row data once the
// advantage statistics are known).  Per wave, rows come in tiles of
// kHeadTile: the tile's activations stay in registers, the head dot products
// are wave reductions, the row results are parked one row per lane, the row
// loss runs once for the whole tile lane-parallel, and the per-row gradients
// come back by v_readlane for the backward through the head and the top
// tanh.  Splitting the nets by wave, with 4-row tiles, brings a wave to 126
// VGPRs (243 with both nets and 8-row tiles), so 4 waves per SIMD stay
// resident instead of 2: 66.4 -> 57.5 us per 65,536-row minibatch
// (rocprofv3, scripts/micro/ppo_prof.sh; 8-row tiles with the split: 65.6).
#ifndef DR_HEAD_TILE
#define DR_HEAD_TILE 4
#endif
constexpr int kHeadTile = DR_HEAD_TILE;
// (round 3 A/B, removed in round 4: the next tile's activation rows loaded
// while this tile computes, +16 VGPRs per wave, slower)

// policy waves: accumulate u[0], u[2..7] (loss terms), u[9..12] (d b_act),
// and per lane d b_pi (4 columns) and d W_act (4 x 4)
__device__ inline void head_policy_wave(const HeadArgs &a, const RowLossConst &c, int lane,
                                        int64_t tile0, int64_t tstride, float u[kHeadFixed],
                                        float sb[4], float sw[4][4]) {
    const int hd = a.hd, c0 = 4 * lane;
    const bool act = c0 < hd;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 wa[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) wa[j] = act ? ld4(a.w_act + j * hd + c0) : z4;
    const float4 zb = (act && a.zb_pi) ? ld4(a.zb_pi + c0) : z4;
    const float ba[4] = {a.b_act[0], a.b_act[1], a.b_act[2], a.b_act[3]};
    for (int64_t tile = tile0; tile * kHeadTile < a.m; tile += tstride) {
        const int64_t r0 = tile * kHeadTile;
        const int nr = (int)min((int64_t)kHeadTile, a.m - r0);
        float4 h[kHeadTile];
#pragma unroll
        for (int i = 0; i < kHeadTile; ++i)
            h[i] = (act && i < nr) ? ld4(a.h_pi + (r0 + i) * hd + c0) : z4;
        // this lane's row (lane < nr): its loss inputs, loaded while the dots run
        const bool own = lane < nr;
        const int64_t rr = r0 + (own ? lane : 0);
        const int64_t ro = a.rows ? (int64_t)a.rows[rr] : rr;
        const float4 ac4 = a.actions[ro];
        const float lp_old = a.aux[3 * ro], A = a.aux[3 * ro + 1];
        if (a.preact) {
#pragma unroll
            for (int i = 0; i < kHeadTile; ++i)
                h[i] = tanh4(add4(h[i], zb));
        }
        float mu[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < kHeadTile; ++i) {
            const bool me = lane == i;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float mj = wave_allsum(dot4(h[i], wa[j])) + ba[j];
                mu[j] = me ? mj : mu[j];
            }
        }
        float gm[4] = {0.f, 0.f, 0.f, 0.f};
        if (own) {
            const float ac[4] = {ac4.x, ac4.y, ac4.z, ac4.w};
            ppo_row_policy(c, mu, ac, lp_old, A, gm, u);
#pragma unroll
            for (int j = 0; j < 4; ++j) u[9 + j] += gm[j];
        }
        const float wq[4][4] = {{wa[0].x, wa[0].y, wa[0].z, wa[0].w},
                                {wa[1].x, wa[1].y, wa[1].z, wa[1].w},
                                {wa[2].x, wa[2].y, wa[2].z, wa[2].w},
                                {wa[3].x, wa[3].y, wa[3].z, wa[3].w}};
#pragma unroll
        for (int i = 0; i < kHeadTile; ++i) {
            // rows past the end (last tile only) carry zero activations and
            // zero gradients (gm = 0 on lanes >= nr): no effect on the sums
            float g[4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
                g[j] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(gm[j]), i));
            const float hq[4] = {h[i].x, h[i].y, h[i].z, h[i].w};
            float gz[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float gh = fmaf(g[3], wq[3][q], fmaf(g[2], wq[2][q],
                                      fmaf(g[1], wq[1][q], g[0] * wq[0][q])));
                gz[q] = gh * (1.0f - hq[q] * hq[q]);
                sb[q] += gz[q];
#pragma unroll
                for (int j = 0; j < 4; ++j) sw[j][q] = fmaf(g[j], hq[q], sw[j][q]);
            }
            if (act && i < nr)
                st4(a.gz_pi + (r0 + i) * hd + c0, make_float4(gz[0], gz[1], gz[2], gz[3]));
        }
    }
}

// value waves: accumulate u[1] (value-loss term), u[13] (d b_val), and per
// lane d b_vf (4 columns) and d W_val (4)
__device__ inline void head_value_wave(const HeadArgs &a, const RowLossConst &c, int lane,
                                       int64_t tile0, int64_t tstride, float u[kHeadFixed],
                                       float sb[4], float sw[4]) {
    const int hd = a.hd, c0 = 4 * lane;
    const bool act = c0 < hd;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    const float4 wv = act ? ld4(a.w_val + c0) : z4;
    const float4 zb = (act && a.zb_vf) ? ld4(a.zb_vf + c0) : z4;
    const float bv = a.b_val[0];
    const float wvq[4] = {wv.x, wv.y, wv.z, wv.w};
    for (int64_t tile = tile0; tile * kHeadTile < a.m; tile += tstride) {
        const int64_t r0 = tile * kHeadTile;
        const int nr = (int)min((int64_t)kHeadTile, a.m - r0);
        float4 h[kHeadTile];
#pragma unroll
        for (int i = 0; i < kHeadTile; ++i)
            h[i] = (act && i < nr) ? ld4(a.h_vf + (r0 + i) * hd + c0) : z4;
        const bool own = lane < nr;
        const int64_t rr = r0 + (own ? lane : 0);
        const int64_t ro = a.rows ? (int64_t)a.rows[rr] : rr;
        const float R = a.aux[3 * ro + 2];
        if (a.preact) {
#pragma unroll
            for (int i = 0; i < kHeadTile; ++i)
                h[i] = tanh4(add4(h[i], zb));
        }
        float v = 0.f;
#pragma unroll
        for (int i = 0; i < kHeadTile; ++i) {
            const float vv = wave_allsum(dot4(h[i], wv)) + bv;
            v = lane == i ? vv : v;
        }
        float gv = 0.f;
        if (own) {
            ppo_row_value(c, R, v, gv, u);
            u[13] += gv;
        }
#pragma unroll
        for (int i = 0; i < kHeadTile; ++i) {
            const float gvi = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(gv), i));
            const float hq[4] = {h[i].x, h[i].y, h[i].z, h[i].w};
            float gz[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                gz[q] = (gvi * wvq[q]) * (1.0f - hq[q] * hq[q]);
                sb[q] += gz[q];
                sw[q] = fmaf(gvi, hq[q], sw[q]);
            }
            if (act && i < nr)
                st4(a.gz_vf + (r0 + i) * hd + c0, make_float4(gz[0], gz[1], gz[2], gz[3]));
        }
    }
}

__global__ __launch_bounds__(kBlock) void ppo_head_kernel(HeadArgs a) {
    extern __shared__ float sh_part[];  // 4 * P
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int hd = a.hd, c0 = 4 * lane;
    const bool act = c0 < hd;
    float amean = 0.f, astd = 1.f;
    if (a.normalize) {
        float m2, cnt;
        merge_stats_block(a.adv_part, a.adv_nb, amean, m2, cnt);
        astd = sqrtf(m2 / (cnt - 1.0f));
    }
    const RowLossConst c = row_loss_const(a.log_std, a.clip, a.vf_coef, a.m, a.normalize,
                                          amean, astd);
    // lane-partial sums of the loss terms and of d b_act / d b_val
    float u[kHeadFixed];
#pragma unroll
    for (int k = 0; k < kHeadFixed; ++k) u[k] = 0.f;
    float sb[4] = {0.f, 0.f, 0.f, 0.f};
    float sw[4][4] = {};
    const bool policy = wid < 2;
    const int64_t tile0 = (int64_t)blockIdx.x * 2 + (wid & 1), tstride = (int64_t)gridDim.x * 2;
    if (policy)
        head_policy_wave(a, c, lane, tile0, tstride, u, sb, sw);
    else
        head_value_wave(a, c, lane, tile0, tstride, u, sb, sw[0]);
    // the lane-partial scalars to wave totals (fixed butterfly order)
#pragma unroll
    for (int k = 0; k < kHeadFixed; ++k) u[k] = wave_allsum(u[k]);
    float *mine = sh_part + wid * a.P;
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < kHeadFixed; ++k) mine[k] = u[k];
    }
    if (act) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            mine[kHeadFixed + c0 + q] = policy ? sb[q] : 0.f;
            mine[kHeadFixed + hd + c0 + q] = policy ? 0.f : sb[q];
#pragma unroll
            for (int j = 0; j < 4; ++j)
                mine[kHeadFixed + 2 * hd + j * hd + c0 + q] = policy ? sw[j][q] : 0.f;
            mine[kHeadFixed + 6 * hd + c0 + q] = policy ? 0.f : sw[0][q];
        }
    }
    __syncthreads();
    const int P = a.P;
    for (int p = threadIdx.x; p < P; p += kBlock)
        a.part[(int64_t)blockIdx.x * P + p] =
            ((sh_part[p] + sh_part[P + p]) + sh_part[2 * P + p]) + sh_part[3 * P + p];
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        a.part[(int64_t)gridDim.x * P + 0] = amean;
        a.part[(int64_t)gridDim.x * P + 1] = astd;
    }
}

// Backward of the first (narrow-input) layer, fused: grad_z = grad_h *
// (1 - h^2) is formed in registers and never stored; per-block partials of
// d b = sum_r grad_z[r,:] and d W = grad_z^T x (n x K) are written instead.
// Replaces tanh_backward (write of grad_z) + the split-K weight-gradient
// GEMM (re-read of grad_z).  Tiles of kFirstTile rows per wave, loads first.
// Partial layout per block (P = (K+1) n): [k*n + c] = dW[c][k], [K*n + c] = db[c].
// A/B build knobs of first_layer_bwd_kernel: rows per tile and the cap on
// blocks per net (scripts/micro/ab_ppo_kern.sh).  4-row tiles fit 115 VGPRs
// and a two-slot LDS reduction 32 KB, so 4 waves per SIMD are resident: 59.0
// -> 56.3 us per minibatch against 8-row tiles / four slots (152 VGPRs, 64
// KB, 2 waves); a next-tile prefetch needed 203 VGPRs and was slower (64.7
// us; removed in round 4 with the four-slot form).
#ifndef DR_FL_TILE
#define DR_FL_TILE 4
#endif
constexpr int kFirstTile = DR_FL_TILE;
// 256 blocks per net (round 3): 52.5-53.2 vs 54.2-54.7 us per minibatch at
// 512 (scripts/micro/round3_z.sh), fewer partials for the deferred finish
#ifndef DR_FL_MAXB
#define DR_FL_MAXB 256
#endif

// With gridDim.y == 2 the launch covers both MLPs (blockIdx.y = net); block
// b of net j writes partial row b * gridDim.y + j, so one column-sum pass
// over (gridDim.y * P)-wide rows reduces both nets.
struct FirstBwdIn {
    const float *gh[2];
    const float *h[2];
};

template <int K>
__global__ __launch_bounds__(kBlock) void first_layer_bwd_kernel(int64_t m, int n,
                                                                 FirstBwdIn in,
                                                                 const float *__restrict__ x,
                                                                 const int32_t *__restrict__ rows,
                                                                 float *__restrict__ part) {
    extern __shared__ float sh_fl[];  // 4 * P
    const float *__restrict__ gh = in.gh[blockIdx.y];
    const float *__restrict__ h = in.h[blockIdx.y];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int c0 = 4 * lane;
    const bool act = c0 < n;
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    float aw[K][4], ab[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
        for (int q = 0; q < 4; ++q) aw[k][q] = 0.f;
    const int64_t nwaves = (int64_t)gridDim.x * 4;
    // loads of one tile: grad_h and h rows (float4 per lane), x row k on lane k
    auto load_tile = [=](int64_t tile, float4 *g, float4 *y, float *xv) {
        const int64_t r0 = tile * kFirstTile;
        const int nr = (int)min((int64_t)kFirstTile, m - r0);
#pragma unroll
        for (int i = 0; i < kFirstTile; ++i) {
            const bool ok = act && i < nr;
            g[i] = ok ? ld4(gh + (r0 + i) * n + c0) : z4;
            y[i] = ok ? ld4(h + (r0 + i) * n + c0) : z4;
            const int64_t xr = rows ? (int64_t)rows[min(r0 + i, m - 1)] : r0 + i;
            xv[i] = (i < nr && lane < K) ? x[xr * K + lane] : 0.f;
        }
    };
    auto use_tile = [&](const float4 *g, const float4 *y, const float *xv) {
#pragma unroll
        for (int i = 0; i < kFirstTile; ++i) {
            const float gq[4] = {g[i].x, g[i].y, g[i].z, g[i].w};
            const float yq[4] = {y[i].x, y[i].y, y[i].z, y[i].w};
            float gz[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                gz[q] = gq[q] * (1.0f - yq[q] * yq[q]);
                ab[q] += gz[q];
            }
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const float xk =
                    __int_as_float(__builtin_amdgcn_readlane(__float_as_int(xv[i]), k));
#pragma unroll
                for (int q = 0; q < 4; ++q) aw[k][q] = fmaf(gz[q], xk, aw[k][q]);
            }
        }
    };
    for (int64_t tile = (int64_t)blockIdx.x * 4 + wid; tile * kFirstTile < m; tile += nwaves) {
        float4 g[kFirstTile], y[kFirstTile];
        float xv[kFirstTile];
        load_tile(tile, g, y, xv);
        use_tile(g, y, xv);
    }
    const int P = (K + 1) * n;
    float *__restrict__ out = part + ((int64_t)blockIdx.x * gridDim.y + blockIdx.y) * P;
    // two slots of P: waves 2 / 3 park their partials, waves 0 / 1 fold theirs
    // in, then the two slots are summed (half the LDS of four slots, so the
    // LDS no longer caps the CU at two blocks)
    float *slot = sh_fl + (wid & 1) * P;
    if (wid >= 2 && act) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
#pragma unroll
            for (int k = 0; k < K; ++k) slot[k * n + c0 + q] = aw[k][q];
            slot[K * n + c0 + q] = ab[q];
        }
    }
    __syncthreads();
    if (wid < 2 && act) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
#pragma unroll
            for (int k = 0; k < K; ++k) slot[k * n + c0 + q] = aw[k][q] + slot[k * n + c0 + q];
            slot[K * n + c0 + q] = ab[q] + slot[K * n + c0 + q];
        }
    }
    __syncthreads();
    for (int p = threadIdx.x; p < P; p += kBlock) out[p] = sh_fl[p] + sh_fl[P + p];
}

// Sum of the grouped partials (ng rows of nets * P) scattered to d W (n,K)
// row-major and d b (n) of each net.
struct FirstBwdOut {
    float *gw[2];
    float *gb[2];
};

// One thread's share of the first-layer finish (see first_layer_finish_kernel);
// returns the square of the gradient entry it wrote.
__device__ inline float first_finish_part(int bx, int ng, int n, int K, int nets,
                                          const float *__restrict__ part, const FirstBwdOut &o) {
    const int P1 = (K + 1) * n;
    const int P = nets * P1;
    const int pp = bx * kBlock + threadIdx.x;
    if (pp >= P) return 0.f;
    const int net = pp >= P1 ? 1 : 0;
    const int p = pp - net * P1;
    float s0 = 0.f, s1 = 0.f;
    int g = 0;
    for (; g + 1 < ng; g += 2) {
        s0 += part[(int64_t)g * P + pp];
        s1 += part[(int64_t)(g + 1) * P + pp];
    }
    if (g < ng) s0 += part[(int64_t)g * P + pp];
    const float s = s0 + s1;
    const int k = p / n, c = p - k * n;
    if (k < K) o.gw[net][c * K + k] = s;
    else o.gb[net][c] = s;
    return s * s;
}

// The same finish from `rows` level-1 partial rows (dr_gemm_x6_bwd_first's
// per-block rows, no grouping launch): a block takes 64 entries, its four
// waves a quarter of the rows each (8 accumulators, 32 loads in flight per
// lane at 128 rows), combined in LDS in a fixed order.
__device__ inline float first_finish_direct(int bx, int rows, int n, int K, int nets,
                                            const float *__restrict__ part, const FirstBwdOut &o) {
    __shared__ float red[4][64];
    const int P1 = (K + 1) * n;
    const int P = nets * P1;
    const int col = threadIdx.x & 63, q = threadIdx.x >> 6;
    const int pp = bx * 64 + col;
    float s = 0.f;
    if (pp < P) {
        const int lo = q * rows / 4, hi = (q + 1) * rows / 4;
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        int r = lo;
        for (; r + 8 <= hi; r += 8) {
#pragma unroll
            for (int u = 0; u < 8; ++u) acc[u] += part[(int64_t)(r + u) * P + pp];
        }
        for (; r < hi; ++r) acc[0] += part[(int64_t)r * P + pp];
        s = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    }
    red[q][col] = s;
    __syncthreads();
    if (q != 0 || pp >= P) return 0.f;
    const float t = (red[0][col] + red[1][col]) + (red[2][col] + red[3][col]);
    const int net = pp >= P1 ? 1 : 0;
    const int p = pp - net * P1;
    const int k = p / n, c = p - k * n;
    if (k < K) o.gw[net][c * K + k] = t;
    else o.gb[net][c] = t;
    return t * t;
}

__global__ __launch_bounds__(kBlock) void first_layer_finish_kernel(int ng, int n, int K,
                                                                    int nets,
                                                                    const float *__restrict__ part,
                                                                    FirstBwdOut o) {
    (void)first_finish_part(blockIdx.x, ng, n, K, nets, part, o);
}

// Gradient outputs of the head step (finish kernel).
struct HeadOut {
    float *g_w_act, *g_b_act, *g_w_val, *g_b_val, *g_b_pi, *g_b_vf, *g_log_std, *stats;
};

// Fixed-order column sums of row groups: out[g][p] = sum of in[b][p] over
// b in [g*gsize, (g+1)*gsize); 8 independent accumulators per thread.
__device__ inline float colsum_range(const float *__restrict__ in, int P, int p, int b0, int b1) {
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int b = b0;
    for (; b + 7 < b1; b += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u) s[u] += in[(int64_t)(b + u) * P + p];
    }
    for (; b < b1; ++b) s[0] += in[(int64_t)b * P + p];
    return ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
}

__global__ __launch_bounds__(kBlock) void colsum_groups_kernel(int nb, int P, int gsize,
                                                               const float *__restrict__ in,
                                                               float *__restrict__ out) {
    const int p = blockIdx.x * kBlock + threadIdx.x;
    if (p >= P) return;
    const int b0 = blockIdx.y * gsize;
    out[(int64_t)blockIdx.y * P + p] = colsum_range(in, P, p, b0, min(nb, b0 + gsize));
}

// first-level row groups of the partial sums (32 / 64 measured 6.62-6.69 vs
// 6.67-6.72 PPO updates/s, round 4)
constexpr int kHeadGroups = 16;

// Entry p of the head's reduced partials to its output (the loss terms to
// `loss`); returns its square for the norm.
__device__ inline float head_store(int p, float s, int hd, float *loss, const HeadOut &o) {
    if (p < kLossK) {
        loss[p] = s;
        return 0.f;
    }
    if (p < 13) {
        o.g_b_act[p - 9] = s;
    } else if (p == 13) {
        o.g_b_val[0] = s;
    } else {
        const int q = p - kHeadFixed;
        if (q < hd) o.g_b_pi[q] = s;
        else if (q < 2 * hd) o.g_b_vf[q - hd] = s;
        else if (q < 6 * hd) o.g_w_act[q - 2 * hd] = s;
        else o.g_w_val[q - 6 * hd] = s;
    }
    return s * s;
}

// Block 0's tail: the loss statistics and the log_std gradient (their
// squares for the norm, from thread 0).
__device__ inline float head_stats(const float *loss, int64_t m, const float *__restrict__ adv_ms,
                                   const float *__restrict__ log_std, float ent_coef,
                                   float vf_coef, const HeadOut &o) {
    float sq = 0.f;
    __syncthreads();
    if (threadIdx.x == 0) {
        const float inv_m = 1.0f / (float)m;
        const float pl = loss[0] * inv_m;
        const float vl = loss[1] * inv_m;
        float H = 0.f;
        for (int j = 0; j < 4; ++j) H += 0.5f + kLogSqrt2Pi + log_std[j];
        const float el = -H;
        for (int j = 0; j < 4; ++j) {
            const float g = loss[4 + j] - ent_coef;
            o.g_log_std[j] = g;
            sq += g * g;
        }
        o.stats[0] = pl + ent_coef * el + vf_coef * vl;
        o.stats[1] = pl;
        o.stats[2] = vl;
        o.stats[3] = el;
        o.stats[4] = loss[2] * inv_m;
        o.stats[5] = loss[3] * inv_m;
        o.stats[6] = adv_ms[0];
        o.stats[7] = adv_ms[1];
    }
    return sq;
}

// One thread's share of the head-gradient finish: the level-2 sum of the
// grouped partials, scattered to the gradient outputs; block bx == 0 also
// forms the loss statistics and the log_std gradient.  Returns the sum of
// squares of the gradient entries this thread wrote (for the norm).
__device__ inline float head_finish_part(int bx, int nb, int P, int hd, int64_t m,
                                         const float *__restrict__ part,
                                         const float *__restrict__ adv_ms,
                                         const float *__restrict__ log_std, float ent_coef,
                                         float vf_coef, const HeadOut &o) {
    __shared__ float loss[kLossK];
    float sq = 0.f;
    const int p = bx * kBlock + threadIdx.x;
    if (p < P) {
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
        int b = 0;
        for (; b + 3 < nb; b += 4) {
            s0 += part[(int64_t)(b + 0) * P + p];
            s1 += part[(int64_t)(b + 1) * P + p];
            s2 += part[(int64_t)(b + 2) * P + p];
            s3 += part[(int64_t)(b + 3) * P + p];
        }
        for (; b < nb; ++b) s0 += part[(int64_t)b * P + p];
        sq = head_store(p, ((s0 + s1) + s2) + s3, hd, loss, o);
    }
    if (bx == 0) sq += head_stats(loss, m, adv_ms, log_std, ent_coef, vf_coef, o);
    return sq;
}

// The head finish from the kernel's nb per-block rows (no grouping launch):
// a block takes 16 entries, its 16 row slices the level-1 groups of the
// grouped path (colsum_range over the same rows), and slice 0 the level-2
// sum in head_finish_part's order: bitwise the grouped path's values.
__device__ inline float head_finish_direct(int bx, int nb, int P, int hd, int64_t m,
                                           const float *__restrict__ part,
                                           const float *__restrict__ adv_ms,
                                           const float *__restrict__ log_std, float ent_coef,
                                           float vf_coef, const HeadOut &o) {
    __shared__ float loss[kLossK];
    __shared__ float red[kHeadGroups][16];
    const int col = threadIdx.x & 15, q = threadIdx.x >> 4;
    const int p = bx * 16 + col;
    const int gsize = (nb + kHeadGroups - 1) / kHeadGroups;
    const int ng = (nb + gsize - 1) / gsize;
    if (p < P && q < ng) {
        const int b0 = q * gsize, b1 = min(nb, b0 + gsize);
        if (b1 - b0 == 64) {
            // the full 64-row group (65,536-row minibatches): every load
            // issued before the sums, which keep colsum_range's order
            float v[64];
#pragma unroll
            for (int r = 0; r < 64; ++r) v[r] = part[(int64_t)(b0 + r) * P + p];
            float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int u = 0; u < 8; ++u) s[u] += v[8 * i + u];
            red[q][col] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
        } else {
            red[q][col] = colsum_range(part, P, p, b0, b1);
        }
    }
    __syncthreads();
    float sq = 0.f;
    if (q == 0 && p < P) {
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
        int b = 0;
        for (; b + 3 < ng; b += 4) {
            s0 += red[b + 0][col];
            s1 += red[b + 1][col];
            s2 += red[b + 2][col];
            s3 += red[b + 3][col];
        }
        for (; b < ng; ++b) s0 += red[b][col];
        sq = head_store(p, ((s0 + s1) + s2) + s3, hd, loss, o);
    }
    if (bx == 0) sq += head_stats(loss, m, adv_ms, log_std, ent_coef, vf_coef, o);
    return sq;
}

__global__ __launch_bounds__(kBlock) void ppo_head_finish_kernel(
    int nb, int P, int hd, int64_t m, const float *__restrict__ part,
    const float *__restrict__ adv_ms, const float *__restrict__ log_std, float ent_coef,
    float vf_coef, HeadOut o) {
    (void)head_finish_part(blockIdx.x, nb, P, hd, m, part, adv_ms, log_std, ent_coef, vf_coef,
                           o);
}


inline int head_blocks(int64_t m) {
    const int64_t b = (m + 4 * kHeadTile - 1) / (4 * kHeadTile);  // >= 1 tile per wave
    return (int)(b < 512 ? b : 512);
}

// ppo_head_kernel: 2 row tiles per block and round (one per wave of a role)
inline int loss_head_blocks(int64_t m) {
    const int64_t b = (m + 2 * kHeadTile - 1) / (2 * kHeadTile);
    return (int)(b < 1024 ? b : 1024);
}

// ---------------------------------------------------------------------------
// clip_grad_norm_ + Adam over one flat fp32 buffer.
// ---------------------------------------------------------------------------
// `scale` multiplies every entry first (1 / world for a summed data-parallel
// gradient; x * 1 is x bitwise, so the single-GPU path is unchanged).
__global__ __launch_bounds__(kBlock) void sumsq_kernel(int64_t n,
                                                       const float *__restrict__ g,
                                                       float *__restrict__ part, float scale) {
    __shared__ float sh[4];
    float acc = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kBlock) {
        const float x = g[i] * scale;
        acc += x * x;
    }
    float x[1] = {acc};
    block_sum<1>(x, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = x[0];
}

// Split-K chunk sum: dst[g*size + i] = sum_c chunks[(g*count + c)*size + i],
// fixed order (16 independent accumulators, then a fixed tree); returns the
// square of the value written.
__device__ inline float chunk_sum_part(int bx, int64_t groups, int count, int64_t size,
                                       const float *__restrict__ chunks,
                                       float *__restrict__ dst) {
    const int64_t e = (int64_t)bx * kBlock + threadIdx.x;
    if (e >= groups * size) return 0.f;
    const int64_t g = e / size, i = e - g * size;
    const float *__restrict__ src = chunks + g * count * size + i;
    float a[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) a[u] = 0.f;
    int c = 0;
    for (; c + 15 < count; c += 16) {
#pragma unroll
        for (int u = 0; u < 16; ++u) a[u] += src[(int64_t)(c + u) * size];
    }
    for (; c < count; ++c) a[0] += src[(int64_t)c * size];
#pragma unroll
    for (int w = 8; w > 0; w >>= 1)
#pragma unroll
        for (int u = 0; u < w; ++u) a[u] += a[u + w];
    dst[e] = a[0];
    return a[0] * a[0];
}

// The whole gradient finish of one fused minibatch step in ONE launch:
// blocks [0, bh) the head's level-2 partial sums (+ loss stats), [bh, +bf)
// the first layer's, the rest the split-K chunk sum of the layers above.
// Every block also writes the sum of squares of the entries it produced, the
// norm partials clip_adam_kernel consumes (replaces 2 finishes, the chunk
// sum and the norm pass: 4 launches).
struct FinishArgs {
    int bh, bf, bc;
    // head (h_direct: h_ng per-block rows at h_part2, summed in the finish)
    int h_ng, h_P, h_hd, h_direct;
    int64_t h_m;
    const float *h_part2, *h_adv_ms, *log_std;
    float ent_coef, vf_coef;
    HeadOut ho;
    // first layer (f_direct > 0: that many level-1 rows, summed here)
    int f_ng, f_n, f_K, f_nets, f_direct;
    const float *f_part2;
    FirstBwdOut fo;
    // split-K chunks
    int64_t c_groups, c_size;
    int c_count;
    const float *chunks;
    float *c_dst;
    float *sq_part;
};

__global__ __launch_bounds__(kBlock) void grad_finish_kernel(FinishArgs a) {
    __shared__ float sh[4];
    int b = blockIdx.x;
    float sq;
    if (b < a.bh) {
        sq = a.h_direct ? head_finish_direct(b, a.h_ng, a.h_P, a.h_hd, a.h_m, a.h_part2,
                                             a.h_adv_ms, a.log_std, a.ent_coef, a.vf_coef, a.ho)
                        : head_finish_part(b, a.h_ng, a.h_P, a.h_hd, a.h_m, a.h_part2, a.h_adv_ms,
                                           a.log_std, a.ent_coef, a.vf_coef, a.ho);
    } else if ((b -= a.bh) < a.bf) {
        sq = a.f_direct ? first_finish_direct(b, a.f_direct, a.f_n, a.f_K, a.f_nets, a.f_part2,
                                              a.fo)
                        : first_finish_part(b, a.f_ng, a.f_n, a.f_K, a.f_nets, a.f_part2, a.fo);
    } else {
        b -= a.bf;
        sq = chunk_sum_part(b, a.c_groups, a.c_count, a.c_size, a.chunks, a.c_dst);
    }
    float x[1] = {sq};
    block_sum<1>(x, sh);
    if (threadIdx.x == 0) a.sq_part[blockIdx.x] = x[0];
}

__global__ __launch_bounds__(kBlock) void clip_adam_kernel(
    int64_t n, float *__restrict__ p, float *__restrict__ g,
    float *__restrict__ m, float *__restrict__ v, const float *__restrict__ part,
    int nb, float max_norm, float w1, float beta2, float one_m_b2,
    float step_size, float bc2_sqrt, const float *__restrict__ sched, float eps,
    float *norm_out, float gscale) {
    // sched (device): this step's (step_size, sqrt(bias_correction2)), written
    // by the host from dr_adam_schedule ahead of a graph replay
    if (sched) {
        step_size = sched[0];
        bc2_sqrt = sched[1];
    }
    // total squared norm: strided per-thread sums of the sumsq partials, then
    // a fixed-shape LDS tree (deterministic; every block gets the same value)
    __shared__ double ssum[kBlock];
    double s = 0.0;
    for (int b = threadIdx.x; b < nb; b += kBlock) s += part[b];
    ssum[threadIdx.x] = s;
    __syncthreads();
    for (int h = kBlock / 2; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h) ssum[threadIdx.x] += ssum[threadIdx.x + h];
        __syncthreads();
    }
    const float total = (float)sqrt(ssum[0]);
    float c = max_norm / (total + 1e-6f);
    c = c < 1.0f ? c : 1.0f;
    if (blockIdx.x == 0 && threadIdx.x == 0 && norm_out) *norm_out = total;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kBlock) {
        const float gi = (g[i] * gscale) * c;   // gscale: sumsq_kernel's scale
        g[i] = gi;
        float mi = m[i];
        mi = mi + w1 * (gi - mi);                    // exp_avg.lerp_(g, 1-b1)
        float vi = v[i] * beta2 + (one_m_b2 * gi) * gi;  // addcmul_: value*t1*t2
        m[i] = mi;
        v[i] = vi;
        const float denom = sqrtf(vi) / bc2_sqrt + eps;
        p[i] = p[i] + (-step_size) * (mi / denom);
    }
}

inline int nblocks_stream(int64_t n) {
    const int64_t b = (n + kBlock - 1) / kBlock;
    return (int)(b < 2048 ? b : 2048);
}

}  // namespace
}  // namespace dr

using namespace dr;

extern "C" {

int dr_gae(int64_t T, int64_t N, const float *rewards, const float *values,
           const uint8_t *episode_starts, const float *last_values,
           const uint8_t *last_dones, double gamma, double gae_lambda,
           float *advantages, float *returns, void *stream) {
    if (T < 1 || N < 1 || !rewards || !values || !episode_starts || !last_values ||
        !last_dones || !advantages || !returns)
        return fail0(DR_ERR_INVALID, "dr_gae: bad arguments");
    const float g32 = (float)gamma;
    const float gl32 = (float)(gamma * gae_lambda);
    hipLaunchKernelGGL(gae_kernel, dim3(grid_for(N)), dim3(kBlock), 0, as_stream(stream),
                       T, N, rewards, values, episode_starts, last_values, last_dones,
                       g32, gl32, advantages, returns);
    return check_launch("dr_gae");
}

int dr_policy_sample(int64_t n, const float *mean, const float *log_std, uint64_t seed,
                     uint64_t counter, float lo, float hi, float *actions_raw,
                     float *actions_clipped, float *logp, void *stream) {
    if (n < 0 || !mean || !log_std) return fail0(DR_ERR_INVALID, "dr_policy_sample: bad arguments");
    if ((((uintptr_t)mean) | ((uintptr_t)actions_raw) | ((uintptr_t)actions_clipped)) & 15)
        return fail0(DR_ERR_INVALID, "dr_policy_sample: (n,4) buffers must be 16-byte aligned");
    if (n == 0) return DR_OK;
    hipLaunchKernelGGL(policy_sample_kernel, dim3(grid_for(n)), dim3(kBlock), 0,
                       as_stream(stream), n, reinterpret_cast<const float4 *>(mean), log_std,
                       (uint32_t)seed, (uint32_t)(seed >> 32), counter,
                       (const uint64_t *)nullptr, lo, hi,
                       reinterpret_cast<float4 *>(actions_raw),
                       reinterpret_cast<float4 *>(actions_clipped), logp);
    return check_launch("dr_policy_sample");
}

int dr_policy_sample_dev(int64_t n, const float *mean, const float *log_std, uint64_t seed,
                         const uint64_t *counter_base, uint64_t counter_offset, float lo,
                         float hi, float *actions_raw, float *actions_clipped, float *logp,
                         void *stream) {
    if (n < 0 || !mean || !log_std || !counter_base)
        return fail0(DR_ERR_INVALID, "dr_policy_sample_dev: bad arguments");
    if ((((uintptr_t)mean) | ((uintptr_t)actions_raw) | ((uintptr_t)actions_clipped)) & 15)
        return fail0(DR_ERR_INVALID,
                     "dr_policy_sample_dev: (n,4) buffers must be 16-byte aligned");
    if (((uintptr_t)counter_base) & 7)
        return fail0(DR_ERR_INVALID, "dr_policy_sample_dev: counter_base must be 8-byte aligned");
    if (n == 0) return DR_OK;
    hipLaunchKernelGGL(policy_sample_kernel, dim3(grid_for(n)), dim3(kBlock), 0,
                       as_stream(stream), n, reinterpret_cast<const float4 *>(mean), log_std,
                       (uint32_t)seed, (uint32_t)(seed >> 32), counter_offset, counter_base, lo,
                       hi, reinterpret_cast<float4 *>(actions_raw),
                       reinterpret_cast<float4 *>(actions_clipped), logp);
    return check_launch("dr_policy_sample_dev");
}

static size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

size_t dr_permutation_workspace_bytes(int64_t n) {
    if (n <= 0) return 0;
    const PermGeom g = perm_geom(n);
    return align_up(sizeof(uint64_t) * n) + align_up(sizeof(int32_t) * n) +
           align_up(sizeof(uint32_t) * g.T * g.B) + align_up(sizeof(uint32_t) * g.B) +
           align_up(sizeof(uint32_t) * (g.B + 1));
}

static int permutation_impl(int64_t n, uint64_t seed, const uint64_t *counter_base,
                            uint64_t counter, int32_t *out, void *workspace,
                            size_t workspace_bytes, void *stream) {
    if (n < 0 || n > 0x7fffffff || !out) return fail0(DR_ERR_INVALID, "dr_permutation: bad arguments");
    if (n == 0) return DR_OK;
    const size_t need = dr_permutation_workspace_bytes(n);
    if (!workspace || workspace_bytes < need)
        return fail0(DR_ERR_INVALID, "dr_permutation: workspace too small");
    const PermGeom g = perm_geom(n);
    char *w = static_cast<char *>(workspace);
    uint64_t *keys = reinterpret_cast<uint64_t *>(w);
    w += align_up(sizeof(uint64_t) * n);
    int32_t *ids = reinterpret_cast<int32_t *>(w);
    w += align_up(sizeof(int32_t) * n);
    uint32_t *hist = reinterpret_cast<uint32_t *>(w);
    w += align_up(sizeof(uint32_t) * g.T * g.B);
    uint32_t *total = reinterpret_cast<uint32_t *>(w);
    w += align_up(sizeof(uint32_t) * g.B);
    uint32_t *start = reinterpret_cast<uint32_t *>(w);
    hipStream_t st = as_stream(stream);
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    const size_t lds = sizeof(uint32_t) * (size_t)g.B;
    hipLaunchKernelGGL(perm_hist_kernel, dim3((unsigned)g.T), dim3(kBlock), lds, st, g, k0, k1,
                       counter, counter_base, keys, hist);
    int rc = check_launch("dr_permutation hist");
    if (rc) return rc;
    hipLaunchKernelGGL(perm_scan_tiles_kernel, dim3((unsigned)((g.B + 63) / 64)), dim3(kBlock), 0, st, g,
                       hist, total);
    if ((rc = check_launch("dr_permutation scan"))) return rc;
    hipLaunchKernelGGL(perm_scan_buckets_kernel, dim3(1), dim3(1024), 0, st, g, total, start);
    if ((rc = check_launch("dr_permutation scan"))) return rc;
    hipLaunchKernelGGL(perm_scatter_kernel, dim3((unsigned)g.T), dim3(kBlock), lds, st, g, keys,
                       hist, start, ids);
    if ((rc = check_launch("dr_permutation scatter"))) return rc;
    // DRONERL_PERM_LDS_CAP (tests only) lowers the LDS capacity so that the
    // global-scratch path of perm_sort_kernel runs on ordinary sizes
    int cap = kPermCap;
    if (const char *e = std::getenv("DRONERL_PERM_LDS_CAP")) {
        const int v = std::atoi(e);
        if (v >= 0 && v < kPermCap) cap = v;
    }
    hipLaunchKernelGGL(perm_sort_kernel, dim3((unsigned)g.B), dim3(kBlock), 0, st, g, k0, k1,
                       counter, counter_base, start, ids, keys, out, cap);
    return check_launch("dr_permutation sort");
}

int dr_permutation(int64_t n, uint64_t seed, uint64_t counter, int32_t *out,
                   void *workspace, size_t workspace_bytes, void *stream) {
    return permutation_impl(n, seed, nullptr, counter, out, workspace, workspace_bytes, stream);
}

int dr_permutation_dev(int64_t n, uint64_t seed, const uint64_t *counter_base,
                       uint64_t counter_offset, int32_t *out, void *workspace,
                       size_t workspace_bytes, void *stream) {
    if (!counter_base || (((uintptr_t)counter_base) & 7))
        return fail0(DR_ERR_INVALID, "dr_permutation_dev: counter_base must be 8-byte aligned");
    return permutation_impl(n, seed, counter_base, counter_offset, out, workspace,
                            workspace_bytes, stream);
}

int dr_gather_rows(int64_t m, int64_t width, const int32_t *idx, const float *src,
                   float *dst, void *stream) {
    if (m < 0 || width < 1 || !idx || !src || !dst)
        return fail0(DR_ERR_INVALID, "dr_gather_rows: bad arguments");
    if (m == 0) return DR_OK;
    hipLaunchKernelGGL(gather_rows_kernel, dim3(grid_for(m * width)), dim3(kBlock), 0,
                       as_stream(stream), m, width, idx, src, dst);
    return check_launch("dr_gather_rows");
}

int dr_gather_minibatch(int64_t m, const int32_t *idx, int64_t obs_dim, const float *obs,
                        const float *actions, const float *aux, float *obs_out,
                        float *actions_out, float *aux_out, float *adv_part, void *stream) {
    if (m < 0 || obs_dim < 1 || !idx || !obs || !actions || !aux || !obs_out || !actions_out ||
        !aux_out)
        return fail0(DR_ERR_INVALID, "dr_gather_minibatch: bad arguments");
    if ((((uintptr_t)actions) | ((uintptr_t)actions_out)) & 15)
        return fail0(DR_ERR_INVALID, "dr_gather_minibatch: action rows must be 16-byte aligned");
    if (m == 0) return DR_OK;
    const int64_t nb_obs = grid_for(m * obs_dim), nb_rows = grid_for(m);
    if (nb_obs + 2 * nb_rows > INT32_MAX)
        return fail0(DR_ERR_INVALID, "dr_gather_minibatch: m too large");
    hipLaunchKernelGGL(gather_minibatch_kernel, dim3((unsigned)(nb_obs + 2 * nb_rows)),
                       dim3(kBlock), 0, as_stream(stream), m, (int)obs_dim, (int)nb_obs,
                       (int)nb_rows, idx, obs, reinterpret_cast<const float4 *>(actions), aux,
                       obs_out, reinterpret_cast<float4 *>(actions_out), aux_out, adv_part);
    return check_launch("dr_gather_minibatch");
}

int dr_pack_rollout_records(int64_t n, int64_t obs_dim, const float *obs, const float *actions,
                            const float *logp, const float *adv, const float *ret,
                            float *records, void *stream) {
    if (n < 0 || obs_dim < 1 || obs_dim > kRecMaxObs || !obs || !actions || !logp || !adv ||
        !ret || !records)
        return fail0(DR_ERR_INVALID, "dr_pack_rollout_records: bad arguments (1 <= obs_dim <= 24)");
    if ((((uintptr_t)actions) | ((uintptr_t)records)) & 15)
        return fail0(DR_ERR_INVALID,
                     "dr_pack_rollout_records: actions and records must be 16-byte aligned");
    if (n == 0) return DR_OK;
    if (n > (int64_t(1) << 31))
        return fail0(DR_ERR_INVALID, "dr_pack_rollout_records: n too large");
    hipLaunchKernelGGL(pack_records_kernel, dim3((unsigned)grid_for(8 * n)), dim3(kBlock), 0,
                       as_stream(stream), n, (int)obs_dim, obs,
                       reinterpret_cast<const float4 *>(actions), logp, adv, ret,
                       reinterpret_cast<float4 *>(records));
    return check_launch("dr_pack_rollout_records");
}

int dr_gather_records(int64_t m, const int32_t *idx, int64_t obs_dim, const float *records,
                      float *obs_out, float *actions_out, float *aux_out, float *adv_part,
                      void *stream) {
    if (m < 0 || obs_dim < 1 || obs_dim > kRecMaxObs || !idx || !records || !obs_out ||
        !actions_out || !aux_out)
        return fail0(DR_ERR_INVALID, "dr_gather_records: bad arguments (1 <= obs_dim <= 24)");
    if ((((uintptr_t)records) | ((uintptr_t)actions_out) | ((uintptr_t)obs_out)) & 15)
        return fail0(DR_ERR_INVALID,
                     "dr_gather_records: records, obs_out and actions_out must be 16-byte aligned");
    if (m == 0) return DR_OK;
    if (grid_for(m) > INT32_MAX) return fail0(DR_ERR_INVALID, "dr_gather_records: m too large");
    hipLaunchKernelGGL(gather_records_kernel, dim3((unsigned)grid_for(m)), dim3(kBlock), 0,
                       as_stream(stream), m, (int)obs_dim, idx,
                       reinterpret_cast<const float4 *>(records), obs_out,
                       reinterpret_cast<float4 *>(actions_out), aux_out, adv_part);
    return check_launch("dr_gather_records");
}

size_t dr_tanh_backward_workspace_bytes(int64_t m, int64_t n) {
    const int64_t nb = (m + kTanhRows - 1) / kTanhRows;
    return align_up(sizeof(float) * (size_t)(nb * n));
}

int dr_tanh_backward(int64_t m, int64_t n, const float *grad_h, const float *h,
                     float *grad_z, float *bias_grad, void *workspace, size_t workspace_bytes,
                     void *stream) {
    if (m < 1 || n < 4 || n % 4 || n > 4 * kBlock || !grad_h || !h || !grad_z || !bias_grad)
        return fail0(DR_ERR_INVALID, "dr_tanh_backward: bad arguments (n % 4, n <= 1024)");
    if ((((uintptr_t)grad_h) | ((uintptr_t)h) | ((uintptr_t)grad_z)) & 15)
        return fail0(DR_ERR_INVALID, "dr_tanh_backward: buffers must be 16-byte aligned");
    if (!workspace || workspace_bytes < dr_tanh_backward_workspace_bytes(m, n))
        return fail0(DR_ERR_INVALID, "dr_tanh_backward: workspace too small");
    const int nb = (int)((m + kTanhRows - 1) / kTanhRows);
    float *part = static_cast<float *>(workspace);
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(tanh_bwd_kernel, dim3(nb), dim3(kBlock), 0, st, m, (int)(n / 4),
                       reinterpret_cast<const float4 *>(grad_h),
                       reinterpret_cast<const float4 *>(h), reinterpret_cast<float4 *>(grad_z),
                       reinterpret_cast<float4 *>(part));
    int rc = check_launch("dr_tanh_backward");
    if (rc) return rc;
    hipLaunchKernelGGL(colsum_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, nb,
                       (int)n, part, bias_grad);
    return check_launch("dr_tanh_backward colsum");
}

size_t dr_ppo_loss_workspace_bytes(int64_t m) {
    const int64_t nb = (m + kBlock - 1) / kBlock;
    return align_up(sizeof(float) * 3 * nb) + align_up(sizeof(float) * (kLossK * nb + 2));
}

int dr_ppo_loss(int64_t m, const float *mean, const float *log_std, const float *values,
                const float *actions, const float *old_logp, const float *advantages,
                const float *returns, int64_t aux_stride, float clip_range, float ent_coef, float vf_coef,
                int normalize_advantage, float *grad_mean, float *grad_values,
                float *grad_log_std, float *stats, void *workspace, size_t workspace_bytes,
                void *stream) {
    if (m < 1 || !mean || !log_std || !values || !actions || !old_logp || !advantages ||
        !returns || !grad_mean || !grad_values || !grad_log_std || !stats)
        return fail0(DR_ERR_INVALID, "dr_ppo_loss: bad arguments");
    if (aux_stride < 1) return fail0(DR_ERR_INVALID, "dr_ppo_loss: aux_stride must be >= 1");
    if ((((uintptr_t)mean) | ((uintptr_t)actions) | ((uintptr_t)grad_mean)) & 15)
        return fail0(DR_ERR_INVALID, "dr_ppo_loss: (m,4) buffers must be 16-byte aligned");
    if (!workspace || workspace_bytes < dr_ppo_loss_workspace_bytes(m))
        return fail0(DR_ERR_INVALID, "dr_ppo_loss: workspace too small");
    // SB3 normalises only when the minibatch has more than one row.
    const int norm = normalize_advantage && m > 1;
    const int nb = (int)grid_for(m);
    float *adv_part = static_cast<float *>(workspace);
    float *part = reinterpret_cast<float *>(static_cast<char *>(workspace) +
                                            align_up(sizeof(float) * 3 * nb));
    hipStream_t st = as_stream(stream);
    if (norm) {
        hipLaunchKernelGGL(adv_stats_kernel, dim3(nb), dim3(kBlock), 0, st, m, advantages,
                           aux_stride, (const int32_t *)nullptr, adv_part);
        int rc = check_launch("dr_ppo_loss stats");
        if (rc) return rc;
    }
    LossArgs a{m, reinterpret_cast<const float4 *>(mean), log_std, values,
               reinterpret_cast<const float4 *>(actions), old_logp, advantages, returns,
               aux_stride, clip_range, ent_coef, vf_coef, norm, adv_part, nb,
               reinterpret_cast<float4 *>(grad_mean), grad_values, part};
    hipLaunchKernelGGL(ppo_loss_kernel, dim3(nb), dim3(kBlock), 0, st, a);
    int rc = check_launch("dr_ppo_loss");
    if (rc) return rc;
    hipLaunchKernelGGL(ppo_loss_finish_kernel, dim3(1), dim3(kBlock), 0, st, m, nb, part,
                       log_std, ent_coef, vf_coef, grad_log_std, stats);
    return check_launch("dr_ppo_loss finish");
}

int dr_adam_schedule(double lr, double beta1, double beta2, int64_t step, float *out) {
    if (!out || step < 1) return fail0(DR_ERR_INVALID, "dr_adam_schedule: bad arguments");
    const double bc1 = 1.0 - std::pow(beta1, (double)step);
    const double bc2 = 1.0 - std::pow(beta2, (double)step);
    out[0] = (float)(lr / bc1);
    out[1] = (float)std::sqrt(bc2);
    return DR_OK;
}

static int launch_adam(int64_t n, float *params, float *grads, float *exp_avg,
                       float *exp_avg_sq, double lr, double beta1, double beta2, double eps,
                       float max_grad_norm, int64_t step, float *grad_norm_out,
                       const float *sq_part, int nsq, hipStream_t st, const char *who,
                       const float *sched = nullptr, float gscale = 1.0f) {
    // torch.optim.Adam scalars, formed in double as torch does on the host.
    const double b1 = beta1, b2 = beta2;
    float ss[2] = {0.f, 1.f};
    if (!sched) dr_adam_schedule(lr, beta1, beta2, step, ss);
    hipLaunchKernelGGL(clip_adam_kernel, dim3(nblocks_stream(n)), dim3(kBlock), 0, st, n,
                       params, grads, exp_avg, exp_avg_sq, sq_part, nsq, max_grad_norm,
                       (float)(1.0 - b1), (float)b2, (float)(1.0 - b2), ss[0], ss[1], sched,
                       (float)eps, grad_norm_out, gscale);
    return check_launch(who);
}

static int first_blocks(int64_t m);

// Block counts of grad_finish_kernel's three segments.
static void finish_blocks(const dr_grad_finish *f, int &bh, int &bf, int &bc) {
    const int64_t hP = kHeadFixed + 7 * f->head_hd;
    bh = !f->head_workspace ? 0
         : f->head_direct ? (int)((hP + 15) / 16)         // head_finish_direct: 16 per block
                          : (int)((hP + kBlock - 1) / kBlock);
    const int64_t fP = 2 * (f->first_k + 1) * f->first_n;
    bf = !f->first_workspace ? 0
         : f->first_rows > 0 ? (int)((fP + 63) / 64)     // first_finish_direct: 64 per block
                             : (int)((fP + kBlock - 1) / kBlock);
    bc = f->chunks ? (int)((f->chunk_groups * f->chunk_size + kBlock - 1) / kBlock) : 0;
}

size_t dr_adam_workspace_bytes(int64_t n) {
    return align_up(sizeof(float) * (size_t)nblocks_stream(n > 0 ? n : 1));
}

int dr_clip_adam(int64_t n, float *params, float *grads, float *exp_avg, float *exp_avg_sq,
                 double lr, double beta1, double beta2, double eps, float max_grad_norm,
                 int64_t step, float *grad_norm_out, void *workspace, size_t workspace_bytes,
                 void *stream) {
    if (n < 1 || !params || !grads || !exp_avg || !exp_avg_sq || step < 1)
        return fail0(DR_ERR_INVALID, "dr_clip_adam: bad arguments");
    if (!workspace || workspace_bytes < dr_adam_workspace_bytes(n))
        return fail0(DR_ERR_INVALID, "dr_clip_adam: workspace too small");
    const int nb = nblocks_stream(n);
    float *part = static_cast<float *>(workspace);
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(sumsq_kernel, dim3(nb), dim3(kBlock), 0, st, n, grads, part, 1.0f);
    int rc = check_launch("dr_clip_adam norm");
    if (rc) return rc;
    return launch_adam(n, params, grads, exp_avg, exp_avg_sq, lr, beta1, beta2, eps,
                       max_grad_norm, step, grad_norm_out, part, nb, st, "dr_clip_adam");
}

size_t dr_grad_finish_workspace_bytes(const dr_grad_finish *f) {
    int bh, bf, bc;
    finish_blocks(f, bh, bf, bc);
    return align_up(sizeof(float) * (size_t)(bh + bf + bc > 0 ? bh + bf + bc : 1));
}

// Validates f and launches grad_finish_kernel (every deferred partial into
// the flat gradient, the norm partials into workspace); *nsq = its blocks.
static int launch_grad_finish(const dr_grad_finish *f, void *workspace, size_t workspace_bytes,
                              hipStream_t st, int *nsq) {
    if (!f) return fail0(DR_ERR_INVALID, "dr_grad_finish: null descriptor");
    if (f->head_workspace && (f->head_m < 1 || f->head_hd < 4 || f->head_hd > 256 ||
                              !f->log_std || !f->g_w_act || !f->g_b_act || !f->g_w_val ||
                              !f->g_b_val || !f->g_b_pi || !f->g_b_vf || !f->g_log_std ||
                              !f->stats))
        return fail0(DR_ERR_INVALID, "dr_grad_finish: bad head arguments");
    if (f->first_workspace && (f->first_m < 1 || f->first_n < 4 || f->first_n > 256 ||
                               f->first_k < 1 || !f->g_w0 || !f->g_b0 || !f->g_w1 || !f->g_b1 ||
                               f->first_rows < 0 || f->first_rows > first_blocks(f->first_m)))
        return fail0(DR_ERR_INVALID, "dr_grad_finish: bad first-layer arguments");
    if (f->chunks && (f->chunk_groups < 1 || f->chunk_count < 1 || f->chunk_size < 1 ||
                      !f->chunk_dst))
        return fail0(DR_ERR_INVALID, "dr_grad_finish: bad chunk arguments");
    if (!workspace || workspace_bytes < dr_grad_finish_workspace_bytes(f))
        return fail0(DR_ERR_INVALID, "dr_grad_finish: workspace too small");
    FinishArgs a{};
    finish_blocks(f, a.bh, a.bf, a.bc);
    if (a.bh + a.bf + a.bc < 1)
        return fail0(DR_ERR_INVALID, "dr_grad_finish: nothing to finish");
    if (f->head_workspace) {
        const int64_t m = f->head_m, hd = f->head_hd;
        const int nb = loss_head_blocks(m);
        const int P = kHeadFixed + 7 * (int)hd;
        const int gsize = (nb + kHeadGroups - 1) / kHeadGroups;
        // the head workspace layout of dr_ppo_head_loss_backward
        const float *part = reinterpret_cast<const float *>(
            static_cast<const char *>(f->head_workspace) +
            align_up(sizeof(float) * 3 * grid_for(m)));
        a.h_ng = (nb + gsize - 1) / gsize;
        a.h_P = P;
        a.h_hd = (int)hd;
        a.h_m = m;
        a.h_part2 = reinterpret_cast<const float *>(reinterpret_cast<const char *>(part) +
                                                    align_up(sizeof(float) * (size_t)(nb * P + 2)));
        a.h_adv_ms = part + (int64_t)nb * P;
        if (f->head_direct) {
            a.h_direct = 1;
            a.h_ng = nb;
            a.h_part2 = part;
        }
        a.log_std = f->log_std;
        a.ent_coef = f->ent_coef;
        a.vf_coef = f->vf_coef;
        a.ho = HeadOut{f->g_w_act, f->g_b_act, f->g_w_val, f->g_b_val,
                       f->g_b_pi,  f->g_b_vf,  f->g_log_std, f->stats};
    }
    if (f->first_workspace) {
        const int nb = first_blocks(f->first_m);
        const int P = 2 * (int)((f->first_k + 1) * f->first_n);
        const int gsize = (nb + kHeadGroups - 1) / kHeadGroups;
        a.f_ng = (nb + gsize - 1) / gsize;
        a.f_n = (int)f->first_n;
        a.f_K = (int)f->first_k;
        a.f_nets = 2;
        a.f_part2 = reinterpret_cast<const float *>(static_cast<const char *>(f->first_workspace) +
                                                    align_up(sizeof(float) * (size_t)(nb * P)));
        a.fo = FirstBwdOut{{f->g_w0, f->g_w1}, {f->g_b0, f->g_b1}};
        if (f->first_rows > 0) {
            a.f_direct = (int)f->first_rows;
            a.f_part2 = static_cast<const float *>(f->first_workspace);
        }
    }
    if (f->chunks) {
        a.c_groups = f->chunk_groups;
        a.c_size = f->chunk_size;
        a.c_count = (int)f->chunk_count;
        a.chunks = f->chunks;
        a.c_dst = f->chunk_dst;
    }
    a.sq_part = static_cast<float *>(workspace);
    *nsq = a.bh + a.bf + a.bc;
    hipLaunchKernelGGL(grad_finish_kernel, dim3(*nsq), dim3(kBlock), 0, st, a);
    return check_launch("dr_grad_finish");
}

static int grad_finish_adam_impl(const dr_grad_finish *f, int64_t n, float *params,
                                 float *grads, float *exp_avg, float *exp_avg_sq, double lr,
                                 double beta1, double beta2, double eps, float max_grad_norm,
                                 int64_t step, const float *sched, float *grad_norm_out,
                                 void *workspace, size_t workspace_bytes, void *stream) {
    if (!f || n < 1 || !params || !grads || !exp_avg || !exp_avg_sq || (step < 1 && !sched))
        return fail0(DR_ERR_INVALID, "dr_grad_finish_clip_adam: bad arguments");
    hipStream_t st = as_stream(stream);
    int nb = 0;
    const int rc = launch_grad_finish(f, workspace, workspace_bytes, st, &nb);
    if (rc) return rc;
    return launch_adam(n, params, grads, exp_avg, exp_avg_sq, lr, beta1, beta2, eps,
                       max_grad_norm, step, grad_norm_out, static_cast<const float *>(workspace),
                       nb, st, "dr_grad_finish_clip_adam", sched);
}

int dr_grad_finish_run(const dr_grad_finish *f, void *workspace, size_t workspace_bytes,
                   void *stream) {
    int nb = 0;
    return launch_grad_finish(f, workspace, workspace_bytes, as_stream(stream), &nb);
}

int dr_clip_adam_sched(int64_t n, float *params, float *grads, float *exp_avg,
                       float *exp_avg_sq, double beta1, double beta2, double eps,
                       float max_grad_norm, float grad_scale, const float *sched,
                       float *grad_norm_out, void *workspace, size_t workspace_bytes,
                       void *stream) {
    if (n < 1 || !params || !grads || !exp_avg || !exp_avg_sq || !sched ||
        (((uintptr_t)sched) & 7) || !(grad_scale > 0.0f))
        return fail0(DR_ERR_INVALID, "dr_clip_adam_sched: bad arguments (sched 8-byte "
                                     "aligned, grad_scale > 0)");
    if (!workspace || workspace_bytes < dr_adam_workspace_bytes(n))
        return fail0(DR_ERR_INVALID, "dr_clip_adam_sched: workspace too small");
    const int nb = nblocks_stream(n);
    float *part = static_cast<float *>(workspace);
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(sumsq_kernel, dim3(nb), dim3(kBlock), 0, st, n, grads, part, grad_scale);
    const int rc = check_launch("dr_clip_adam_sched norm");
    if (rc) return rc;
    return launch_adam(n, params, grads, exp_avg, exp_avg_sq, 0.0, beta1, beta2, eps,
                       max_grad_norm, 0, grad_norm_out, part, nb, st, "dr_clip_adam_sched", sched,
                       grad_scale);
}

int dr_grad_finish_clip_adam(const dr_grad_finish *f, int64_t n, float *params, float *grads,
                             float *exp_avg, float *exp_avg_sq, double lr, double beta1,
                             double beta2, double eps, float max_grad_norm, int64_t step,
                             float *grad_norm_out, void *workspace, size_t workspace_bytes,
                             void *stream) {
    return grad_finish_adam_impl(f, n, params, grads, exp_avg, exp_avg_sq, lr, beta1, beta2,
                                 eps, max_grad_norm, step, nullptr, grad_norm_out, workspace,
                                 workspace_bytes, stream);
}

int dr_grad_finish_clip_adam_sched(const dr_grad_finish *f, int64_t n, float *params,
                                   float *grads, float *exp_avg, float *exp_avg_sq, double lr,
                                   double beta1, double beta2, double eps, float max_grad_norm,
                                   const float *sched, float *grad_norm_out, void *workspace,
                                   size_t workspace_bytes, void *stream) {
    if (!sched || (((uintptr_t)sched) & 7))
        return fail0(DR_ERR_INVALID,
                     "dr_grad_finish_clip_adam_sched: sched must be 8-byte aligned");
    return grad_finish_adam_impl(f, n, params, grads, exp_avg, exp_avg_sq, lr, beta1, beta2,
                                 eps, max_grad_norm, 0, sched, grad_norm_out, workspace,
                                 workspace_bytes, stream);
}


static int launch_linear_tanh(const char *who, int nets, int64_t m, int64_t k, int64_t n,
                              const float *x, const int32_t *rows, const LayerPair &lp,
                              void *stream) {
    if (m < 1 || !x || n < 4 || n > 256 || (n & 3))
        return fail0(DR_ERR_INVALID, std::string(who) +
                                         ": bad arguments (need 4 <= n <= 256, n % 4 == 0)");
    for (int j = 0; j < nets; ++j) {
        if (!lp.w[j] || !lp.b[j] || !lp.h[j])
            return fail0(DR_ERR_INVALID, std::string(who) + ": null weight / bias / output");
        if ((((uintptr_t)lp.h[j]) | ((uintptr_t)lp.w[j])) & 15)
            return fail0(DR_ERR_INVALID, std::string(who) + ": h and w must be 16-byte aligned");
    }
    hipStream_t st = as_stream(stream);
    const int64_t nbl = (m + DR_LT_RPB - 1) / DR_LT_RPB;    // >= RPB / 4 rows per wave
    const int nb = (int)(nbl < DR_LT_MAXB ? nbl : DR_LT_MAXB);
    switch (k) {
#define DR_LT_CASE(K)                                                                      \
    case K:                                                                                \
        hipLaunchKernelGGL((linear_tanh_kernel<K, false>), dim3(nb, nets), dim3(kBlock), 0, st, \
                           m, (int)n, x, rows, lp, X6Aux{});                               \
        break;
        DR_LT_CASE(4) DR_LT_CASE(8) DR_LT_CASE(12) DR_LT_CASE(15) DR_LT_CASE(16)
        DR_LT_CASE(18) DR_LT_CASE(24) DR_LT_CASE(32)
#undef DR_LT_CASE
        default:
            return fail0(DR_ERR_UNSUPPORTED,
                         std::string(who) + ": k must be one of 4, 8, 12, 15, 16, 18, 24, 32");
    }
    return check_launch(who);
}

int dr_linear_tanh(int64_t m, int64_t k, int64_t n, const float *x, const int32_t *rows,
                   const float *w, const float *b, float *h, void *stream) {
    const LayerPair lp{{w, nullptr}, {b, nullptr}, {h, nullptr}};
    return launch_linear_tanh("dr_linear_tanh", 1, m, k, n, x, rows, lp, stream);
}

int dr_linear_tanh2(int64_t m, int64_t k, int64_t n, const float *x, const int32_t *rows,
                    const float *w0, const float *b0, float *h0, const float *w1,
                    const float *b1, float *h1, void *stream) {
    const LayerPair lp{{w0, w1}, {b0, b1}, {h0, h1}};
    return launch_linear_tanh("dr_linear_tanh2", 2, m, k, n, x, rows, lp, stream);
}

int dr_linear_tanh2_x6(int64_t m, int64_t k, int64_t n, const float *x, const int32_t *rows,
                       const float *w0, const float *b0, float *h0, const float *w1,
                       const float *b1, float *h1, const float *w256, void *img, void *ximg,
                       void *stream) {
    const char *who = "dr_linear_tanh2_x6";
    if (m < 1 || !x || n != 256 || k != 15 || !w0 || !b0 || !h0 || !w1 || !b1 || !h1 ||
        !w256 || !img || ((((uintptr_t)h0) | ((uintptr_t)h1) | ((uintptr_t)w0) |
                           ((uintptr_t)w1) | ((uintptr_t)img) | ((uintptr_t)ximg)) & 15))
        return fail0(DR_ERR_INVALID, std::string(who) +
                                         ": bad arguments (k 15, n 256, 16-byte aligned "
                                         "outputs, weights and images)");
    if (ximg && (m % 128 || m > (int64_t(1) << 26)))
        return fail0(DR_ERR_INVALID, std::string(who) + ": ximg needs m a multiple of 128");
    const LayerPair lp{{w0, w1}, {b0, b1}, {h0, h1}};
    const int64_t nbl = (m + DR_LT_RPB - 1) / DR_LT_RPB;
    const int nb = (int)(nbl < DR_LT_MAXB ? nbl : DR_LT_MAXB);
    const int64_t naux = 2 * kAuxWBlocks + (ximg ? (2 * m + kBlock - 1) / kBlock : 0);
    const int gx = (int)(naux > nb ? naux : nb);
    hipLaunchKernelGGL((linear_tanh_kernel<15, true>), dim3(gx, 3), dim3(kBlock), 0,
                       as_stream(stream), m, 256, x, rows, lp,
                       X6Aux{w256, static_cast<uint8_t *>(img), static_cast<uint8_t *>(ximg)});
    return check_launch(who);
}

int dr_policy_heads(int64_t m, int64_t hd, int preact, const float *h_pi, const float *h_vf,
                    const float *zb_pi, const float *zb_vf, const float *w_act, const float *b_act, const float *w_val,
                    const float *b_val, float *mean, float *value, void *stream) {
    if (m < 1 || hd < 4 || hd > 256 || (hd & 3) || !h_pi || !h_vf || !w_act || !b_act ||
        !w_val || !b_val || !mean || !value)
        return fail0(DR_ERR_INVALID, "dr_policy_heads: bad arguments");
    if ((((uintptr_t)h_pi) | ((uintptr_t)h_vf) | ((uintptr_t)w_act) | ((uintptr_t)w_val) |
         ((uintptr_t)mean)) & 15)
        return fail0(DR_ERR_INVALID, "dr_policy_heads: buffers must be 16-byte aligned");
    if ((zb_pi || zb_vf) && !preact)
        return fail0(DR_ERR_INVALID, "dr_policy_heads: zb_pi / zb_vf need preact");
    if ((((uintptr_t)zb_pi) | ((uintptr_t)zb_vf)) & 15)
        return fail0(DR_ERR_INVALID, "dr_policy_heads: zb_pi / zb_vf must be 16-byte aligned");
    hipLaunchKernelGGL(policy_heads_kernel, dim3(head_blocks(m)), dim3(kBlock), 0,
                       as_stream(stream), m, (int)hd, preact, h_pi, h_vf, zb_pi, zb_vf, w_act, b_act,
                       w_val, b_val,
                       reinterpret_cast<float4 *>(mean), value);
    return check_launch("dr_policy_heads");
}

size_t dr_ppo_head_workspace_bytes(int64_t m, int64_t hd) {
    const int64_t nb = (m + kBlock - 1) / kBlock;
    const int64_t P = kHeadFixed + 7 * hd;
    return align_up(sizeof(float) * 3 * nb) +
           align_up(sizeof(float) * (size_t)(loss_head_blocks(m > 0 ? m : 1) * P + 2)) +
           align_up(sizeof(float) * (size_t)(kHeadGroups * P));
}

int dr_ppo_head_loss_backward(int64_t m, int64_t hd, int preact, const float *h_pi,
                              const float *h_vf, const float *zb_pi, const float *zb_vf,
                              const float *w_act, const float *b_act, const float *w_val,
                              const float *b_val, const float *log_std, const float *actions,
                              const float *aux, const int32_t *rows, float clip_range,
                              float ent_coef,
                              float vf_coef, int normalize_advantage, float *gz_pi,
                              float *gz_vf, float *g_w_act, float *g_b_act, float *g_w_val,
                              float *g_b_val, float *g_b_pi, float *g_b_vf, float *g_log_std,
                              float *stats, int defer, void *workspace,
                              size_t workspace_bytes, void *stream) {
    if (m < 1 || hd < 4 || hd > 256 || (hd & 3) || !h_pi || !h_vf || !w_act || !b_act ||
        !w_val || !b_val || !log_std || !actions || !aux || !gz_pi || !gz_vf || !g_w_act ||
        !g_b_act || !g_w_val || !g_b_val || !g_b_pi || !g_b_vf || !g_log_std || !stats)
        return fail0(DR_ERR_INVALID, "dr_ppo_head_loss_backward: bad arguments");
    if ((((uintptr_t)h_pi) | ((uintptr_t)h_vf) | ((uintptr_t)w_act) | ((uintptr_t)w_val) |
         ((uintptr_t)actions) | ((uintptr_t)gz_pi) | ((uintptr_t)gz_vf)) & 15)
        return fail0(DR_ERR_INVALID,
                     "dr_ppo_head_loss_backward: row buffers must be 16-byte aligned");
    if ((zb_pi || zb_vf) && !preact)
        return fail0(DR_ERR_INVALID, "dr_ppo_head_loss_backward: zb_pi / zb_vf need preact");
    if ((((uintptr_t)zb_pi) | ((uintptr_t)zb_vf)) & 15)
        return fail0(DR_ERR_INVALID,
                     "dr_ppo_head_loss_backward: zb_pi / zb_vf must be 16-byte aligned");
    if (!workspace || workspace_bytes < dr_ppo_head_workspace_bytes(m, hd))
        return fail0(DR_ERR_INVALID, "dr_ppo_head_loss_backward: workspace too small");
    const int norm = normalize_advantage && m > 1;
    const int anb = (int)grid_for(m);
    float *adv_part = static_cast<float *>(workspace);
    float *part = reinterpret_cast<float *>(static_cast<char *>(workspace) +
                                            align_up(sizeof(float) * 3 * anb));
    hipStream_t st = as_stream(stream);
    // normalize_advantage == 2: dr_gather_minibatch already wrote the
    // advantage partials to the head of the workspace
    if (norm && normalize_advantage != 2) {
        hipLaunchKernelGGL(adv_stats_kernel, dim3(anb), dim3(kBlock), 0, st, m, aux + 1,
                           (int64_t)3, rows, adv_part);
        int rc = check_launch("dr_ppo_head_loss_backward stats");
        if (rc) return rc;
    }
    const int nb = loss_head_blocks(m);
    const int P = kHeadFixed + 7 * (int)hd;
    HeadArgs a{m, (int)hd, preact, h_pi, h_vf, zb_pi, zb_vf, w_act, b_act, w_val, b_val, log_std,
               reinterpret_cast<const float4 *>(actions), aux, rows, clip_range, ent_coef,
               vf_coef, norm, adv_part, anb, gz_pi, gz_vf, part, P};
    hipLaunchKernelGGL(ppo_head_kernel, dim3(nb), dim3(kBlock), sizeof(float) * 4 * P, st, a);
    int rc = check_launch("dr_ppo_head_loss_backward");
    if (rc) return rc;
    // defer 2: the per-block rows are summed by the finish (head_direct)
    if (defer == 2) return DR_OK;
    // two-level fixed-order reduction of the nb x P partials
    float *part2 = reinterpret_cast<float *>(
        reinterpret_cast<char *>(part) + align_up(sizeof(float) * (size_t)(nb * P + 2)));
    const int gsize = (nb + kHeadGroups - 1) / kHeadGroups;
    const int ng = (nb + gsize - 1) / gsize;
    hipLaunchKernelGGL(colsum_groups_kernel, dim3((P + kBlock - 1) / kBlock, ng), dim3(kBlock),
                       0, st, nb, P, gsize, part, part2);
    rc = check_launch("dr_ppo_head_loss_backward groups");
    if (rc) return rc;
    // defer: the level-2 sum is left to dr_grad_finish_clip_adam
    if (defer) return DR_OK;
    HeadOut o{g_w_act, g_b_act, g_w_val, g_b_val, g_b_pi, g_b_vf, g_log_std, stats};
    hipLaunchKernelGGL(ppo_head_finish_kernel, dim3((P + kBlock - 1) / kBlock), dim3(kBlock),
                       0, st, ng, P, (int)hd, m, part2, part + (int64_t)nb * P, log_std,
                       ent_coef, vf_coef, o);
    return check_launch("dr_ppo_head_loss_backward finish");
}


static int first_blocks(int64_t m) {
    const int64_t b = (m + 4 * kFirstTile - 1) / (4 * kFirstTile);
    return (int)(b < DR_FL_MAXB ? b : DR_FL_MAXB);
}

static size_t first_ws_bytes(int nets, int64_t m, int64_t k, int64_t n) {
    const int64_t P = nets * (k + 1) * n;
    return align_up(sizeof(float) * (size_t)(first_blocks(m > 0 ? m : 1) * P)) +
           align_up(sizeof(float) * (size_t)(kHeadGroups * P));
}

size_t dr_first_layer_backward_workspace_bytes(int64_t m, int64_t k, int64_t n) {
    return first_ws_bytes(1, m, k, n);
}

size_t dr_first_layer_backward2_workspace_bytes(int64_t m, int64_t k, int64_t n) {
    return first_ws_bytes(2, m, k, n);
}

static int launch_first_bwd(const char *who, int nets, int64_t m, int64_t k, int64_t n,
                            const FirstBwdIn &in, const float *x, const int32_t *rows,
                            const FirstBwdOut &o, void *workspace, size_t workspace_bytes,
                            void *stream, int defer = 0) {
    if (m < 1 || !x || n < 4 || n > 256 || (n & 3))
        return fail0(DR_ERR_INVALID, std::string(who) + ": bad arguments");
    for (int j = 0; j < nets; ++j) {
        if (!in.gh[j] || !in.h[j] || !o.gw[j] || !o.gb[j])
            return fail0(DR_ERR_INVALID, std::string(who) + ": bad arguments");
        if ((((uintptr_t)in.gh[j]) | ((uintptr_t)in.h[j])) & 15)
            return fail0(DR_ERR_INVALID,
                         std::string(who) + ": grad_h / h must be 16-byte aligned");
    }
    if (!workspace || workspace_bytes < first_ws_bytes(nets, m, k, n))
        return fail0(DR_ERR_INVALID, std::string(who) + ": workspace too small");
    const int nb = first_blocks(m);
    const int P1 = (int)((k + 1) * n);
    const int P = nets * P1;
    float *part = static_cast<float *>(workspace);
    float *part2 = reinterpret_cast<float *>(static_cast<char *>(workspace) +
                                             align_up(sizeof(float) * (size_t)(nb * P)));
    hipStream_t st = as_stream(stream);
    const size_t lds = sizeof(float) * 2 * P1;
    switch (k) {
#define DR_FL_CASE(K)                                                                      \
    case K:                                                                                \
        if (lds > 65536)                                                                   \
            (void)hipFuncSetAttribute(reinterpret_cast<const void *>(first_layer_bwd_kernel<K>), \
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
        hipLaunchKernelGGL(first_layer_bwd_kernel<K>, dim3(nb, nets), dim3(kBlock), lds, st, \
                           m, (int)n, in, x, rows, part);                                  \
        break;
        DR_FL_CASE(4) DR_FL_CASE(8) DR_FL_CASE(12) DR_FL_CASE(15) DR_FL_CASE(16)
        DR_FL_CASE(18) DR_FL_CASE(24) DR_FL_CASE(32)
#undef DR_FL_CASE
        default:
            return fail0(DR_ERR_UNSUPPORTED,
                         std::string(who) + ": k must be one of 4, 8, 12, 15, 16, 18, 24, 32");
    }
    int rc = check_launch(who);
    if (rc) return rc;
    const int gsize = (nb + kHeadGroups - 1) / kHeadGroups;
    const int ng = (nb + gsize - 1) / gsize;
    hipLaunchKernelGGL(colsum_groups_kernel, dim3((P + kBlock - 1) / kBlock, ng), dim3(kBlock),
                       0, st, nb, P, gsize, part, part2);
    rc = check_launch(who);
    if (rc || defer) return rc;     // defer: level 2 in dr_grad_finish_clip_adam
    hipLaunchKernelGGL(first_layer_finish_kernel, dim3((P + kBlock - 1) / kBlock), dim3(kBlock),
                       0, st, ng, (int)n, (int)k, nets, part2, o);
    return check_launch(who);
}

extern "C++" {
namespace dr {   // gemm_x6.hip
size_t gemm_x6_x_bytes(int64_t m);
int gemm_x6_split_x_launch(int64_t m, int k, const float *x, void *ximg, hipStream_t st);
int gemm_x6_fl_launch(int batch, int64_t m, const float *gz, const void *img, const float *h,
                      const void *ximg, float *part, hipStream_t st);
int gemm_x6_fl_rows(int batch, int64_t m);
}  // namespace dr
}

size_t dr_gemm_x6_x_bytes(int64_t m) { return gemm_x6_x_bytes(m); }

int dr_gemm_x6_split_x(int64_t m, int64_t k, const float *x, void *ximg, void *stream) {
    if (m < 128 || m % 128 || m > (int64_t(1) << 26) || k < 1 || k > 15 || !x || !ximg ||
        (((uintptr_t)ximg) & 15))
        return fail0(DR_ERR_INVALID, "dr_gemm_x6_split_x: bad arguments (m a positive multiple "
                                     "of 128, 1 <= k <= 15, ximg 16-byte aligned)");
    if (gemm_x6_split_x_launch(m, (int)k, x, ximg, as_stream(stream)))
        return fail0(DR_ERR_HIP, std::string("dr_gemm_x6_split_x: ") +
                                     hipGetErrorString(hipGetLastError()));
    return DR_OK;
}

// grad_h1 = grad_z W (the 256 x 256 layer's input gradient, both nets) never
// stored: the first layer's backward (grad_z1 = grad_h1 (1 - h1^2), its
// weight and bias gradients) fused into the GEMM's epilogue, leaving in
// `workspace` exactly what dr_first_layer_backward2(..., defer = 1) leaves
// there (the level-1 grouped partials) for dr_grad_finish.
int64_t dr_gemm_x6_bwd_first_rows(int64_t m) {
    if (m < 128 || m % 128 || m > (int64_t(1) << 26)) return 0;
    return gemm_x6_fl_rows(2, m);
}

int dr_gemm_x6_bwd_first(int64_t batch, int64_t m, int64_t k, const float *grad_z,
                         const void *img, const float *h, const void *ximg, void *workspace,
                         size_t workspace_bytes, int direct, void *stream) {
    const int64_t n = 256;
    if (batch != 2 || m < 128 || m % 128 || m > (int64_t(1) << 26) || k < 1 || k > 15 ||
        !grad_z || !img || !h || !ximg || !workspace ||
        ((((uintptr_t)grad_z) | ((uintptr_t)img) | ((uintptr_t)h) | ((uintptr_t)ximg)) & 15))
        return fail0(DR_ERR_INVALID, "dr_gemm_x6_bwd_first: bad arguments (batch 2, m a positive "
                                     "multiple of 128, 1 <= k <= 15, 16-byte aligned pointers)");
    if (workspace_bytes < first_ws_bytes(2, m, k, n))
        return fail0(DR_ERR_INVALID, "dr_gemm_x6_bwd_first: workspace too small");
    hipStream_t st = as_stream(stream);
    // the fused kernel writes 16 x 256 partials per net (features 0 .. 14,
    // the bias at 15); the workspace's per-net stride is (k + 1) x 256, so
    // k < 15 is laid out by the features it has
    if (k != 15)
        return fail0(DR_ERR_UNSUPPORTED, "dr_gemm_x6_bwd_first: k must be 15 (the drone obs)");
    const int nb_fl = first_blocks(m);
    const int P = (int)(2 * (k + 1) * n);
    float *part = static_cast<float *>(workspace);
    float *part2 = reinterpret_cast<float *>(static_cast<char *>(workspace) +
                                             align_up(sizeof(float) * (size_t)(nb_fl * P)));
    // the kernel writes one partial row per block and net: the workspace
    // holds first_blocks(m) of them, checked before the launch (a device
    // with more CUs than DR_FL_MAXB x 2 is refused, not overrun)
    const int want = gemm_x6_fl_rows(2, m);
    if (want < 1 || want > nb_fl)
        return fail0(DR_ERR_UNSUPPORTED, "dr_gemm_x6_bwd_first: the kernel's grid exceeds the "
                                         "workspace's partial rows on this device");
    const int per = gemm_x6_fl_launch(2, m, grad_z, img, h, ximg, part, st);
    if (per != want)
        return fail0(DR_ERR_HIP, std::string("dr_gemm_x6_bwd_first: ") +
                                     hipGetErrorString(hipGetLastError()));
    // direct: the per-block rows stay at the workspace start for a finish
    // with first_rows = dr_gemm_x6_bwd_first_rows(m) (no level-1 launch)
    if (direct) return DR_OK;
    // level 1 into the group count dr_grad_finish expects of this m
    const int gsize_fl = (nb_fl + kHeadGroups - 1) / kHeadGroups;
    const int ng = (nb_fl + gsize_fl - 1) / gsize_fl;
    const int gsize = (per + ng - 1) / ng;
    hipLaunchKernelGGL(colsum_groups_kernel, dim3((P + kBlock - 1) / kBlock, ng), dim3(kBlock),
                       0, st, per, P, gsize, part, part2);
    return check_launch("dr_gemm_x6_bwd_first");
}

int dr_first_layer_backward(int64_t m, int64_t k, int64_t n, const float *grad_h,
                            const float *h, const float *x, const int32_t *rows, float *grad_w,
                            float *grad_b, void *workspace, size_t workspace_bytes,
                            void *stream) {
    const FirstBwdIn in{{grad_h, nullptr}, {h, nullptr}};
    const FirstBwdOut o{{grad_w, nullptr}, {grad_b, nullptr}};
    return launch_first_bwd("dr_first_layer_backward", 1, m, k, n, in, x, rows, o, workspace,
                            workspace_bytes, stream);
}

int dr_first_layer_backward2(int64_t m, int64_t k, int64_t n, const float *x,
                             const int32_t *rows, const float *grad_h0, const float *h0,
                             float *grad_w0, float *grad_b0, const float *grad_h1,
                             const float *h1, float *grad_w1, float *grad_b1, int defer,
                             void *workspace, size_t workspace_bytes, void *stream) {
    const FirstBwdIn in{{grad_h0, grad_h1}, {h0, h1}};
    const FirstBwdOut o{{grad_w0, grad_w1}, {grad_b0, grad_b1}};
    return launch_first_bwd("dr_first_layer_backward2", 2, m, k, n, in, x, rows, o, workspace,
                            workspace_bytes, stream, defer);
}

}  // extern "C"
