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

#include <hipcub/hipcub.hpp>

#include <cmath>
#include <string>

#include "common.h"

#pragma clang fp contract(off)

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
    uint32_t k0, uint32_t k1, uint64_t counter, float lo, float hi,
    float4 *__restrict__ a_raw, float4 *__restrict__ a_clip,
    float *__restrict__ logp) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
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
        lp += (-(d * d) / (2.0f * var) - logf(sd)) - kLogSqrt2Pi;
    }
    if (a_raw) a_raw[i] = make_float4(a[0], a[1], a[2], a[3]);
    if (a_clip)
        a_clip[i] = make_float4(fminf(fmaxf(a[0], lo), hi), fminf(fmaxf(a[1], lo), hi),
                                fminf(fmaxf(a[2], lo), hi), fminf(fmaxf(a[3], lo), hi));
    if (logp) logp[i] = lp;
}

// Random 64-bit sort keys for the permutation.
__global__ __launch_bounds__(kBlock) void perm_keys_kernel(
    int64_t n, uint32_t k0, uint32_t k1, uint64_t counter,
    uint64_t *__restrict__ keys, int32_t *__restrict__ vals) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const u32x4 r = philox4x32_10(
        u32x4{(uint32_t)i, (uint32_t)((uint64_t)i >> 32), (uint32_t)counter,
              TAG_PERM ^ (uint32_t)(counter >> 32)},
        k0, k1);
    keys[i] = ((uint64_t)r.x << 32) | r.y;
    vals[i] = (int32_t)i;
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
    int64_t m, const float *__restrict__ adv, int64_t stride, float *__restrict__ part) {
    __shared__ float sh[8];
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t cnt = min((int64_t)kBlock, m - (int64_t)blockIdx.x * kBlock);
    const float ai = i < m ? adv[i * stride] : 0.f;
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
    float acc[kLossK] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (i < a.m) {
        const float ls[4] = {a.log_std[0], a.log_std[1], a.log_std[2], a.log_std[3]};
        const float4 mu4 = a.mean[i], ac4 = a.actions[i];
        const float mu[4] = {mu4.x, mu4.y, mu4.z, mu4.w};
        const float ac[4] = {ac4.x, ac4.y, ac4.z, ac4.w};
        float lp = 0.f, zz[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float sd = expf(ls[j]);
            const float d = ac[j] - mu[j];
            const float var = sd * sd;
            zz[j] = d / var;             // d logp / d mu_j
            lp += (-(d * d) / (2.0f * var) - logf(sd)) - kLogSqrt2Pi;
        }
        float A = a.adv[i * a.stride];
        if (a.normalize) A = (A - amean) / (astd + 1e-8f);
        const float logr = lp - a.old_logp[i * a.stride];
        const float r = expf(logr);
        const float lo = 1.0f - a.clip, hi = 1.0f + a.clip;
        const float rc = fminf(fmaxf(r, lo), hi);
        const float l1 = A * r, l2 = A * rc;
        const float inv_m = 1.0f / (float)a.m;
        // policy_loss = -mean(min(l1, l2))
        acc[0] = -fminf(l1, l2);
        float g1 = l1 < l2 ? 1.f : (l1 == l2 ? 0.5f : 0.f);
        float g2 = l2 < l1 ? 1.f : (l1 == l2 ? 0.5f : 0.f);
        const float dclamp = (r >= lo && r <= hi) ? 1.f : 0.f;
        const float dr = -(g1 * A + g2 * A * dclamp) * inv_m;  // dL/dratio
        const float dlp = dr * r;                              // dL/dlogp
        // value loss: vf_coef * mean((R - V)^2)
        const float v = a.values[i];
        const float R = a.ret[i * a.stride];
        const float e = R - v;
        acc[1] = e * e;
        a.grad_values[i] = a.vf_coef * (2.0f * (v - R)) * inv_m;
        acc[2] = (fabsf(r - 1.0f) > a.clip) ? 1.f : 0.f;
        acc[3] = (r - 1.0f) - logr;                       // approx_kl term
        a.grad_mean[i] = make_float4(dlp * zz[0], dlp * zz[1], dlp * zz[2], dlp * zz[3]);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float d = ac[j] - mu[j];
            const float sd = expf(ls[j]);
            // d logp / d log_std_j = d^2 / var - 1
            acc[4 + j] = dlp * ((d * d) / (sd * sd) - 1.0f);
        }
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
// clip_grad_norm_ + Adam over one flat fp32 buffer.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void sumsq_kernel(int64_t n,
                                                       const float *__restrict__ g,
                                                       float *__restrict__ part) {
    __shared__ float sh[4];
    float acc = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kBlock) {
        const float x = g[i];
        acc += x * x;
    }
    float x[1] = {acc};
    block_sum<1>(x, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = x[0];
}

__global__ __launch_bounds__(kBlock) void clip_adam_kernel(
    int64_t n, float *__restrict__ p, float *__restrict__ g,
    float *__restrict__ m, float *__restrict__ v, const float *__restrict__ part,
    int nb, float max_norm, float w1, float beta2, float one_m_b2,
    float step_size, float bc2_sqrt, float eps, float *norm_out) {
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
        const float gi = g[i] * c;
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
                       (uint32_t)seed, (uint32_t)(seed >> 32), counter, lo, hi,
                       reinterpret_cast<float4 *>(actions_raw),
                       reinterpret_cast<float4 *>(actions_clipped), logp);
    return check_launch("dr_policy_sample");
}

static size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

size_t dr_permutation_workspace_bytes(int64_t n) {
    if (n <= 0) return 0;
    size_t temp = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, temp, (uint64_t *)nullptr,
                                       (uint64_t *)nullptr, (int32_t *)nullptr,
                                       (int32_t *)nullptr, (int)n, 0, 64, (hipStream_t)0);
    return align_up(sizeof(uint64_t) * n) * 2 + align_up(sizeof(int32_t) * n) + align_up(temp);
}

int dr_permutation(int64_t n, uint64_t seed, uint64_t counter, int32_t *out,
                   void *workspace, size_t workspace_bytes, void *stream) {
    if (n < 0 || n > 0x7fffffff || !out) return fail0(DR_ERR_INVALID, "dr_permutation: bad arguments");
    if (n == 0) return DR_OK;
    const size_t need = dr_permutation_workspace_bytes(n);
    if (!workspace || workspace_bytes < need)
        return fail0(DR_ERR_INVALID, "dr_permutation: workspace too small");
    char *w = static_cast<char *>(workspace);
    uint64_t *k_in = reinterpret_cast<uint64_t *>(w);
    w += align_up(sizeof(uint64_t) * n);
    uint64_t *k_out = reinterpret_cast<uint64_t *>(w);
    w += align_up(sizeof(uint64_t) * n);
    int32_t *v_in = reinterpret_cast<int32_t *>(w);
    w += align_up(sizeof(int32_t) * n);
    size_t temp = need - (size_t)(w - static_cast<char *>(workspace));
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(perm_keys_kernel, dim3(grid_for(n)), dim3(kBlock), 0, st, n,
                       (uint32_t)seed, (uint32_t)(seed >> 32), counter, k_in, v_in);
    int rc = check_launch("dr_permutation keys");
    if (rc) return rc;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(w, temp, k_in, k_out, v_in, out, (int)n,
                                                      0, 64, st);
    if (e != hipSuccess)
        return fail0(DR_ERR_HIP, std::string("dr_permutation sort: ") + hipGetErrorString(e));
    return DR_OK;
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
                           aux_stride, adv_part);
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
    hipLaunchKernelGGL(sumsq_kernel, dim3(nb), dim3(kBlock), 0, st, n, grads, part);
    int rc = check_launch("dr_clip_adam norm");
    if (rc) return rc;
    // torch.optim.Adam scalars, formed in double as torch does on the host.
    const double b1 = beta1, b2 = beta2;
    const double bc1 = 1.0 - std::pow(b1, (double)step);
    const double bc2 = 1.0 - std::pow(b2, (double)step);
    const float step_size = (float)(lr / bc1);
    const float bc2_sqrt = (float)std::sqrt(bc2);
    hipLaunchKernelGGL(clip_adam_kernel, dim3(nb), dim3(kBlock), 0, st, n, params, grads,
                       exp_avg, exp_avg_sq, part, nb, max_grad_norm, (float)(1.0 - b1),
                       (float)b2, (float)(1.0 - b2), step_size, bc2_sqrt, (float)eps,
                       grad_norm_out);
    return check_launch("dr_clip_adam");
}

}  // extern "C"
