// Batched quadrotor environment for MI355X (gfx950).
//
// One HIP thread owns one env for the whole step: the state lives in HBM as a
// struct of arrays (15 arrays of N: pos xyz, vel xyz, euler xyz, omega xyz,
// target xyz, then step / ep_num / eps / monitor counters), so every state
// load and store of a wave is one contiguous 512 B (f64) or 256 B (f32)
// transaction.  Actions arrive as (N,4) f32 (one 16 B load per lane).  The
// (N,15) f32 observation rows (60 B, not 16 B aligned per env) are staged
// through LDS and leave the block as contiguous float4 stores.
//
// Physics: the reference's op order, restated from
//   DroneEnv.step            /root/reference/drone.py:81-159
//   DroneEnv._rotation_matrix /root/reference/drone.py:161-174 (column 2 only)
//   DroneEnv._euler_angle_rates /root/reference/drone.py:176-186
//   DroneEnv.reset           /root/reference/drone.py:48-75
//   DroneEnv._get_obs        /root/reference/drone.py:77-79
//   VectorizedDroneEnv.*     /root/reference/vectorized_drone.py:38-216
// compiled with -ffp-contract=off so no product/sum pair is fused into an FMA
// that numpy would round twice.  The state scalar S is double (reference
// precision) or float (throughput mode).

#include <cstdlib>
#include <cstring>
#include <hip/hip_ext.h>
#include <new>
#include <string>

#include "common.h"
#include "trig.h"

#pragma clang fp contract(off)

namespace dr {
namespace {

// Physical constants (drone.py:14-43, 263; vectorized_drone.py:13-33).
constexpr double kG = 9.81;
constexpr double kMass = 1.0;
constexpr double kIxx = 0.005, kIyy = 0.005, kIzz = 0.01;
constexpr double kArm = 0.5;
constexpr double kFactor = kArm / 1.4142135623730951;  // L / np.sqrt(2)
constexpr float kKyaw32 = 0.01f;  // python float * np.float32 -> f32 (NEP 50)
constexpr double kDt = 0.02;

#ifndef DR_STRIDE_PAD
#define DR_STRIDE_PAD 0
#endif
// DR_STAMPS (diagnostic builds only): per-wave s_memrealtime / s_memtime
// stamps at phase boundaries of env_step_kernel into a module-scope array,
// read back by dr_diag_stamps (scripts/micro/stamps.py).  Never set in the
// product build; no output element is computed from a stamp.
#ifndef DR_STAMPS
#define DR_STAMPS 0
#endif
#if DR_STAMPS
__device__ unsigned long long g_stamps[16384 * 8];
#define DR_STAMP(k)                                                            \
    do {                                                                       \
        __builtin_amdgcn_sched_barrier(0);                                     \
        const unsigned long long t__ = __builtin_amdgcn_s_memrealtime();       \
        const unsigned w__ = blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);   \
        const unsigned long long m__ = __ballot(1);                          \
        if ((int)(threadIdx.x & 63) == __ffsll((long long)m__) - 1 && w__ < 16384) \
            g_stamps[w__ * 8 + (k)] = t__;                                     \
        __builtin_amdgcn_sched_barrier(0);                                     \
    } while (0)
#else
#define DR_STAMP(k) \
    do {            \
    } while (0)
#endif
// 1: obs staged per wave (no block barrier); 0: per block
#ifndef DR_WAVE_STAGE
#define DR_WAVE_STAGE 1
#endif
// 1 (A/B builds only; measured no gain): the Philox block of the reset draws
// is computed for every lane right after the loads are issued (keyed by
// ep_num + 1, loaded first), instead of in the divergent reset branch
#ifndef DR_HOIST_RESET
#define DR_HOIST_RESET 0
#endif
// waves per workgroup of env_step_kernel (A/B builds: 1, 2, 4)
#ifndef DR_ENV_WPB
#define DR_ENV_WPB 4
#endif
constexpr int kEnvBlock = 64 * DR_ENV_WPB;
// steps per group of the rollout kernels' next-reset Philox draw-ahead
constexpr int kResetAhead = 8;

// 1: the observation is formed once, after the auto-reset (the terminal
// obs only when requested); 0: formed before the reset and again for the
// reset rows
#ifndef DR_OBS_ONCE
#define DR_OBS_ONCE 1
#endif

// 1: per-step outputs and state are written with nontemporal stores.  They
// stream to HBM while the kernel runs instead of sitting dirty in L2 until
// the end-of-kernel writeback (4-9 % faster from 65,536 to 4M envs).
// 1: the step kernel's loads are all waited for before its first store
// (see env_step_kernel); 0 (A/B only): the compiler's own wait placement
#ifndef DR_LOADS_LANDED
#define DR_LOADS_LANDED 1
#endif
#ifndef DR_NT_STORES
#define DR_NT_STORES 1
#endif
// State loads: nontemporal (NTL) only in the large-batch launch form, where
// they measured faster; at 131,072 envs they measured 28 % slower.
template <bool NTL, typename T>
__device__ inline T ld_in(const T *p) {
    if constexpr (NTL) return __builtin_nontemporal_load(p);
    else return *p;
}
template <typename T>
__device__ inline void st_out(T *p, T x) {
    if (DR_NT_STORES) store_nt(p, x);
    else *p = x;
}
// N of the Euler angles at once: the fast path runs unconditionally for
// all N (independent chains interleave; the polynomial constants are
// materialised once), the library path only for out-of-range lanes.  Each
// angle's result depends on that angle alone.
template <int N, typename S>
__device__ inline void m_sincos_n(const S *x, S *s, S *c) {
    if constexpr (sizeof(S) == 8) {
        // trig.h: 3-FMA reduction + shared polynomials (<= 1 ulp); the
        // library sincos only for |x| >= 2^19 rad, inf and NaN (a branch no
        // lane usually takes)
        int fast = 1;
#pragma unroll
        for (int k = 0; k < N; ++k) {
            const SinCos t = sincos_medium(x[k]);
            s[k] = t.s;
            c[k] = t.c;
            fast &= (int)sincos_fast_range(x[k]);
        }
        if (!fast) {
#pragma unroll
            for (int k = 0; k < N; ++k)
                if (!sincos_fast_range(x[k])) sincos(x[k], &s[k], &c[k]);
        }
    } else {
        // f32 state mode: trig.h's sincosf_medium (f64 reduction, f32
        // polynomials, <= 2 ulp); the library sincosf only out of range
        int fast = 1;
#pragma unroll
        for (int k = 0; k < N; ++k) {
            const SinCosF t = sincosf_medium(x[k]);
            s[k] = t.s;
            c[k] = t.c;
            fast &= (int)sincosf_fast_range(x[k]);
        }
        if (!fast) {
#pragma unroll
            for (int k = 0; k < N; ++k)
                if (!sincosf_fast_range(x[k])) sincosf(x[k], &s[k], &c[k]);
        }
    }
}
template <typename S>
__device__ inline void m_sincos3(const S x[3], S s[3], S c[3]) {
    m_sincos_n<3>(x, s, c);
}
__device__ inline double m_sqrt(double x) { return sqrt(x); }
__device__ inline float m_sqrt(float x) { return sqrtf(x); }

__device__ inline double m_fma(double a, double b, double c) { return fma(a, b, c); }
__device__ inline float m_fma(float a, float b, float c) { return fmaf(a, b, c); }

// x / d given rd = RN(1/d): q = RN(x*rd), then one Markstein correction with
// the exact FMA remainder, giving the correctly rounded quotient (up to
// rare 1-ulp cases) in 3 instructions instead of the ~10 of an IEEE divide.
template <typename S>
__device__ inline S div_rcp(S x, S d, S rd) {
    const S q = x * rd;
    const S r = m_fma(-q, d, x);
    return m_fma(r, rd, q);
}

enum : int { F_POS = 0, F_VEL = 3, F_EUL = 6, F_OMG = 9, F_TGT = 12, F_N = 15 };

template <typename S>
struct EnvView {
    S *f;             // F_N arrays, array k at f + k * stride
    int64_t stride;
    int32_t *step;
    int32_t *ep_num;
    double *eps;
    float *ep_ret;
    int32_t *ep_len;
    float *mot;       // moving variant: 9 f32 arrays (a xyz, w xyz, ph xyz)
    int64_t n;
    int64_t env_id_offset;
    const double *host_u;  // DR_RNG_HOST_UNIFORMS buffer, else nullptr
    uint32_t seed_lo, seed_hi;
    int32_t max_steps;
    S dt;
    __host__ __device__ S *field(int k) const { return f + k * stride; }
};

// Byte offsets of the per-env arrays inside a handle's one allocation of
// `sp` (stride) elements per array: F_N state arrays of S, then eps (f64),
// step, ep_num (i32), the VecMonitor return (f32) and length (i32), then the
// moving variant's 9 f32 motion arrays.  Shared by view_of and the step
// kernel, which forms its array bases from (f, stride) in scalar registers.
template <typename S>
struct Layout {
    __host__ __device__ static int64_t eps(int64_t sp) { return (int64_t)F_N * sp * sizeof(S); }
    __host__ __device__ static int64_t step(int64_t sp) { return eps(sp) + sp * 8; }
    __host__ __device__ static int64_t ep_num(int64_t sp) { return step(sp) + sp * 4; }
    __host__ __device__ static int64_t ep_ret(int64_t sp) { return ep_num(sp) + sp * 4; }
    __host__ __device__ static int64_t ep_len(int64_t sp) { return ep_ret(sp) + sp * 4; }
    __host__ __device__ static int64_t mot(int64_t sp) { return ep_len(sp) + sp * 4; }
};

// The step kernel's per-field base pointers (f + k * stride), passed as
// separate uniform kernel arguments so each SoA access is an SGPR base plus
// one shared 32-bit lane offset (the compiler folds f + k*stride + i*8 into
// per-field 64-bit VGPR address arithmetic otherwise).  Kernel-argument
// preloading into SGPRs (gfx950) was measured as the alternative: slower by
// 0.1 us at 65,536 envs (the scalar address chain it needs costs more than
// the one scalar-load round trip it saves).
template <typename S>
struct FieldPtrs {
    S *p[F_N];
    int32_t *step, *ep_num;
    double *eps;
};

struct StepIO {
    const float *actions;
    float *obs;
    float *rew;
    uint8_t *done;
    float *term_obs;
    float *ep_ret_out;
    int32_t *ep_len_out;
    int auto_reset;
    // MON only, nullable: 1 where the episode ended at the step limit
    // without a crash (the gymnasium TimeLimit "truncated" flag)
    uint8_t *trunc_out;
};

// The five reset draws of env i starting episode `ep_new`, in the reference
// order: pos x, pos y, target x, y, z (drone.py:57,73).  mode: 0 Philox,
// 1 host buffer, 2 constant 0.5 (constructor reset in host-uniform mode).
// NU = 5 (gym) or 14 (moving: the 5 gym draws, then 9 motion draws; the
// first 5 are the gym variant's, so eps = 0 reproduces it exactly).
template <int NU, typename S>
__device__ inline void reset_uniforms(const EnvView<S> &v, int64_t i,
                                      int32_t ep_new, int mode, double u[NU],
                                      const u32x4 *pre = nullptr) {
    if (mode == 1) {
#pragma unroll
        for (int k = 0; k < NU; ++k) u[k] = v.host_u[i * NU + k];
        return;
    }
    if (mode == 2) {
#pragma unroll
        for (int k = 0; k < NU; ++k) u[k] = 0.5;
        return;
    }
    const uint64_t gid = (uint64_t)(v.env_id_offset + i);
#pragma unroll
    for (int b = 0; b < (NU + 3) / 4; ++b) {
        // pre: the blocks already drawn for this (episode, env)
        const u32x4 r = pre ? pre[b]
                            : philox4x32_10(u32x4{(uint32_t)ep_new, (uint32_t)gid,
                                                  (uint32_t)(gid >> 32), TAG_RESET | (uint32_t)b},
                                            v.seed_lo, v.seed_hi);
        const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (4 * b + k < NU) u[4 * b + k] = u01_w32(w[k]);
    }
}

// DroneEnv.reset (drone.py:48-75) on registers st[F_N]; updates ep_num/eps
// in memory, returns the new step counter (0).
template <typename S>
__device__ inline void gym_reset_regs(const EnvView<S> &v, int64_t i, int mode,
                                      S st[F_N], int32_t ep_old, double eps,
                                      const u32x4 *pre0 = nullptr) {
    const int32_t ep_new = ep_old + 1;        // ep_num += 1          (61)
    if (ep_new % 2000 == 0) {                 // curriculum bump      (68-70)
        eps += 0.1;
        v.eps[i] = eps;
    }
    double u[5];
    if (mode == 0) {
        // Philox block 0 = (pos x, pos y, target x, target y); block 1 word
        // 0 = target z.  The target draws are multiplied by eps, and 0 * u
        // is exactly +0 for the uniforms in [0,1): while the curriculum is
        // at eps == 0 (the first 2000 episodes of every env) block 1 cannot
        // change any result bit, so it is skipped.
        const uint64_t gid = (uint64_t)(v.env_id_offset + i);
        const u32x4 r0 = pre0 ? *pre0
                              : philox4x32_10(u32x4{(uint32_t)ep_new, (uint32_t)gid,
                                                    (uint32_t)(gid >> 32), TAG_RESET},
                                              v.seed_lo, v.seed_hi);
        u[0] = u01_w32(r0.x);
        u[1] = u01_w32(r0.y);
        u[2] = u01_w32(r0.z);
        u[3] = u01_w32(r0.w);
        u[4] = 0.0;
        if (eps != 0.0) {
            const u32x4 r1 = philox4x32_10(
                u32x4{(uint32_t)ep_new, (uint32_t)gid, (uint32_t)(gid >> 32), TAG_RESET | 1u},
                v.seed_lo, v.seed_hi);
            u[4] = u01_w32(r1.x);
        }
    } else {
        reset_uniforms<5>(v, i, ep_new, mode, u);
    }
    DR_STAMP(6);
    v.ep_num[i] = ep_new;
    st[F_POS + 0] = (S)(u[0] - 0.5);          // (57)
    st[F_POS + 1] = (S)(u[1] - 0.5);
    st[F_POS + 2] = (S)1.0;
#pragma unroll
    for (int k = 3; k < 12; ++k) st[k] = (S)0;   // vel, euler, omega (58-60)
    st[F_TGT + 0] = (S)(eps * u[2]);          // (73)
    st[F_TGT + 1] = (S)(eps * u[3]);
    st[F_TGT + 2] = (S)(eps * u[4] + 1.0 + 0.0);
    DR_STAMP(7);
}

// The state DroneEnv.reset would start episode ep_old + 1 from (drone.py:
// 48-75), formed from that episode's first Philox block r0 exactly as
// gym_reset_regs forms it (the curriculum bump, then the draws, the same
// expressions), so that a reset inside the split-physics rollout kernel is a
// register copy of state prepared when the block was drawn, off the step in
// which some lane of the wave resets (round 5).
template <typename S>
struct GymNext {
    S px, py, tx, ty, tz;
    double eps;               // eps after episode ep_old + 1's curriculum bump
    bool bump;                // ep_old + 1 bumps the curriculum
};
template <typename S>
__device__ inline GymNext<S> gym_next_reset(const EnvView<S> &v, uint64_t gid, int32_t ep_old,
                                            double eps, const u32x4 &r0) {
    const int32_t ep_new = ep_old + 1;
    GymNext<S> g;
    g.bump = ep_new % 2000 == 0;
    if (g.bump) eps += 0.1;
    double u4 = 0.0;
    if (eps != 0.0) {
        const u32x4 r1 = philox4x32_10(
            u32x4{(uint32_t)ep_new, (uint32_t)gid, (uint32_t)(gid >> 32), TAG_RESET | 1u},
            v.seed_lo, v.seed_hi);
        u4 = u01_w32(r1.x);
    }
    g.px = (S)(u01_w32(r0.x) - 0.5);
    g.py = (S)(u01_w32(r0.y) - 0.5);
    g.tx = (S)(eps * u01_w32(r0.z));
    g.ty = (S)(eps * u01_w32(r0.w));
    g.tz = (S)(eps * u4 + 1.0 + 0.0);
    g.eps = eps;
    return g;
}

template <typename S>
__device__ inline void vec_reset_regs(S st[F_N]) {
    // VectorizedDroneEnv.reset: every env at (0.1,0.1,0.1), at rest
    // (vectorized_drone.py:50-53); fixed target (0,0,10) (line 30).
#pragma unroll
    for (int k = 0; k < 3; ++k) st[F_POS + k] = (S)0.1;
#pragma unroll
    for (int k = 3; k < 12; ++k) st[k] = (S)0;
    st[F_TGT + 0] = (S)0;
    st[F_TGT + 1] = (S)0;
    st[F_TGT + 2] = (S)10.0;
}

// ---- moving-target variant (DR_VARIANT_MOVING) ----
// target_k(s) = c_k + a_k sin(w_k s dt + ph_k), velocity a_k w_k cos(...),
// evaluated in f32 (the motion is this build's spec, not the reference's).
template <typename S>
__device__ inline void moving_target(const S c[3], const float mp[9], int32_t s,
                                     float dt, S tgt[3], float tvel[3]) {
    const float t = (float)s * dt;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        float sn, cs;
        sincosf(mp[3 + k] * t + mp[6 + k], &sn, &cs);
        tgt[k] = c[k] + (S)(mp[k] * sn);
        tvel[k] = mp[k] * mp[3 + k] * cs;
    }
}

// DroneEnv.reset plus the motion draws: pos / zeroed rates / centre exactly
// as gym_reset_regs (centre = the gym target), a = eps * U, w = 0.5 + 1.5 U
// rad/s, ph = 2 pi U.
template <typename S>
__device__ inline void moving_reset_regs(const EnvView<S> &v, int64_t i, int mode,
                                         S st[F_N], S c[3], float mp[9],
                                         int32_t ep_old, double eps,
                                         const u32x4 *pre4 = nullptr) {
    const int32_t ep_new = ep_old + 1;
    double u[14];
    reset_uniforms<14>(v, i, ep_new, mode, u, pre4);
    if (ep_new % 2000 == 0) {
        eps += 0.1;
        v.eps[i] = eps;
    }
    v.ep_num[i] = ep_new;
    st[F_POS + 0] = (S)(u[0] - 0.5);
    st[F_POS + 1] = (S)(u[1] - 0.5);
    st[F_POS + 2] = (S)1.0;
#pragma unroll
    for (int k = 3; k < 12; ++k) st[k] = (S)0;
    c[0] = (S)(eps * u[2]);
    c[1] = (S)(eps * u[3]);
    c[2] = (S)(eps * u[4] + 1.0 + 0.0);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        mp[k] = (float)(eps * u[5 + k]);
        mp[3 + k] = (float)(0.5 + 1.5 * u[8 + k]);
        mp[6 + k] = (float)(6.283185307179586 * u[11 + k]);
    }
}

template <typename S, int OD>
__device__ inline void make_obs(const S st[F_N], float ob[OD],
                                const float *tvel = nullptr) {
    // _get_obs: f32(concat(pos, vel, euler, omega[, target - pos]))  (79)
#pragma unroll
    for (int k = 0; k < 12; ++k) ob[k] = (float)st[k];
    if constexpr (OD >= 15) {
#pragma unroll
        for (int k = 0; k < 3; ++k) ob[12 + k] = (float)(st[F_TGT + k] - st[F_POS + k]);
    }
    if constexpr (OD == 18) {
#pragma unroll
        for (int k = 0; k < 3; ++k) ob[15 + k] = tvel[k];
    }
}

// One physics step on registers.  Returns the reward, sets `crash` (z<0 or
// |p|>50).  VAR selects the two places the variants differ (W row 3 and the
// reward form / bonus radius).
// The action's motor mixes (drone.py:106, 113-117): total thrust and the
// three torques' f32 sums, before any state is involved.
struct MotorMix {
    float thr, phi, theta, psi;
};
__device__ inline MotorMix motor_mix(float4 act) {
    const float a0 = act.x, a1 = act.y, a2 = act.z, a3 = act.w;
    return MotorMix{((a0 + a1) + a2) + a3, ((a0 + a1) - a2) - a3,
                    ((-a0 + a1) + a2) - a3, ((a0 - a1) + a2) - a3};
}

template <typename S, int VAR>
__device__ inline S physics_step_mixed(S st[F_N], MotorMix mx, S dt, bool &crash) {
    // thrust / torques (drone.py:106, 113-117): f32 sums, f64 factor product,
    // the yaw torque stays f32.
    const float thr = mx.thr;
    const S tau_phi = (S)kFactor * (S)mx.phi;
    const S tau_theta = (S)kFactor * (S)mx.theta;
    const float tau_psi = kKyaw32 * mx.psi;

    // One sincos per angle: a shared range reduction yields exactly the
    // separate sin() and cos() results at half the instructions.
    S sn[3], cs[3];
    m_sincos3(&st[F_EUL], sn, cs);
    DR_STAMP(1);
    const S sph = sn[0], cph = cs[0], sth = sn[1], cth = cs[1], sps = sn[2], cps = cs[2];
    // R(old euler) column 2 (drone.py:169-173): thrust is body-z only.
    const S r02 = cps * sth * cph + sps * sph;
    const S r12 = sps * sth * cph - cps * sph;
    const S r22 = cth * cph;
    const S T = (S)thr;
    const S acc0 = (S)0 + (r02 * T) / (S)kMass;      // (124)
    const S acc1 = (S)0 + (r12 * T) / (S)kMass;
    const S acc2 = (S)(-kG) + (r22 * T) / (S)kMass;
    st[F_VEL + 0] += acc0 * dt;                      // (127)
    st[F_VEL + 1] += acc1 * dt;
    st[F_VEL + 2] += acc2 * dt;
#pragma unroll
    for (int k = 0; k < 3; ++k) st[F_POS + k] += st[F_VEL + k] * dt;  // (128)

    // Euler-angle rates from the OLD omega (131-132, 176-186).
    const S w0 = st[F_OMG + 0], w1 = st[F_OMG + 1], w2 = st[F_OMG + 2];
    // tan(theta) from the shared sincos (np.tan rounds once; this rounds the
    // quotient once more: <= 2 ulp apart, far inside the parity bar).
    const S sec = (S)1 / cth;        // the only IEEE divide; also vd:116
    const S tth = div_rcp(sth, cth, sec);
    S ed2;
    if constexpr (VAR != DR_VARIANT_VECTORIZED) {
        ed2 = ((S)0 * w0 + div_rcp(sph, cth, sec) * w1) +
              div_rcp(cph, cth, sec) * w2;                             // (184)
    } else {
        ed2 = ((S)0 * w0 + (sph * sec) * w1) + (cph * sec) * w2;
    }
    const S ed0 = ((S)1 * w0 + (sph * tth) * w1) + (cph * tth) * w2;
    const S ed1 = ((S)0 * w0 + cph * w1) + (-sph) * w2;
    st[F_EUL + 0] += ed0 * dt;
    st[F_EUL + 1] += ed1 * dt;
    st[F_EUL + 2] += ed2 * dt;

    // Angular dynamics, diagonal inertia, old omega (135-139).
    const S wd0 = div_rcp(tau_phi - (S)(kIyy - kIzz) * w1 * w2, (S)kIxx, (S)(1.0 / kIxx));
    const S wd1 = div_rcp(tau_theta - (S)(kIzz - kIxx) * w0 * w2, (S)kIyy, (S)(1.0 / kIyy));
    const S wd2 = div_rcp((S)tau_psi - (S)(kIxx - kIyy) * w0 * w1, (S)kIzz, (S)(1.0 / kIzz));
    st[F_OMG + 0] += wd0 * dt;
    st[F_OMG + 1] += wd1 * dt;
    st[F_OMG + 2] += wd2 * dt;

    // Reward on the new position (142-148; vectorized_drone.py:204-207).
    const S dx = st[F_POS + 0] - st[F_TGT + 0];
    const S dy = st[F_POS + 1] - st[F_TGT + 1];
    const S dz = st[F_POS + 2] - st[F_TGT + 2];
    const S d = m_sqrt((dx * dx + dy * dy) + dz * dz);
    S r;
    if constexpr (VAR != DR_VARIANT_VECTORIZED) {
        r = (S)0.01 * -d;
        if (d < (S)0.05) r += (S)1;
    } else {
        r = (S)(-0.01) * d;
        if (d < (S)1) r += (S)1;
    }
    // Termination (154; vectorized_drone.py:211).  NaN compares false.
    const S px = st[F_POS + 0], py = st[F_POS + 1], pz = st[F_POS + 2];
    // norm(p) > 50  <=>  |p|^2 > 2500 exactly: sqrt is correctly rounded and
    // the next representable square above 2500 already rounds above 50
    // (f64 and f32 alike); NaN compares false either way.
    const S pn2 = (px * px + py * py) + pz * pz;
    crash = (pz < (S)0) || (pn2 > (S)2500);
    return r;
}

template <typename S, int VAR>
__device__ inline S physics_step(S st[F_N], float4 act, S dt, bool &crash) {
    return physics_step_mixed<S, VAR>(st, motor_mix(act), dt, crash);
}

// Per-wave variant: each wave stages its own 64 rows (3,840 B) and writes
// them out with no workgroup barrier, so a wave delayed by a reset or a late
// load does not hold back the other three waves of its block.
template <int OD, int RPW = 64>
__device__ inline void store_obs_wave(float *sh_block, const float ob[OD],
                                      float *dst_all, int64_t n) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float *sh = sh_block + w * RPW * OD;
    if (lane < RPW) {
#pragma unroll
        for (int k = 0; k < OD; ++k) sh[lane * OD + k] = ob[k];
    }
    // DS ops of one wave execute in order; the barrier only pins the
    // compiler's schedule (no workgroup s_barrier is emitted)
    __builtin_amdgcn_wave_barrier();
    const int64_t wbase = (int64_t)blockIdx.x * (DR_ENV_WPB * RPW) + w * RPW;
    const int64_t nvalid = (n - wbase) < RPW ? (n - wbase) : RPW;
    if (nvalid <= 0) return;
    float *dst = dst_all + wbase * OD;
    if (nvalid == RPW && (((uintptr_t)dst) & 15) == 0) {
        const float4 *s4 = reinterpret_cast<const float4 *>(sh);
        float4 *d4 = reinterpret_cast<float4 *>(dst);
#pragma unroll
        for (int q = lane; q < RPW * OD / 4; q += 64) st_out(&d4[q], s4[q]);
    } else {
        for (int q = lane; q < (int)nvalid * OD; q += 64) dst[q] = sh[q];
    }
}

template <int OD>
__device__ inline void store_obs_block(float *sh, const float ob[OD],
                                       float *dst_all, int64_t base,
                                       int64_t n) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int k = 0; k < OD; ++k) sh[tid * OD + k] = ob[k];
    __syncthreads();
    const int64_t nvalid = (n - base) < kBlock ? (n - base) : kBlock;
    float *dst = dst_all + base * OD;
    const int total = (int)nvalid * OD;
    if (nvalid == kBlock && (((uintptr_t)dst) & 15) == 0) {
        const float4 *s4 = reinterpret_cast<const float4 *>(sh);
        float4 *d4 = reinterpret_cast<float4 *>(dst);
#pragma unroll
        for (int q = tid; q < kBlock * OD / 4; q += kBlock) d4[q] = s4[q];
    } else {
        for (int q = tid; q < total; q += kBlock) dst[q] = sh[q];
    }
}

// Element i of a per-env array at a uniform (SGPR) base: the byte offset
// i * sizeof(T) is formed in 32 bits (dr_create caps a handle at 2^28 envs),
// so every SoA access of a wave is one `global_load/store ... v_off, s[base]`
// sharing ONE offset VGPR per element size, with no per-field 64-bit address
// arithmetic ahead of the loads.
template <typename T>
__device__ inline T *at(T *base, int64_t i) {
    return reinterpret_cast<T *>(reinterpret_cast<char *>(base) +
                                 (uint32_t)((uint32_t)i * (uint32_t)sizeof(T)));
}
template <typename T>
__device__ inline const T *at(const T *base, int64_t i) {
    return reinterpret_cast<const T *>(reinterpret_cast<const char *>(base) +
                                       (uint32_t)((uint32_t)i * (uint32_t)sizeof(T)));
}

// HU: reset draws from the host-uniform ring (parity mode).  A template
// parameter, not a runtime branch, so the Philox reset path holds no global
// load: a load there would make the waitcnt pass drain every outstanding
// store of the wave (vmcnt counts stores too) before the reset could finish.
//
// Entry: lanes past the batch end (ragged n, half-populated waves) load the
// last env's row instead of branching around the loads and only their
// stores are masked, so the kernel's first basic block holds every
// kernel-argument load and every state load: one scalar-load round trip
// before the first global load is issued, not two.
template <typename S, int VAR, bool MON, int RPW, bool HU, bool NTL>
__global__ __launch_bounds__(kEnvBlock) void env_step_kernel(EnvView<S> v,
                                                             StepIO io, FieldPtrs<S> fp) {
    constexpr int OD = VAR == DR_VARIANT_GYM ? 15 : (VAR == DR_VARIANT_MOVING ? 18 : 12);
    constexpr bool GYMLIKE = VAR != DR_VARIANT_VECTORIZED;
    __shared__ float4 sh4[kEnvBlock * OD / 4];
    // Every kernel argument the state loads need is materialised here, in
    // ONE batch of scalar loads: the compiler otherwise issues them in three
    // dependent rounds (n, then the field pointers, then the rest), each a
    // full scalar-memory round trip ahead of the first state load.
    asm volatile("" ::"s"(v.n), "s"(fp.p[0]), "s"(fp.p[1]), "s"(fp.p[2]), "s"(fp.p[3]),
                 "s"(fp.p[4]), "s"(fp.p[5]), "s"(fp.p[6]), "s"(fp.p[7]), "s"(fp.p[8]),
                 "s"(fp.p[9]), "s"(fp.p[10]), "s"(fp.p[11]), "s"(fp.p[12]), "s"(fp.p[13]),
                 "s"(fp.p[14]), "s"(io.actions), "s"(fp.step), "s"(fp.ep_num), "s"(fp.eps));
    __builtin_amdgcn_sched_barrier(0);
    const int64_t n_ = v.n;
    const float4 *const actions = reinterpret_cast<const float4 *>(io.actions);
    int32_t *const p_step = fp.step;
    int32_t *const p_epn = fp.ep_num;
    double *const p_eps = fp.eps;
    const int64_t base = (int64_t)blockIdx.x * (DR_ENV_WPB * RPW);
    const int lane_ = threadIdx.x & 63;
    // env of this lane; lanes >= RPW of a half-populated wave own none
    const int64_t i_own = lane_ < RPW ? base + (threadIdx.x >> 6) * RPW + lane_ : n_;
    const bool live = i_own < n_;
    const int64_t i = live ? i_own : n_ - 1;           // in-bounds row for dead lanes
    DR_STAMP(0);
    float ob[OD];
    S st[F_N];
    int32_t ep_old = 0;
    if constexpr (GYMLIKE && DR_HOIST_RESET) ep_old = *at(p_epn, i);
    // Issue order = landing order: euler and omega first so the three
    // sincos range reductions start while pos / vel / target are still in
    // flight (s_waitcnt vmcnt counts oldest-first).
#pragma unroll
    for (int k = F_EUL; k < F_EUL + 3; ++k) st[k] = ld_in<NTL>(at(fp.p[k], i));
    __builtin_amdgcn_sched_barrier(0);     // keep the issue order (euler first)
#pragma unroll
    for (int k = F_OMG; k < F_OMG + 3; ++k) st[k] = ld_in<NTL>(at(fp.p[k], i));
    const float4 act = *at(actions, i);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < F_EUL; ++k) st[k] = ld_in<NTL>(at(fp.p[k], i));
    S cen[3];
    float mp[9], tvel[3];
    if constexpr (VAR == DR_VARIANT_GYM) {
#pragma unroll
        for (int k = F_TGT; k < F_N; ++k) st[k] = ld_in<NTL>(at(fp.p[k], i));
    } else if constexpr (VAR == DR_VARIANT_MOVING) {
#pragma unroll
        for (int k = 0; k < 3; ++k) cen[k] = *at(fp.p[F_TGT + k], i);
#pragma unroll
        for (int k = 0; k < 9; ++k) mp[k] = *at(v.mot + k * v.stride, i);
    } else {
        st[F_TGT + 0] = (S)0;
        st[F_TGT + 1] = (S)0;
        st[F_TGT + 2] = (S)10.0;
    }
    int32_t step = ld_in<NTL>(at(p_step, i));
    // needed only if this env resets; loaded up front so a reset does not
    // stall the wave on a dependent global load (+12 B per step, counted in
    // the measured traffic, not in the 305 B algorithmic)
    double eps_old = 0.0;
    if constexpr (GYMLIKE) {
        if (!DR_HOIST_RESET) ep_old = *at(p_epn, i);
        // eps loaded with the state: the Philox reset path holds no global
        // load (6-8 % faster at 65,536-131,072 envs than loading it in the reset)
        eps_old = *at(p_eps, i);
    }
    // VecMonitor counters: also loaded up front (a load after the physics
    // would put one more full memory latency on every wave)
    float ret0 = 0.f;
    int32_t len0 = 0;
    if constexpr (MON) {
        ret0 = *at(v.ep_ret, i);
        len0 = *at(v.ep_len, i);
    }
    // Every load is issued before any arithmetic: without this the
    // scheduler interleaves the first sincos with the loads and its
    // s_waitcnt holds back the issue of the remaining ones by a full memory
    // latency.
    __builtin_amdgcn_sched_barrier(0);
    u32x4 pre0{};
    if constexpr (VAR == DR_VARIANT_GYM && DR_HOIST_RESET) {
        if constexpr (!HU) {
            const uint64_t gid = (uint64_t)(v.env_id_offset + i);
            pre0 = philox4x32_10(u32x4{(uint32_t)(ep_old + 1), (uint32_t)gid,
                                       (uint32_t)(gid >> 32), TAG_RESET},
                                 v.seed_lo, v.seed_hi);
        }
    }
    if constexpr (VAR == DR_VARIANT_MOVING) {
        // the reward and obs of this step see the target at the NEW step
        moving_target(cen, mp, step + 1, (float)v.dt, &st[F_TGT], tvel);
    }

    bool crash;
    const S r = physics_step<S, VAR>(st, act, v.dt, crash);
    DR_STAMP(2);
    step += 1;                                             // (155)
    const bool done = live && (crash || (step >= v.max_steps));   // (156-157)
    const float rf = (float)r;                             // SB3 f32 buffer
#if DR_LOADS_LANDED
    // Every value loaded up front has landed before the first store is
    // issued (they were issued first and the physics took longer than
    // their latency, so this waits for nothing).  Without it the compiler
    // places the waits for the late-used ones (ep_num / eps in the reset
    // branch, the VecMonitor counters, the step counter) at their uses,
    // after the rew / done (and terminal obs) stores: vmcnt(0) there drains
    // those stores as well -- vmcnt counts both, in issue order -- once
    // in the reset branch and again where it rejoins, for every wave.
    asm volatile("" ::"v"(step), "v"(ep_old), "v"(eps_old), "v"(ret0), "v"(len0));
#pragma unroll
    for (int k = 0; k < F_N; ++k) asm volatile("" ::"v"(st[k]));
#endif
    if (live) {
        st_out(at(io.rew, i), rf);
        st_out(at(io.done, i), (uint8_t)done);
    }
#if !DR_OBS_ONCE
    make_obs<S, OD>(st, ob, tvel);
#endif

    float ret = 0.f;
    int32_t len = 0;
    if constexpr (MON) {
        ret = ret0 + rf;                                   // VecMonitor
        len = len0 + 1;
    }
    if constexpr (GYMLIKE) {
        if (done && io.auto_reset) {
            // DummyVecEnv: keep the terminal obs, reset in the same step.
            if (io.term_obs) {
#if DR_OBS_ONCE
                make_obs<S, OD>(st, ob, tvel);
#endif
#pragma unroll
                for (int k = 0; k < OD; ++k) io.term_obs[i * OD + k] = ob[k];
            }
            step = 0;
            if constexpr (VAR == DR_VARIANT_GYM) {
                gym_reset_regs(v, i, HU ? 1 : 0, st, ep_old, eps_old,
                               DR_HOIST_RESET ? &pre0 : nullptr);
#pragma unroll
                for (int k = F_TGT; k < F_N; ++k) *at(fp.p[k], i) = st[k];
            } else {
                moving_reset_regs(v, i, HU ? 1 : 0, st, cen, mp, ep_old, eps_old);
#pragma unroll
                for (int k = 0; k < 3; ++k) *at(fp.p[F_TGT + k], i) = cen[k];
#pragma unroll
                for (int k = 0; k < 9; ++k) *at(v.mot + k * v.stride, i) = mp[k];
                moving_target(cen, mp, 0, (float)v.dt, &st[F_TGT], tvel);
            }
#if !DR_OBS_ONCE
            make_obs<S, OD>(st, ob, tvel);
#endif
        }
    }
#if DR_OBS_ONCE
    // ONE observation pass over the post-reset state (the terminal obs is
    // formed inside the reset branch only when the caller keeps it)
    make_obs<S, OD>(st, ob, tvel);
#endif
    if constexpr (MON) {
        if (io.trunc_out && live) *at(io.trunc_out, i) = (uint8_t)(done && !crash);
        if (done) {               // VecMonitor: report, then restart counters
            *at(io.ep_ret_out, i) = ret;
            *at(io.ep_len_out, i) = len;
            ret = 0.f;
            len = 0;
        }
        if (live) {
            *at(v.ep_ret, i) = ret;
            *at(v.ep_len, i) = len;
        }
    }
    DR_STAMP(3);
    if (live) {
#pragma unroll
        for (int k = 0; k < 12; ++k) st_out(at(fp.p[k], i), st[k]);
        st_out(at(p_step, i), step);
    }
    DR_STAMP(4);
    if (!live) {
#pragma unroll
        for (int k = 0; k < OD; ++k) ob[k] = 0.f;
    }
#if DR_WAVE_STAGE
    store_obs_wave<OD, RPW>(reinterpret_cast<float *>(sh4), ob, io.obs, v.n);
#else
    store_obs_block<OD>(reinterpret_cast<float *>(sh4), ob, io.obs, base, v.n);
#endif
    DR_STAMP(5);
}

// ----------------------------------------------------------------------------
// K-step rollout: K successive steps of the same batch in ONE launch, the
// state held in registers between steps.  Equivalent, output for output and
// bit for bit, to K env_step_kernel launches (dr_step with no terminal obs,
// no VecMonitor) on actions[t] -- or, GEN, on the random policy's actions
// generated in-kernel with random_actions_kernel's exact Philox draw for
// step step0 + t.  This is the random-policy rollout loop (a = sample();
// obs, r, done = env.step(a), K times; drone.py:81-159 per step, the
// DummyVecEnv auto-reset in between) with the per-step state round trip
// through HBM and the per-launch gap removed: per env-step it moves the
// outputs (obs 4*OD + rew 4 + done 1 B) and the action (16 B, none when
// GEN), plus the state once per launch.
//
// Every step's outputs are stored as they are formed (rew / done per lane,
// obs through the per-wave LDS staging), so the stores of step t drain
// while step t+1 computes; actions are loaded two steps ahead.  The fields
// a reset changes outside the 12 dynamic ones (target,
// motion; ep_num / eps are written by the reset itself) are written back
// at the end only for lanes that reset during the launch.
// ----------------------------------------------------------------------------
struct RolloutIO {
    const float *actions;   // (K, n, 4); unused when GEN
    float *act_out;         // GEN: optional (K, n, 4) copy of the drawn actions
    float *obs;             // (K, n, OD)
    float *rew;             // (K, n)
    uint8_t *done;          // (K, n)
    int32_t k;
    uint32_t a_k0, a_k1;    // action Philox key
    uint64_t a_step0;
    float a_lo, a_span;
    int auto_reset;
};

template <typename S, int VAR, int RPW, bool GEN>
__global__ __launch_bounds__(kEnvBlock) void env_rollout_kernel(EnvView<S> v, RolloutIO io,
                                                                FieldPtrs<S> fp) {
    constexpr int OD = VAR == DR_VARIANT_GYM ? 15 : (VAR == DR_VARIANT_MOVING ? 18 : 12);
    constexpr bool GYMLIKE = VAR != DR_VARIANT_VECTORIZED;
    __shared__ float4 sh4[kEnvBlock * OD / 4];
    const int64_t n_ = v.n;
    const int64_t base = (int64_t)blockIdx.x * (DR_ENV_WPB * RPW);
    const int lane_ = threadIdx.x & 63;
    const int64_t i_own = lane_ < RPW ? base + (threadIdx.x >> 6) * RPW + lane_ : n_;
    const bool live = i_own < n_;
    const int64_t i = live ? i_own : n_ - 1;
    const uint64_t gid = (uint64_t)(v.env_id_offset + i);
    S st[F_N];
#pragma unroll
    for (int k = F_EUL; k < F_N - 3; ++k) st[k] = *at(fp.p[k], i);
#pragma unroll
    for (int k = 0; k < F_EUL; ++k) st[k] = *at(fp.p[k], i);
    S cen[3];
    float mp[9], tvel[3];
    if constexpr (VAR == DR_VARIANT_GYM) {
#pragma unroll
        for (int k = F_TGT; k < F_N; ++k) st[k] = *at(fp.p[k], i);
    } else if constexpr (VAR == DR_VARIANT_MOVING) {
#pragma unroll
        for (int k = 0; k < 3; ++k) cen[k] = *at(fp.p[F_TGT + k], i);
#pragma unroll
        for (int k = 0; k < 9; ++k) mp[k] = *at(v.mot + k * v.stride, i);
    } else {
        st[F_TGT + 0] = (S)0;
        st[F_TGT + 1] = (S)0;
        st[F_TGT + 2] = (S)10.0;
    }
    int32_t step = *at(fp.step, i);
    int32_t ep_num = 0;
    double eps = 0.0;
    if constexpr (GYMLIKE) {
        ep_num = *at(fp.ep_num, i);
        eps = *at(fp.eps, i);
    }
    bool reset_any = false;
    float ob[OD];

    // The Philox keys (reset draws; GEN: actions) are re-declared opaque
    // once per step, so the compiler cannot hoist the 10-round key
    // schedules out of the loop: hoisted, their 40 words spilled to VGPR
    // lanes, and every round paid a v_readlane plus a hazard s_nop.
    EnvView<S> vk = v;
    // The Philox blocks of a lane's NEXT reset (episode ep_num + 1; gym:
    // block 0 = pos x, y and target x, y; moving: all four) are drawn ahead, for every lane
    // whose draw is used up, at the first step of each group of
    // kResetAhead steps -- a wave-wide pass once per group instead of the
    // reset branch's Philox, which a wave runs at almost every step (≈86 % of
    // waves hold a resetting env at each step under the random policy).  A
    // lane resetting twice within one group draws in the branch as before;
    // the draws are the same Philox words either way.
    constexpr int NB = VAR == DR_VARIANT_MOVING ? 4 : 1;   // Philox blocks per reset
    u32x4 nd[NB] = {};
    bool nd_ok = false;
    // the step limit in a VGPR: under the kernel's SGPR pressure the
    // compiler otherwise re-reads it from the kernel arguments at every
    // step (a scalar load and its wait on the critical path)
    int32_t max_steps;
    asm volatile("v_mov_b32 %0, %1" : "=v"(max_steps) : "s"(v.max_steps));
    // one step from the action's motor mixes: the body of env_step_kernel
    // on registers
    auto step_one = [&](const MotorMix mx, const int t) {
        asm volatile("" : "+s"(vk.seed_lo), "+s"(vk.seed_hi));
        if constexpr (GYMLIKE) {
            if (t % kResetAhead == 0 && !nd_ok) {
#pragma unroll
                for (int b = 0; b < NB; ++b)
                    nd[b] = philox4x32_10(u32x4{(uint32_t)(ep_num + 1), (uint32_t)gid,
                                                (uint32_t)(gid >> 32), TAG_RESET | (uint32_t)b},
                                          vk.seed_lo, vk.seed_hi);
                nd_ok = true;
            }
        }
        if constexpr (VAR == DR_VARIANT_MOVING)
            moving_target(cen, mp, step + 1, (float)v.dt, &st[F_TGT], tvel);
        bool crash;
        const S r = physics_step_mixed<S, VAR>(st, mx, v.dt, crash);
        step += 1;
        const bool done = live && (crash || (step >= max_steps));
        const int64_t row = (int64_t)t * n_;
        if (live) {
            st_out(at(io.rew + row, i), (float)r);
            st_out(at(io.done + row, i), (uint8_t)done);
        }
        if constexpr (GYMLIKE) {
            if (done && io.auto_reset) {
                step = 0;
                reset_any = true;
                if constexpr (VAR == DR_VARIANT_GYM) {
                    gym_reset_regs(vk, i, 0, st, ep_num, eps, nd_ok ? &nd[0] : nullptr);
                    nd_ok = false;
                } else {
                    moving_reset_regs(vk, i, 0, st, cen, mp, ep_num, eps, nd_ok ? nd : nullptr);
                    nd_ok = false;
                    moving_target(cen, mp, 0, (float)v.dt, &st[F_TGT], tvel);
                }
                // the curriculum counters gym/moving_reset_regs just wrote
                // (drone.py:61, 68-70), carried on in registers
                ep_num += 1;
                if (ep_num % 2000 == 0) eps += 0.1;
            }
        }
        make_obs<S, OD>(st, ob, tvel);
        if (!live) {
#pragma unroll
            for (int k = 0; k < OD; ++k) ob[k] = 0.f;
        }
        // (plain stores for these outputs measured the same: 60.2 / 62.2 us
        // per 32-step launch at 65,536 envs)
        store_obs_wave<OD, RPW>(reinterpret_cast<float *>(sh4), ob, io.obs + row * OD, n_);
    };

    if constexpr (GEN) {
        for (int t = 0; t < io.k; ++t) {
            const uint64_t s = io.a_step0 + (uint64_t)t;
            uint32_t ak0 = io.a_k0, ak1 = io.a_k1;
            asm volatile("" : "+s"(ak0), "+s"(ak1));
            const u32x4 r = philox4x32_10(
                u32x4{(uint32_t)s, (uint32_t)(s >> 32), (uint32_t)gid,
                      TAG_ACTION ^ (uint32_t)(gid >> 32)},
                ak0, ak1);
            const float4 act = make_float4(io.a_lo + io.a_span * u01_f32(r.x),
                                           io.a_lo + io.a_span * u01_f32(r.y),
                                           io.a_lo + io.a_span * u01_f32(r.z),
                                           io.a_lo + io.a_span * u01_f32(r.w));
            if (io.act_out && live)
                st_out(at(reinterpret_cast<float4 *>(io.act_out) + (int64_t)t * n_, i), act);
            step_one(motor_mix(act), t);
        }
    } else {
        // Each action is loaded ahead into the registers the action two
        // steps earlier just vacated (right after its motor mixes, its only
        // use), by an asm load the compiler does not track: its own waitcnt
        // pass, at a loop back edge, waits vmcnt(0) for any load in flight
        // -- draining every store of the step as well (vmcnt counts both,
        // in issue order).  The hand-placed wait below counts only stores
        // that a wave with a live lane always issues (a wave with none
        // stores nothing and its lanes' results are discarded).  The first
        // two actions are ordinary loads.
        typedef float f4v __attribute__((ext_vector_type(4)));
        const float4 *const acts = reinterpret_cast<const float4 *>(io.actions);
        const float4 a_first = *at(acts, i);
        const float4 b_first = io.k > 1 ? *at(acts + n_, i) : a_first;
        f4v a = {a_first.x, a_first.y, a_first.z, a_first.w};
        f4v b = {b_first.x, b_first.y, b_first.z, b_first.w};
        // every preheader load landed before the loop: otherwise the
        // compiler places the waits for them at their first uses inside
        // the loop (ep_num / eps in the reset branch, a state component in
        // the physics), where they run every step as vmcnt(0)
        asm volatile("" ::"v"(ep_num), "v"(eps), "v"(a), "v"(b), "v"(step));
#pragma unroll
        for (int k = 0; k < F_N; ++k) asm volatile("" ::"v"(st[k]));
        if constexpr (VAR == DR_VARIANT_MOVING) {
#pragma unroll
            for (int k = 0; k < 3; ++k) asm volatile("" ::"v"(cen[k]));
#pragma unroll
            for (int k = 0; k < 9; ++k) asm volatile("" ::"v"(mp[k]));
        }
        // Two steps ahead, in two registers that alternate (the loop is
        // unrolled by two so each keeps its role): step t's action was
        // loaded at the top of step t-2; younger than that load are step
        // t-2's rew / done stores, step t-1's action load (when issued) and
        // step t-1's rew / done stores, so vmcnt(4) waits for it and no
        // further.  One step ahead left part of the HBM latency exposed
        // (62.9 us per 32-step launch with 335 MB of distinct actions
        // against 50.5 with one cache-resident action set).
        auto act_step = [&](f4v &r, const int t) {
            if (t >= 2) {
                // younger than step t's action load (issued at the top of step
                // t - 2): each of steps t - 2 and t - 1 issues its reward,
                // done and NQ obs-row stores, step t - 1 the next load
                asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
            }
            const MotorMix mx = motor_mix(make_float4(r.x, r.y, r.z, r.w));
            asm volatile("" ::"v"(mx.thr), "v"(mx.phi), "v"(mx.theta), "v"(mx.psi));
            __builtin_amdgcn_sched_barrier(0);
            if (t + 2 < io.k) {
                const float4 *pa = at(acts + (int64_t)(t + 2) * n_, i);
                asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(pa) : "memory");
            }
            __builtin_amdgcn_sched_barrier(0);
            step_one(mx, t);
        };
        for (int t = 0; t < io.k; t += 2) {
            act_step(a, t);
            if (t + 1 < io.k) act_step(b, t + 1);
        }
        // a wave with no live lane never waited for its loads: none may
        // still be writing registers the code below reuses
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (live) {
#pragma unroll
        for (int k = 0; k < 12; ++k) st_out(at(fp.p[k], i), st[k]);
        st_out(at(fp.step, i), step);
        if (reset_any) {
            if constexpr (VAR == DR_VARIANT_GYM) {
#pragma unroll
                for (int k = F_TGT; k < F_N; ++k) *at(fp.p[k], i) = st[k];
            } else if constexpr (VAR == DR_VARIANT_MOVING) {
#pragma unroll
                for (int k = 0; k < 3; ++k) *at(fp.p[F_TGT + k], i) = cen[k];
#pragma unroll
                for (int k = 0; k < 9; ++k) *at(v.mot + k * v.stride, i) = mp[k];
            }
        }
    }
}

// ----------------------------------------------------------------------------
// Warp-specialised K-step rollout (dr_rollout's default launch form).
// 512-thread blocks of 256 envs: waves 0-3, the PHYSICS waves (one per SIMD),
// run the steps on registers exactly as env_rollout_kernel does, with no
// global load inside the step loop (its only global stores are a reset's
// ep_num / eps); waves 4-7, the MEMORY waves
// (wave p + 4 shares SIMD p with physics wave p), move the bytes: each loads
// its partner's actions by LDS-DMA kWsAhead + 1 steps ahead into a ring of
// LDS slots (GEN: draws the random policy's actions into them), and streams
// its partner's finished outputs -- obs rows, reward, done, staged in LDS by
// the physics wave -- to HBM.  One s_barrier per step hands the slots over.  At one physics wave per SIMD, env_rollout_kernel's
// wave issues its own stores and action loads between steps (the write
// stream alone is ~0.9 us per step at 65,536 envs); here
// that issue and its back-pressure sit on the memory waves, beside the
// physics.
//
// Outputs are bitwise those of env_rollout_kernel (the same physics, reset
// and Philox code on the same registers; only where the bytes travel
// differs); tests/test_rollout_gpu.py checks both forms against K dr_step.
//
// Step t / phase t (B_t = the barrier that ends physics step t):
//   physics: action t from slot t % NA (landed before B_(t-1)), the step,
//            outputs into slot t & 1, lgkmcnt(0), B_t
//   memory:  after B_(t-1): LDS-DMA action t + D + 1 into slot (t + D + 1) % NA
//            (its previous action, t - 1, was read before B_(t-1)); load
//            slot (t - 1) & 1 and store it to HBM (physics writes that slot
//            again only after B_t); wait for action t + 1 (vmcnt, counted by
//            hand: vmcnt counts loads and stores in issue order), B_t.
//   After the last barrier the memory waves store step K - 1's outputs.
// ----------------------------------------------------------------------------
constexpr int kWsEnvs = 256;                 // envs per block: 4 physics waves
constexpr int kWsThreads = 2 * kWsEnvs;
// D: how many steps ahead of the physics the memory waves issue an action
// load (the physics wave reads action t at the top of step t; the
// hand-counted waits below are generic in D; vmcnt holds at most 63, so
// S_OPS + D * (S_OPS + 1) must stay below it).  Ring slots: D + 2.
constexpr int kWsAhead = 2;                  // D
constexpr int kWsNA = kWsAhead + 2;          // action ring slots


// global_load_lds_dwordx4: lane l's 16 bytes land at LDS byte lds_base + 16 l
// (the wave's 64 actions as one 1-KB slot).  It clobbers m0, which the
// compiler reserves (and sets before each of its own uses).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ inline void ws_glds16(const void *gptr, uint32_t lds_base) {
    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
                 ::"v"(gptr), "s"(lds_base)
                 : "memory", "m0");
}
#pragma clang diagnostic pop


template <int OD>
struct WsLds {
    float obs[2][kWsEnvs * OD];              // per slot: 4 waves x 64 rows x OD
    float rew[2][kWsEnvs];
    uint8_t done[2][kWsEnvs];
    float4 act[kWsNA][kWsEnvs];
};

template <typename S, int VAR, bool GEN>
__global__ __launch_bounds__(kWsThreads) void env_rollout_ws_kernel(EnvView<S> v, RolloutIO io,
                                                                    FieldPtrs<S> fp) {
    constexpr int OD = VAR == DR_VARIANT_GYM ? 15 : (VAR == DR_VARIANT_MOVING ? 18 : 12);
    constexpr bool GYMLIKE = VAR != DR_VARIANT_VECTORIZED;
    constexpr int NQ = (64 * OD / 4 + 63) / 64;  // float4 rows-stores per lane and step
    // the hand-counted wait assumes NQ obs + 1 reward + 1 done store per phase
    constexpr int S_OPS = NQ + 2;
    static_assert(S_OPS + kWsAhead * (S_OPS + 1) <= 63,
                  "the action-load wait count must fit vmcnt");
    __shared__ __attribute__((aligned(16))) WsLds<OD> sh;
    const int64_t n_ = v.n;
    const int K = io.k;
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int p = wid & 3;                        // physics wave / partner index
    const int64_t wbase = (int64_t)blockIdx.x * kWsEnvs + p * 64;
    const int64_t i_own = wbase + lane;
    const bool live = i_own < n_;
    const int64_t i = live ? i_own : n_ - 1;

    if (wid >= 4) {
        // ---------------- memory wave ----------------
        const int64_t nvalid = (n_ - wbase) < 64 ? (n_ - wbase) : 64;
        // full: 64 live rows and 16-byte aligned obs rows at every step; else
        // (the ragged last wave) scalar stores and vmcnt(0) waits
        const bool full = nvalid == 64 && (((uintptr_t)io.obs) & 15) == 0 &&
                          ((n_ * OD) & 3) == 0;
        const float4 *acts = reinterpret_cast<const float4 *>(io.actions);
        // GEN: the memory wave draws the random policy's action itself
        // (random_actions_kernel's Philox word for step a_step0 + t) into the
        // slot, off the physics wave's instruction stream
        const uint64_t gid = (uint64_t)(v.env_id_offset + i);
        auto load_act = [&](int t) {
            if constexpr (GEN) {
                const uint64_t s = io.a_step0 + (uint64_t)t;
                uint32_t ak0 = io.a_k0, ak1 = io.a_k1;
                asm volatile("" : "+s"(ak0), "+s"(ak1));
                const u32x4 r = philox4x32_10(
                    u32x4{(uint32_t)s, (uint32_t)(s >> 32), (uint32_t)gid,
                          TAG_ACTION ^ (uint32_t)(gid >> 32)},
                    ak0, ak1);
                const float4 act = make_float4(io.a_lo + io.a_span * u01_f32(r.x),
                                               io.a_lo + io.a_span * u01_f32(r.y),
                                               io.a_lo + io.a_span * u01_f32(r.z),
                                               io.a_lo + io.a_span * u01_f32(r.w));
                sh.act[t % kWsNA][p * 64 + lane] = act;
                if (io.act_out && live)
                    st_out(at(reinterpret_cast<float4 *>(io.act_out) + (int64_t)t * n_, i), act);
            } else if (nvalid > 0) {
                ws_glds16(at(acts + (int64_t)t * n_, i),
                          (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)
                              &sh.act[t % kWsNA][p * 64]);
            }
        };
        auto store_out = [&](int t) {
            if (nvalid <= 0) return;
            const int so = t & 1;
            const int64_t row = (int64_t)t * n_;
            const float *src = &sh.obs[so][p * 64 * OD];
            float *dst = io.obs + (row + wbase) * OD;
            const float r = sh.rew[so][p * 64 + lane];
            const uint8_t d = sh.done[so][p * 64 + lane];
            if (full) {
                float4 q[NQ];
#pragma unroll
                for (int j = 0; j < NQ; ++j)
                    if (j * 64 + lane < 64 * OD / 4)
                        q[j] = reinterpret_cast<const float4 *>(src)[j * 64 + lane];
#pragma unroll
                for (int j = 0; j < NQ; ++j)
                    if (j * 64 + lane < 64 * OD / 4)
                        st_out(reinterpret_cast<float4 *>(dst) + j * 64 + lane, q[j]);
            } else {
                for (int q = lane; q < (int)nvalid * OD; q += 64) st_out(dst + q, src[q]);
            }
            if (live) {
                st_out(at(io.rew + row, i_own), r);
                st_out(at(io.done + row, i_own), d);
            }
        };
        for (int t = 0; t <= kWsAhead && t < K; ++t) load_act(t);
        if (!GEN) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // actions 0 .. D
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // B_(-1)
        for (int t = 0; t < K; ++t) {
            if (t + kWsAhead + 1 < K) load_act(t + kWsAhead + 1);
            if (t >= 1) store_out(t - 1);
            // action a = t + 1 must have landed before B_t (actions 0 .. D
            // did before B_(-1)).  It was issued first in phase q = a - D - 1
            // = t - D; younger in the steady state: q's S_OPS stores and D
            // phases of one load and S_OPS stores; elsewhere at least this
            // phase's S_OPS stores (t >= 1 here).  A ragged wave waits for
            // every op.
            constexpr int AH = kWsAhead;
            if (!GEN && t + 1 < K && t + 1 > kWsAhead) {
                __builtin_amdgcn_sched_barrier(0);
                if (!full)
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                else if (t >= AH + 1 && t + kWsAhead + 1 < K)
                    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(S_OPS + AH * (S_OPS + 1))
                                 : "memory");
                else
                    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(S_OPS) : "memory");
            }
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // B_t
        }
        if (K > 0) store_out(K - 1);
        return;
    }

    // ---------------- physics wave ----------------
    const uint64_t gid = (uint64_t)(v.env_id_offset + i);
    S st[F_N];
#pragma unroll
    for (int k = F_EUL; k < F_N - 3; ++k) st[k] = *at(fp.p[k], i);
#pragma unroll
    for (int k = 0; k < F_EUL; ++k) st[k] = *at(fp.p[k], i);
    S cen[3];
    float mp[9], tvel[3];
    if constexpr (VAR == DR_VARIANT_GYM) {
#pragma unroll
        for (int k = F_TGT; k < F_N; ++k) st[k] = *at(fp.p[k], i);
    } else if constexpr (VAR == DR_VARIANT_MOVING) {
#pragma unroll
        for (int k = 0; k < 3; ++k) cen[k] = *at(fp.p[F_TGT + k], i);
#pragma unroll
        for (int k = 0; k < 9; ++k) mp[k] = *at(v.mot + k * v.stride, i);
    } else {
        st[F_TGT + 0] = (S)0;
        st[F_TGT + 1] = (S)0;
        st[F_TGT + 2] = (S)10.0;
    }
    int32_t step = *at(fp.step, i);
    int32_t ep_num = 0;
    double eps = 0.0;
    if constexpr (GYMLIKE) {
        ep_num = *at(fp.ep_num, i);
        eps = *at(fp.eps, i);
    }
    // every state load landed before the loop (else the compiler waits for
    // them at their first uses inside it, as vmcnt(0))
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bool reset_any = false;
    float ob[OD];
    EnvView<S> vk = v;
    // the next reset's Philox blocks drawn ahead, once per group of
    // kResetAhead steps (env_rollout_kernel)
    constexpr int NB = VAR == DR_VARIANT_MOVING ? 4 : 1;
    u32x4 nd[NB] = {};
    bool nd_ok = false;
    int32_t max_steps;
    asm volatile("v_mov_b32 %0, %1" : "=v"(max_steps) : "s"(v.max_steps));
    asm volatile("s_barrier" ::: "memory");                          // B_(-1)
    for (int t = 0; t < K; ++t) {
        asm volatile("" : "+s"(vk.seed_lo), "+s"(vk.seed_hi));
        const float4 a_cur = sh.act[t % kWsNA][p * 64 + lane];
        const MotorMix mx = motor_mix(a_cur);
        if constexpr (GYMLIKE) {
            if (t % kResetAhead == 0 && !nd_ok) {
#pragma unroll
                for (int b = 0; b < NB; ++b)
                    nd[b] = philox4x32_10(u32x4{(uint32_t)(ep_num + 1), (uint32_t)gid,
                                                (uint32_t)(gid >> 32), TAG_RESET | (uint32_t)b},
                                          vk.seed_lo, vk.seed_hi);
                nd_ok = true;
            }
        }
        if constexpr (VAR == DR_VARIANT_MOVING)
            moving_target(cen, mp, step + 1, (float)v.dt, &st[F_TGT], tvel);
        bool crash;
        S r;
        r = physics_step_mixed<S, VAR>(st, mx, v.dt, crash);
        step += 1;
        const bool done = live && (crash || (step >= max_steps));
        if constexpr (GYMLIKE) {
            const bool rs = done && io.auto_reset;
            if (rs) {
                step = 0;
                reset_any = true;
                // a second reset within the group: draw its blocks here (the
                // same words the reset would draw; always passing the array
                // keeps it in registers -- a pointer-or-null argument put it
                // on the scratch stack)
                if (!nd_ok) {
#pragma unroll
                    for (int b = 0; b < NB; ++b)
                        nd[b] = philox4x32_10(u32x4{(uint32_t)(ep_num + 1), (uint32_t)gid,
                                                    (uint32_t)(gid >> 32),
                                                    TAG_RESET | (uint32_t)b},
                                              vk.seed_lo, vk.seed_hi);
                }
                if constexpr (VAR == DR_VARIANT_GYM) {
                    gym_reset_regs(vk, i, 0, st, ep_num, eps, &nd[0]);
                } else {
                    moving_reset_regs(vk, i, 0, st, cen, mp, ep_num, eps, nd);
                    moving_target(cen, mp, 0, (float)v.dt, &st[F_TGT], tvel);
                }
                nd_ok = false;
                ep_num += 1;
                if (ep_num % 2000 == 0) eps += 0.1;
            }
        }
        make_obs<S, OD>(st, ob, tvel);
        if (!live) {
#pragma unroll
            for (int k = 0; k < OD; ++k) ob[k] = 0.f;
        }
        const int so = t & 1;
        float *srow = &sh.obs[so][(p * 64 + lane) * OD];
#pragma unroll
        for (int k = 0; k < OD; ++k) srow[k] = ob[k];
        sh.rew[so][p * 64 + lane] = (float)r;
        sh.done[so][p * 64 + lane] = (uint8_t)done;
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // B_t
    }
    if (live) {
#pragma unroll
        for (int k = 0; k < 12; ++k) st_out(at(fp.p[k], i), st[k]);
        st_out(at(fp.step, i), step);
        if (reset_any) {
            if constexpr (VAR == DR_VARIANT_GYM) {
#pragma unroll
                for (int k = F_TGT; k < F_N; ++k) *at(fp.p[k], i) = st[k];
            } else if constexpr (VAR == DR_VARIANT_MOVING) {
#pragma unroll
                for (int k = 0; k < 3; ++k) *at(fp.p[F_TGT + k], i) = cen[k];
#pragma unroll
                for (int k = 0; k < 9; ++k) *at(v.mot + k * v.stride, i) = mp[k];
            }
        }
    }
}

// ----------------------------------------------------------------------------
// Split-physics K-step rollout (gym variant, actions read from HBM).  The
// warp-specialised kernel's physics wave, split by DATA into two waves on the
// same SIMD, so that two dependent f64 chains interleave where one wave per
// SIMD left the VALU idle about half of its cycles (two physics waves per
// SIMD were measured to hide 24 % per env):
//   * the TRANSLATION wave (waves 0-3) owns pos / vel / target, the step
//     counter, the curriculum and the reset draws: the yaw's sincos, R's
//     column 2 from the step's Euler sincos, acceleration, velocity,
//     position, reward, crash, done, the reset, and the obs fields pos / vel
//     / target - pos;
//   * the ROTATION wave (waves 4-7) owns the Euler angles and body rates:
//     the roll and pitch sincos, the Euler rates and the angular update, and
//     the obs fields euler / omega;
//   * the MEMORY waves (8-11) load actions and stream outputs as in the
//     warp-specialised kernel.
// Wave p, p + 4 and p + 8 share SIMD p.  The two halves of a step touch
// disjoint state; what crosses is the roll / pitch sincos and the yaw
// (rotation -> translation, formed one step ahead from the updated angles,
// through a double-buffered LDS slot) and the done flag (translation ->
// rotation, read one phase later: a reset zeroes the angles and rates before
// the next step, and their sincos is then exactly (+0, 1), which both waves
// substitute).  The rotation wave therefore writes step t's euler / omega
// obs fields in phase t + 1, and the memory waves store step t's outputs in
// phase t + 2 from three output slots.  Every expression is
// physics_step_mixed's, in its order: outputs bitwise those of the other
// kernels (tests/test_rollout_gpu.py).  Each angle's sincos depends on that
// angle alone, so the yaw's moving waves changes no bit: 41.6-43.3 vs
// 42.6-44.7 us per 32-step launch (round 4, alternating on one box; without
// the rotation wave's sincos altogether, a wrong-result diagnostic build,
// 33.3-34.4 us: that sincos was the launch's critical path).
// ----------------------------------------------------------------------------
// The translation wave stages the squared target distance and the memory
// wave forms the reward from it (the same sqrt and reward arithmetic, off the
// translation wave's instruction stream): 41.3-41.9 vs 43.0-44.2 us per
// 32-step launch against the translation wave forming it (round 3).
constexpr int kAbThreads = 3 * kWsEnvs;   // 4 translation + 4 rotation + 4 memory waves
constexpr int kAbOut = 3;                 // output slots

template <typename S, int OD>
struct AbLds {
    float obs[kAbOut][kWsEnvs * OD];
    S d2[kAbOut][kWsEnvs];                // squared target distance
    uint8_t done[kAbOut][kWsEnvs];
    float4 act[kWsNA][kWsEnvs];
    S sc[2][4][kWsEnvs];                  // sin phi, theta, cos phi, theta
    S psi[2][kWsEnvs];                    // the yaw itself
};

template <typename S, bool GEN>
__global__ __launch_bounds__(kAbThreads) void env_rollout_ab_kernel(EnvView<S> v, RolloutIO io,
                                                                    FieldPtrs<S> fp) {
    constexpr int OD = 15;
    constexpr int NQ = (64 * OD / 4 + 63) / 64;
    constexpr int S_OPS = NQ + 2;
    static_assert(S_OPS + kWsAhead * (S_OPS + 1) <= 63, "the action-load wait count must fit vmcnt");
    __shared__ __attribute__((aligned(16))) AbLds<S, OD> sh;
    const int64_t n_ = v.n;
    const int K = io.k;
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int p = wid & 3;
    const int role = wid >> 2;                    // 0 translation, 1 rotation, 2 memory
    const int ps = p * 64 + lane;                 // this lane's env within the block
    const int64_t wbase = (int64_t)blockIdx.x * kWsEnvs + p * 64;
    const int64_t i_own = wbase + lane;
    const bool live = i_own < n_;
    const int64_t i = live ? i_own : n_ - 1;

    if (role == 2) {
        // ---------------- memory wave (env_rollout_ws_kernel's, stores two
        // phases behind the translation wave, three output slots) ----------
        const int64_t nvalid = (n_ - wbase) < 64 ? (n_ - wbase) : 64;
        const bool full = nvalid == 64 && (((uintptr_t)io.obs) & 15) == 0 &&
                          ((n_ * OD) & 3) == 0;
        const float4 *acts = reinterpret_cast<const float4 *>(io.actions);
        const uint64_t gid = (uint64_t)(v.env_id_offset + i);
        auto load_act = [&](int t) {
            if constexpr (GEN) {
                const uint64_t s = io.a_step0 + (uint64_t)t;
                uint32_t ak0 = io.a_k0, ak1 = io.a_k1;
                asm volatile("" : "+s"(ak0), "+s"(ak1));
                const u32x4 r = philox4x32_10(
                    u32x4{(uint32_t)s, (uint32_t)(s >> 32), (uint32_t)gid,
                          TAG_ACTION ^ (uint32_t)(gid >> 32)},
                    ak0, ak1);
                const float4 act = make_float4(io.a_lo + io.a_span * u01_f32(r.x),
                                               io.a_lo + io.a_span * u01_f32(r.y),
                                               io.a_lo + io.a_span * u01_f32(r.z),
                                               io.a_lo + io.a_span * u01_f32(r.w));
                sh.act[t % kWsNA][ps] = act;
                if (io.act_out && live)
                    st_out(at(reinterpret_cast<float4 *>(io.act_out) + (int64_t)t * n_, i), act);
            } else if (nvalid > 0) {
                ws_glds16(at(acts + (int64_t)t * n_, i),
                          (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)
                              &sh.act[t % kWsNA][p * 64]);
            }
        };
        auto store_out = [&](int t) {
            if (nvalid <= 0) return;
            const int so = t % kAbOut;
            const int64_t row = (int64_t)t * n_;
            const float *src = &sh.obs[so][p * 64 * OD];
            float *dst = io.obs + (row + wbase) * OD;
            // physics_step_mixed's reward (gym variant) from the staged d^2
            const S dd = m_sqrt(sh.d2[so][ps]);
            S rr = (S)0.01 * -dd;
            if (dd < (S)0.05) rr += (S)1;
            const float r = (float)rr;
            const uint8_t d = sh.done[so][ps];
            if (full) {
                float4 q[NQ];
#pragma unroll
                for (int j = 0; j < NQ; ++j)
                    if (j * 64 + lane < 64 * OD / 4)
                        q[j] = reinterpret_cast<const float4 *>(src)[j * 64 + lane];
#pragma unroll
                for (int j = 0; j < NQ; ++j)
                    if (j * 64 + lane < 64 * OD / 4)
                        st_out(reinterpret_cast<float4 *>(dst) + j * 64 + lane, q[j]);
            } else {
                for (int q = lane; q < (int)nvalid * OD; q += 64) st_out(dst + q, src[q]);
            }
            if (live) {
                st_out(at(io.rew + row, i_own), r);
                st_out(at(io.done + row, i_own), d);
            }
        };
        for (int t = 0; t <= kWsAhead && t < K; ++t) load_act(t);
        if (!GEN) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");        // actions 0 .. D
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // B_(-1)
        for (int t = 0; t < K; ++t) {
            if (t + kWsAhead + 1 < K) load_act(t + kWsAhead + 1);
            if (t >= 2) store_out(t - 2);
            // action t + 1 lands before B_t.  Issued in phase q = t - D;
            // younger in the steady state (q >= 2, loads through phase t):
            // q's S_OPS stores and D phases of one load and S_OPS stores;
            // otherwise at least this phase's S_OPS stores (t >= D >= 2).
            if (!GEN && t + 1 < K && t + 1 > kWsAhead) {
                __builtin_amdgcn_sched_barrier(0);
                if (!full)
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                else if (t >= kWsAhead + 2 && t + kWsAhead + 1 < K)
                    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(S_OPS + kWsAhead * (S_OPS + 1))
                                 : "memory");
                else
                    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(S_OPS) : "memory");
            }
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // B_t
        }
        asm volatile("s_barrier" ::: "memory");   // B_K: step K - 1's euler / omega staged
        if (K >= 2) store_out(K - 2);
        if (K >= 1) store_out(K - 1);
        return;
    }

    if (role == 1) {
        // ---------------- rotation wave ----------------
        S eul[3], omg[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            eul[k] = *at(fp.p[F_EUL + k], i);
            omg[k] = *at(fp.p[F_OMG + k], i);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        S sn[2], cs[2];
        m_sincos_n<2>(eul, sn, cs);
        sh.psi[0][ps] = eul[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            sh.sc[0][k][ps] = sn[k];
            sh.sc[0][2 + k][ps] = cs[k];
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // B_(-1)
        // the reset of step t - 1 (done flag staged by the translation wave
        // before B_(t-1)) and the obs fields of step t - 1
        auto after_step = [&](int tp) {
            const bool rs = io.auto_reset && sh.done[tp % kAbOut][ps];
            if (rs) {
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    eul[k] = (S)0;
                    omg[k] = (S)0;
                }
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    sn[k] = (S)0;      // sincos(+0) = (+0, 1) exactly
                    cs[k] = (S)1;
                }
            }
            float *srow = &sh.obs[tp % kAbOut][ps * OD];
#pragma unroll
            for (int k = 0; k < 3; ++k) {     // dead lanes' rows are never stored
                srow[F_EUL + k] = (float)eul[k];
                srow[F_OMG + k] = (float)omg[k];
            }
        };
        for (int t = 0; t < K; ++t) {
            const float4 a_cur = sh.act[t % kWsNA][ps];
            if (t >= 1) after_step(t - 1);
            const MotorMix mx = motor_mix(a_cur);
            // physics_step_mixed's angular part, in its order
            const S tau_phi = (S)kFactor * (S)mx.phi;
            const S tau_theta = (S)kFactor * (S)mx.theta;
            const float tau_psi = kKyaw32 * mx.psi;
            const S sph = sn[0], cph = cs[0], sth = sn[1], cth = cs[1];
            const S w0 = omg[0], w1 = omg[1], w2 = omg[2];
            const S sec = (S)1 / cth;
            const S tth = div_rcp(sth, cth, sec);
            const S ed2 = ((S)0 * w0 + div_rcp(sph, cth, sec) * w1) + div_rcp(cph, cth, sec) * w2;
            const S ed0 = ((S)1 * w0 + (sph * tth) * w1) + (cph * tth) * w2;
            const S ed1 = ((S)0 * w0 + cph * w1) + (-sph) * w2;
            eul[0] += ed0 * v.dt;
            eul[1] += ed1 * v.dt;
            eul[2] += ed2 * v.dt;
            const S wd0 = div_rcp(tau_phi - (S)(kIyy - kIzz) * w1 * w2, (S)kIxx, (S)(1.0 / kIxx));
            const S wd1 = div_rcp(tau_theta - (S)(kIzz - kIxx) * w0 * w2, (S)kIyy, (S)(1.0 / kIyy));
            const S wd2 = div_rcp((S)tau_psi - (S)(kIxx - kIyy) * w0 * w1, (S)kIzz, (S)(1.0 / kIzz));
            omg[0] += wd0 * v.dt;
            omg[1] += wd1 * v.dt;
            omg[2] += wd2 * v.dt;
            // the next step's sincos (of the angles before any reset of this
            // step: the translation wave substitutes (+0, 1) after one)
            m_sincos_n<2>(eul, sn, cs);
            if (t + 1 < K) {
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    sh.sc[(t + 1) & 1][k][ps] = sn[k];
                    sh.sc[(t + 1) & 1][2 + k][ps] = cs[k];
                }
                sh.psi[(t + 1) & 1][ps] = eul[2];
            }
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // B_t
        }
        if (K >= 1) after_step(K - 1);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // B_K
        if (live) {
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                st_out(at(fp.p[F_EUL + k], i), eul[k]);
                st_out(at(fp.p[F_OMG + k], i), omg[k]);
            }
        }
        return;
    }

    // ---------------- translation wave ----------------
    const uint64_t gid = (uint64_t)(v.env_id_offset + i);
    S st[F_N];                // euler / omega entries unused here
#pragma unroll
    for (int k = 0; k < F_EUL; ++k) st[k] = *at(fp.p[k], i);
#pragma unroll
    for (int k = F_TGT; k < F_N; ++k) st[k] = *at(fp.p[k], i);
#pragma unroll
    for (int k = F_EUL; k < F_TGT; ++k) st[k] = (S)0;
    int32_t step = *at(fp.step, i);
    int32_t ep_num = *at(fp.ep_num, i);
    double eps = *at(fp.eps, i);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bool reset_any = false, prev_rs = false;
    EnvView<S> vk = v;
    // the next reset's state, prepared when its Philox block is drawn (once
    // per group of kResetAhead steps for the lanes whose draw was used)
    GymNext<S> nx = {};
    bool nd_ok = false;
    int32_t max_steps;
    asm volatile("v_mov_b32 %0, %1" : "=v"(max_steps) : "s"(v.max_steps));
    auto draw_next = [&]() {
        const u32x4 r0 = philox4x32_10(u32x4{(uint32_t)(ep_num + 1), (uint32_t)gid,
                                             (uint32_t)(gid >> 32), TAG_RESET},
                                       vk.seed_lo, vk.seed_hi);
        nx = gym_next_reset(vk, gid, ep_num, eps, r0);
    };
    asm volatile("s_barrier" ::: "memory");                          // B_(-1)
    for (int t = 0; t < K; ++t) {
        asm volatile("" : "+s"(vk.seed_lo), "+s"(vk.seed_hi));
        const float4 a_cur = sh.act[t % kWsNA][ps];
        // the yaw's sincos here (only R's column 2 needs it), the roll and
        // pitch's from the rotation wave
        S sn[3], cs[3];
        const S psi = sh.psi[t & 1][ps];
        m_sincos_n<1>(&psi, &sn[2], &cs[2]);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            sn[k] = prev_rs ? (S)0 : (k < 2 ? sh.sc[t & 1][k][ps] : sn[k]);
            cs[k] = prev_rs ? (S)1 : (k < 2 ? sh.sc[t & 1][2 + k][ps] : cs[k]);
        }
        const MotorMix mx = motor_mix(a_cur);
        if (t % kResetAhead == 0 && !nd_ok) {
            draw_next();
            nd_ok = true;
        }
        // physics_step_mixed's translational part, in its order
        const float thr = mx.thr;
        const S sph = sn[0], cph = cs[0], sth = sn[1], cth = cs[1], sps = sn[2], cps = cs[2];
        const S r02 = cps * sth * cph + sps * sph;
        const S r12 = sps * sth * cph - cps * sph;
        const S r22 = cth * cph;
        const S T = (S)thr;
        const S acc0 = (S)0 + (r02 * T) / (S)kMass;
        const S acc1 = (S)0 + (r12 * T) / (S)kMass;
        const S acc2 = (S)(-kG) + (r22 * T) / (S)kMass;
        st[F_VEL + 0] += acc0 * v.dt;
        st[F_VEL + 1] += acc1 * v.dt;
        st[F_VEL + 2] += acc2 * v.dt;
#pragma unroll
        for (int k = 0; k < 3; ++k) st[F_POS + k] += st[F_VEL + k] * v.dt;
        const S dx = st[F_POS + 0] - st[F_TGT + 0];
        const S dy = st[F_POS + 1] - st[F_TGT + 1];
        const S dz = st[F_POS + 2] - st[F_TGT + 2];
        const S dist2 = (dx * dx + dy * dy) + dz * dz;
        const S px = st[F_POS + 0], py = st[F_POS + 1], pz = st[F_POS + 2];
        const S pn2 = (px * px + py * py) + pz * pz;
        const bool crash = (pz < (S)0) || (pn2 > (S)2500);
        step += 1;
        const bool done = live && (crash || (step >= max_steps));
        const bool rs = done && io.auto_reset;
        const int so = t % kAbOut;
        // staged before the reset: the squared distance is of the pre-reset
        // position (otherwise the compiler sinks it below the reset branch and
        // keeps both states live, with a copy of each per step)
        sh.d2[so][ps] = dist2;
        sh.done[so][ps] = (uint8_t)done;
        if (rs) {
            // gym_reset_regs on the prepared state (a second reset within
            // the group draws here, as the reset itself would)
            step = 0;
            reset_any = true;
            if (!nd_ok) draw_next();
            ep_num += 1;
            vk.ep_num[i] = ep_num;
            eps = nx.eps;
            if (nx.bump) vk.eps[i] = eps;
            st[F_POS + 0] = nx.px;
            st[F_POS + 1] = nx.py;
            st[F_POS + 2] = (S)1.0;
#pragma unroll
            for (int k = F_VEL; k < F_VEL + 3; ++k) st[k] = (S)0;
            st[F_TGT + 0] = nx.tx;
            st[F_TGT + 1] = nx.ty;
            st[F_TGT + 2] = nx.tz;
            nd_ok = false;
        }
        prev_rs = rs;
        float *srow = &sh.obs[so][ps * OD];
        // a dead lane's (i >= n) row is staged but never stored (the memory
        // wave stores the live rows only), so it needs no zeroing
#pragma unroll
        for (int k = 0; k < F_EUL; ++k) srow[k] = (float)st[k];
#pragma unroll
        for (int k = 0; k < 3; ++k) srow[12 + k] = (float)(st[F_TGT + k] - st[F_POS + k]);
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // B_t
    }
    asm volatile("s_barrier" ::: "memory");                          // B_K
    if (live) {
#pragma unroll
        for (int k = 0; k < F_EUL; ++k) st_out(at(fp.p[k], i), st[k]);
        st_out(at(fp.step, i), step);
        if (reset_any) {
#pragma unroll
            for (int k = F_TGT; k < F_N; ++k) *at(fp.p[k], i) = st[k];
        }
    }
}


// Reset (all envs, or those with mask[i] != 0) and write every env's obs.
// mode: 0 Philox, 1 host uniforms, 2 constant 0.5.  `init` additionally
// clears ep_num / eps / monitor counters first (constructor).
template <typename S, int VAR>
__global__ __launch_bounds__(kBlock) void env_reset_kernel(EnvView<S> v,
                                                           const uint8_t *mask,
                                                           float *obs, int mode,
                                                           int init) {
    constexpr int OD = VAR == DR_VARIANT_GYM ? 15 : (VAR == DR_VARIANT_MOVING ? 18 : 12);
    __shared__ float4 sh4[kBlock * OD / 4];
    const int64_t base = (int64_t)blockIdx.x * kBlock;
    const int64_t i = base + threadIdx.x;
    float ob[OD];
    if (i < v.n) {
        if (init) {
            v.ep_num[i] = 0;
            v.eps[i] = 0.0;
            v.ep_ret[i] = 0.f;
            v.ep_len[i] = 0;
        }
        S st[F_N];
        float tvel[3] = {0.f, 0.f, 0.f};
        const bool doit = (mask == nullptr) || mask[i];
        if (doit) {
            if constexpr (VAR == DR_VARIANT_GYM) {
                gym_reset_regs(v, i, mode, st, v.ep_num[i], v.eps[i]);
            } else if constexpr (VAR == DR_VARIANT_MOVING) {
                float mp[9];
                moving_reset_regs(v, i, mode, st, &st[F_TGT], mp, v.ep_num[i], v.eps[i]);
#pragma unroll
                for (int k = 0; k < 9; ++k) v.mot[k * v.stride + i] = mp[k];
            } else {
                vec_reset_regs(st);
            }
#pragma unroll
            for (int k = 0; k < F_N; ++k) v.field(k)[i] = st[k];
            v.step[i] = 0;
        } else {
#pragma unroll
            for (int k = 0; k < F_N; ++k) st[k] = v.field(k)[i];
        }
        if constexpr (VAR == DR_VARIANT_MOVING) {
            // stored target = the centre; the obs sees the target at `step`
            S cen[3] = {st[F_TGT], st[F_TGT + 1], st[F_TGT + 2]};
            float mp[9];
#pragma unroll
            for (int k = 0; k < 9; ++k) mp[k] = v.mot[k * v.stride + i];
            moving_target(cen, mp, v.step[i], (float)v.dt, &st[F_TGT], tvel);
        }
        make_obs<S, OD>(st, ob, tvel);
    } else {
#pragma unroll
        for (int k = 0; k < OD; ++k) ob[k] = 0.f;
    }
    if (obs) store_obs_block<OD>(reinterpret_cast<float *>(sh4), ob, obs, base, v.n);
}

template <typename S>
__global__ void get_field_kernel(EnvView<S> v, int field, void *out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= v.n) return;
    if (field <= DR_FIELD_TARGET) {
        double *o = static_cast<double *>(out);
#pragma unroll
        for (int k = 0; k < 3; ++k) o[i * 3 + k] = (double)v.field(field * 3 + k)[i];
    } else if (field == DR_FIELD_STEP) {
        static_cast<int32_t *>(out)[i] = v.step[i];
    } else if (field == DR_FIELD_EP_NUM) {
        static_cast<int32_t *>(out)[i] = v.ep_num[i];
    } else if (field == DR_FIELD_EPS) {
        static_cast<double *>(out)[i] = v.eps[i];
    } else if (field == DR_FIELD_EP_RETURN) {
        static_cast<float *>(out)[i] = v.ep_ret[i];
    } else if (field == DR_FIELD_EP_LENGTH) {
        static_cast<int32_t *>(out)[i] = v.ep_len[i];
    } else if (field == DR_FIELD_MOTION) {
#pragma unroll
        for (int k = 0; k < 9; ++k) static_cast<float *>(out)[i * 9 + k] = v.mot[k * v.stride + i];
    }
}

template <typename S>
__global__ void gather_field_kernel(EnvView<S> v, int field, const int32_t *ids, int64_t k,
                                    void *out) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= k) return;
    const int64_t i = ids[j];
    if (i < 0 || i >= v.n) return;
    if (field <= DR_FIELD_TARGET) {
        double *o = static_cast<double *>(out);
#pragma unroll
        for (int c = 0; c < 3; ++c) o[j * 3 + c] = (double)v.field(field * 3 + c)[i];
    } else if (field == DR_FIELD_STEP) {
        static_cast<int32_t *>(out)[j] = v.step[i];
    } else if (field == DR_FIELD_EP_NUM) {
        static_cast<int32_t *>(out)[j] = v.ep_num[i];
    } else if (field == DR_FIELD_EPS) {
        static_cast<double *>(out)[j] = v.eps[i];
    } else if (field == DR_FIELD_EP_RETURN) {
        static_cast<float *>(out)[j] = v.ep_ret[i];
    } else if (field == DR_FIELD_EP_LENGTH) {
        static_cast<int32_t *>(out)[j] = v.ep_len[i];
    } else if (field == DR_FIELD_MOTION) {
#pragma unroll
        for (int c = 0; c < 9; ++c) static_cast<float *>(out)[j * 9 + c] = v.mot[c * v.stride + i];
    }
}

template <typename S>
__global__ void set_field_kernel(EnvView<S> v, int field, const void *in) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= v.n) return;
    if (field <= DR_FIELD_TARGET) {
        const double *p = static_cast<const double *>(in);
#pragma unroll
        for (int k = 0; k < 3; ++k) v.field(field * 3 + k)[i] = (S)p[i * 3 + k];
    } else if (field == DR_FIELD_STEP) {
        v.step[i] = static_cast<const int32_t *>(in)[i];
    } else if (field == DR_FIELD_EP_NUM) {
        v.ep_num[i] = static_cast<const int32_t *>(in)[i];
    } else if (field == DR_FIELD_EPS) {
        v.eps[i] = static_cast<const double *>(in)[i];
    } else if (field == DR_FIELD_EP_RETURN) {
        v.ep_ret[i] = static_cast<const float *>(in)[i];
    } else if (field == DR_FIELD_EP_LENGTH) {
        v.ep_len[i] = static_cast<const int32_t *>(in)[i];
    } else if (field == DR_FIELD_MOTION) {
#pragma unroll
        for (int k = 0; k < 9; ++k) v.mot[k * v.stride + i] = static_cast<const float *>(in)[i * 9 + k];
    }
}

__global__ __launch_bounds__(kBlock) void random_actions_kernel(
    int64_t n, uint32_t k0, uint32_t k1, int64_t env_off, uint64_t step,
    float lo, float span, float4 *out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint64_t gid = (uint64_t)(env_off + i);
    const u32x4 r = philox4x32_10(
        u32x4{(uint32_t)step, (uint32_t)(step >> 32), (uint32_t)gid,
              TAG_ACTION ^ (uint32_t)(gid >> 32)},
        k0, k1);
    out[i] = make_float4(lo + span * u01_f32(r.x), lo + span * u01_f32(r.y),
                         lo + span * u01_f32(r.z), lo + span * u01_f32(r.w));
}

}  // namespace
}  // namespace dr

// ============================================================================
// C ABI
// ============================================================================
using namespace dr;

struct dr_handle {
    dr_config cfg{};
    int64_t n = 0;
    int64_t stride = 0;
    int obs_dim = 15;
    // envs per wave of env_step_kernel: 64, or 32 (half-populated waves:
    // twice the waves in flight); chosen by batch size in dr_create
    int rpw = 64;
    bool nt_loads = false;  // nontemporal state loads (large batches)
    void *mem = nullptr;
    const double *host_u = nullptr;
    std::string err;
};

namespace dr {
static thread_local std::string g_err;
void set_global_error(const std::string &msg) { g_err = msg; }
const char *global_error() { return g_err.c_str(); }
}  // namespace dr

namespace {

int fail(dr_handle *h, int code, const std::string &msg) {
    if (h)
        h->err = msg;
    else
        set_global_error(msg);
    return code;
}

template <typename S>
EnvView<S> view_of(const dr_handle *h) {
    EnvView<S> v{};
    char *m = static_cast<char *>(h->mem);
    const int64_t sp = h->stride;
    v.f = reinterpret_cast<S *>(m);
    v.stride = sp;
    v.eps = reinterpret_cast<double *>(m + Layout<S>::eps(sp));
    v.step = reinterpret_cast<int32_t *>(m + Layout<S>::step(sp));
    v.ep_num = reinterpret_cast<int32_t *>(m + Layout<S>::ep_num(sp));
    v.ep_ret = reinterpret_cast<float *>(m + Layout<S>::ep_ret(sp));
    v.ep_len = reinterpret_cast<int32_t *>(m + Layout<S>::ep_len(sp));
    v.mot = h->cfg.variant == DR_VARIANT_MOVING ? reinterpret_cast<float *>(m + Layout<S>::mot(sp))
                                                 : nullptr;
    v.n = h->n;
    v.env_id_offset = h->cfg.env_id_offset;
    v.host_u = h->host_u;
    v.seed_lo = (uint32_t)h->cfg.seed;
    v.seed_hi = (uint32_t)(h->cfg.seed >> 32);
    v.max_steps = h->cfg.max_steps;
    v.dt = (S)h->cfg.dt;
    return v;
}

size_t state_bytes(int64_t stride, int dtype, int variant) {
    const size_t s = dtype == DR_STATE_F64 ? sizeof(double) : sizeof(float);
    const size_t mot = variant == DR_VARIANT_MOVING ? 9 * sizeof(float) : 0;
    return (size_t)F_N * stride * s + (size_t)stride * (8 + 4 + 4 + 4 + 4 + mot);
}

inline hipStream_t as_stream(void *s) { return static_cast<hipStream_t>(s); }

template <typename S, int VAR>
int launch_reset(dr_handle *h, const uint8_t *mask, float *obs, int mode,
                 int init, hipStream_t st) {
    EnvView<S> v = view_of<S>(h);
    hipLaunchKernelGGL((env_reset_kernel<S, VAR>), dim3(grid_for(h->n)),
                       dim3(kBlock), 0, st, v, mask, obs, mode, init);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return fail(h, DR_ERR_HIP, std::string("env_reset_kernel: ") + hipGetErrorString(e));
    return DR_OK;
}

int dispatch_reset(dr_handle *h, const uint8_t *mask, float *obs, int mode,
                   int init, hipStream_t st) {
    const bool f64 = h->cfg.state_dtype == DR_STATE_F64;
    if (h->cfg.variant == DR_VARIANT_GYM)
        return f64 ? launch_reset<double, DR_VARIANT_GYM>(h, mask, obs, mode, init, st)
                   : launch_reset<float, DR_VARIANT_GYM>(h, mask, obs, mode, init, st);
    if (h->cfg.variant == DR_VARIANT_MOVING)
        return f64 ? launch_reset<double, DR_VARIANT_MOVING>(h, mask, obs, mode, init, st)
                   : launch_reset<float, DR_VARIANT_MOVING>(h, mask, obs, mode, init, st);
    return f64 ? launch_reset<double, DR_VARIANT_VECTORIZED>(h, mask, obs, mode, init, st)
               : launch_reset<float, DR_VARIANT_VECTORIZED>(h, mask, obs, mode, init, st);
}

template <typename S, int VAR, bool MON>
int launch_step(dr_handle *h, const StepIO &io, hipStream_t st) {
    EnvView<S> v = view_of<S>(h);
    FieldPtrs<S> fp;
    for (int k = 0; k < F_N; ++k) fp.p[k] = v.field(k);
    fp.step = v.step;
    fp.ep_num = v.ep_num;
    fp.eps = v.eps;
    bool launched = false;
    if (!launched && VAR != DR_VARIANT_VECTORIZED && v.host_u) {   // parity mode
        if (h->rpw == 32)
            hipLaunchKernelGGL((env_step_kernel<S, VAR, MON, 32, true, false>),
                               dim3(grid_for(h->n, DR_ENV_WPB * 32)), dim3(kEnvBlock), 0, st,
                               v, io, fp);
        else
            hipLaunchKernelGGL((env_step_kernel<S, VAR, MON, 64, true, false>),
                               dim3(grid_for(h->n, DR_ENV_WPB * 64)), dim3(kEnvBlock), 0, st,
                               v, io, fp);
        launched = true;
    }
    if (!launched) {
        const dim3 g64(grid_for(h->n, DR_ENV_WPB * 64)), g32(grid_for(h->n, DR_ENV_WPB * 32));
        switch (h->rpw * 2 + (int)h->nt_loads) {
            case 64:
                hipLaunchKernelGGL((env_step_kernel<S, VAR, MON, 32, false, false>), g32,
                                   dim3(kEnvBlock), 0, st, v, io, fp);
                break;
            case 65:
                hipLaunchKernelGGL((env_step_kernel<S, VAR, MON, 32, false, true>), g32,
                                   dim3(kEnvBlock), 0, st, v, io, fp);
                break;
            case 129:
                hipLaunchKernelGGL((env_step_kernel<S, VAR, MON, 64, false, true>), g64,
                                   dim3(kEnvBlock), 0, st, v, io, fp);
                break;
            default:
                hipLaunchKernelGGL((env_step_kernel<S, VAR, MON, 64, false, false>), g64,
                                   dim3(kEnvBlock), 0, st, v, io, fp);
        }
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return fail(h, DR_ERR_HIP, std::string("env_step_kernel: ") + hipGetErrorString(e));
    return DR_OK;
}

template <bool MON>
int dispatch_step(dr_handle *h, const StepIO &io, hipStream_t st) {
    const bool f64 = h->cfg.state_dtype == DR_STATE_F64;
    if (h->cfg.variant == DR_VARIANT_GYM)
        return f64 ? launch_step<double, DR_VARIANT_GYM, MON>(h, io, st)
                   : launch_step<float, DR_VARIANT_GYM, MON>(h, io, st);
    if (h->cfg.variant == DR_VARIANT_MOVING)
        return f64 ? launch_step<double, DR_VARIANT_MOVING, MON>(h, io, st)
                   : launch_step<float, DR_VARIANT_MOVING, MON>(h, io, st);
    return f64 ? launch_step<double, DR_VARIANT_VECTORIZED, MON>(h, io, st)
               : launch_step<float, DR_VARIANT_VECTORIZED, MON>(h, io, st);
}

template <typename S, int VAR, bool GEN>
int launch_rollout(dr_handle *h, const RolloutIO &io, hipStream_t st, hipEvent_t e0,
                   hipEvent_t e1) {
    EnvView<S> v = view_of<S>(h);
    FieldPtrs<S> fp;
    for (int k = 0; k < F_N; ++k) fp.p[k] = v.field(k);
    fp.step = v.step;
    fp.ep_num = v.ep_num;
    fp.eps = v.eps;
    // The warp-specialised form while its grid is at most one block per CU
    // (n <= 256 x CUs: 65,536 envs on MI355X), where one physics wave per
    // SIMD has nothing else to overlap with; above that the one-role kernel
    // already runs two or more waves per SIMD, and the warp-specialised one
    // measured equal (gym, 131,072 / 1,048,576 envs) or slower (in-kernel
    // policy at 2^20; the moving variant, whose 175 VGPRs fit one 512-thread
    // block per CU).  DRONERL_ROLLOUT_WS=0 / 1 forces either (A/B).
    static const int ws_env = [] {
        const char *r = std::getenv("DRONERL_ROLLOUT_WS");
        return r ? (std::atoi(r) != 0 ? 1 : 0) : -1;
    }();
    const bool ws = ws_env >= 0 ? ws_env == 1 : h->n <= (int64_t)kWsEnvs * device_cu_count();
    // with events: hipExtLaunchKernelGGL binds them to the dispatch packet's
    // own start / end timestamps (no extra packets in the queue)
    if (ws) {
        if constexpr (VAR == DR_VARIANT_GYM && !GEN) {
            // the split-physics form of the warp-specialised kernel (gym
            // variant, actions read from HBM; with the in-kernel policy its
            // memory waves' Philox draws share the SIMD with two physics
            // waves and it measured slower, so GEN keeps the one-physics-wave
            // form)
            const dim3 grid(grid_for(h->n, kWsEnvs)), block(kAbThreads);
            if (e0 || e1)
                hipExtLaunchKernelGGL((env_rollout_ab_kernel<S, GEN>), grid, block, 0, st, e0,
                                      e1, 0, v, io, fp);
            else
                hipLaunchKernelGGL((env_rollout_ab_kernel<S, GEN>), grid, block, 0, st, v, io,
                                   fp);
        } else {
            const dim3 grid(grid_for(h->n, kWsEnvs)), block(kWsThreads);
            if (e0 || e1)
                hipExtLaunchKernelGGL((env_rollout_ws_kernel<S, VAR, GEN>), grid, block, 0, st,
                                      e0, e1, 0, v, io, fp);
            else
                hipLaunchKernelGGL((env_rollout_ws_kernel<S, VAR, GEN>), grid, block, 0, st, v,
                                   io, fp);
        }
    } else {
        const dim3 grid(grid_for(h->n, DR_ENV_WPB * 64)), block(kEnvBlock);
        if (e0 || e1)
            hipExtLaunchKernelGGL((env_rollout_kernel<S, VAR, 64, GEN>), grid, block, 0, st, e0,
                                  e1, 0, v, io, fp);
        else
            hipLaunchKernelGGL((env_rollout_kernel<S, VAR, 64, GEN>), grid, block, 0, st, v, io,
                               fp);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return fail(h, DR_ERR_HIP, std::string("env_rollout_kernel: ") + hipGetErrorString(e));
    return DR_OK;
}

template <bool GEN>
int dispatch_rollout(dr_handle *h, const RolloutIO &io, hipStream_t st, hipEvent_t e0,
                     hipEvent_t e1) {
    const bool f64 = h->cfg.state_dtype == DR_STATE_F64;
    if (h->cfg.variant == DR_VARIANT_GYM)
        return f64 ? launch_rollout<double, DR_VARIANT_GYM, GEN>(h, io, st, e0, e1)
                   : launch_rollout<float, DR_VARIANT_GYM, GEN>(h, io, st, e0, e1);
    if (h->cfg.variant == DR_VARIANT_MOVING)
        return f64 ? launch_rollout<double, DR_VARIANT_MOVING, GEN>(h, io, st, e0, e1)
                   : launch_rollout<float, DR_VARIANT_MOVING, GEN>(h, io, st, e0, e1);
    return f64 ? launch_rollout<double, DR_VARIANT_VECTORIZED, GEN>(h, io, st, e0, e1)
               : launch_rollout<float, DR_VARIANT_VECTORIZED, GEN>(h, io, st, e0, e1);
}

int check_rng(dr_handle *h) {
    if (h->cfg.rng_mode == DR_RNG_HOST_UNIFORMS && h->host_u == nullptr &&
        h->cfg.variant != DR_VARIANT_VECTORIZED)
        return fail(h, DR_ERR_INVALID,
                    "rng_mode DR_RNG_HOST_UNIFORMS: call dr_set_reset_uniforms first");
    return DR_OK;
}

}  // namespace

extern "C" {

int dr_abi_version(void) { return DR_ABI_VERSION; }

int dr_create(const dr_config *cfg_in, dr_handle **out) {
    if (!cfg_in || !out) return fail(nullptr, DR_ERR_INVALID, "dr_create: null argument");
    *out = nullptr;
    dr_config cfg = *cfg_in;
    if (cfg.num_envs < 1) return fail(nullptr, DR_ERR_INVALID, "dr_create: num_envs must be >= 1");
    if (cfg.variant != DR_VARIANT_GYM && cfg.variant != DR_VARIANT_VECTORIZED &&
        cfg.variant != DR_VARIANT_MOVING)
        return fail(nullptr, DR_ERR_INVALID, "dr_create: unknown variant");
    if (cfg.state_dtype != DR_STATE_F64 && cfg.state_dtype != DR_STATE_F32)
        return fail(nullptr, DR_ERR_INVALID, "dr_create: unknown state_dtype");
    if (cfg.rng_mode != DR_RNG_PHILOX && cfg.rng_mode != DR_RNG_HOST_UNIFORMS)
        return fail(nullptr, DR_ERR_INVALID, "dr_create: unknown rng_mode");
    // 32-bit per-array byte offsets in the step kernel (float4 actions:
    // 16 B x 2^28 = 4 GiB); shard larger batches over several handles
    if (cfg.num_envs > (int64_t)1 << 28)
        return fail(nullptr, DR_ERR_INVALID, "dr_create: num_envs above 2^28 per handle");
    if (cfg.max_steps == 0) cfg.max_steps = cfg.variant == DR_VARIANT_VECTORIZED ? 1000 : 200;
    if (cfg.max_steps < 0) return fail(nullptr, DR_ERR_INVALID, "dr_create: max_steps < 0");
    if (cfg.dt == 0.0) cfg.dt = kDt;
    if (cfg.variant == DR_VARIANT_VECTORIZED) cfg.auto_reset = 0;

    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(nullptr, DR_ERR_HIP, "dr_create: no HIP device available");
    if (cfg.device < 0 || cfg.device >= ndev)
        return fail(nullptr, DR_ERR_INVALID, "dr_create: device ordinal out of range");

    dr_handle *h = new (std::nothrow) dr_handle();
    if (!h) return fail(nullptr, DR_ERR_NOMEM, "dr_create: host allocation failed");
    h->cfg = cfg;
    h->n = cfg.num_envs;
    // SoA arrays are `stride` elements apart.  A pure power-of-two spacing
    // would put the 17 concurrently streamed arrays at congruent addresses
    // (same HBM channel bits); DR_STRIDE_PAD elements of skew break that.
    h->stride = (cfg.num_envs + 63) / 64 * 64 + DR_STRIDE_PAD;
    h->obs_dim = cfg.variant == DR_VARIANT_GYM ? 15 : (cfg.variant == DR_VARIANT_MOVING ? 18 : 12);
    // Launch form by batch size, from the measured sweep
    // (scripts/micro/ab_sweep.sh, profiles/r01_env_launch_sweep.txt):
    // [0, 384k) 64 rows/wave; [384k, 1.5M) 32 + nontemporal state loads;
    // [1.5M, 3M) 32; [3M, ...) 64 + nontemporal state loads.
    // The moving variant (9 more f32 arrays per env) and the f32 state mode
    // have sweeps of their own: moving always 64 rows/wave, nontemporal
    // state loads from 384k envs up; f32 state 64 rows/wave with plain loads
    // below 3M envs, 32 + nontemporal loads from 3M up.
    {
        const int64_t n = cfg.num_envs, k = (int64_t)1 << 10;
        if (cfg.variant == DR_VARIANT_MOVING) {
            h->rpw = 64;
            h->nt_loads = n >= 384 * k;
        } else if (cfg.state_dtype == DR_STATE_F32) {
            h->rpw = n >= 3072 * k ? 32 : 64;
            h->nt_loads = n >= 3072 * k;
        } else {
            h->rpw = (n >= 384 * k && n < 3072 * k) ? 32 : 64;
            h->nt_loads = (n >= 384 * k && n < 1536 * k) || n >= 3072 * k;
        }
    }
    if (const char *r = std::getenv("DRONERL_ROWS_PER_WAVE")) {
        const int v = std::atoi(r);
        if (v == 32 || v == 64) h->rpw = v;
    }
    if (const char *r = std::getenv("DRONERL_NT_LOADS")) h->nt_loads = std::atoi(r) != 0;

    DeviceGuard g(cfg.device);
    const size_t bytes = state_bytes(h->stride, cfg.state_dtype, cfg.variant);
    hipError_t e = hipMalloc(&h->mem, bytes);
    if (e != hipSuccess) {
        delete h;
        return fail(nullptr, DR_ERR_NOMEM, std::string("dr_create: hipMalloc: ") + hipGetErrorString(e));
    }
    // Constructor reset (drone.py:46): ep_num 0 -> 1.
    const int mode = cfg.rng_mode == DR_RNG_PHILOX ? 0 : 2;
    int rc = dispatch_reset(h, nullptr, nullptr, mode, 1, nullptr);
    if (rc == DR_OK) {
        e = hipDeviceSynchronize();
        if (e != hipSuccess) rc = fail(h, DR_ERR_HIP, hipGetErrorString(e));
    }
    if (rc != DR_OK) {
        set_global_error(h->err);
        (void)hipFree(h->mem);
        delete h;
        return rc;
    }
    *out = h;
    return DR_OK;
}

int dr_destroy(dr_handle *h) {
    if (!h) return DR_OK;
    DeviceGuard g(h->cfg.device);
    if (h->mem) {
        // The caller's streams may still use the state: drain first.
        (void)hipDeviceSynchronize();
        (void)hipFree(h->mem);
    }
    delete h;
    return DR_OK;
}

int64_t dr_num_envs(const dr_handle *h) { return h ? h->n : -1; }
int dr_obs_dim(const dr_handle *h) { return h ? h->obs_dim : -1; }

int dr_reset(dr_handle *h, float *obs_out, void *stream) {
    if (!h) return fail(nullptr, DR_ERR_INVALID, "dr_reset: null handle");
    if (!obs_out) return fail(h, DR_ERR_INVALID, "dr_reset: obs_out is null");
    int rc = check_rng(h);
    if (rc) return rc;
    DeviceGuard g(h->cfg.device);
    return dispatch_reset(h, nullptr, obs_out, h->host_u ? 1 : 0, 0, as_stream(stream));
}

int dr_reset_masked(dr_handle *h, const uint8_t *mask, float *obs_out, void *stream) {
    if (!h) return fail(nullptr, DR_ERR_INVALID, "dr_reset_masked: null handle");
    if (!mask) return fail(h, DR_ERR_INVALID, "dr_reset_masked: mask is null");
    if (h->cfg.variant == DR_VARIANT_VECTORIZED)
        return fail(h, DR_ERR_UNSUPPORTED, "dr_reset_masked: vectorized variant resets globally");
    int rc = check_rng(h);
    if (rc) return rc;
    DeviceGuard g(h->cfg.device);
    return dispatch_reset(h, mask, obs_out, h->host_u ? 1 : 0, 0, as_stream(stream));
}

static int step_common(dr_handle *h, const float *actions, float *obs_out,
                       float *rew_out, uint8_t *done_out, float *term_obs_out,
                       float *ep_ret_out, int32_t *ep_len_out, bool mon,
                       void *stream, uint8_t *trunc_out = nullptr) {
    if (!h) return fail(nullptr, DR_ERR_INVALID, "dr_step: null handle");
    if (!actions || !obs_out || !rew_out || !done_out)
        return fail(h, DR_ERR_INVALID, "dr_step: actions/obs/rew/done must be non-null");
    if (((uintptr_t)actions) & 15)
        return fail(h, DR_ERR_INVALID, "dr_step: actions must be 16-byte aligned");
    if (mon && (!ep_ret_out || !ep_len_out))
        return fail(h, DR_ERR_INVALID, "dr_step_monitored: episode outputs must be non-null");
    if (h->cfg.auto_reset) {
        int rc = check_rng(h);
        if (rc) return rc;
    }
    StepIO io{actions, obs_out, rew_out, done_out, term_obs_out, ep_ret_out,
              ep_len_out, h->cfg.auto_reset, trunc_out};
    DeviceGuard g(h->cfg.device);
    return mon ? dispatch_step<true>(h, io, as_stream(stream))
               : dispatch_step<false>(h, io, as_stream(stream));
}

int dr_step(dr_handle *h, const float *actions, float *obs_out, float *rew_out,
            uint8_t *done_out, float *terminal_obs_out, void *stream) {
    return step_common(h, actions, obs_out, rew_out, done_out, terminal_obs_out,
                       nullptr, nullptr, false, stream);
}

int dr_step_monitored(dr_handle *h, const float *actions, float *obs_out,
                      float *rew_out, uint8_t *done_out, float *terminal_obs_out,
                      float *ep_return_out, int32_t *ep_length_out, void *stream) {
    return step_common(h, actions, obs_out, rew_out, done_out, terminal_obs_out,
                       ep_return_out, ep_length_out, true, stream);
}

int dr_step_monitored_trunc(dr_handle *h, const float *actions, float *obs_out,
                            float *rew_out, uint8_t *done_out, float *terminal_obs_out,
                            float *ep_return_out, int32_t *ep_length_out,
                            uint8_t *truncated_out, void *stream) {
    if (!truncated_out)
        return fail(h, DR_ERR_INVALID, "dr_step_monitored_trunc: truncated_out is null");
    return step_common(h, actions, obs_out, rew_out, done_out, terminal_obs_out,
                       ep_return_out, ep_length_out, true, stream, truncated_out);
}

static int rollout_common(dr_handle *h, int32_t k, RolloutIO io, bool gen, void *stream,
                          void *start_event = nullptr, void *stop_event = nullptr) {
    if (!h) return fail(nullptr, DR_ERR_INVALID, "dr_rollout: null handle");
    if (k < 0) return fail(h, DR_ERR_INVALID, "dr_rollout: k < 0");
    if (!io.obs || !io.rew || !io.done)
        return fail(h, DR_ERR_INVALID, "dr_rollout: obs/rew/done must be non-null");
    if (!gen && !io.actions) return fail(h, DR_ERR_INVALID, "dr_rollout: actions is null");
    if ((((uintptr_t)io.actions) & 15) || (((uintptr_t)io.act_out) & 15))
        return fail(h, DR_ERR_INVALID, "dr_rollout: actions must be 16-byte aligned");
    // per-step output offsets t * n are formed in 64 bits, the per-env
    // offset in 32 (as dr_step); K * n rows must still fit one allocation
    if ((int64_t)k * h->n > ((int64_t)1 << 31))
        return fail(h, DR_ERR_INVALID, "dr_rollout: k * num_envs above 2^31");
    if (h->cfg.variant != DR_VARIANT_VECTORIZED && h->cfg.auto_reset &&
        h->cfg.rng_mode != DR_RNG_PHILOX)
        return fail(h, DR_ERR_UNSUPPORTED,
                    "dr_rollout: host-supplied reset uniforms change per step; use dr_step");
    if (k == 0) return DR_OK;
    io.k = k;
    io.auto_reset = h->cfg.auto_reset;
    DeviceGuard g(h->cfg.device);
    const hipEvent_t e0 = static_cast<hipEvent_t>(start_event);
    const hipEvent_t e1 = static_cast<hipEvent_t>(stop_event);
    return gen ? dispatch_rollout<true>(h, io, as_stream(stream), e0, e1)
               : dispatch_rollout<false>(h, io, as_stream(stream), e0, e1);
}

int dr_rollout(dr_handle *h, int32_t k, const float *actions, float *obs_out, float *rew_out,
               uint8_t *done_out, void *stream) {
    RolloutIO io{};
    io.actions = actions;
    io.obs = obs_out;
    io.rew = rew_out;
    io.done = done_out;
    return rollout_common(h, k, io, false, stream);
}

int dr_rollout_timed(dr_handle *h, int32_t k, const float *actions, float *obs_out,
                     float *rew_out, uint8_t *done_out, void *stream, void *start_event,
                     void *stop_event) {
    RolloutIO io{};
    io.actions = actions;
    io.obs = obs_out;
    io.rew = rew_out;
    io.done = done_out;
    return rollout_common(h, k, io, false, stream, start_event, stop_event);
}

int dr_rollout_random(dr_handle *h, int32_t k, uint64_t action_seed, int64_t action_step0,
                      float lo, float hi, float *actions_out, float *obs_out, float *rew_out,
                      uint8_t *done_out, void *stream) {
    RolloutIO io{};
    io.act_out = actions_out;
    io.obs = obs_out;
    io.rew = rew_out;
    io.done = done_out;
    io.a_k0 = (uint32_t)action_seed;
    io.a_k1 = (uint32_t)(action_seed >> 32);
    io.a_step0 = (uint64_t)action_step0;
    io.a_lo = lo;
    io.a_span = hi - lo;
    return rollout_common(h, k, io, true, stream);
}

int dr_get_state(dr_handle *h, int field, void *out, void *stream) {
    if (!h) return fail(nullptr, DR_ERR_INVALID, "dr_get_state: null handle");
    if (!out) return fail(h, DR_ERR_INVALID, "dr_get_state: out is null");
    if (field < DR_FIELD_POS || field > DR_FIELD_MOTION)
        return fail(h, DR_ERR_INVALID, "dr_get_state: unknown field");
    if (field == DR_FIELD_MOTION && h->cfg.variant != DR_VARIANT_MOVING)
        return fail(h, DR_ERR_INVALID, "dr_get_state: motion exists only for DR_VARIANT_MOVING");
    DeviceGuard g(h->cfg.device);
    if (h->cfg.state_dtype == DR_STATE_F64)
        hipLaunchKernelGGL(get_field_kernel<double>, dim3(grid_for(h->n)), dim3(kBlock), 0,
                           as_stream(stream), view_of<double>(h), field, out);
    else
        hipLaunchKernelGGL(get_field_kernel<float>, dim3(grid_for(h->n)), dim3(kBlock), 0,
                           as_stream(stream), view_of<float>(h), field, out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(h, DR_ERR_HIP, std::string("get_field: ") + hipGetErrorString(e));
    return DR_OK;
}

int dr_gather_state(dr_handle *h, int field, const int32_t *env_ids, int64_t k, void *out,
                    void *stream) {
    if (!h) return fail(nullptr, DR_ERR_INVALID, "dr_gather_state: null handle");
    if (!env_ids || !out || k < 0) return fail(h, DR_ERR_INVALID, "dr_gather_state: bad arguments");
    if (field < DR_FIELD_POS || field > DR_FIELD_MOTION)
        return fail(h, DR_ERR_INVALID, "dr_gather_state: unknown field");
    if (field == DR_FIELD_MOTION && h->cfg.variant != DR_VARIANT_MOVING)
        return fail(h, DR_ERR_INVALID, "dr_gather_state: motion exists only for DR_VARIANT_MOVING");
    if (k == 0) return DR_OK;
    DeviceGuard g(h->cfg.device);
    if (h->cfg.state_dtype == DR_STATE_F64)
        hipLaunchKernelGGL(gather_field_kernel<double>, dim3(grid_for(k)), dim3(kBlock), 0,
                           as_stream(stream), view_of<double>(h), field, env_ids, k, out);
    else
        hipLaunchKernelGGL(gather_field_kernel<float>, dim3(grid_for(k)), dim3(kBlock), 0,
                           as_stream(stream), view_of<float>(h), field, env_ids, k, out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(h, DR_ERR_HIP, std::string("gather_field: ") + hipGetErrorString(e));
    return DR_OK;
}

int dr_set_state(dr_handle *h, int field, const void *in, void *stream) {
    if (!h) return fail(nullptr, DR_ERR_INVALID, "dr_set_state: null handle");
    if (!in) return fail(h, DR_ERR_INVALID, "dr_set_state: in is null");
    if (field < DR_FIELD_POS || field > DR_FIELD_MOTION)
        return fail(h, DR_ERR_INVALID, "dr_set_state: unknown field");
    if (field == DR_FIELD_MOTION && h->cfg.variant != DR_VARIANT_MOVING)
        return fail(h, DR_ERR_INVALID, "dr_set_state: motion exists only for DR_VARIANT_MOVING");
    DeviceGuard g(h->cfg.device);
    if (h->cfg.state_dtype == DR_STATE_F64)
        hipLaunchKernelGGL(set_field_kernel<double>, dim3(grid_for(h->n)), dim3(kBlock), 0,
                           as_stream(stream), view_of<double>(h), field, in);
    else
        hipLaunchKernelGGL(set_field_kernel<float>, dim3(grid_for(h->n)), dim3(kBlock), 0,
                           as_stream(stream), view_of<float>(h), field, in);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(h, DR_ERR_HIP, std::string("set_field: ") + hipGetErrorString(e));
    return DR_OK;
}

int dr_set_reset_uniforms(dr_handle *h, const double *u_dev) {
    if (!h) return fail(nullptr, DR_ERR_INVALID, "dr_set_reset_uniforms: null handle");
    if (h->cfg.rng_mode != DR_RNG_HOST_UNIFORMS)
        return fail(h, DR_ERR_INVALID, "dr_set_reset_uniforms: handle uses DR_RNG_PHILOX");
    h->host_u = u_dev;
    return DR_OK;
}

int dr_set_seed(dr_handle *h, uint64_t seed) {
    if (!h) return fail(nullptr, DR_ERR_INVALID, "dr_set_seed: null handle");
    h->cfg.seed = seed;
    return DR_OK;
}

int dr_random_actions(int64_t n, uint64_t seed, int64_t env_id_offset,
                      int64_t step, float lo, float hi, float *out, void *stream) {
    if (n < 0 || !out) return fail(nullptr, DR_ERR_INVALID, "dr_random_actions: bad arguments");
    if (((uintptr_t)out) & 15) return fail(nullptr, DR_ERR_INVALID, "dr_random_actions: out must be 16-byte aligned");
    if (n == 0) return DR_OK;
    hipLaunchKernelGGL(random_actions_kernel, dim3(grid_for(n)), dim3(kBlock), 0,
                       as_stream(stream), n, (uint32_t)seed, (uint32_t)(seed >> 32),
                       env_id_offset, (uint64_t)step, lo, hi - lo,
                       reinterpret_cast<float4 *>(out));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return fail(nullptr, DR_ERR_HIP, std::string("random_actions: ") + hipGetErrorString(e));
    return DR_OK;
}

#if DR_STAMPS
int dr_diag_stamps(void *host_out, size_t bytes) {
    hipError_t e = hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_stamps), bytes, 0,
                                       hipMemcpyDeviceToHost);
    return e == hipSuccess ? DR_OK : DR_ERR_HIP;
}
#endif

const char *dr_last_error(const dr_handle *h) {
    return h ? h->err.c_str() : global_error();
}

}  // extern "C"
