/*
 * oracle/ppo_ref.c -- CPU restatements used to check the PPO-side kernels.
 *
 * TEST INFRASTRUCTURE ONLY (see drone_ref.c).  Contents:
 *   oracle_philox4x32_10   Philox4x32-10 (Salmon et al. SC'11), checked
 *                          against the Random123 known-answer vectors in
 *                          tests/test_oracle.py; the GPU generator must match
 *                          it bit for bit.
 *   oracle_gae_f32         stable-baselines3 RolloutBuffer
 *                          .compute_returns_and_advantage in f32 with numpy's
 *                          NEP-50 rounding (SB3 is not vendored
 *                          in the reference -> "parity unpinned"; call site
 *                          /root/reference/train.py:63).
 */
#include <stdint.h>

void oracle_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2],
                          uint32_t out[4]) {
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0;
        c1 = lo1;
        c2 = n2;
        c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0;
    out[1] = c1;
    out[2] = c2;
    out[3] = c3;
}

/* rewards/values/starts (T,N) time-major; last_values/last_dones (N). */
void oracle_gae_f32(int64_t T, int64_t N, const float *rew, const float *val,
                    const uint8_t *starts, const float *last_val,
                    const uint8_t *last_done, double gamma, double lam,
                    float *adv, float *ret) {
    const float g = (float)gamma;
    const float gl = (float)(gamma * lam);
    for (int64_t n = 0; n < N; ++n) {
        float last = 0.0f;
        for (int64_t t = T - 1; t >= 0; --t) {
            float nnt, nv;
            if (t == T - 1) {
                nnt = 1.0f - (float)last_done[n];
                nv = last_val[n];
            } else {
                nnt = 1.0f - (float)starts[(t + 1) * N + n];
                nv = val[(t + 1) * N + n];
            }
            const int64_t o = t * N + n;
            float delta = (rew[o] + (g * nv) * nnt) - val[o];
            last = delta + (gl * nnt) * last;
            adv[o] = last;
            ret[o] = last + val[o];
        }
    }
}
